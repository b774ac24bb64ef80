// nwk_gotoh.hip -- nw_align_gotoh: the affine-gap variant (the
// build defines it, oracle/nw_oracle.c nwo_pair_affine restates it) as
// bit-sliced thermometer planes, one bit per DP cell.
//
// The step (nwk_gotoh_planes.h) works in G-space (ge subtracted per step)
// relative to G_diag: a difference v / h in [-go, go + 2 ge] is held as
// 2 (go + ge) planes, a gap offset min(e, go) / min(f, go) as go planes, and
// every output plane is an OR of (plane AND NOT plane) terms -- one
// v_bitop3_b32 per term for 32 cells.  C5's scoring (pxy 3, go 3, ge 1) is
// ~175 VALU per wave-step for 32 cells against nw_align_pka's ~7.4 per cell.
//
// Layout (nw_align_bits' anti-diagonal bands): a wave owns a 2048-row band;
// bit b of lane t is row R0 + 32 t + b + 1 at (1-based) column s - 32 t - b at
// step s.  A cell's left neighbour is the same bit one step earlier; its upper
// neighbour is the bit below one step earlier (a 1-bit funnel shift with lane
// t - 1's top bit through DPP wave_shr:1).  Lane 0 bit 0 reads the band
// above's last row: that row (lane 63 bit 31, column s - 2047) goes to an LDS
// ring each step, and at the end of every 32-step segment its next complete
// 32 columns are packed by ballot into one word per h / f plane and published
// as self-tagged granules {epoch:32 | word:32}, which the band below polls
// with atomic reads (the coherence point: a plain load can hit a stale line in
// the reading XCD's L2) and stages in LDS as the DPP fill-in of lane 0.
//
// Storage: four words per lane and step -- D (X == S: the diagonal candidate
// is the minimum), F-source (f == 0: H came from F), E-extend (eL < go) and
// F-extend (fU < go), exactly the decisions of nwo_pair_affine's walk
// (oracle/nw_oracle.c:240-256) -- in 4-step blocks of 4 KB, one 8-byte store
// per word every two steps (512 B contiguous across the wave), only the
// blocks within bits_w columns of the diagonal when windowed.
//
// Traceback: the wave that finishes a pair's last band walks the three-state
// walk from (m, n) on the scalar unit over tiles of 128 steps x 64 rows held
// in VGPRs (lane L = steps 64 u + L and 64 u + 64 + L, two row-lanes x four
// words), the next tile along the diagonal prefetched, one v_readlane per word
// per move; a gap's first column is emitted as 'u' / 'l'
// (the finalize charges go + ge there, ge elsewhere).  A cell outside the
// stored blocks flags the pair for a wider re-run (FillArgs::retry).
#include "nwk_bits_dev.h"
#include "nwk_gotoh_planes.h"

namespace nwk {
namespace {

using namespace gotoh_bits;

template <class C>
struct GGeo {
  static constexpr int NQ1 = C::NQ > 0 ? C::NQ : 1;  // gap-offset planes held (go = 0: one dummy)
  static constexpr int kPl = C::NV + C::NQ;          // planes handed down: h, then f
  static constexpr int kPs = (kPl + 3) & ~3;         // LDS / granule stride per column / chunk
  static_assert(kPl <= 64, "one granule per lane");
};

// At least NWK_GOTOH_WPE waves per SIMD: the step is issue-bound and a lone
// wave issues a VALU op only every ~8 cycles, so occupancy is
// what fills the SIMD.  5 (96 VGPRs) since round 6: with the segment loop
// split in three the fill loops do not spill at 96 (the spills left are per
// band task), C5 6.58-6.63k -> 6.85k GCUPS; 4 waves take 112 VGPRs.
#ifndef NWK_GOTOH_WPE
#define NWK_GOTOH_WPE 5
#endif
#ifndef NWK_GOTOH_STEPSTORE
#define NWK_GOTOH_STEPSTORE 0
#endif

// Waits until lanes 0 .. kPl - 1 hold granules tagged `epoch` (v: their last
// reads).  A chunk's granules are one store instruction of the producing wave,
// so only the last plane's lane polls -- one atomic read (at the coherence
// point) per try, backing off 0.1 -> 1.6 us -- and once it has arrived every
// stale lane re-reads.  (Every lane re-reading per try made the polls ~30% of
// the launch's WRITE_SIZE: an atomic read counts as a write.)  Bounded like
// bits_wait: ~4 s of wall time, or another wave's failure.
template <int kPl>
__device__ __noinline__ u64 gran_wait(const u64* p, unsigned epoch, u64 v, unsigned* err) {
  const int lane = threadIdx.x & 63;
  const bool mine = lane < kPl;
  const u64 t0 = __builtin_amdgcn_s_memrealtime();
  int nap = 1;
  for (;;) {
    if (__all(!mine || (unsigned)(v >> 32) == epoch)) return v;
    if (__builtin_amdgcn_readfirstlane(__hip_atomic_load((gu32*)err, BITS_RLX)) != 0u) return 0;
    if (__builtin_amdgcn_s_memrealtime() - t0 > 400000000ull) {
      if (lane == 0) atomicOr(err, 1u);
      return 0;
    }
    const unsigned sent = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(v >> 32), kPl - 1);
    if (sent != epoch) {
      for (int z = 0; z < nap; ++z) __builtin_amdgcn_s_sleep(4);
      nap = nap < 16 ? 2 * nap : 16;
      if (lane == kPl - 1) v = __hip_atomic_fetch_add((gu64*)p, bits_opaque_zero(), BITS_RLX);
    } else if (mine && (unsigned)(v >> 32) != epoch) {
      v = __hip_atomic_fetch_add((gu64*)p, bits_opaque_zero(), BITS_RLX);
    }
  }
}

// ---- traceback ---------------------------------------------------------------

struct Walk {
  int i, j, st, k;  // cell, state (0 H, 1 F, 2 E), moves emitted
  int b, q;         // bit of the cell's row in its row-lane, tile lane of its step
};

// n copies of move c: bytes k .. k + n - 1 of the reversed move string, staged
// in the VGPR outv (lane L holds bytes 4 L .. 4 L + 3 of the current 256) and
// flushed 256 B at a time
__device__ __forceinline__ void emit_run(Walk& w, unsigned c, int n, unsigned& outv, unsigned* ops, int lane) {
  const unsigned rep = c * 0x01010101u;
  while (n > 0) {
    const int kk = w.k & 255, m = n < 256 - kk ? n : 256 - kk;
    int lo = kk - 4 * lane, hi = kk + m - 4 * lane;
    lo = lo < 0 ? 0 : (lo > 4 ? 4 : lo);
    hi = hi < 0 ? 0 : (hi > 4 ? 4 : hi);
    outv |= rep & (unsigned)(((1ull << (8 * hi)) - 1) ^ ((1ull << (8 * lo)) - 1));
    w.k += m;
    n -= m;
    if ((w.k & 255) == 0) {
      ops[(int64_t)((w.k >> 8) - 1) * 64 + lane] = outv;
      outv = 0;
    }
  }
}

// A walk tile: row-lanes 2 g, 2 g + 1 of a band (rows 64 g .. + 63) by steps
// 64 u .. 64 u + 127.  A diagonal run crosses it corner to corner (two steps
// per row), so a tile serves ~64 moves; while the walk crosses one, the tile
// it is predicted to enter next is already loading (gtile_load into nx, copied
// to tw at the switch).
struct GKey {
  int band, g, u;
};

__device__ __forceinline__ GKey gkey_of(int i, int j) {
  const int r = i - 1, rl = r & (kBR - 1), s = j + rl;
  return GKey{r >> 11, rl >> 6, s >= 128 ? (s >> 6) - 1 : 0};
}

// nx[p][h][w]: lane L's word w of row-lane 2 g + h at step 64 u + 64 p + L.  In
// the 4-step block layout a uint4 holds row-lane 2 g at an even / odd step in
// x / y and row-lane 2 g + 1 in z / w; a lane loads only its parity's two dwords.
__device__ __forceinline__ void gtile_load(const FillArgs& a, const PairDesc& pd, GKey k, int lane,
                                           unsigned (&nx)[2][2][4]) {
  const int nblk = pd.bits_nblk, blo = gotoh_blk_lo(k.band, pd.m, pd.n, pd.bits_w);
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const int ss = 64 * k.u + 64 * p + lane;
    int rel = (ss >> 2) - blo;
    rel = rel < 0 ? 0 : (rel >= nblk ? nblk - 1 : rel);  // (steps outside the stored blocks are never read)
    const unsigned* bp =
        a.mat + pd.mat_off + ((int64_t)k.band * nblk + rel) * 1024 + (ss & 2) * 64 + 4 * k.g + (lane & 1);
#pragma unroll
    for (int wd = 0; wd < 4; ++wd) {
      nx[p][0][wd] = bp[wd * 256];
      nx[p][1][wd] = bp[wd * 256 + 2];
    }
  }
}

// Moves inside row-lane h = H, step part P of the tile (oracle/nw_oracle.c:241-256),
// one run at a time: the cell's words are lane q - 64 P (q = its step - 64 u),
// and every cell a run can reach inside the part is one lane, so a ballot finds
// where it breaks (a move at a time ran ~550 cycles a move; runs average ~5.5
// moves on C5).  Returns when the walk reaches row or column 0, leaves the
// row-lane (b < 0) or the part (q < qlo), or has emitted kcap moves.
//   H: D while the D bit is set (diagonal: lane -2, bit -1); at the first cell
//      without it the F-source bit picks F or E (no move yet);
//   F: UP moves (lane -1, bit -1), 'U' while the F-extend bit is set, then 'u'
//      back to H; E: the same leftwards (lane -1, same bit) on the E-extend bit.
template <int H, int P>
__device__ __forceinline__ void walk_rl(const unsigned (&tw)[2][2][4], Walk& w, int qlo, int kcap, unsigned& outv,
                                        unsigned* ops, int lane) {
  const int lo = qlo - 64 * P;  // lowest tile lane the part may read
  while (w.i > 0 && w.j > 0 && w.q >= qlo && w.k < kcap && w.b >= 0) {
    const int ql = w.q - 64 * P, b = w.b, dl = ql - lane;
    const int room = kcap - w.k;
    if (w.st == 0) {
      const int t = dl >> 1;
      const bool ok = dl >= 0 && !(dl & 1) && t <= b && lane >= lo;
      const unsigned bit = (tw[P][H][0] >> ((unsigned)(b - t) & 31u)) & 1u;
      const u64 brk = __ballot(ok && !bit);
      const int tlim = (b < ((ql - lo) >> 1) ? b : (ql - lo) >> 1) + 1;
      const int ts = brk ? (ql - (63 - __builtin_clzll(brk))) >> 1 : tlim;
      int cap = w.i < w.j ? w.i : w.j;
      cap = cap < room ? cap : room;
      const int n = ts < cap ? ts : cap;
      emit_run(w, 'D', n, outv, ops, lane);
      w.i -= n;
      w.j -= n;
      w.b -= n;
      w.q -= 2 * n;
      if (n == ts && ts < tlim) {
        const unsigned f = (unsigned)__builtin_amdgcn_readlane((int)tw[P][H][1], w.q - 64 * P);
        w.st = (f >> w.b) & 1u ? 1 : 2;
      }
    } else if (w.st == 1) {
      const bool ok = dl >= 0 && dl <= b && lane >= lo;
      const unsigned bit = (tw[P][H][3] >> ((unsigned)(b - dl) & 31u)) & 1u;
      const u64 brk = __ballot(ok && !bit);
      const int tlim = (b < ql - lo ? b : ql - lo) + 1;
      const int ts = brk ? ql - (63 - __builtin_clzll(brk)) : tlim;
      const int cap = w.i < room ? w.i : room;
      const bool close = ts < tlim && ts < cap;
      const int n = close ? ts : (tlim < cap ? tlim : cap);
      emit_run(w, 'U', n, outv, ops, lane);
      if (close) {
        emit_run(w, 'u', 1, outv, ops, lane);
        w.st = 0;
      }
      const int mv = n + (close ? 1 : 0);
      w.i -= mv;
      w.b -= mv;
      w.q -= mv;
    } else {
      const bool ok = dl >= 0 && lane >= lo;
      const unsigned bit = (tw[P][H][2] >> (unsigned)b) & 1u;
      const u64 brk = __ballot(ok && !bit);
      const int tlim = ql - lo + 1;
      const int ts = brk ? ql - (63 - __builtin_clzll(brk)) : tlim;
      const int cap = w.j < room ? w.j : room;
      const bool close = ts < tlim && ts < cap;
      const int n = close ? ts : (tlim < cap ? tlim : cap);
      emit_run(w, 'L', n, outv, ops, lane);
      if (close) {
        emit_run(w, 'l', 1, outv, ops, lane);
        w.st = 0;
      }
      const int mv = n + (close ? 1 : 0);
      w.j -= mv;
      w.q -= mv;
    }
  }
}

__device__ __forceinline__ void trace_gotoh(const FillArgs& a, const PairDesc& pd, int lane) {
  Walk w{pd.m, pd.n, 0, 0, 0, 0};
  unsigned outv = 0;
  unsigned* ops = reinterpret_cast<unsigned*>(a.ops + pd.ops_off);
  const int nblk = pd.bits_nblk, kcap = pd.m + pd.n;
  unsigned tw[2][2][4];
  unsigned nx[2][2][4];
  GKey cur{-1, 0, 0}, pre{-1, 0, 0};
  int slo = 0, shi = -1;
  bool out = false;
  u64 n_sw = 0, n_dem = 0, c_wait = 0;  // (verbose >= 2 timeline: tile switches, demand loads, cycles waiting on tiles)
  const u64 c0 = a.stamps ? __builtin_amdgcn_s_memtime() : 0;
  if (a.dbg_corrupt == pd.slot + 1) {
    // (tests of the fill-vs-walk guard) flip the stored D bit of cell (m, n):
    // row-lane rl / 32, bit rl % 32 of the D word at step n + rl
    const int r = pd.m - 1, band = r >> 11, rl = r & (kBR - 1), s = pd.n + rl;
    const int rel = (s >> 2) - gotoh_blk_lo(band, pd.m, pd.n, pd.bits_w);
    if (lane == 0 && (unsigned)rel < (unsigned)nblk)
      __hip_atomic_fetch_xor((gu32*)(a.mat + pd.mat_off + ((int64_t)band * nblk + rel) * 1024 + (s & 2) * 64 +
                                     2 * (rl >> 5) + (s & 1)),
                             1u << (rl & 31), BITS_RLX);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  while (w.i > 0 && w.j > 0 && w.k < kcap) {
    const int r = w.i - 1, band = r >> 11, rl = r & (kBR - 1), g = rl >> 6, s = w.j + rl;
    if (band != cur.band || g != cur.g || s < 64 * cur.u || s > 64 * cur.u + 127) {
      // the tile holding the cell: the prefetched one if it does, else loaded now
      ++n_sw;
      if (!(band == pre.band && g == pre.g && s >= 64 * pre.u && s <= 64 * pre.u + 127)) {
        pre = gkey_of(w.i, w.j);
        gtile_load(a, pd, pre, lane, nx);
        ++n_dem;
      }
      const u64 tw0 = a.stamps ? __builtin_amdgcn_s_memtime() : 0;
#pragma unroll
      for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int h = 0; h < 2; ++h)
#pragma unroll
          for (int wd = 0; wd < 4; ++wd) tw[p][h][wd] = nx[p][h][wd];
      if (a.stamps) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        c_wait += __builtin_amdgcn_s_memtime() - tw0;
      }
      cur = pre;
      const int blo = gotoh_blk_lo(band, pd.m, pd.n, pd.bits_w);
      slo = 4 * blo;
      shi = 4 * (blo + nblk) - 1;
      // the next tile: where a diagonal run from this cell leaves this one (rows
      // or steps, whichever run out first)
      const int q = s - 64 * cur.u, ro = rl & 63;
      const int d = ro + 1 < (q >> 1) + 1 ? ro + 1 : (q >> 1) + 1;
      if (w.i - d >= 1 && w.j - d >= 1) {
        pre = gkey_of(w.i - d, w.j - d);
        gtile_load(a, pd, pre, lane, nx);
      } else {
        pre.band = -1;
      }
    }
    if (s < slo || s > shi) {  // the path left the stored window
      out = true;
      break;
    }
    w.b = rl & 31;
    w.q = s - 64 * cur.u;
    const int qmin = slo > 64 * cur.u ? slo - 64 * cur.u : 0;
    const int h = (rl >> 5) & 1, part = w.q >> 6;
    const int qlo = qmin > 64 * part ? qmin : 64 * part;
    switch (2 * h + part) {
      case 0: walk_rl<0, 0>(tw, w, qlo, kcap, outv, ops, lane); break;
      case 1: walk_rl<0, 1>(tw, w, qlo, kcap, outv, ops, lane); break;
      case 2: walk_rl<1, 0>(tw, w, qlo, kcap, outv, ops, lane); break;
      default: walk_rl<1, 1>(tw, w, qlo, kcap, outv, ops, lane); break;
    }
  }
  const bool bad = !out && w.i > 0 && w.j > 0;  // more moves than m + n: inconsistent words
  if (bad && lane == 0) atomicOr(a.err, 16u);
  if ((w.k & 255) && lane < (((w.k & 255) + 3) >> 2)) ops[(int64_t)(w.k >> 8) * 64 + lane] = outv;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (a.stamps && lane == 0) {  // trace cycles, tile-wait cycles, moves, switches / demand loads
    u64* x = a.stamps + 8 * pd.slot;
    x[2] = __builtin_amdgcn_s_memtime() - c0;
    x[3] = c_wait;
    x[4] = (u64)w.k;
    x[5] = (n_sw << 32) | n_dem;
  }
  if (lane == 0) {
    a.oplen[pd.slot] = out ? 0 : w.k;
    a.endij[pd.slot] = out ? make_int2(pd.m, pd.n) : make_int2(w.i, w.j);
    if (out) a.retry[pd.slot] = 1;
  }
}

// ---- fill ----------------------------------------------------------------------

// (scorings with more planes than C5's 8 + 3 keep 4 waves: at 96 VGPRs their step spills)
template <int GO, int GE>
constexpr int gotoh_wpe() { return 2 * (GO + GE) + GO <= 11 ? NWK_GOTOH_WPE : 4; }

template <int PXY, int GO, int GE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(gotoh_wpe<GO, GE>()))) void nw_align_gotoh(FillArgs a) {
  using C = Cfg<GO, GE, PXY>;
  using G = GGeo<C>;
  constexpr int NV = C::NV, NQ1 = G::NQ1, kPl = G::kPl, kPs = G::kPs;
  __shared__ __attribute__((aligned(16))) unsigned cons_all[4][32 * kPs];
  __shared__ __attribute__((aligned(16))) unsigned ring_all[4][64 * kPs];
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  unsigned* cons = cons_all[wid];
  unsigned* ring = ring_all[wid];
  // verbose >= 2 timeline (FillArgs::stamps, layout in nwk_runtime.cpp)
  if (a.stamps && threadIdx.x == 0) atomicMin(a.stamps + 11 * a.ntasks_pairs, (u64)__builtin_amdgcn_s_memrealtime());
  for (;;) {
    unsigned tk = 0;
    if (lane == 0) tk = atomicAdd(a.counter, 1u);
    tk = __builtin_amdgcn_readfirstlane(tk);
    if (tk >= (unsigned)a.ntasks) return;
    // wave-uniform exit (a per-lane load would make the task loop divergent)
    if (__builtin_amdgcn_readfirstlane(__hip_atomic_load((gu32*)a.err, BITS_RLX)) != 0u) return;
    const u64 t_task = a.stamps ? __builtin_amdgcn_s_memtime() : 0;
    u64 cyc_wait = 0;
    const int2 task = a.tasks[tk];
    const PairDesc pd = a.pairs[task.x];
    const int band = task.y;
    const int R0 = band * kBR;
    // code bit planes of rows R0 + 32 lane + b (rows past m: code 0, never traced)
    unsigned x0 = 0, x1 = 0;
    {
      const int base = R0 + 32 * lane;
      const int nv = pd.m - base;
      const uint8_t* xc = a.codes + pd.x_off + base;
#pragma unroll
      for (int b = 0; b < 32; ++b) {
        const unsigned cd = b < nv ? (unsigned)xc[b] : 0u;
        x0 |= (cd & 1u) << b;
        x1 |= ((cd >> 1) & 1u) << b;
      }
    }
    const int kmax = pd.n >> 5;  // last 32-column chunk holding a real column
    const int nw = kmax + 1;
    const bool from_above = band > 0, to_below = band + 1 < pd.nbands;
    const u64* gin = reinterpret_cast<const u64*>(a.bnd) + pd.bnd_off + (int64_t)(from_above ? band - 1 : 0) * nw * kPs;
    u64* gout = a.bnd + pd.bnd_off + (int64_t)band * nw * kPs;
    const bool gl = lane < kPl;
    u64 g = 0;
    if (from_above && gl) g = __hip_atomic_load((gu64*)(gin + lane), BITS_RLX);
    // left border: v(1, 0) = -go (row 1 only), v(i > 1, 0) = 0; e = +inf (saturated)
    uint32_t v[NV], e[NQ1], h[NV], f[NQ1];
    const uint32_t row1 = (band == 0 && lane == 0) ? 1u : 0u;
#pragma unroll
    for (int p = 0; p < NV; ++p) {
      v[p] = p < GO ? ~row1 : 0u;
      h[p] = 0u;
    }
#pragma unroll
    for (int q = 0; q < NQ1; ++q) e[q] = f[q] = C::NQ > 0 ? ~0u : 0u;
    // storage: the band's 4-step blocks blo .. blo + nblk (all of them when not windowed)
    const int nblk = pd.bits_nblk, blo = gotoh_blk_lo(band, pd.m, pd.n, pd.bits_w);
    unsigned* mb = a.mat + pd.mat_off + (int64_t)band * nblk * 1024 + lane * 2;
    // y windows: chunk q (columns 32 q .. 32 q + 31) is y position 32 q - 1; at
    // segment j lane t takes chunk j - t (lo) and chunk j - t - 1 (hi)
    const unsigned* ywp = a.yw + 2 * (pd.e_off - 1 - 32 * (int64_t)lane);
    unsigned hi0 = ywp[-64], hi1 = ywp[-63], lo0 = ywp[0], lo1 = ywp[1];
    const int nseg = kmax + 65;  // the last chunk is published after segment kmax + 64
    bool ok = true;
    // fill-vs-walk guard: with v = G(i-1, j) - G(i, j) = VLO + (its planes set)
    // and G(0, n) = go, H(m, n) = go + (m + n) ge - sum_i v(i, n); row
    // 32 t + b reaches column n at step n + 32 t + b (segments kmax ..)
    // At step s exactly one row of the band is at column n: band row r = s - n
    // (lane r / 32, bit r % 32), so the scalar unit reads it (v_readlane) and
    // no VGPR lives across the loop for the guard (a per-lane counter and row
    // mask made the C5 instantiation spill 33 VGPRs)
    const int capn = a.endv ? pd.n : -100000;
    const int rows_m = pd.m - R0;  // band rows < m
    int cnt = 0;                   // (uniform) planes set over this band's rows < m at column n
    // one 32-step segment j; false: the hand-off failed (the task ends)
    auto segment = [&](int j, auto mask_t, auto end_t) -> bool {
      // --- the row above for lane 0's columns 32 j .. 32 j + 31 -> cons (bit 31 per column)
      {
        unsigned w = 0;  // lane p < kPl: plane p's word (bit r = column 32 j + r)
        if (!from_above) {
          // row 0: h(0, 1) = -go (no plane set), h(0, c > 1) = 0 (planes < go), f = +inf
          const unsigned h0 = j == 0 ? ~3u : ~0u;  // (columns 0 and 1 cleared in chunk 0)
          w = lane < GO ? h0 : (lane < NV ? 0u : ~0u);
        } else if (j <= kmax) {
          if (!__all(!gl || (unsigned)(g >> 32) == a.epoch)) {
            const u64 tw = a.stamps ? __builtin_amdgcn_s_memtime() : 0;
            g = gran_wait<kPl>(gin + (int64_t)j * kPs + lane, a.epoch, g, a.err);
            if (a.stamps) cyc_wait += __builtin_amdgcn_s_memtime() - tw;
            if (!__all(!gl || (unsigned)(g >> 32) == a.epoch)) return false;
          }
          w = (unsigned)g;
          if (j < kmax && gl) g = __hip_atomic_load((gu64*)(gin + (int64_t)(j + 1) * kPs + lane), BITS_RLX);
        }
        unsigned ev[kPs];
#pragma unroll
        for (int p = 0; p < kPs; ++p)
          ev[p] = p < kPl ? (((unsigned)__builtin_amdgcn_readlane((int)w, p) >> (lane & 31)) & 1u) << 31 : 0u;
        if (lane < 32) {
#pragma unroll
          for (int p = 0; p < kPs; p += 4)
            *reinterpret_cast<uint4*>(cons + lane * kPs + p) = make_uint4(ev[p], ev[p + 1], ev[p + 2], ev[p + 3]);
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
      }
      const unsigned* yn = ywp + 64 * (j + 1);
      const unsigned nlo0 = yn[0], nlo1 = yn[1];
      {
        constexpr bool MASK = decltype(mask_t)::value;
        constexpr bool END = decltype(end_t)::value;
        unsigned dq[4][2];
#pragma unroll 4
        for (int r = 0; r < 32; ++r) {
          const int s = 32 * j + r;
          const unsigned sh = 31u - (unsigned)r;
          const unsigned y0 = __builtin_amdgcn_alignbit(hi0, lo0, sh);
          const unsigned y1 = __builtin_amdgcn_alignbit(hi1, lo1, sh);
          const uint32_t match = ~((x0 ^ y0) | (x1 ^ y1));
          unsigned inj[kPs];
#pragma unroll
          for (int p = 0; p < kPs; p += 4) {
            const uint4 c4 = *reinterpret_cast<const uint4*>(cons + r * kPs + p);
            inj[p] = c4.x;
            inj[p + 1] = c4.y;
            inj[p + 2] = c4.z;
            inj[p + 3] = c4.w;
          }
          uint32_t U[NV], fU[NQ1];
#pragma unroll
          for (int p = 0; p < NV; ++p) {
            const unsigned T = (unsigned)__builtin_amdgcn_update_dpp((int)inj[p], (int)h[p], 0x138, 0xf, 0xf, false);
            U[p] = __builtin_amdgcn_alignbit(h[p], T, 31);
          }
          if constexpr (C::NQ > 0) {
#pragma unroll
            for (int p = 0; p < NQ1; ++p) {
              const unsigned T =
                  (unsigned)__builtin_amdgcn_update_dpp((int)inj[NV + p], (int)f[p], 0x138, 0xf, 0xf, false);
              fU[p] = __builtin_amdgcn_alignbit(f[p], T, 31);
            }
          } else {
            fU[0] = 0u;
          }
          uint32_t D, Fs, Ee, Fe, vn[NV], en[NQ1];
          step<C>(match, v, e, U, fU, vn, en, h, f, D, Fs, Ee, Fe);
#pragma unroll
          for (int p = 0; p < NV; ++p) v[p] = vn[p];
          if constexpr (END) {  // column n: band row r = s - n (rows < m)
            const int rr = s - capn;
            if ((unsigned)rr < (unsigned)kBR && rr < rows_m) {
#pragma unroll
              for (int p = 0; p < NV; ++p)
                cnt += (int)(((unsigned)__builtin_amdgcn_readlane((int)vn[p], rr >> 5) >> (rr & 31)) & 1u);
            }
          }
#pragma unroll
          for (int q = 0; q < NQ1; ++q) e[q] = en[q];
          if constexpr (MASK) {  // columns <= 0 keep the left border
            const int lim = s - 32 * lane;
            const uint32_t M = lim <= 0 ? ~0u : (lim >= 32 ? 0u : ~((1u << lim) - 1u));
#pragma unroll
            for (int p = 0; p < NV; ++p) v[p] = (v[p] & ~M) | ((p < GO ? ~row1 : 0u) & M);
            if constexpr (C::NQ > 0) {
#pragma unroll
              for (int q = 0; q < NQ1; ++q) e[q] |= M;
            }
          }
          if (to_below && lane == 63) {  // the band's last row at column s - 2047
            unsigned ow[kPs];
#pragma unroll
            for (int p = 0; p < kPs; ++p) ow[p] = p < NV ? h[p] : (p < kPl ? f[p - NV] : 0u);
            unsigned* en_ = ring + ((s - 2047) & 63) * kPs;
#pragma unroll
            for (int p = 0; p < kPs; p += 4)
              *reinterpret_cast<uint4*>(en_ + p) = make_uint4(ow[p], ow[p + 1], ow[p + 2], ow[p + 3]);
          }
#if NWK_GOTOH_STEPSTORE
          // four words per lane and step, one 4-byte store each (the layout of
          // the 8-byte form below; no staging registers live across steps)
          {
            const int rel = (s >> 2) - blo;
            if ((unsigned)rel < (unsigned)nblk) {
              unsigned* q = mb + (int64_t)rel * 1024 + (s & 2) * 64 + (s & 1);
              __builtin_nontemporal_store(D, q);
              __builtin_nontemporal_store(Fs, q + 256);
              __builtin_nontemporal_store(Ee, q + 512);
              __builtin_nontemporal_store(Fe, q + 768);
            }
          }
#else
          // four words per lane and step; every 2 steps one 8-byte store per
          // word, 512 B contiguous across the wave
          dq[0][r & 1] = D;
          dq[1][r & 1] = Fs;
          dq[2][r & 1] = Ee;
          dq[3][r & 1] = Fe;
          if ((r & 1) == 1) {
            const int rel = (s >> 2) - blo;
            if ((unsigned)rel < (unsigned)nblk) {
              typedef unsigned u2 __attribute__((ext_vector_type(2)));
#pragma unroll
              for (int w4 = 0; w4 < 4; ++w4)
                __builtin_nontemporal_store(u2{dq[w4][0], dq[w4][1]},
                                            reinterpret_cast<u2*>(mb + (int64_t)rel * 1024 + w4 * 256 + (s & 2) * 64));
            }
          }
#endif
        }
      }
      hi0 = lo0;
      hi1 = lo1;
      lo0 = nlo0;
      lo1 = nlo1;
      // --- publish chunk k = j - 64 (columns 32 k .. + 31, complete after this segment)
      const int k = j - 64;
      if (to_below && k >= 0 && k <= kmax) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        unsigned word = 0;
#pragma unroll
        for (int p = 0; p < kPl; ++p) {
          const unsigned bit = lane < 32 ? ring[((32 * k + lane) & 63) * kPs + p] >> 31 : 0u;
          const unsigned wd = (unsigned)__ballot(bit != 0u);
          word = lane == p ? wd : word;
        }
        if (gl) __hip_atomic_store((gu64*)(gout + (int64_t)k * kPs + lane), ((u64)a.epoch << 32) | word, BITS_RLX);
      }
      return true;
    };
    // three loops, one per form of the step (a branch between the forms inside
    // one loop made the segment loop irreducible, and the compiler shuffled and
    // spilled registers at every segment): columns <= 0 masked in the first 65
    // segments (with the guard's end value for pairs shorter than that), the
    // plain steps, then the segments that reach column n
    int j = 0;
    const int j1 = nseg < 65 ? nseg : 65;
    for (; j < j1 && ok; ++j) ok = segment(j, std::true_type{}, std::true_type{});
    for (; j < kmax && ok; ++j) ok = segment(j, std::false_type{}, std::false_type{});
    for (; j < nseg && ok; ++j) ok = segment(j, std::false_type{}, std::true_type{});
    if (!ok) return;
    if (a.endv) {  // this band's part of H(m, n) (+ the border terms once, band 0)
      const int rows = min(kBR, pd.m - R0);
      const int part = rows * GO - cnt + (band == 0 ? GO + (pd.m + pd.n) * GE : 0);
      if (lane == 0) __hip_atomic_fetch_add((gu32*)(a.endv + pd.slot), (unsigned)part, BITS_RLX);
    }
    if (a.stamps && lane == 0) {  // per pair: band cycles, of which waiting on the band above
      atomicAdd(a.stamps + 8 * pd.slot + 6, (u64)(__builtin_amdgcn_s_memtime() - t_task));
      atomicAdd(a.stamps + 8 * pd.slot + 7, cyc_wait);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned prev = 0;
    if (lane == 0) prev = __hip_atomic_fetch_add((gu32*)(a.done + pd.slot), 1u, BITS_RLX);
    prev = __builtin_amdgcn_readfirstlane(prev);
    if (prev + 1u == (unsigned)pd.nbands) {  // the pair's last band: every band has released
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      // the walk is one latency-bound wave: let it issue ahead of the SIMD's fill waves
      __builtin_amdgcn_s_setprio(3);
      if (a.stamps && lane == 0) a.stamps[8 * pd.slot] = __builtin_amdgcn_s_memrealtime();
      if (!a.dbg_notrace) {
        trace_gotoh(a, pd, lane);
      } else if (lane == 0) {
        a.oplen[pd.slot] = 0;
        a.endij[pd.slot] = make_int2(pd.m, pd.n);
      }
      if (a.stamps && lane == 0) a.stamps[8 * pd.slot + 1] = __builtin_amdgcn_s_memrealtime();
      __builtin_amdgcn_s_setprio(0);
    }
  }
}

template <int PXY, int GO, int GE>
hipError_t gotoh_launch(const FillArgs& a, int grid, hipStream_t s) {
  hipLaunchKernelGGL((nw_align_gotoh<PXY, GO, GE>), dim3(grid), dim3(256), 0, s, a);
  return hipGetLastError();
}

template <int PXY, int GO, int GE>
int gotoh_occ() {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, reinterpret_cast<const void*>(&nw_align_gotoh<PXY, GO, GE>), 256,
                                                   0) != hipSuccess)
    return 1;
  return n > 0 ? n : 1;
}

struct GotohEntry {
  int pxy, go, ge;
  hipError_t (*launch)(const FillArgs&, int, hipStream_t);
  int (*occ)();
};

// The scorings instantiated (pxy, go, ge): C5's (3, 3, 1); the reference's
// linear 3/2 and 5/1 as their degenerate affine case (go = 0, ge = pgap); and
// the affine scorings of the GPU tests.  Others run on nw_align_pka /
// nw_align_affine.
#define NWK_GOTOH_ENTRY(p, o, e) {p, o, e, gotoh_launch<p, o, e>, gotoh_occ<p, o, e>},
const GotohEntry kGotohSet[] = {
    NWK_GOTOH_ENTRY(3, 3, 1)
    NWK_GOTOH_ENTRY(3, 0, 2) NWK_GOTOH_ENTRY(5, 0, 1) NWK_GOTOH_ENTRY(3, 0, 1)
    NWK_GOTOH_ENTRY(3, 4, 1) NWK_GOTOH_ENTRY(1, 2, 2) NWK_GOTOH_ENTRY(2, 1, 1) NWK_GOTOH_ENTRY(4, 2, 2)
    NWK_GOTOH_ENTRY(4, 2, 1) NWK_GOTOH_ENTRY(2, 4, 2) NWK_GOTOH_ENTRY(3, 5, 2) NWK_GOTOH_ENTRY(9, 3, 2)
};
#undef NWK_GOTOH_ENTRY

const GotohEntry* gotoh_find(int pxy, int go, int ge) {
  for (const auto& g : kGotohSet)
    if (g.pxy == pxy && g.go == go && g.ge == ge) return &g;
  return nullptr;
}

}  // namespace

bool gotoh_admissible(int pxy, int go, int ge, int alpha) { return alpha <= 4 && gotoh_find(pxy, go, ge) != nullptr; }

int gotoh_granules(int go, int ge) { return (2 * (go + ge) + go + 3) & ~3; }

hipError_t launch_gotoh(const FillArgs& a, int pxy, int go, int ge, int grid, hipStream_t s) {
  const GotohEntry* g = gotoh_find(pxy, go, ge);
  return g ? g->launch(a, grid, s) : hipErrorInvalidValue;
}

int gotoh_blocks_per_cu(int pxy, int go, int ge) {
  const GotohEntry* g = gotoh_find(pxy, go, ge);
  return g ? g->occ() : 1;
}

}  // namespace nwk
