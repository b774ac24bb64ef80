// nwk_kernels.hip -- CDNA4 (gfx950) kernels of the all-pairs NW engine.
//
// Reference hot loop (submit/xuliny-seqalkway.cpp:476-488, oracle
// seqalign-mpi-skeleton.cpp:211-226):
//     dp[i][j] = x[i-1]==y[j-1] ? dp[i-1][j-1]
//                               : min(dp[i-1][j-1]+pxy, dp[i-1][j]+pgap, dp[i][j-1]+pgap)
// and its traceback (skel:236-262, sub:502-531).
//
// The fill runs in G-space, G[i][j] = H[i][j] - (i+j)*pgap, a bijective
// relabelling of the reference matrix in which the two gap moves cost 0 and
// the diagonal move costs K = pxy - 2*pgap (mismatch) or -2*pgap (match):
//     G = min(G[i-1][j-1] + K(x_i, y_j), G[i-1][j], G[i][j-1])
// (for pxy, pgap >= 0 the match shortcut equals this minimum; kLiteral keeps
// the shortcut literally for negative penalties).  Every border cell of G is
// 0.  The traceback's equality tests are preserved exactly:
//     dp[i-1][j-1]+pxy == dp[i][j]  <=>  G[i-1][j-1] + (pxy-2pgap) == G[i][j]
//     dp[i-1][j]+pgap  == dp[i][j]  <=>  G[i-1][j] == G[i][j]
// and for pxy, pgap >= 0 both differences lie in [-(2pgap+pxy), 0], so the
// matrix is stored as G mod 2^W with 2^W > 2pgap+pxy (W = 4 for the
// reference's 3/2): equality mod 2^W is then exact equality.
//
// Work decomposition: a wave owns a band of 512 rows (8 per lane) of one
// pair and sweeps it as a skewed anti-diagonal: at step s lane t computes
// column j = s - t + 1 for its 8 rows.  up/diag for the lane's first row come
// from lane t-1 through DPP wave_shr:1; lane 0 gets them from the band above
// through 8-byte {epoch, value} granules in HBM (written sc1, polled sc1 --
// MI355X_MICROARCH.md "R2") staged in a per-wave LDS ring and read back with
// broadcast ds_read_b128.  Bands are dequeued from one atomic head in
// dependency order, so a wave only ever waits on a band dequeued earlier.
#include "nwk_internal.h"

namespace nwk {

typedef unsigned long long u64;
typedef __attribute__((address_space(1))) u64 gu64;
typedef __attribute__((address_space(1))) unsigned gu32;

#define RLX_AGENT __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT

__device__ __forceinline__ u64 ld_granule(const u64* p) {
  return __hip_atomic_load((gu64*)p, RLX_AGENT);
}
__device__ __forceinline__ void st_granule(u64* p, unsigned epoch, int v) {
  __hip_atomic_store((gu64*)p, ((u64)epoch << 32) | (unsigned)v, RLX_AGENT);
}

// Polls until every lane's granule carries `epoch` and returns it.  Bounded:
// gives up after ~4 s of wall time (s_memrealtime runs at 100 MHz) or when
// another wave has already failed, so a hand-off bug ends the grid instead of
// hanging it; the caller tells success from the returned tags.
__device__ __noinline__ u64 wait_granules(const u64* p, unsigned epoch, u64 v, unsigned* err) {
  const u64 t0 = __builtin_amdgcn_s_memrealtime();
  for (;;) {
    if (__all((unsigned)(v >> 32) == epoch)) return v;
    __builtin_amdgcn_s_sleep(4);
    if (__hip_atomic_load((gu32*)err, RLX_AGENT) != 0u) return 0;
    if (__builtin_amdgcn_s_memrealtime() - t0 > 400000000ull) {
      if ((threadIdx.x & 63) == 0) atomicOr(err, 1u);
      return 0;
    }
    v = ld_granule(p);
  }
}

// One DP cell in G-space.  xq: substitution profile (kProfile) or the row's
// byte (+0x100 for rows past m, never equal).  ysh: the column's E byte
// shifted to bit 0 (kProfile reads bits [4:0] = code*8).
template <int MODE>
__device__ __forceinline__ int cell(int dg, int up, int left, unsigned ysh, unsigned xq, int K0,
                                    int K1) {
  if constexpr (MODE == kProfile) {
    const int sub = __builtin_amdgcn_sbfe((int)xq, ysh, 8);
    return min(min(dg + sub, up), left);
  } else if constexpr (MODE == kCompare) {
    const int sub = ((ysh & 0xffu) == xq) ? K0 : K1;
    return min(min(dg + sub, up), left);
  } else {
    const int mm = min(min(dg + K1, up), left);
    return ((ysh & 0xffu) == xq) ? dg + K0 : mm;
  }
}

// Eight wavefront steps s0..s0+7 (s0 % 8 == 0).
//   bslot: LDS ring holding B[s0+1 .. s0+8] (the band-above row, G-space)
//   mptr:  this lane's store pointer for the block's first dword row
template <int MODE, int W, bool MASK>
__device__ __forceinline__ void step_block(int s0, int lane, int (&h)[kRows], int& Up, int& stage,
                                           unsigned (&acc)[kRows], const unsigned (&xq)[kRows],
                                           unsigned e0, unsigned e1, const int* bslot,
                                           unsigned* mptr, int K0, int K1) {
  constexpr int SPD = 32 / W;
  const int4 bA = *reinterpret_cast<const int4*>(bslot);
  const int4 bB = *reinterpret_cast<const int4*>(bslot + 4);
  const int bv[8] = {bA.x, bA.y, bA.z, bA.w, bB.x, bB.y, bB.z, bB.w};
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    // lane 63's last-row value of the previous step enters the publish window
    stage = __builtin_amdgcn_update_dpp(h[kRows - 1], stage, 0x130 /*wave_shl:1*/, 0xf, 0xf, false);
    // up of the lane's first row: lane t-1's last row (previous step); lane 0: B[s+1]
    const int up0 = __builtin_amdgcn_update_dpp(bv[k], h[kRows - 1], 0x138 /*wave_shr:1*/, 0xf, 0xf, false);
    const int dg0 = Up;
    Up = up0;
    const unsigned ysh = (k < 4 ? e0 : e1) >> (8 * (k & 3));
    int hn[kRows];
#pragma unroll
    for (int r = 0; r < kRows; ++r)
      hn[r] = cell<MODE>(r ? h[r - 1] : dg0, r ? hn[r - 1] : up0, h[r], ysh, xq[r], K0, K1);
    if constexpr (MASK) {  // columns j <= 0 stay on the border (G = 0)
      const bool valid = (s0 + k) >= lane;
#pragma unroll
      for (int r = 0; r < kRows; ++r) hn[r] = valid ? hn[r] : 0;
    }
#pragma unroll
    for (int r = 0; r < kRows; ++r) h[r] = hn[r];
    if constexpr (W < 32) {
#pragma unroll
      for (int r = 0; r < kRows; ++r) acc[r] = __builtin_amdgcn_alignbit((unsigned)h[r], acc[r], W);
    }
    if ((k % SPD) == SPD - 1) {
#pragma unroll
      for (int r = 0; r < kRows; ++r)
        __builtin_nontemporal_store(W < 32 ? acc[r] : (unsigned)h[r], mptr + ((k / SPD) * kRows + r) * kWave);
    }
  }
}

template <int MODE, int W>
__global__ __launch_bounds__(256) void nw_fill(FillArgs a) {
  constexpr int SPD = 32 / W;
  __shared__ __attribute__((aligned(16))) int ring_all[4][128];
  const int lane = threadIdx.x & 63;
  int* ring = ring_all[threadIdx.x >> 6];

  for (;;) {
    unsigned tk = 0;
    if (lane == 0) tk = atomicAdd(a.counter, 1u);
    tk = __builtin_amdgcn_readfirstlane(tk);
    if (tk >= (unsigned)a.ntasks) return;
    if (__hip_atomic_load((gu32*)a.err, RLX_AGENT) != 0u) return;
    const int2 task = a.tasks[tk];
    const PairDesc pd = a.pairs[task.x];
    const int band = task.y;
    const int row0 = band * kBandRows + lane * kRows;  // 0-based first row of this lane

    unsigned xq[kRows];
#pragma unroll
    for (int r = 0; r < kRows; ++r) {
      const int row = row0 + r;
      const unsigned c = row < pd.m ? a.codes[pd.x_off + row] : 0x100u;
      if constexpr (MODE == kProfile) {
        const unsigned cc = c & 0xffu;
        unsigned p = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) p |= ((unsigned)(cc == (unsigned)q ? a.K0 : a.K1) & 0xffu) << (8 * q);
        xq[r] = p;
      } else {
        xq[r] = c;
      }
    }

    const bool from_above = band > 0;
    const bool to_below = band + 1 < pd.nbands;
    const int64_t bstride = (int64_t)pd.nchunks * 64;
    const u64* gin = reinterpret_cast<const u64*>(a.bnd) + pd.bnd_off + (int64_t)(band - 1) * bstride + lane;
    u64* gout = a.bnd + pd.bnd_off + (int64_t)band * bstride + lane;
    const unsigned* Ep = a.E + pd.e_off - lane;
    unsigned* mptr = a.mat + pd.mat_off + (int64_t)band * band_dwords(W, pd.sblocks) + lane;

    int h[kRows];
    unsigned acc[kRows];
#pragma unroll
    for (int r = 0; r < kRows; ++r) { h[r] = 0; acc[r] = 0; }
    int Up = 0, stage = 0;
    u64 pend = 0;
    if (from_above && pd.nchunks > 0) pend = ld_granule(gin);
    unsigned e0 = Ep[0], e1 = Ep[4];
    bool ok = true;

    for (int sb = 0; sb < pd.sblocks; ++sb) {
      // --- band-above row for this super-block: B[64sb+1 .. 64sb+64] = chunk sb+1
      int bval = 0;
      if (from_above && sb < pd.nchunks) {
        if (!__all((unsigned)(pend >> 32) == a.epoch)) {
          pend = wait_granules(gin + 64 * sb, a.epoch, pend, a.err);
          if (!__all((unsigned)(pend >> 32) == a.epoch)) { ok = false; break; }
        }
        bval = (int)(unsigned)pend;
        if (sb + 1 < pd.nchunks) pend = ld_granule(gin + 64 * (sb + 1));
      }
      int* slot = ring + (sb & 1) * 64;
      slot[lane] = bval;
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();

      for (int blk = 0; blk < 8; ++blk) {
        const int s0 = sb * 64 + blk * 8;
        const unsigned ne0 = Ep[s0 + 8], ne1 = Ep[s0 + 12];  // next block's columns
        if (sb == 0)
          step_block<MODE, W, true>(s0, lane, h, Up, stage, acc, xq, e0, e1, slot + blk * 8, mptr, a.K0, a.K1);
        else
          step_block<MODE, W, false>(s0, lane, h, Up, stage, acc, xq, e0, e1, slot + blk * 8, mptr, a.K0, a.K1);
        mptr += (8 / SPD) * kRows * kWave;
        e0 = ne0;
        e1 = ne1;
      }
      // --- publish chunk sb (columns 64sb-63 .. 64sb of our last row) for band+1
      if (to_below && sb >= 1 && sb <= pd.nchunks) st_granule(gout + 64 * (sb - 1), a.epoch, stage);
      __builtin_amdgcn_wave_barrier();
    }
    if (!ok) return;
  }
}

// ---------------------------------------------------------------------------
// Traceback (skel:236-262 / sub:502-531 priority: DIAG on match > DIAG if
// diag+pxy==H > UP if up+pgap==H > LEFT) on the stored G mod 2^W.
//
// One wave per pair.  The walk itself is sequential and uniform (all lanes
// run it, so its state lives in SGPRs); the wave's lanes only move data:
// the stored matrix is staged in LDS one tile at a time -- a band's 512 rows
// x TC dword columns (+ overlap below) -- by LDS-DMA (global_load_lds_dword),
// and the next tile down the band is prefetched while the walk runs.  Each
// step then costs one round of broadcast ds_reads instead of dependent HBM
// loads.  Ops are emitted reversed, 4 per dword, by lane 0.
// ---------------------------------------------------------------------------
typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void gbl_void;

template <int W>
__device__ __forceinline__ unsigned getG_global(const unsigned* M, const PairDesc& pd, int64_t bdw, int i, int j) {
  if (i == 0 || j == 0) return 0u;
  constexpr int SPD = 32 / W;
  const int w = i - 1;
  const int b = w / kBandRows;
  const int wr = w - b * kBandRows;
  const int t = wr / kRows;
  const int r = wr - t * kRows;
  const int s = j - 1 + t;
  const unsigned d = M[pd.mat_off + (int64_t)b * bdw + ((int64_t)(s / SPD) * kRows + r) * kWave + t];
  if constexpr (W == 32) return d;
  else return (d >> (W * (s % SPD))) & ((1u << W) - 1u);
}

struct Five { unsigned v[5]; };

template <int W>
__device__ __noinline__ Five tb_fallback(const unsigned* mat, const PairDesc& pd, int64_t bdw, const uint8_t* xg,
                                         const uint8_t* yg, int ci, int cj, bool xin, bool yin, bool fg, bool fu,
                                         bool fd, int shg, int shu, int shd, Five in) {
  Five o = in;
  if (!xin && ci >= 1) o.v[0] = xg[ci - 1];
  if (!yin && cj >= 1) o.v[1] = yg[cj - 1];
  if (fg) o.v[2] = getG_global<W>(mat, pd, bdw, ci, cj) << shg;
  if (fu) o.v[3] = getG_global<W>(mat, pd, bdw, ci - 1, cj) << shu;
  if (fd) o.v[4] = getG_global<W>(mat, pd, bdw, ci - 1, cj - 1) << shd;
  return o;
}

typedef __attribute__((address_space(3))) unsigned lds_u32;
__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(uintptr_t)(const lds_u32*)p;
}

template <int W>
__global__ __launch_bounds__(64) void nw_traceback(TraceArgs a) {
  constexpr int SPD = 32 / W;
  constexpr int TC = 8;                      // dword columns per tile window
  constexpr int TS = TC * SPD;               // steps per tile window
  constexpr int OV = (11 + SPD - 1) / SPD;   // columns kept below the window: a block reaches s-10
  constexpr int CC = TC + OV;
  constexpr int TILE = CC * kRows * kWave;
  constexpr int YLO = 96;                    // y window starts 96 columns below the tile's first step
  constexpr unsigned MASK = W == 32 ? 0xffffffffu : ((1u << (W & 31)) - 1u);
  static_assert(TS + YLO <= 256, "y window must fit one DMA");
  __shared__ __attribute__((aligned(16))) unsigned tile[2][TILE];
  __shared__ __attribute__((aligned(16))) unsigned xs[2][kBandRows / 4];
  __shared__ __attribute__((aligned(16))) unsigned ys[2][64];

  const int lane = threadIdx.x;
  const PairDesc pd = a.pairs[blockIdx.x];
  const int64_t bdw = band_dwords(W, pd.sblocks);
  const int ncols = 64 * pd.sblocks / SPD;
  const uint8_t* xg = a.codes + pd.x_off;
  const uint8_t* yg = a.codes + pd.y_off;

  // Stage tile (b, q) into buffer buf by LDS-DMA: dword columns
  // [TC*q - OV, TC*q + TC), the band's x codes and the y codes of columns
  // [TS*q - YLO, TS*q - YLO + 256).  Completion = this wave's vmcnt.
  auto issue = [&](int buf, int b, int q) {
    const unsigned* src = a.mat + pd.mat_off + (int64_t)b * bdw + lane;
    for (int cc = 0; cc < CC; ++cc) {
      const int c = TC * q - OV + cc;
      if (c < 0 || c >= ncols) continue;
#pragma unroll
      for (int r = 0; r < kRows; ++r)
        __builtin_amdgcn_global_load_lds((gbl_void*)(src + ((int64_t)c * kRows + r) * kWave),
                                         (lds_void*)&tile[buf][(cc * kRows + r) * kWave], 4, 0, 0);
    }
    const unsigned* xsrc = reinterpret_cast<const unsigned*>(xg + (int64_t)b * kBandRows);
    __builtin_amdgcn_global_load_lds((gbl_void*)(xsrc + lane), (lds_void*)&xs[buf][0], 4, 0, 0);
    __builtin_amdgcn_global_load_lds((gbl_void*)(xsrc + 64 + lane), (lds_void*)&xs[buf][64], 4, 0, 0);
    const unsigned* ysrc = reinterpret_cast<const unsigned*>(yg + (int64_t)TS * q - YLO);
    __builtin_amdgcn_global_load_lds((gbl_void*)(ysrc + lane), (lds_void*)&ys[buf][0], 4, 0, 0);
  };
  // The walk reads LDS only through inline asm, so the compiler does not
  // make every read wait for the in-flight DMA: this drain is the one wait.
  auto drain = []() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); };

  uint8_t* ops = a.ops + pd.ops_off;
  int i = pd.m, j = pd.n, L = 0;
  unsigned opw = 0;
  int tb = -1, tq = 0, cur = 0, pb = -1, pq = 0;
  // this lane's cell of the 8x8 block anchored at (i, j): (i - li, j - lj)
  const int li = lane >> 3, lj = lane & 7;

  while (i > 0 && j > 0) {
    {  // ---- make the tile holding the block current
      const int w = (i - 1) & (kBandRows - 1);
      const int b = (i - 1) / kBandRows;
      const int s = j - 1 + (w >> 3);
      if (b != tb || s < TS * tq) {
        const int q = s / TS;
        drain();
        if (!(b == pb && q == pq)) {
          issue(cur ^ 1, b, q);
          drain();
        }
        cur ^= 1;
        tb = b;
        tq = q;
        pb = -1;
        if (q > 0) {
          issue(cur ^ 1, b, q - 1);
          pb = b;
          pq = q - 1;
        }
      }
    }
    // ---- every lane decides the traceback move of one cell of the block
    const int ci = i - li, cj = j - lj;
    const int slo = TS * tq - OV * SPD, shi = TS * tq + TS;
    const unsigned tbase = lds_addr(&tile[cur][0]);
    // address of G(ii, jj) in the tile, or ~0u when outside (border / other band / window)
    auto gaddr = [&](int ii, int jj, int& sh) -> unsigned {
      if (ii <= 0 || jj <= 0) { sh = -1; return ~0u; }
      const int ww = ii - 1 - tb * kBandRows;
      const int tt = ww >> 3, rr = ww & 7, ss = jj - 1 + tt;
      sh = W * (ss & (SPD - 1));
      if (ww < 0 || ss < slo || ss >= shi) return ~1u;
      return tbase + 4u * (unsigned)(((ss / SPD - (TC * tq - OV)) * kRows + rr) * kWave + tt);
    };
    int shg, shu, shd;
    const unsigned ag = gaddr(ci, cj, shg), au = gaddr(ci - 1, cj, shu), ad = gaddr(ci - 1, cj - 1, shd);
    const int wx = ci - 1 - tb * kBandRows, wy = cj - 1 - (TS * tq - YLO);
    const bool xin = ci >= 1 && wx >= 0, yin = cj >= 1 && wy >= 0 && wy < 256;
    const unsigned ax = xin ? lds_addr(&xs[cur][0]) + (unsigned)wx : lds_addr(&xs[cur][0]);
    const unsigned ay = yin ? lds_addr(&ys[cur][0]) + (unsigned)wy : lds_addr(&ys[cur][0]);
    const unsigned z = tbase;
    unsigned vx, vy, vg, vu, vd;
    asm volatile(
        "ds_read_u8 %0, %5\n\t"
        "ds_read_u8 %1, %6\n\t"
        "ds_read_b32 %2, %7\n\t"
        "ds_read_b32 %3, %8\n\t"
        "ds_read_b32 %4, %9\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(vx), "=&v"(vy), "=&v"(vg), "=&v"(vu), "=&v"(vd)
        : "v"(ax), "v"(ay), "v"(ag < ~1u ? ag : z), "v"(au < ~1u ? au : z), "v"(ad < ~1u ? ad : z)
        : "memory");
    // rare: cells of the band above / outside the staged window -> global,
    // in a non-inlined call so the wait for those loads (which also drains
    // the tile prefetch) stays on this path.
    if ((!xin && ci >= 1) || (!yin && cj >= 1) || ag == ~1u || au == ~1u || ad == ~1u) {
      const Five f = tb_fallback<W>(a.mat, pd, bdw, xg, yg, ci, cj, xin, yin, ag == ~1u, au == ~1u, ad == ~1u,
                                    shg, shu, shd, Five{vx, vy, vg, vu, vd});
      vx = f.v[0]; vy = f.v[1]; vg = f.v[2]; vu = f.v[3]; vd = f.v[4];
    }
    const unsigned g = ag == ~0u ? 0u : (vg >> shg) & MASK;
    const unsigned gu = au == ~0u ? 0u : (vu >> shu) & MASK;
    const unsigned gd = ad == ~0u ? 0u : (vd >> shd) & MASK;
    const bool isD = (vx & 0xffu) == (vy & 0xffu) || ((gd + (unsigned)a.K1 - g) & MASK) == 0u;
    const bool isU = !isD && ((gu - g) & MASK) == 0u;
    const unsigned long long mD = __ballot(isD), mU = __ballot(isU);
    // ---- sequential walk through the block on the two masks (SALU only)
    int di = 0, dj = 0;
    while (di < 8 && dj < 8 && i - di > 0 && j - dj > 0) {
      const int k = di * 8 + dj;
      const unsigned op = ((mD >> k) & 1ull) ? 'D' : ((mU >> k) & 1ull) ? 'U' : 'L';
      opw |= op << (8 * (L & 3));
      if ((L & 3) == 3) {
        if (lane == 0) *reinterpret_cast<unsigned*>(ops + (L & ~3)) = opw;
        opw = 0;
      }
      ++L;
      di += op != 'L';
      dj += op != 'U';
    }
    i -= di;
    j -= dj;
  }
  if ((L & 3) != 0 && lane == 0) *reinterpret_cast<unsigned*>(ops + (L & ~3)) = opw;
  drain();
  if (lane == 0) {
    a.oplen[pd.slot] = L;
    a.endij[pd.slot] = make_int2(i, j);
  }
}

// ---------------------------------------------------------------------------
template <int MODE, int W>
static hipError_t fill_w(const FillArgs& a, int grid, hipStream_t s) {
  hipLaunchKernelGGL((nw_fill<MODE, W>), dim3(grid), dim3(256), 0, s, a);
  return hipGetLastError();
}

template <int MODE>
static hipError_t fill_m(int bits, const FillArgs& a, int grid, hipStream_t s) {
  switch (bits) {
    case 4: return fill_w<MODE, 4>(a, grid, s);
    case 8: return fill_w<MODE, 8>(a, grid, s);
    case 16: return fill_w<MODE, 16>(a, grid, s);
    case 32: return fill_w<MODE, 32>(a, grid, s);
  }
  return hipErrorInvalidValue;
}

hipError_t launch_fill(int mode, int bits, const FillArgs& a, int grid, hipStream_t s) {
  switch (mode) {
    case kProfile: return fill_m<kProfile>(bits, a, grid, s);
    case kCompare: return fill_m<kCompare>(bits, a, grid, s);
    case kLiteral: return bits == 32 ? fill_w<kLiteral, 32>(a, grid, s) : hipErrorInvalidValue;
  }
  return hipErrorInvalidValue;
}

template <int MODE, int W>
static int occ_w() {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, reinterpret_cast<const void*>(&nw_fill<MODE, W>), 256, 0) != hipSuccess)
    return 1;
  return n > 0 ? n : 1;
}

int fill_blocks_per_cu(int mode, int bits) {
  if (mode == kLiteral) return occ_w<kLiteral, 32>();
  const bool p = mode == kProfile;
  switch (bits) {
    case 4: return p ? occ_w<kProfile, 4>() : occ_w<kCompare, 4>();
    case 8: return p ? occ_w<kProfile, 8>() : occ_w<kCompare, 8>();
    case 16: return p ? occ_w<kProfile, 16>() : occ_w<kCompare, 16>();
    default: return p ? occ_w<kProfile, 32>() : occ_w<kCompare, 32>();
  }
}

hipError_t launch_traceback(int bits, const TraceArgs& a, hipStream_t s) {
  const int grid = a.npairs;  // one wave per pair
  if (grid == 0) return hipSuccess;
  switch (bits) {
    case 4: hipLaunchKernelGGL((nw_traceback<4>), dim3(grid), dim3(64), 0, s, a); break;
    case 8: hipLaunchKernelGGL((nw_traceback<8>), dim3(grid), dim3(64), 0, s, a); break;
    case 16: hipLaunchKernelGGL((nw_traceback<16>), dim3(grid), dim3(64), 0, s, a); break;
    case 32: hipLaunchKernelGGL((nw_traceback<32>), dim3(grid), dim3(64), 0, s, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace nwk
