// nwk_bits.hip -- bit-sliced anti-diagonal fill (mode kBits, kernel nw_align_bits)
// for the reference's linear-gap recurrence (skel:211-226, sub:478-487) with
// pxy >= 0, pgap in {1, 2} and at most four distinct symbols.
//
// Difference form.  In G-space (G = H - (i+j) pgap) every
// cell's vertical and horizontal differences
//     v(i,j) = G[i-1][j] - G[i][j],   h(i,j) = G[i][j-1] - G[i][j]
// lie in [0, 2 pgap], and with U = h(i-1,j), L = v(i,j-1)
//     D = max(S, U, L),  S = 2 pgap (match) or 2 pgap - pxy (mismatch)
//     v(i,j) = D - U,    h(i,j) = D - L.
// Borders are all zero.  The reference's traceback (skel:229-262: DIAG on a
// match, DIAG if H_diag + pxy == H, UP if H_up + pgap == H, else LEFT) needs
// two bits per cell: diag = match | (D == S_mismatch), and plane 0 of v
// (stored raw: UP is v == 0).
//
// Bit slicing.  A value x in [0, NP], NP = 2 pgap, is held as NP thermometer
// planes t_k = [x > k].  Then max is OR, and D - U is the convolution
//     t_k(D - U) = OR_j (~t_j(U) & t_{j+k}(D)),
// so one 32-bit VALU op evaluates one plane term for 32 cells.  Bit b of lane
// t is row 32 t + b of a 2048-row band; at step s that row is at column
// s - 32 t - b (one anti-diagonal per step), so a cell's left neighbour is the
// same bit one step earlier and its upper neighbour is the bit below one step
// earlier -- a 1-bit funnel shift with lane t-1's top bit (DPP wave_shr:1).
// Lane 0's bit 0 takes the band above's last row instead: per 64-column chunk
// that row arrives as 2 NP self-tagged granules {epoch:32 | 32 plane bits}.
//
// Per step and lane: ~46 VALU ops for 32 cells (pk2: ~44 for 16), the stored
// traceback is 2 bits per cell (pk2: 4) and the hand-off 2 NP bits per column.
// The traceback reads the (diag, up) bits back: a scalar walk over 64-step x
// 64-row tiles staged in VGPRs (one v_readlane per bit word and move).
//
// Stored layout per band: 8-step block B = s >> 3 owns 1024 dwords; the diag
// bits of step s for lane t sit at dword B * 1024 + ((s & 7) >> 2) * 256 +
// 4 t + (s & 3), the up bits 512 dwords further.  Each of a block's four
// 16-byte stores thus writes 1 KB contiguous across the wave (whole lines:
// a lane-major 64-byte-stride layout wrote partial lines at ~1.1 TB/s).  A
// band has 64 * sblocks steps (sblocks = nchunks + 32: the last row runs 2047
// columns behind the first).  Windowed storage (PairDesc::bits_w > 0) keeps
// only bits_nblk blocks per band, from block bits_blk_lo(band) on: the band's
// steps within bits_w columns of the diagonal j = i n / m; a traceback that
// leaves them flags the pair for a full-storage re-run (FillArgs::retry).
#include "nwk_bits_dev.h"

namespace nwk {
namespace {

// Eight steps s0 .. s0+7 (s0 % 8 == 0) of one band.
//   x0, x1   code bit planes of this lane's 32 rows
//   yp, w    y windows: previous half and this 32-step half (bit 31 - q of w =
//            code of column s_half - 32 lane + q)
//   H, V     h and v planes of the previous step
//   cons     LDS: band-above row, entry (column & 63) * NP + k (bit 31)
//   ring     LDS: this band's last row at this block's entries: step s0 + q writes entry
//            q + 1 (the caller passes the ring + ((s0 & 127) * NP): entry (s & 127) + 1
//            holds column s - 2047, so column c is at entry ((c - 1) & 127) + 1 -- immediate
//            offsets from one address per block, no per-step address arithmetic)
//   eh       MASK blocks: this lane's bit-0 column at step s0 (columns < 0 keep
//            v = 0; strips: the column within the current row pass, so a bit
//            entering column 0 of its next pass sees the left border)
//   sto      the block is inside the pair's stored blocks (uniform); lsto: this
//            lane's words hold a cell of the storage window (bits_lane_stored)
//   END      steps that may hold column capc = n - 1: the bit there (row 32 lane
//            + s - capc - 32 lane) adds its vertical difference to cnt when its
//            row is < m (rowm) -- the fill-vs-walk guard's end value, FillArgs::endv
template <int NP, int SR, bool MASK, bool PROD, bool END = false>
__device__ __forceinline__ void bits_block(int s0, int lane, unsigned x0, unsigned x1, unsigned yp0, unsigned yp1,
                                           unsigned w0, unsigned w1, unsigned (&H)[NP], unsigned (&V)[NP],
                                           const unsigned* cons, unsigned* ring, unsigned* st, bool sto, int eh,
                                           bool lsto, int capc = 0, unsigned rowm = 0, int* cnt = nullptr) {
  unsigned dw[8], uw[8];
  // the band-above entries are read one step ahead (an LDS read's latency
  // would otherwise sit on every step's dependence chain)
  unsigned injn[NP];
  auto read_inj = [&](int s) {
    if constexpr (NP == 4) {
      const uint4 e = *reinterpret_cast<const uint4*>(cons + (s & 63) * 4);
      injn[0] = e.x; injn[1] = e.y; injn[2] = e.z; injn[3] = e.w;
    } else {
      const uint2 e = *reinterpret_cast<const uint2*>(cons + (s & 63) * 2);
      injn[0] = e.x; injn[1] = e.y;
    }
  };
  read_inj(s0);
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    const int s = s0 + q;
    unsigned inj[NP];
#pragma unroll
    for (int k = 0; k < NP; ++k) inj[k] = injn[k];
    if (q < 7) read_inj(s + 1);
    const unsigned sh = 31u - (unsigned)(s & 31);
    const unsigned y0 = __builtin_amdgcn_alignbit(yp0, w0, sh);
    const unsigned y1 = __builtin_amdgcn_alignbit(yp1, w1, sh);
#if NWK_BITS_BOP3
    const unsigned match = BOP3(x0 ^ y0, x1, y1, ~(kA | (kB ^ kC)));  // ~((x0^y0) | (x1^y1))
    unsigned U[NP], D[NP], Vn[NP], Hn[NP];
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      // lane t-1's plane word (lane 0: the band above), its bit 31 enters at bit 0
      const unsigned T = (unsigned)__builtin_amdgcn_update_dpp((int)inj[k], (int)H[k], 0x138 /*wave_shr:1*/, 0xf, 0xf, false);
      U[k] = __builtin_amdgcn_alignbit(H[k], T, 31);
      D[k] = k < SR ? ~0u : BOP3(match, U[k], V[k], kA | kB | kC);
    }
    bits_diffs<NP, SR>(U, D, Vn);
    bits_diffs<NP, SR>(V, D, Hn);
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      V[k] = Vn[k];
      H[k] = Hn[k];
    }
    if constexpr (SR < 0) dw[q] = match;
    else if constexpr (SR >= NP) dw[q] = ~0u;
    else dw[q] = BOP3(match, D[SR], D[SR], kA | ~kB);  // match | ~D_SR
    uw[q] = V[0];  // stored raw: the traceback's UP test is v == 0 (bit clear)
#else
    const unsigned mism = (x0 ^ y0) | (x1 ^ y1);
    const unsigned match = ~mism;
    unsigned nU[NP], nV[NP], D[NP];
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      // lane t-1's plane word (lane 0: the band above), its bit 31 enters at bit 0
      const unsigned T = (unsigned)__builtin_amdgcn_update_dpp((int)inj[k], (int)H[k], 0x138 /*wave_shr:1*/, 0xf, 0xf, false);
      const unsigned U = __builtin_amdgcn_alignbit(H[k], T, 31);
      nU[k] = ~U;
      nV[k] = ~V[k];
      D[k] = k < SR ? ~0u : (match | U | V[k]);
    }
#pragma unroll
    for (int k = 0; k < NP; ++k) {
      unsigned vk = nU[0] & D[k], hk = nV[0] & D[k];
#pragma unroll
      for (int j = 1; j + k < NP; ++j) {
        vk |= nU[j] & D[j + k];
        hk |= nV[j] & D[j + k];
      }
      V[k] = vk;
      H[k] = hk;
    }
    if constexpr (SR < 0) dw[q] = match;
    else if constexpr (SR >= NP) dw[q] = ~0u;
    else dw[q] = match | ~D[SR];
    uw[q] = V[0];
#endif
    if constexpr (MASK) {  // columns < 0 keep v = 0 (the left border seen by column 0)
      const int e = eh + q;
      const unsigned M = e >= 31 ? ~0u : (e < 0 ? 0u : (2u << e) - 1u);
#pragma unroll
      for (int k = 0; k < NP; ++k) V[k] &= M;
    }
    if constexpr (END) {
      const int bb = s - capc - 32 * lane;
      const unsigned mk = (unsigned)bb < 32u ? (1u << bb) & rowm : 0u;
#pragma unroll
      for (int k = 0; k < NP; ++k) *cnt += __builtin_popcount(V[k] & mk);
    }
    if constexpr (PROD) {  // lane 63 bit 31 = the band's last row at column s - 2047
      if (lane == 63) {
        unsigned* e = ring + (q + 1) * NP;
        if constexpr (NP == 4) *reinterpret_cast<uint4*>(e) = make_uint4(H[0], H[1], H[2], H[3]);
        else *reinterpret_cast<uint2*>(e) = make_uint2(H[0], H[1]);
      }
    }
    // a 4-step half's words go out as soon as they are complete (two 16-byte
    // stores, each 1 KB contiguous across the wave): 8 fewer live registers
    // than storing the whole block at its end
    if ((q & 3) == 3) {
      typedef unsigned u4 __attribute__((ext_vector_type(4)));
      const int h = q >> 2;
#ifdef NWK_BITS_NOSTORE  // A/B: fill without the traceback matrix (traces read garbage; time with NWK_NOTRACE)
      if (dw[4 * h] == 0x9e3779b9u && uw[4 * h + 3] == 0x7f4a7c15u) *st = dw[4 * h + 1] ^ uw[4 * h + 2];
#else
      // sto: the block is inside the pair's stored window (PairDesc::bits_w);
      // lsto per lane: the active lanes are contiguous, so the stores stay whole lines
      if (sto && lsto) {
        __builtin_nontemporal_store(u4{dw[4 * h], dw[4 * h + 1], dw[4 * h + 2], dw[4 * h + 3]},
                                    reinterpret_cast<u4*>(st + 256 * h));
        __builtin_nontemporal_store(u4{uw[4 * h], uw[4 * h + 1], uw[4 * h + 2], uw[4 * h + 3]},
                                    reinterpret_cast<u4*>(st + 512 + 256 * h));
      }
#endif
    }
  }
}

// Windowed storage writes only the lane words that hold a cell within w
// columns of the diagonal: lane words of one 8-step block cover rows R .. R+31
// (R = the lane's bit-0 row) at columns e - b (e = bit 0's column, b = bit), so
// dev = c m - i n over them spans [(e - 31) m - (R + 31) n, (e + 7) m - R n]
// (e at the block's first step).  hi = (e + 7) m - R n; the words are kept iff
// that span meets [-w m, w m].  The trace checks every cell it reads against
// the same |dev| <= w m (a kept cell's words were written) and flags the pair
// for a full re-run when its path leaves.  With w >= 2048 rows' worth this
// keeps nearly every word; at C4's w = 1024 about half of them, which halves
// the HBM writes of the stored blocks.
__device__ __forceinline__ bool bits_lane_stored(int64_t hi, int64_t lim, int64_t hlim) {
  return hi >= -lim && hi <= hlim;  // hlim = w m + 38 m + 31 n: the span's low end <= w m
}

// Traceback of one pair from (m, n) over the stored (diag, up) bits.
//
// Tiles are 64 steps (grid-aligned: ts = s | 63; lane L holds step ts - L) by
// four row-lanes ta .. ta - 3 (128 rows; the current row is in ta or below),
// eight dwords per lane.  While the walk crosses one tile, the next one along
// the steps (ts - 64, anchored at the row-lane the walk entered with) is
// already loading.
//
// Inside a tile the walk runs on the scalar unit over 64-bit lane masks.  A
// D move goes from (row r, lane L) to (r - 1, L + 2), so every cell of a
// diagonal run has the same key K = r + (L >> 1) and lies on lanes of L's
// parity.  Each lane re-indexes its column of bits by key (a per-lane funnel
// shift, once per tile): then one ballot per key gives, for every lane at
// once, whether its cell on that key's diagonal is a D move (Dm) or an UP
// move (Um).  A run from (L, K) stops at the first lane >= L of L's parity
// whose Dm bit is clear; that cell moves U or L as Um says, and the next run
// starts one lane on, at key K + (L & 1) - [U].  A run costs ~20 scalar
// instructions and two ballots only when its key is new, instead of a vector
// round trip per run.  The moves of a tile are written once, when it is left:
// lanes visited in lane order, each at its rank among the visited lanes
// (v_mbcnt), through a 1 KB LDS ring flushed to ops[].
__device__ __forceinline__ void trace_bits(const FillArgs& a, const PairDesc& pd, unsigned char* obuf, int lane,
                                           unsigned* prog, int& o_len, int2& o_end, bool& o_out) {
  const int nblk = pd.bits_nblk, win = pd.bits_w;
  const int64_t bdw = (int64_t)nblk * 1024;  // dwords per band
  // Storage map.  Banded tasks: band b's step s = c + r (its own numbering),
  // stored blocks bits_blk_lo(b) .. + nblk at b * bdw.  Strips (pd.bits_np =
  // n' > 0, one wave sweeps every band): s = c + r + b n' (the strip's
  // numbering); windowed, band b keeps blocks strip_blk_lo(b) .. + nblk at
  // b * bdw; full storage is one region of nblk blocks from block 0.
  const int snp = pd.bits_np;
  const bool sfull = snp > 0 && win <= 0;
  const unsigned* mat = a.mat + pd.mat_off;
  uint8_t* ops = a.ops + pd.ops_off;
  const unsigned ob = (unsigned)(uintptr_t)obuf;
  int Lc = 0, flushed = 0;
  auto flush = [&](int upto) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const int from = flushed & ~3;
    for (int o = from + 4 * lane; o < upto; o += 256) {
      unsigned v;
      asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(ob + (unsigned)(o & (kTraceRing - 1)))
                   : "memory");
      *reinterpret_cast<unsigned*>(ops + o) = v;
    }
    flushed = upto;
  };
  // position: band b, band row r (0..2047, -1 = the row above the band), column c (0-based)
  int b = (pd.m - 1) / kBR, r = (pd.m - 1) % kBR, c = pd.n - 1;
  if (a.dbg_notrace) c = -1;  // NWK_NOTRACE (fill timing): no moves, the walk "ends" at (m, n)
  int tb = -1, ts = 0, ta = 0, blo = 0, slo = 0;
  unsigned vd[4] = {0, 0, 0, 0}, vu[4] = {0, 0, 0, 0};
  // Tiles come in batches of kNB consecutive step-tiles: tile j of a batch
  // covers steps bts - 64 j - 63 .. bts - 64 j, row-lanes bpa[j] .. bpa[j] - 3
  // (anchored where the walk is predicted to enter it).  The walk crosses the
  // current batch (c*) while the next one (n*) is in flight; the next batch's
  // registers are read only after everything has arrived, so the compiler's
  // waits never stall the walk on it.  A tile is eight loads with addresses
  // clamped into the band's storage (cells off the stored steps or above row
  // 0 are never read: the walk's jmax excludes them).
  unsigned cd[kNB][4], cu[kNB][4], nd[kNB][4], nu[kNB][4];
  int cts = -1, cb = -1, cpa[kNB], nts = -1, nbb = -1, npa[kNB];
#pragma unroll
  for (int j = 0; j < kNB; ++j) cpa[j] = npa[j] = 0;
  // rows per step along the pair (16.16): predicts the row a tile ahead is entered at
  const int64_t slope = ((int64_t)pd.m << 16) / ((int64_t)pd.m + pd.n);
  auto load_tile = [&](int ts_, int ta_, unsigned (&d)[4], unsigned (&u)[4]) {
    int sl = ts_ - lane;
    int rel = (sl >> 3) - blo;
    const bool okl = sl >= 0 && (unsigned)rel < (unsigned)nblk;
    sl = okl ? sl : 0;
    rel = okl ? rel : 0;
    const unsigned* p0 =
        mat + (sfull ? 0 : (int64_t)b * bdw) + (int64_t)rel * 1024 + ((sl & 7) >> 2) * 256 + (sl & 3);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int rl = ta_ - k < 0 ? 0 : ta_ - k;
      d[k] = __builtin_nontemporal_load(p0 + 4 * rl);
      u[k] = __builtin_nontemporal_load(p0 + 512 + 4 * rl);
    }
  };
  // row-lane anchor of the tile k tiles ahead: the walk at (r, lane L) reaches
  // its top step after 64 k - L steps, ~slope rows per step; 24 rows of slack above
  auto predict = [&](int k, int L) {
    const int rp = r - (int)(((int64_t)(64 * k - L) * slope) >> 16);
    const int pa = (rp + 24) >> 5;
    return pa < 0 ? 0 : (pa > kBR / 32 - 1 ? kBR / 32 - 1 : pa);
  };
  bool bad = false, out = false;
  // verbose >= 2 timeline: walk cycles, runs, tiles entered, batches loaded (demand / ahead)
  const u64 tc0 = a.stamps ? __builtin_amdgcn_s_memtime() : 0;
  unsigned n_runs = 0, n_tiles = 0, n_dem = 0, n_ahead = 0;
#if NWK_TRACE_PROF
  u64 p_sw = 0, p_win = 0, p_walk = 0, p_out = 0, p_wait = 0, p_nb = 0;
#endif
  // windowed storage keeps only the lane words holding a cell within win
  // columns of the diagonal (bits_lane_stored): dev = c m - i n of the current
  // cell (i = b 2048 + r), |dev| <= win m, else the path has left them
  const int64_t lim = (int64_t)win * pd.m, dD = (int64_t)pd.n - pd.m, wmargin = 64 * ((int64_t)pd.m + pd.n);
  const bool lwin = bits_lane_window(win);
  auto devof = [&]() { return (int64_t)c * pd.m - (int64_t)(b * kBR + r) * pd.n; };
  if (lwin && c >= 0) {
    const int64_t dev = devof();
    if (dev > lim || dev < -lim) out = true;
  }
  constexpr u64 kEven = 0x5555555555555555ull;
  while (!out && c >= 0 && (b > 0 || r >= 0)) {
    if (r < 0) {  // into the band above
      --b;
      r += kBR;
    }
    const int t = r >> 5;
    int s = c + r + (snp > 0 ? b * snp : 0);
    if (b != tb) {
      blo = snp > 0 ? strip_blk_lo(b, pd.m, pd.n, snp, win) : bits_blk_lo(b, pd.m, pd.n, win);
      blo = __builtin_amdgcn_readfirstlane(blo);  // (uniform: keep the walk's bounds in SGPRs)
      slo = 8 * blo;  // lowest stored step of band b
    }
    if ((unsigned)((s >> 3) - blo) >= (unsigned)nblk) {  // the path left the stored window
      out = true;
      break;
    }
#if NWK_TRACE_PROF
    const u64 pt0 = __builtin_amdgcn_s_memtime();
#endif
    BITS_PROG(0x50000000u | ((unsigned)(Lc & 0xfff) << 16) | ((unsigned)(r & 0xff) << 8) | (unsigned)(c & 0xff));
    if (Lc - flushed >= kTraceRing - 128) flush(Lc & ~3);  // (a tile adds <= 64 moves to the ring)
    if (b != tb || s > ts || s <= ts - 64 || t > ta || t < ta - 3) {
      const int sg = s | 63;
      int j = (cts - sg) >> 6;
      if (!(b == cb && sg <= cts && j < kNB && t <= cpa[j] && t >= cpa[j] - 3)) {  // not in the current batch
        const int jn = (nts - sg) >> 6;
        if (!(b == nbb && sg <= nts && jn < kNB && t <= npa[jn] && t >= npa[jn] - 3)) {
          // nor in the next one: load the batch starting at this tile
          ++n_dem;
          nts = sg;
          nbb = b;
#pragma unroll
          for (int i = 0; i < kNB; ++i) {
            npa[i] = i == 0 ? t : predict(i, sg - s);
            load_tile(nts - 64 * i, npa[i], nd[i], nu[i]);
          }
        }
#if NWK_TRACE_PROF
        const u64 pw0 = __builtin_amdgcn_s_memtime();
#endif
        __builtin_amdgcn_s_waitcnt(waitcnt_vm(0));
#if NWK_TRACE_PROF
        p_wait += __builtin_amdgcn_s_memtime() - pw0;
        ++p_nb;
#endif
        cts = nts;
        cb = nbb;
#pragma unroll
        for (int i = 0; i < kNB; ++i) {
          cpa[i] = npa[i];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            cd[i][k] = nd[i][k];
            cu[i][k] = nu[i][k];
          }
        }
        j = (cts - sg) >> 6;
        // the batch after it goes out now
        nts = cts - 64 * kNB;
        nbb = nts >= slo ? b : -1;
        if (nbb >= 0) {
          ++n_ahead;
#pragma unroll
          for (int i = 0; i < kNB; ++i) {
            npa[i] = predict(kNB + i - j, sg - s);
            load_tile(nts - 64 * i, npa[i], nd[i], nu[i]);
          }
        }
      }
      ts = __builtin_amdgcn_readfirstlane(cts - 64 * j);
      {
        int pa = cpa[0];
#pragma unroll
        for (int i = 1; i < kNB; ++i) pa = j == i ? cpa[i] : pa;
        ta = __builtin_amdgcn_readfirstlane(pa);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        unsigned dd = cd[0][k], uu = cu[0][k];
#pragma unroll
        for (int i = 1; i < kNB; ++i) {
          dd = j == i ? cd[i][k] : dd;
          uu = j == i ? cu[i][k] : uu;
        }
        vd[k] = dd;
        vu[k] = uu;
      }
      tb = b;
      ++n_tiles;
    }
#if NWK_TRACE_PROF
    const u64 pt1 = __builtin_amdgcn_s_memtime();
    p_sw += pt1 - pt0;
#endif
    // Key window: keys Kb .. Kb + 31 around the entry key.  Lane l's bit i is
    // its cell at row Kb + i - (l >> 1): bit q = that row - 32 (ta - 3) + 32 of
    // the column {0, vd[3], vd[2], vd[1], vd[0], 0} (rows outside the tile read 0).
    int L = ts - s;
    const int Kb = r + (L >> 1) - 20;
    const int rowlo = ta > 3 ? 32 * (ta - 3) : 0;  // lowest row of the tile
    unsigned WD, WU;
    {
      const int q = Kb - (lane >> 1) - 32 * (ta - 3) + 32;
      const int dq = q >> 5, sh = q & 31;
      const bool ok = q >= 0 && q < 160;
      const unsigned dlo = dq == 1 ? vd[3] : dq == 2 ? vd[2] : dq == 3 ? vd[1] : dq == 4 ? vd[0] : 0u;
      const unsigned dhi = dq == 0 ? vd[3] : dq == 1 ? vd[2] : dq == 2 ? vd[1] : dq == 3 ? vd[0] : 0u;
      const unsigned ulo = dq == 1 ? vu[3] : dq == 2 ? vu[2] : dq == 3 ? vu[1] : dq == 4 ? vu[0] : ~0u;
      const unsigned uhi = dq == 0 ? vu[3] : dq == 1 ? vu[2] : dq == 2 ? vu[1] : dq == 3 ? vu[0] : ~0u;
      WD = ok ? __builtin_amdgcn_alignbit(dhi, dlo, sh) : 0u;
      WU = ok ? __builtin_amdgcn_alignbit(uhi, ulo, sh) : ~0u;  // stored up word: 0 = UP
    }
#if NWK_TRACE_PROF
    const u64 pt2 = __builtin_amdgcn_s_memtime();
    p_win += pt2 - pt1;
#endif
    const bool wchk = lwin && [&] {
      const int64_t dev = devof();
      return dev > lim - wmargin || dev < -lim + wmargin;
    }();
    u64 vD = 0, vU = 0, vL = 0;  // lanes visited by D / U / L moves in this tile
    // The run loop, all scalar; a second copy checks the stored lane words
    // (windowed storage, only in tiles near the window's edge).
    auto walk = [&](auto chk) {
      constexpr bool kChk = decltype(chk)::value;
      int Kc = -(1 << 30);
      u64 Dm = 0, Um = 0;
      for (;;) {
        if constexpr (kChk) {  // this cell must be inside the stored lane words
          const int64_t dev = devof();
          if (dev > lim || dev < -lim) {
            out = true;
            return;
          }
        }
        if (a.stamps) ++n_runs;
        const int K = r + (L >> 1);
        if (K != Kc) {
          const int i = K - Kb;
          if ((unsigned)i > 31u) return;  // off the key window: re-window (same tile)
          Dm = __builtin_amdgcn_ballot_w64((WD >> i) & 1u);
          Um = __builtin_amdgcn_ballot_w64(!((WU >> i) & 1u));
          Kc = K;
        }
        // the run's cells j = 0 .. jmax are readable: in the tile's lanes and
        // rows, columns >= 0, stored steps (>= slo)
        const int jmax = smin(smin((63 - L) >> 1, r - rowlo), smin(c, (s - slo) >> 1));
        const u64 par = (L & 1) ? ~kEven : kEven;
        const u64 stops = ~Dm & par & (~0ull << L);
        const int lend = L + 2 * jmax + 2;  // first lane past the readable cells
        const int ls = min(stops ? (int)__builtin_ctzll(stops) : lend, lend);
        const int jn = (ls - L) >> 1;  // D moves: cells 0 .. jn - 1
        if constexpr (kChk) {
          if (dD != 0) {  // dev is linear along the run: check its far end
            const int64_t de = devof() + (int64_t)(ls < lend ? jn : jmax) * dD;
            if (de > lim || de < -lim) {
              out = true;
              return;
            }
          }
        }
        vD |= par & (ls >= 64 ? ~0ull : ((1ull << ls) - 1)) & (~0ull << L);
        r -= jn;
        c -= jn;
        s -= 2 * jn;
        if (ls >= lend) return;  // the run leaves the tile
        // cell jn stops the run: U or L
        const u64 bit = 1ull << ls;
        const int u = (Um & bit) ? 1 : 0;
        vU |= u ? bit : 0ull;
        vL |= u ? 0ull : bit;
        r -= u;
        c -= 1 - u;
        s -= 1;
        L = ls + 1;
        if ((L > 63) | (c < 0) | (r < rowlo) | (s < slo)) return;
      }
    };
    if (wchk) {
      walk(std::true_type{});
    } else {
      // The common case, ~28 scalar instructions a run.  The walk carries
      // three lane bounds that a D run leaves unchanged: A = L + 2 (r - rowlo)
      // (the tile's top row), B = L + 2 c (column 0) and LL (the last stored
      // step); a U stop moves them by (-1, +1), an L stop by (+1, -1), and the
      // key by (ls & 1) - [U].  r and c are recovered from A, B and L at the
      // end.  The D lanes are not collected per run but rebuilt once from the
      // stops below.
      const int LL = smin(63, ts - slo);  // last lane whose step is stored
      const int L0 = L;
      u64 vS = 0;  // lanes of the runs' stopping cells (U or L moves)
      int Kc = -(1 << 30);
      u64 SE = 0, SO = 0, Um = 0;  // the key's stops on even / odd lanes, its U cells
      int A = L + 2 * (r - rowlo), B = L + 2 * c, K = r + (L >> 1);
      for (;;) {
        const int bnd = smin(smin(A, B), LL);
        if (L > bnd) break;  // the current cell is outside the tile
        ++n_runs;
        if (K != Kc) {
          const int i = K - Kb;
          if ((unsigned)i > 31u) break;  // off the key window: re-window (same tile)
          const u64 Dm = __builtin_amdgcn_ballot_w64((WD >> i) & 1u);
          Um = __builtin_amdgcn_ballot_w64(!((WU >> i) & 1u));
          SE = ~Dm & kEven;
          SO = ~Dm & ~kEven;
          Kc = K;
        }
        const int lend = L + ((bnd - L) & ~1) + 2;  // first lane past the readable cells
        const u64 stops = ((L & 1) ? SO : SE) & (~0ull << L);
        const int ls = sminu(sff1(stops), lend);  // (no stop: ff1 = -1)
        if (ls >= lend) {  // the run leaves the tile
          L = lend;
          break;
        }
        vS |= 1ull << ls;
        const int u = (int)((Um >> ls) & 1ull);
        vU |= (u64)u << ls;
        A += 1 - 2 * u;
        B += 2 * u - 1;
        K += (ls & 1) - u;
        L = ls + 1;
      }
      r = rowlo + ((A - L) >> 1);
      c = (B - L) >> 1;
      // D lanes: in [L0, L), not a stop, an even offset from the start of their run
      const u64 starts = (1ull << L0) | (vS << 1);
      const u64 sb = (starts & ((2ull << lane) - 1)) | 1ull;
      const int a0 = 63 - __builtin_clzll(sb);
      vD = __builtin_amdgcn_ballot_w64(lane >= L0 && lane < L && !((vS >> lane) & 1u) && !((lane - a0) & 1));
      vL = vS & ~vU;
    }
#if NWK_TRACE_PROF
    const u64 pt3 = __builtin_amdgcn_s_memtime();
    p_walk += pt3 - pt2;
#endif
    // the tile's moves, in lane order, into the ring
    {
      const u64 vis = vD | vU | vL;
      const unsigned rank = __builtin_amdgcn_mbcnt_hi((unsigned)(vis >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)vis, 0u));
      const unsigned ch = ((vU >> lane) & 1u) ? 'U' : ((vL >> lane) & 1u) ? 'L' : 'D';
      if ((vis >> lane) & 1u)
        asm volatile("ds_write_b8 %0, %1" ::"v"(ob + (unsigned)((Lc + (int)rank) & (kTraceRing - 1))), "v"(ch)
                     : "memory");
      Lc += __builtin_popcountll(vis);
    }
#if NWK_TRACE_PROF
    p_out += __builtin_amdgcn_s_memtime() - pt3;
#endif
    if (out) break;
    if (Lc > pd.m + pd.n) {
      bad = true;
      break;
    }
  }
  if (bad && lane == 0) atomicOr(a.err, 16u);
  if (a.stamps && lane == 0) {
    u64* x = a.stamps + 8 * pd.slot;
    x[2] = __builtin_amdgcn_s_memtime() - tc0;
#if NWK_TRACE_PROF  // {tile switch | key window} {walk | move output} {load wait | batches} cycles
    x[3] = (p_sw << 32) | p_win;
    x[4] = (p_walk << 32) | p_out;
    x[5] = (p_wait << 32) | p_nb;
#else
    x[3] = n_runs;
    x[4] = (u64)Lc;
    x[5] = ((u64)n_tiles << 32) | ((u64)n_dem << 16) | n_ahead;
#endif
  }
  flush(Lc);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // out of the window: a placeholder result (no moves) and the re-run flag;
  // otherwise the walk ends on the border: row b * 2048 + r + 1, column c + 1
  o_len = out ? 0 : Lc;
  o_end = (a.dbg_notrace || out) ? make_int2(pd.m, pd.n) : make_int2(b * kBR + r + 1, c + 1);
  o_out = out;
  if (lane == 0) {
    a.oplen[pd.slot] = o_len;
    a.endij[pd.slot] = o_end;
    if (out) a.retry[pd.slot] = 1;
  }
}

template <int NP, int SR, bool FUSE>
__global__ __launch_bounds__(256) NWK_BITS_OCC void nw_align_bits(FillArgs a) {
  __shared__ __attribute__((aligned(16))) unsigned cons_all[4][64 * NP];
  __shared__ __attribute__((aligned(16))) unsigned ring_all[4][129 * NP];
  __shared__ __attribute__((aligned(16))) unsigned char obuf_all[4][kTraceRing];
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  unsigned* prog = a.prog ? a.prog + blockIdx.x * 4 + wid : nullptr;  // NWK_WATCHDOG markers
  unsigned* cons = cons_all[wid];
  unsigned* ring = ring_all[wid];
  constexpr int NG = 2 * NP;  // granules per 64-column chunk
  // verbose >= 2 timeline (FillArgs::stamps, layout in nwk_runtime.cpp)
  if (a.stamps && threadIdx.x == 0) atomicMin(a.stamps + 11 * a.ntasks_pairs, (u64)__builtin_amdgcn_s_memrealtime());

  for (;;) {
    if constexpr (FUSE) {  // queued pairs to hash: whole groups between fill tasks
      while (hq_hash(a, lane, false)) {
      }
    }
    unsigned tk = 0;
    if (lane == 0) tk = atomicAdd(a.counter, 1u);
    tk = __builtin_amdgcn_readfirstlane(tk);
    BITS_PROG(0x10000000u | tk);
    if (tk >= (unsigned)a.ntasks) {
      if constexpr (FUSE) hq_drain(a, lane);
      BITS_PROG(0x60000000u);
      return;
    }
    // wave-uniform exit (a per-lane load would make the task loop divergent)
    if (__builtin_amdgcn_readfirstlane(__hip_atomic_load((gu32*)a.err, BITS_RLX)) != 0u) return;
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
    unsigned H[NP], V[NP];
#pragma unroll
    for (int k = 0; k < NP; ++k) H[k] = V[k] = 0u;
    const bool from_above = band > 0;
    const bool to_below = band + 1 < pd.nbands;
    const int nch = pd.nchunks, nsb = pd.sblocks;
    const u64* gin = reinterpret_cast<const u64*>(a.bnd) + pd.bnd_off + (int64_t)(from_above ? band - 1 : 0) * nch * NG;
    u64* gout = a.bnd + pd.bnd_off + (int64_t)band * nch * NG;
    const int nblk = pd.bits_nblk, blo = bits_blk_lo(band, pd.m, pd.n, pd.bits_w);
    unsigned* mb = a.mat + pd.mat_off + (int64_t)band * nblk * 1024 + lane * 4;
    // windowed, w < 2048: per-lane store predicate (bits_lane_stored) for rows
    // R0 + 32 lane ..; hi of the block at step s0 = hi0 + s0 m
    const bool lwin = bits_lane_window(pd.bits_w);
    const int64_t lim = (int64_t)pd.bits_w * pd.m, hlim = lim + 38ll * pd.m + 31ll * pd.n;
    const int64_t hi0 = (int64_t)(7 - 32 * lane) * pd.m - (int64_t)(R0 + 32 * lane) * pd.n;
    // y windows: lane t's window for the half starting at step s_h is position s_h - 32 t
    const unsigned* ywp = a.yw + 2 * (pd.e_off - 32 * (int64_t)lane);
    unsigned yp0 = 0, yp1 = 0;
    unsigned wa0 = ywp[0], wa1 = ywp[1], wb0 = ywp[64], wb1 = ywp[65];
    const bool gl = lane < NG;
    u64 g = 0;
    if (from_above && gl) g = __hip_atomic_load((gu64*)(gin + lane), BITS_RLX);
    bool ok = true;
    const u64 t_task = a.stamps ? __builtin_amdgcn_s_memtime() : 0;
    u64 cyc_wait = 0, cyc_wait0 = 0, n_wait = 0;
    // fill-vs-walk guard: G(m, n) = -sum of v down column n; row 32 t + b
    // reaches column n - 1 (0-based) at step n - 1 + 32 t + b: super-blocks sbe ..
    const int capc = pd.n - 1;
    const bool want_end = a.endv != nullptr;
    const int sbe = want_end ? capc >> 6 : nsb;
    const int capx = want_end ? capc : -100000;
    int cnt = 0;
    unsigned rowm;
    {
      const int nvr = pd.m - R0 - 32 * lane;
      rowm = nvr >= 32 ? ~0u : (nvr <= 0 ? 0u : (1u << nvr) - 1u);
    }

    for (int sb = 0; sb < nsb; ++sb) {
      BITS_PROG(0x20000000u | (unsigned)sb);
      // --- band-above row for columns 64 sb .. 64 sb + 63 -> cons
      if (from_above && sb < nch) {
        if (!__all(!gl || (unsigned)(g >> 32) == a.epoch)) {
          const u64 tw = a.stamps ? __builtin_amdgcn_s_memtime() : 0;
          g = bits_wait(gin + (int64_t)sb * NG + lane, gl, a.epoch, g, a.err);
          if (a.stamps) {
            const u64 d = __builtin_amdgcn_s_memtime() - tw;
            cyc_wait += d;
            if (sb == 0) cyc_wait0 = d;
            ++n_wait;
          }
          if (!__all(!gl || (unsigned)(g >> 32) == a.epoch)) { ok = false; break; }
        }
        const unsigned dat = (unsigned)g;
        unsigned e[NP];
#pragma unroll
        for (int k = 0; k < NP; ++k) {
          const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)dat, 2 * k);
          const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)dat, 2 * k + 1);
          const unsigned w = lane < 32 ? lo : hi;
          e[k] = (w >> (lane & 31)) << 31;
        }
        if constexpr (NP == 4) *reinterpret_cast<uint4*>(cons + lane * 4) = make_uint4(e[0], e[1], e[2], e[3]);
        else *reinterpret_cast<uint2*>(cons + lane * 2) = make_uint2(e[0], e[1]);
      } else if (sb == 0 || sb == nch) {  // top border (band 0) / past the last chunk: zeros
        if constexpr (NP == 4) *reinterpret_cast<uint4*>(cons + lane * 4) = make_uint4(0, 0, 0, 0);
        else *reinterpret_cast<uint2*>(cons + lane * 2) = make_uint2(0, 0);
      }
      if (from_above && sb + 1 < nch && gl) g = __hip_atomic_load((gu64*)(gin + (int64_t)(sb + 1) * NG + lane), BITS_RLX);
      // next super-block's windows
      const unsigned* wn = ywp + 128 * (sb + 1);
      const unsigned na0 = wn[0], na1 = wn[1], nb0 = wn[64], nb1 = wn[65];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();

      const bool mask = sb < 32;
      const bool prod = to_below && sb >= 31;
      unsigned* const ring_sb = ring + ((64 * sb) & 127) * NP;
#pragma unroll
      for (int blk = 0; blk < 8; ++blk) {
        const int s0 = 64 * sb + 8 * blk;
        unsigned* const rblk = ring_sb + 8 * blk * NP;  // (s0 & 127) = (64 sb & 127) + 8 blk
        const unsigned w0 = blk < 4 ? wa0 : wb0, w1 = blk < 4 ? wa1 : wb1;
        const int rel = (s0 >> 3) - blo;
        const bool sto = (unsigned)rel < (unsigned)nblk;
        unsigned* st = mb + (int64_t)rel * 1024;
        const int eh = s0 - 32 * lane;
        bool ls = true;
        if (lwin) ls = bits_lane_stored(hi0 + (int64_t)s0 * pd.m, lim, hlim);
        if (mask) {  // (the masked super-blocks always take the guard's END form)
          if (prod)
            bits_block<NP, SR, true, true, true>(s0, lane, x0, x1, yp0, yp1, w0, w1, H, V, cons, rblk, st, sto, eh, ls,
                                                 capx, rowm, &cnt);
          else
            bits_block<NP, SR, true, false, true>(s0, lane, x0, x1, yp0, yp1, w0, w1, H, V, cons, rblk, st, sto, eh, ls,
                                                  capx, rowm, &cnt);
        } else if (sb >= sbe) {
          if (prod)
            bits_block<NP, SR, false, true, true>(s0, lane, x0, x1, yp0, yp1, w0, w1, H, V, cons, rblk, st, sto, eh, ls,
                                                  capx, rowm, &cnt);
          else
            bits_block<NP, SR, false, false, true>(s0, lane, x0, x1, yp0, yp1, w0, w1, H, V, cons, rblk, st, sto, eh,
                                                   ls, capx, rowm, &cnt);
        } else {
          if (prod) bits_block<NP, SR, false, true>(s0, lane, x0, x1, yp0, yp1, w0, w1, H, V, cons, rblk, st, sto, eh, ls);
          else bits_block<NP, SR, false, false>(s0, lane, x0, x1, yp0, yp1, w0, w1, H, V, cons, rblk, st, sto, eh, ls);
        }
        if ((blk & 3) == 3) {  // end of a 32-step half: its window becomes the previous one
          yp0 = w0;
          yp1 = w1;
        }
      }
      wa0 = na0; wa1 = na1; wb0 = nb0; wb1 = nb1;
      // --- publish chunk q = sb - 32 of this band's last row (complete after this super-block)
      if (to_below && sb >= 32 && sb - 32 < nch) {
        const int q = sb - 32;
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        const unsigned* e = ring + ((((64 * q + lane) - 1) & 127) + 1) * NP;
        unsigned val = 0;
#pragma unroll
        for (int k = 0; k < NP; ++k) {
          const u64 m64 = __ballot((e[k] >> 31) != 0u);
          val = lane == 2 * k ? (unsigned)m64 : val;
          val = lane == 2 * k + 1 ? (unsigned)(m64 >> 32) : val;
        }
        if (gl) __hip_atomic_store((gu64*)(gout + (int64_t)q * NG + lane), ((u64)a.epoch << 32) | val, BITS_RLX);
      }
    }
    BITS_PROG(0x30000000u);
    if (!ok) return;
    if (want_end) {  // this band's part of H(m, n): - sum v (+ (m + n) pgap once, band 0)
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o);
      if (lane == 0)
        __hip_atomic_fetch_add((gu32*)(a.endv + pd.slot), (unsigned)(band == 0 ? (pd.m + pd.n) * a.pgap - cnt : -cnt),
                               BITS_RLX);
    }
    if (a.stamps && lane == 0) {  // per pair: band cycles, of which waiting on the band above
      atomicAdd(a.stamps + 8 * pd.slot + 6, (u64)(__builtin_amdgcn_s_memtime() - t_task));
      atomicAdd(a.stamps + 8 * pd.slot + 7, cyc_wait);
      atomicAdd(a.stamps + 8 * a.ntasks_pairs + 3 * pd.slot, cyc_wait0);
      atomicAdd(a.stamps + 8 * a.ntasks_pairs + 3 * pd.slot + 1, n_wait);
      atomicAdd(a.stamps + 8 * a.ntasks_pairs + 3 * pd.slot + 2, (u64)nsb);
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
      // (NWK_NOTRACE runs trace_bits too, with no moves: a separate branch here
      // made the compiler's task-loop structure hang on single-band pairs)
      BITS_PROG(0x40000000u);
      if (a.stamps && lane == 0) a.stamps[8 * pd.slot] = __builtin_amdgcn_s_memrealtime();
#if NWK_TRACE_PRIO
      // the walk is one latency-bound wave: let it issue ahead of the SIMD's fill waves
      __builtin_amdgcn_s_setprio(3);
#endif
      int tlen;
      int2 tend;
      bool tout;
      trace_bits(a, pd, obuf_all[wid], lane, prog, tlen, tend, tout);
#if NWK_TRACE_PRIO
      __builtin_amdgcn_s_setprio(0);
#endif
      if constexpr (FUSE) {
        const bool ok_rows = !tout && fin_rows(a, pd, lane, tlen, tend);
        hq_push(a, pd, lane, ok_rows);
      }
      if (a.stamps && lane == 0) a.stamps[8 * pd.slot + 1] = __builtin_amdgcn_s_memrealtime();
      BITS_PROG(0x56000000u);
    }
  }
}

// Rolling strips (mode kBitsStrip): one wave sweeps ALL bands of a pair.
// Lane bit p (= 32 lane + b) runs rows p, p + 2048, p + 4096, ... : at step s
// its virtual column is v = s - p, its row pass k = v / n' and its column
// v % n' (n' = a multiple of 64, at least n + 32: the 32+ columns past n are
// junk).  When a bit leaves its pass it enters column 0 of row p + 2048 (k + 1):
//   * its left input must be the border (v = 0): the MASK blocks clear V of
//     the bits that have not yet entered the pass, as the banded kernel does
//     for columns < 0 -- those bits are in the junk columns of the pass before;
//   * its row code changes: a lane switches x to its next pass's rows at the
//     32-step half where its bit 0 enters the pass (its bits 1..31 are still
//     in junk columns, so their codes do not matter);
//   * lane 0 bit 0 (row 2048 (k + 1)) reads the pass above's last row (lane
//     63 bit 31, row 2048 k + 2047) -- produced by this same wave n' - 2047
//     steps earlier, so it goes through an LDS ring of one 64-column chunk per
//     slot (hand[], 2 NP packed dwords per chunk) instead of HBM granules, and
//     nothing ever waits.
// Against 2048-row band tasks (each band sweeps n + 2048 steps, the skew paid
// per band) a strip pays the 2047-step skew once per pair, and it needs no
// inter-wave hand-off.  The price is the pair's latency (one wave does all
// nb x n' steps), so the runtime picks strips for jobs with many pairs per
// wave slot (C4: 32,640 pairs of 8k on 4,096 slots).
// y windows: the column sequence's usual windows, indexed by the wrapped
// column (32-step halves are 32-aligned and n' is a multiple of 64, so a
// window never straddles the wrap).  Row codes: the row sequence's y windows,
// bit-reversed (bit b = row 32 lane + b).  Storage: the strip's 8-step blocks
// in order (full), or per band the blocks strip_blk_lo(band) .. + nblk of its
// W-column diagonal window (the runtime keeps the bands' windows disjoint).
template <int NP, int SR, bool FUSE>
__global__ __launch_bounds__(256) NWK_BITS_OCC void nw_align_strip(FillArgs a) {
  __shared__ __attribute__((aligned(16))) unsigned cons_all[4][64 * NP];
  __shared__ __attribute__((aligned(16))) unsigned ring_all[4][129 * NP];
  __shared__ __attribute__((aligned(16))) unsigned char obuf_all[4][kTraceRing];
  extern __shared__ __attribute__((aligned(16))) unsigned hand_all[];  // [4][a.strip_ring]
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  unsigned* prog = a.prog ? a.prog + blockIdx.x * 4 + wid : nullptr;  // NWK_WATCHDOG markers
  unsigned* cons = cons_all[wid];
  unsigned* ring = ring_all[wid];
  unsigned* hand = hand_all + wid * a.strip_ring;
  constexpr int NG = 2 * NP;  // packed dwords per 64-column chunk of a pass's last row

  for (;;) {
    if constexpr (FUSE) {
      while (hq_hash(a, lane, false)) {
      }
    }
    unsigned tk = 0;
    if (lane == 0) tk = atomicAdd(a.counter, 1u);
    tk = __builtin_amdgcn_readfirstlane(tk);
    BITS_PROG(0x10000000u | tk);
    if (tk >= (unsigned)a.ntasks) {
      if constexpr (FUSE) hq_drain(a, lane);
      BITS_PROG(0x60000000u);
      return;
    }
    if (__builtin_amdgcn_readfirstlane(__hip_atomic_load((gu32*)a.err, BITS_RLX)) != 0u) return;
    const PairDesc pd = a.pairs[a.tasks[tk].x];
    const int np = pd.bits_np, nch = np >> 6, nb = pd.nbands, nsb = pd.sblocks;
    if (a.stamps && lane == 0) a.stamps[8 * pd.slot + 6] = __builtin_amdgcn_s_memrealtime();
    // row code planes of pass 0 and (ahead) pass 1: bit b = row 2048 k + 32 lane + b
    const unsigned* xw = a.yw + 2 * (pd.xw_off + 32 * (int64_t)lane);
    unsigned x0 = __builtin_bitreverse32(xw[0]), x1 = __builtin_bitreverse32(xw[1]);
    unsigned nx0 = 0, nx1 = 0;
    if (nb > 1) {
      nx0 = __builtin_bitreverse32(xw[2 * kBR]);
      nx1 = __builtin_bitreverse32(xw[2 * kBR + 1]);
    }
    unsigned H[NP], V[NP];
#pragma unroll
    for (int k = 0; k < NP; ++k) H[k] = V[k] = 0u;
    // y windows by wrapped column: ua / ub = this lane's bit-0 column at the
    // start of the super-block's two halves (negative before pass 0 starts)
    const unsigned* yb = a.yw + 2 * pd.e_off;
    int ua = -32 * lane, ub = ua + 32;
    unsigned wa0 = yb[2 * ua], wa1 = yb[2 * ua + 1], wb0 = yb[2 * ub], wb1 = yb[2 * ub + 1];
    unsigned yp0 = 0, yp1 = 0;
    const bool win = pd.bits_w > 0;
    const int nblk = pd.bits_nblk;
    int kw = 0, blo = win ? strip_blk_lo(0, pd.m, pd.n, np, pd.bits_w) : 0;  // current storage window
    // windowed, w < 2048: per-lane store predicate (bits_lane_stored) for the
    // rows of the lane's current pass; hi = (e + 7) m - R n, e = bit 0's column
    const bool lwin = bits_lane_window(pd.bits_w);
    const int64_t lim = (int64_t)pd.bits_w * pd.m, hlim = lim + 38ll * pd.m + 31ll * pd.n;
    int64_t negRn = -(int64_t)(32 * lane) * pd.n;
    unsigned* mb = a.mat + pd.mat_off + lane * 4;
    int q0 = 0, k0 = 0;  // lane 0 bit 0: chunk and pass of this super-block
    int pslot = 0;       // hand[] slot of the chunk published at the end of this super-block (sb >= 32)

    for (int sb = 0; sb < nsb; ++sb) {
      BITS_PROG(0x20000000u | (unsigned)sb);
      // --- pass k0's row above (pass k0 - 1's last row) for columns 64 q0 .. + 63 -> cons
      if (k0 > 0) {
        const unsigned dat = lane < NG ? hand[q0 * NG + lane] : 0u;
        unsigned e[NP];
#pragma unroll
        for (int k = 0; k < NP; ++k) {
          const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)dat, 2 * k);
          const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)dat, 2 * k + 1);
          const unsigned w = lane < 32 ? lo : hi;
          e[k] = (w >> (lane & 31)) << 31;
        }
        if constexpr (NP == 4) *reinterpret_cast<uint4*>(cons + lane * 4) = make_uint4(e[0], e[1], e[2], e[3]);
        else *reinterpret_cast<uint2*>(cons + lane * 2) = make_uint2(e[0], e[1]);
      } else if (sb == 0) {  // pass 0: the top border (zeros)
        if constexpr (NP == 4) *reinterpret_cast<uint4*>(cons + lane * 4) = make_uint4(0, 0, 0, 0);
        else *reinterpret_cast<uint2*>(cons + lane * 2) = make_uint2(0, 0);
      }
      // next super-block's windows (wrapped), and ahead of a pass boundary the
      // next pass's row codes (lane t switches to them t / 2 super-blocks later)
      int na = ua + 64;
      if (na >= np) na -= np;
      int nbw = na + 32;
      if (nbw >= np) nbw -= np;
      const unsigned na0 = yb[2 * na], na1 = yb[2 * na + 1], nb0 = yb[2 * nbw], nb1 = yb[2 * nbw + 1];
      if (q0 == nch - 1 && k0 > 0 && k0 + 1 < nb) {  // (pass 1's codes were loaded with the task)
        nx0 = __builtin_bitreverse32(xw[2 * (int64_t)kBR * (k0 + 1)]);
        nx1 = __builtin_bitreverse32(xw[2 * (int64_t)kBR * (k0 + 1) + 1]);
      }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();

      const bool mask = q0 < 32;  // some lane's bit 0 enters a pass in this super-block
      const bool prod = sb >= 31;
      unsigned* const ring_sb = ring + ((64 * sb) & 127) * NP;
#pragma unroll
      for (int blk = 0; blk < 8; ++blk) {
        const int s0 = 64 * sb + 8 * blk;
        unsigned* const rblk = ring_sb + 8 * blk * NP;  // (s0 & 127) = (64 sb & 127) + 8 blk
        const unsigned w0 = blk < 4 ? wa0 : wb0, w1 = blk < 4 ? wa1 : wb1;
        const int uh = blk < 4 ? ua : ub;
        if ((blk & 3) == 0 && mask) {  // this lane's bit 0 enters pass >= 1 here: switch the row codes
          const bool sw = uh == 0 && s0 > 32 * lane;
          x0 = sw ? nx0 : x0;
          x1 = sw ? nx1 : x1;
          negRn -= sw ? (int64_t)kBR * pd.n : 0;
        }
        const int eh = uh + 8 * (blk & 3);
        const int K = 8 * sb + blk;  // the block's index in the strip
        bool sto = true;
        unsigned* st = mb + (int64_t)K * 1024;
        if (win) {
          while (kw < nb && K >= blo + nblk) {
            ++kw;
            blo = kw < nb ? strip_blk_lo(kw, pd.m, pd.n, np, pd.bits_w) : 0;
          }
          sto = kw < nb && K >= blo;
          st = mb + ((int64_t)kw * nblk + (K - blo)) * 1024;
        }
        bool ls = true;
        if (lwin) ls = bits_lane_stored((int64_t)(eh + 7) * pd.m + negRn, lim, hlim);
        if (mask) {
          if (prod) bits_block<NP, SR, true, true>(s0, lane, x0, x1, yp0, yp1, w0, w1, H, V, cons, rblk, st, sto, eh, ls);
          else bits_block<NP, SR, true, false>(s0, lane, x0, x1, yp0, yp1, w0, w1, H, V, cons, rblk, st, sto, eh, ls);
        } else {
          if (prod) bits_block<NP, SR, false, true>(s0, lane, x0, x1, yp0, yp1, w0, w1, H, V, cons, rblk, st, sto, eh, ls);
          else bits_block<NP, SR, false, false>(s0, lane, x0, x1, yp0, yp1, w0, w1, H, V, cons, rblk, st, sto, eh, ls);
        }
        if ((blk & 3) == 3) {  // end of a 32-step half: its window becomes the previous one
          yp0 = w0;
          yp1 = w1;
        }
      }
      wa0 = na0; wa1 = na1; wb0 = nb0; wb1 = nb1;
      ua = na;
      ub = nbw;
      // --- chunk sb - 32 of the strip's last-row stream (lane 63 bit 31) is complete: into hand[]
      if (sb >= 32) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        const unsigned* e = ring + ((((64 * sb + lane) - 1) & 127) + 1) * NP;
        unsigned val = 0;
#pragma unroll
        for (int k = 0; k < NP; ++k) {
          const u64 m64 = __ballot((e[k] >> 31) != 0u);
          val = lane == 2 * k ? (unsigned)m64 : val;
          val = lane == 2 * k + 1 ? (unsigned)(m64 >> 32) : val;
        }
        if (lane < NG) hand[pslot * NG + lane] = val;
        if (++pslot == nch) pslot = 0;
      }
      if (++q0 == nch) {
        q0 = 0;
        ++k0;
      }
    }
    BITS_PROG(0x30000000u);
    // the trace reads this wave's own stores
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (a.stamps && lane == 0) a.stamps[8 * pd.slot] = __builtin_amdgcn_s_memrealtime();
    BITS_PROG(0x40000000u);
    int tlen;
    int2 tend;
    bool tout;
    trace_bits(a, pd, obuf_all[wid], lane, prog, tlen, tend, tout);
    if constexpr (FUSE) {
      const bool ok_rows = !tout && fin_rows(a, pd, lane, tlen, tend);
      hq_push(a, pd, lane, ok_rows);
    }
    if (a.stamps && lane == 0) a.stamps[8 * pd.slot + 1] = __builtin_amdgcn_s_memrealtime();
    BITS_PROG(0x56000000u);
  }
}

template <int NP, int SR>
hipError_t bits_launch(const FillArgs& a, int grid, hipStream_t s) {
  if (a.fuse_fin) hipLaunchKernelGGL((nw_align_bits<NP, SR, true>), dim3(grid), dim3(256), 0, s, a);
  else hipLaunchKernelGGL((nw_align_bits<NP, SR, false>), dim3(grid), dim3(256), 0, s, a);
  return hipGetLastError();
}

template <int NP, int SR>
hipError_t strip_launch(const FillArgs& a, int grid, hipStream_t s) {
  if (a.fuse_fin) hipLaunchKernelGGL((nw_align_strip<NP, SR, true>), dim3(grid), dim3(256), (size_t)4 * a.strip_ring * 4, s, a);
  else hipLaunchKernelGGL((nw_align_strip<NP, SR, false>), dim3(grid), dim3(256), (size_t)4 * a.strip_ring * 4, s, a);
  return hipGetLastError();
}

template <int NP, int SR>
int strip_occ(int ring_dwords) {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, reinterpret_cast<const void*>(&nw_align_strip<NP, SR, false>), 256,
                                                   (size_t)4 * ring_dwords * 4) != hipSuccess)
    return 1;
  return n > 0 ? n : 1;
}

template <int NP, int SR>
int bits_occ() {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, reinterpret_cast<const void*>(&nw_align_bits<NP, SR, false>), 256, 0) !=
      hipSuccess)
    return 1;
  return n > 0 ? n : 1;
}

}  // namespace

// SR = 2 pgap - pxy clamped to [-1, NP]: the mismatch score's thermometer level
int bits_sr(int pxy, int pgap) {
  const int np = 2 * pgap, sr = np - pxy;
  return sr < -1 ? -1 : (sr > np ? np : sr);
}

bool bits_admissible(int pxy, int pgap, int alpha) { return pxy >= 0 && (pgap == 1 || pgap == 2) && alpha <= 4; }

hipError_t launch_bits(const FillArgs& a, int pxy, int pgap, int grid, hipStream_t s) {
  const int sr = bits_sr(pxy, pgap);
  if (pgap == 1) {
    switch (sr) {
      case -1: return bits_launch<2, -1>(a, grid, s);
      case 0: return bits_launch<2, 0>(a, grid, s);
      case 1: return bits_launch<2, 1>(a, grid, s);
      default: return bits_launch<2, 2>(a, grid, s);
    }
  }
  if (pgap == 2) {
    switch (sr) {
      case -1: return bits_launch<4, -1>(a, grid, s);
      case 0: return bits_launch<4, 0>(a, grid, s);
      case 1: return bits_launch<4, 1>(a, grid, s);
      case 2: return bits_launch<4, 2>(a, grid, s);
      case 3: return bits_launch<4, 3>(a, grid, s);
      default: return bits_launch<4, 4>(a, grid, s);
    }
  }
  return hipErrorInvalidValue;
}

int bits_blocks_per_cu(int pgap) { return pgap == 1 ? bits_occ<2, 1>() : bits_occ<4, 1>(); }

hipError_t launch_strip(const FillArgs& a, int pxy, int pgap, int grid, hipStream_t s) {
  const int sr = bits_sr(pxy, pgap);
  if (pgap == 1) {
    switch (sr) {
      case -1: return strip_launch<2, -1>(a, grid, s);
      case 0: return strip_launch<2, 0>(a, grid, s);
      case 1: return strip_launch<2, 1>(a, grid, s);
      default: return strip_launch<2, 2>(a, grid, s);
    }
  }
  if (pgap == 2) {
    switch (sr) {
      case -1: return strip_launch<4, -1>(a, grid, s);
      case 0: return strip_launch<4, 0>(a, grid, s);
      case 1: return strip_launch<4, 1>(a, grid, s);
      case 2: return strip_launch<4, 2>(a, grid, s);
      case 3: return strip_launch<4, 3>(a, grid, s);
      default: return strip_launch<4, 4>(a, grid, s);
    }
  }
  return hipErrorInvalidValue;
}

int strip_blocks_per_cu(int pgap, int ring_dwords) {
  return pgap == 1 ? strip_occ<2, 1>(ring_dwords) : strip_occ<4, 1>(ring_dwords);
}

}  // namespace nwk
