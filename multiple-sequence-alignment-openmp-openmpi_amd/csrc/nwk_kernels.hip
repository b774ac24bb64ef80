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
#include "nwk_prof.h"

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

// The block loops' prefetch loads (next super-block's E / SEL words and
// band-above granules, issued one super-block ahead) and their waits.
//
// Until round 6 these were inline-asm loads the compiler did not track, waited
// for by a COUNTED s_waitcnt after the block's stores (the compiler's own
// loop-header vmcnt(0) would make every block wait for the previous block's
// stores).  That form is unsound: the compiler believes an asm output is ready
// when the asm statement ends, and where it needs the "+v" operands of the
// wait in other registers (a join of the block variants) it copies the
// in-flight destinations BEFORE the wait -- v_mov of a register the load has
// not written yet.  A late load then leaves the previous super-block's value
// in the copy; for a granule that is the previous chunk's (same epoch: it
// passes the tag check), so a band pair computes from a wrong upper row.  This
// was nw_align_pka's intermittent wrong penalty (round 5: 2-6% of runs of its
// windowed job, found in round 6 by the fill-vs-walk guard, which saw the
// FILL's H(m, n) below the true minimum, and then in the ISA: nw_align_pka
// .LBB7_113 copies v85/v131/v[16:17]/v[18:19] before the s_waitcnt; the same
// shape in nw_align, nw_align_pk, nw_align_pk2 and nw_align_affine).  The
// loads are now ordinary (compiler-tracked) loads, which the compiler waits
// for before any use or copy; NWK_ASM_PREFETCH=1 builds the old form (A/B).
#ifndef NWK_ASM_PREFETCH
#define NWK_ASM_PREFETCH 0
#endif
#if NWK_ASM_PREFETCH
__device__ __forceinline__ void asm_load_E(const unsigned* p, unsigned& e0, unsigned& e1) {
  asm volatile("global_load_dword %0, %2, off\n\tglobal_load_dword %1, %2, off offset:16"
               : "=&v"(e0), "=&v"(e1)
               : "v"(p)
               : "memory");
}
__device__ __forceinline__ void asm_load_E2(const unsigned* p, unsigned& e0, unsigned& e1) {
  asm volatile("global_load_dword %0, %2, off\n\tglobal_load_dword %1, %2, off offset:256"
               : "=&v"(e0), "=&v"(e1)
               : "v"(p)
               : "memory");
}
__device__ __forceinline__ void asm_load_granule(const u64* p, u64& v) {
  asm volatile("global_load_dwordx2 %0, %1, off sc1" : "=&v"(v) : "v"(p) : "memory");
}
// Waits until at most N vector-memory ops are outstanding; the "+v" operands
// order every later use of those registers after the wait.
template <int N>
__device__ __forceinline__ void wait_vm_keep(unsigned& a, unsigned& b, u64& c) {
  static_assert(N >= 0 && N <= 63, "vmcnt is 6 bits");
  asm volatile("s_waitcnt vmcnt(%3)" : "+v"(a), "+v"(b), "+v"(c) : "n"(N) : "memory");
}
#else
__device__ __forceinline__ void asm_load_E(const unsigned* p, unsigned& e0, unsigned& e1) {
  e0 = p[0];
  e1 = p[4];
}
__device__ __forceinline__ void asm_load_E2(const unsigned* p, unsigned& e0, unsigned& e1) {
  e0 = p[0];
  e1 = p[64];
}
// (an 8-byte sc1 load: a granule is read untorn)
__device__ __forceinline__ void asm_load_granule(const u64* p, u64& v) { v = __hip_atomic_load((gu64*)p, RLX_AGENT); }
template <int N>
__device__ __forceinline__ void wait_vm_keep(unsigned&, unsigned&, u64&) {}
#endif

// The same, but waits for every outstanding op when `all` (wave-uniform) is
// set -- one asm block, so the compiler never copies a register between two
// differently counted waits (a copy made before the wait reads the old value).
#if NWK_ASM_PREFETCH
template <int N>
__device__ __forceinline__ void wait_vm_keep_or_all(bool all, unsigned& a, unsigned& b, u64& c) {
  static_assert(N >= 0 && N <= 63, "vmcnt is 6 bits");
  asm volatile(
      "s_cmp_eq_u32 %[all], 0\n\t"
      "s_cbranch_scc1 .Lnwk_keep%=\n\t"
      "s_waitcnt vmcnt(0)\n"
      ".Lnwk_keep%=:\n\t"
      "s_waitcnt vmcnt(%[n])"
      : "+v"(a), "+v"(b), "+v"(c)
      : [all] "s"(__builtin_amdgcn_readfirstlane(all ? 1 : 0)), [n] "n"(N)
      : "memory", "scc");
}
#else
template <int N>
__device__ __forceinline__ void wait_vm_keep_or_all(bool, unsigned&, unsigned&, u64&) {}
#endif

// A zero the optimiser cannot see: LLVM rewrites an idempotent atomic RMW
// (add 0) into a plain atomic load, which can be served by a stale copy in
// this XCD's L2.  A real RMW is performed at the coherence point.
__device__ __forceinline__ unsigned long long opaque_zero64() {
  unsigned long long z = 0;
  asm volatile("" : "+v"(z));
  return z;
}
__device__ __forceinline__ unsigned opaque_zero32() {
  unsigned z = 0;
  asm volatile("" : "+v"(z));
  return z;
}

// Polls until every lane's granule carries `epoch` and returns it.  Bounded:
// gives up after ~4 s of wall time (s_memrealtime runs at 100 MHz) or when
// another wave has already failed, so a hand-off bug ends the grid instead of
// hanging it; the caller tells success from the returned tags.
// Each re-read below is a 64-lane atomic performed at the memory side, and
// WRITE_SIZE counts it (nw_align_pka on 200k pairs: polls were ~1/3 of the
// kernel's HBM writes, tools/pka_write_probe.py), so a wait backs off: the
// sleep doubles from ~0.1 us to ~1.6 us (s_sleep n = 64 n cycles) -- a
// 64-column chunk takes a band ~15 us, so the wait still ends within ~10%.
#ifndef NWK_WALK_JUMP  // trace_pair_affine<LIN>: a block's path by pointer doubling
#define NWK_WALK_JUMP 2
#endif
#ifndef NWK_POLL_SLEEP_MAX
#define NWK_POLL_SLEEP_MAX 32
#endif
__device__ __forceinline__ void poll_sleep(int& n) {
  switch (n) {  // s_sleep takes an immediate
    case 2: __builtin_amdgcn_s_sleep(2); break;
    case 4: __builtin_amdgcn_s_sleep(4); break;
    case 8: __builtin_amdgcn_s_sleep(8); break;
    case 16: __builtin_amdgcn_s_sleep(16); break;
    default: __builtin_amdgcn_s_sleep(NWK_POLL_SLEEP_MAX); break;
  }
  n = n < NWK_POLL_SLEEP_MAX ? 2 * n : n;
}
__device__ __noinline__ u64 wait_granules(const u64* p, unsigned epoch, u64 v, unsigned* err) {
  const u64 t0 = __builtin_amdgcn_s_memrealtime();
  int nap = 2;
  for (;;) {
    if (__all((unsigned)(v >> 32) == epoch)) return v;
    poll_sleep(nap);
    if (__hip_atomic_load((gu32*)err, RLX_AGENT) != 0u) return 0;
    if (__builtin_amdgcn_s_memrealtime() - t0 > 400000000ull) {
      if ((threadIdx.x & 63) == 0) atomicOr(err, 1u);
      return 0;
    }
    // Re-read through an atomic: it is performed at the coherence point, so a
    // stale copy of the line in this XCD's L2 (left by the first, too-early
    // load) cannot keep the poll spinning.  The tag makes any copy safe to
    // USE; only liveness needs the coherent re-read.  A chunk's granules are
    // published by one 64-lane store, so only the first stale lane polls (a
    // sentinel, 8 bytes instead of 512 per poll); once it has arrived every
    // stale lane re-reads.
    const int lane = threadIdx.x & 63;
    const u64 stale = __ballot((unsigned)(v >> 32) != epoch);
    const int l = __builtin_ctzll(stale);
    u64 pv = 0;
    if (lane == l) pv = __hip_atomic_fetch_add((gu64*)p, opaque_zero64(), RLX_AGENT);
    if ((unsigned)__builtin_amdgcn_readlane((int)(pv >> 32), l) == epoch) {
      if ((stale >> lane) & 1ull) v = __hip_atomic_fetch_add((gu64*)p, opaque_zero64(), RLX_AGENT);
    }
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
// CAPT: the block of cell (m, n): hs := every row's G after step s0 + kcap
// (the fill-vs-walk guard's end value, FillArgs::endv)
template <int MODE, int W, bool MASK, bool CAPT = false>
__device__ __forceinline__ void step_block(int s0, int lane, int (&h)[kRows], int& Up, int& stage,
                                           unsigned (&acc)[kRows], const unsigned (&xq)[kRows],
                                           unsigned e0, unsigned e1, const int* bslot,
                                           unsigned* mptr, int K0, int K1, bool store, int kcap, int (&hs)[kRows]) {
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
    unsigned ysh = (k < 4 ? e0 : e1) >> (8 * (k & 3));
    // opaque per step: stops the compiler hoisting all 64 lookups of the
    // block to its top (64 live VGPRs -> 3 instead of 5 waves per SIMD)
    asm volatile("" : "+v"(ysh));
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
    if constexpr (CAPT) {
      if (k == kcap) {
#pragma unroll
        for (int r = 0; r < kRows; ++r) hs[r] = hn[r];
      }
    }
    if constexpr (W < 32) {
#pragma unroll
      for (int r = 0; r < kRows; ++r) acc[r] = __builtin_amdgcn_alignbit((unsigned)h[r], acc[r], W);
    }
    if ((k % SPD) == SPD - 1 && store) {  // (linear-space fill pass: boundary rows only)
#pragma unroll
      for (int r = 0; r < kRows; ++r)
        __builtin_nontemporal_store(W < 32 ? acc[r] : (unsigned)h[r], mptr + ((k / SPD) * kRows + r) * kWave);
    }
    // keep each step's substitution lookups inside the step: hoisting all 64
    // of a block costs ~64 VGPRs and with them 2 waves per SIMD
    __builtin_amdgcn_sched_barrier(0);
  }
}

// ---------------------------------------------------------------------------
// Traceback (skel:236-262 / sub:502-531 priority: DIAG on match > DIAG if
// diag+pxy==H > UP if up+pgap==H > LEFT) on the stored G mod 2^W.
//
// Fused into the fill kernel: the wave that finishes a pair's last band
// (told by the pair's band counter, after every band wave released its
// stores) traces that pair, while the other waves keep filling later pairs.
// Per 8x8 block of cells anchored at the current cell, every lane decides
// the move of one cell (one round of LDS reads), two ballots give the D and
// U masks, and the sequential walk through the block runs on those masks in
// scalar code.  The matrix is staged in LDS by LDS-DMA one tile at a time:
// 16 lanes x 8 rows of one band x TC dword columns (+ overlap below), with
// the next tile down the band prefetched.  Ops are emitted reversed, 4 per
// dword, by lane 0.
// ---------------------------------------------------------------------------
typedef __attribute__((address_space(3))) void lds_void;
typedef const __attribute__((address_space(1))) void gbl_void;
typedef __attribute__((address_space(3))) unsigned lds_u32;

__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(uintptr_t)(const lds_u32*)p;
}

// Stored-matrix layouts (LY).
//  0 plain  (nw_align, W bits):  per band, dword (c*8 + r)*64 + t holds row r of
//           lane t for steps [c*SPD, (c+1)*SPD), SPD = 32/W; cell (row 8t+r,
//           column j) is step s = j-1+t, bits W*(s%SPD).
//  1 packed (nw_align_pk, W = 4): dword (g*4 + q)*64 + t holds rows q and q+4
//           of lane t for steps [4g, 4g+4); cell (8t+r, j) is step
//           s = j-1+2t+h (h = r>>2: rows 4..7 run one column behind rows
//           0..3), nibble at bit 8*(2*(s&1)+h) + 4*((s>>1)&1).
//  2 band pairs (nw_align_pk2, W = 4): bands 2p and 2p+1 share one region of
//           2 band_dwords; dword (g*8 + r)*64 + t holds row r of lane t of
//           both bands for steps [4g, 4g+4); cell (8t+r, j) of band 2p+h is
//           step s = j-1+t+64h (the odd band runs 64 columns behind), nibble
//           at bit 8*(2*(s&1)+h) + 4*((s>>1)&1).
template <int W, int LY>
struct Lay {
  static constexpr int SPC = 32 / W;  // steps per column unit
  static constexpr int RPC = kRows;   // dwords per column unit per lane
  __device__ static int hb(int b) { (void)b; return 0; }
  __device__ static int64_t base(int b, int64_t bdw) { return (int64_t)b * bdw; }
  __device__ static int step(int t, int r, int j, int h) { (void)r; (void)h; return j - 1 + t; }
  __device__ static int slot(int r) { return r; }
  __device__ static int shift(int s, int r, int h) { (void)r; (void)h; return W == 32 ? 0 : W * (s & (SPC - 1)); }
};
template <>
struct Lay<4, 1> {
  static constexpr int SPC = 4;
  static constexpr int RPC = 4;
  __device__ static int hb(int b) { (void)b; return 0; }
  __device__ static int64_t base(int b, int64_t bdw) { return (int64_t)b * bdw; }
  __device__ static int step(int t, int r, int j, int h) { (void)h; return j - 1 + 2 * t + (r >> 2); }
  __device__ static int slot(int r) { return r & 3; }
  __device__ static int shift(int s, int r, int h) { (void)h; return 8 * (2 * (s & 1) + (r >> 2)) + 4 * ((s >> 1) & 1); }
};
template <>
struct Lay<4, 2> {
  static constexpr int SPC = 4;
  static constexpr int RPC = kRows;
  __device__ static int hb(int b) { return b & 1; }
  __device__ static int64_t base(int b, int64_t bdw) { return (int64_t)(b >> 1) * 2 * bdw; }
  __device__ static int step(int t, int r, int j, int h) { (void)r; return j - 1 + t + 64 * h; }
  __device__ static int slot(int r) { return r; }
  __device__ static int shift(int s, int r, int h) { (void)r; return 8 * (2 * (s & 1) + h) + 4 * ((s >> 1) & 1); }
};

template <int W, int LY = 0>
struct TbConf {
  using L = Lay<W, LY>;
  static constexpr int SPC = L::SPC;
  static constexpr int TC = LY == 1 ? 32 : LY == 2 ? 16 : 8;  // column units per window
  static constexpr int TS = TC * SPC;               // steps per window
  // column units below the window: a block reaches 10 (plain, LY 2) / 12 (LY 1) steps below its cell
  static constexpr int OV = LY == 1 ? 4 : (11 + SPC - 1) / SPC;
  static constexpr int CC = TC + OV;
  static constexpr int TL = 16;                     // lanes (8-row groups) per tile
  static constexpr int TILE = CC * L::RPC * TL;     // dwords
#ifndef NWK_PK_TB_NB
#define NWK_PK_TB_NB 1
#endif
  // tile buffers: 1 (LDS per block bounds the plain kernels' fill occupancy) or 2 (next window prefetched)
  static constexpr int NB = LY ? NWK_PK_TB_NB : 1;
  static constexpr int YLO = 96;                    // plain: y window starts 96 columns below the window
  static_assert(TILE % 64 == 0, "tile = whole DMA instructions");
  static_assert(L::RPC % 4 == 0, "a DMA covers 4 dword rows x 16 lanes");
  static_assert(LY || TS + YLO <= 256, "y window must fit one DMA");
  static_assert(LY != 1 || (TS + 56 <= 256 && 2 * 63 + 48 + 3 <= kCodesFrontPad), "y window (LY 1)");
  static_assert(LY != 2 || (TS + 64 <= 256 && 63 + 64 + 48 + 3 <= kCodesFrontPad), "y window (LY 2)");
  static_assert(LY || YLO <= kCodesFrontPad, "y windows must stay inside the codes buffer");
  // first y column (0-based) of the 256-byte window staged for step window q, lanes [t0, t0+16), half h
  __device__ static int ywin(int q, int t0, int h) {
    if constexpr (LY == 1) return (TS * q - 2 * t0 - 48) & ~3;
    else if constexpr (LY == 2) return (TS * q - t0 - 64 * h - 48) & ~3;
    else { (void)t0; (void)h; return TS * q - YLO; }
  }
};

template <int W, int LY = 0>
struct TbLds {
  unsigned tile[TbConf<W, LY>::NB][TbConf<W, LY>::TILE];
  unsigned xs[TbConf<W, LY>::NB][64];
  unsigned ys[TbConf<W, LY>::NB][64];
  unsigned obuf[64];   // 256-byte ring of traceback moves, flushed to HBM in dwords
};

template <int W, int LY = 0>
__device__ __forceinline__ unsigned getG_global(const unsigned* M, const PairDesc& pd, int64_t bdw, int i, int j) {
  if (i == 0 || j == 0) return 0u;
  using L = Lay<W, LY>;
  const int w = i - 1;
  const int b = w / kBandRows;
  const int wr = w - b * kBandRows;
  const int t = wr / kRows;
  const int r = wr - t * kRows;
  const int h = L::hb(b);
  const int s = L::step(t, r, j, h);
  const unsigned d = M[pd.mat_off + L::base(b, bdw) + ((int64_t)(s / L::SPC) * L::RPC + L::slot(r)) * kWave + t];
  if constexpr (W == 32) return d;
  else return (d >> L::shift(s, r, h)) & ((1u << W) - 1u);
}

struct Five { unsigned v[5]; };

// Rare cells (band above, outside the staged window) come from global memory
// in a non-inlined call, so the wait for those loads -- which also drains the
// tile prefetch -- stays on this path.
template <int W, int LY>
__device__ __noinline__ Five tb_fallback(const unsigned* mat, const PairDesc& pd, int64_t bdw, const uint8_t* xg,
                                         const uint8_t* yg, int ci, int cj, bool fx, bool fy, bool fg, bool fu,
                                         bool fd, int shg, int shu, int shd, Five in) {
  Five o = in;
  if (fx) o.v[0] = xg[ci - 1];
  if (fy) o.v[1] = yg[cj - 1];
  if (fg) o.v[2] = getG_global<W, LY>(mat, pd, bdw, ci, cj) << shg;
  if (fu) o.v[3] = getG_global<W, LY>(mat, pd, bdw, ci - 1, cj) << shu;
  if (fd) o.v[4] = getG_global<W, LY>(mat, pd, bdw, ci - 1, cj - 1) << shd;
  return o;
}

// A traceback segment.  The whole-pair trace starts at (m, n) with no
// records.  Speculative segments (nw_align_pk2) start on a task boundary row;
// every segment stops its walk on each record row (multiple of kRecRows) and
// there claims or matches a per-row record {column, segment, move index}: a
// match means the two paths are identical from that cell on, so the segment
// ends with a merge link (SegOut.mseg / midx) that the gather kernel follows.
struct SegCtx {
  uint8_t* ops;                    // this segment's move buffer (reversed moves)
  int i0, j0;                      // start cell
  int seg;                         // segment id (task index) for records
  unsigned long long* recs;        // per pair [m / kRecRows + 1][2] records, nullptr: none
  const unsigned* tdone;           // per pair task-done flags, nullptr: all done
  int task_shift;                  // band -> task: b >> task_shift
  const unsigned* resolved;        // speculative segments: the pair's chain is complete -> abort (mseg -4)
  int stop = 0;                    // linear-space groups: the walk ends on entering this row (a band top)
};
struct SegOut {
  int len, ei, ej;                 // moves, end cell
  int mseg, midx;                  // merged into segment mseg at its move midx (-1: ran to the border)
};
constexpr int kRecRows = 128;
constexpr int kRecSlots = 32;  // per record row (open addressing by column; a full row just skips the check)
// record: bit 63 valid | column (22 bits) << 41 | segment (14 bits) << 27 | move index (27 bits)
__device__ __forceinline__ unsigned long long rec_pack(int col, int seg, int idx) {
  return (1ull << 63) | ((unsigned long long)col << 41) | ((unsigned long long)seg << 27) | (unsigned long long)idx;
}

template <int W, int LY = 0>
__device__ __forceinline__ SegOut trace_pair(const FillArgs& a, const PairDesc& pd, TbLds<W, LY>& L, int lane,
                                             const SegCtx& sc) {
  using C = TbConf<W, LY>;
  using Y = Lay<W, LY>;
  constexpr int SPC = Y::SPC;
  constexpr int RPC = Y::RPC;
  constexpr unsigned MASK = W == 32 ? 0xffffffffu : ((1u << (W & 31)) - 1u);
  const int64_t bdw = band_dwords(W, pd.sblocks);
  const int ncols = 64 * pd.sblocks / SPC;
  const uint8_t* xg = a.codes + pd.x_off;
  const uint8_t* yg = a.codes + pd.y_off;
  const unsigned* mb = a.mat + pd.mat_off;
  const bool prof = a.stamps != nullptr;
  unsigned long long cy_sw = 0, cy_blk = 0, cy_walk = 0, n_blk = 0, n_sw = 0, tA = 0, tB;

  // Stage tile (b, q, t0) into buffer buf by LDS-DMA: lanes [t0, t0+16) of
  // band b, column units [TC*q - OV, TC*q + TC) (clamped), the x codes of
  // rows [512b + 8t0, +256) and the y codes of columns [ywin(q, t0), +256).
  // DMA k covers column unit k/(RPC/4), dword rows 4(k%(RPC/4)) + lane/16,
  // lanes t0 + lane%16.
  const int lane_off = (lane >> 4) * kWave + (lane & 15);
  auto issue = [&](int buf, int b, int q, int t0) {
    const unsigned* src = mb + Y::base(b, bdw) + t0 + lane_off;
#pragma unroll
    for (int k = 0; k < C::TILE / 64; ++k) {
      int c = C::TC * q - C::OV + k / (RPC / 4);
      c = c < 0 ? 0 : (c >= ncols ? ncols - 1 : c);
      __builtin_amdgcn_global_load_lds((gbl_void*)(src + (int64_t)c * (RPC * kWave) + 4 * (k % (RPC / 4)) * kWave),
                                       (lds_void*)&L.tile[buf][64 * k], 4, 0, 0);
    }
    const unsigned* xsrc = reinterpret_cast<const unsigned*>(xg + (int64_t)b * kBandRows + 8 * t0);
    __builtin_amdgcn_global_load_lds((gbl_void*)(xsrc + lane), (lds_void*)&L.xs[buf][0], 4, 0, 0);
    const unsigned* ysrc = reinterpret_cast<const unsigned*>(yg + C::ywin(q, t0, Y::hb(b)));
    __builtin_amdgcn_global_load_lds((gbl_void*)(ysrc + lane), (lds_void*)&L.ys[buf][0], 4, 0, 0);
  };
  // The walk reads LDS only through inline asm, so the compiler does not
  // make every read wait for the in-flight DMA: this drain is the one wait.
  auto drain = []() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); };

  uint8_t* ops = sc.ops;
  int i = sc.i0, j = sc.j0, Lc = 0, flushed = 0;
  int mseg = -1, midx = 0, last_rec = -1, task_ok = 1 << 30;  // tasks >= task_ok are known done
  int tb = -1, tq = 0, tt0 = 0, cur = 0, pb = -1, pq = 0, pt0 = 0, yw = 0;
  const unsigned ob = lds_addr(&L.obuf[0]);
  // Moves go to an LDS ring (ds_write_b8, no VMEM) and reach HBM as whole
  // dwords: a store in flight would otherwise make every drain() wait for it.
  auto flush = [&](int upto) {  // copy ring bytes [flushed, upto) (upto % 4 == 0 or final)
    const int from = flushed & ~3;
    for (int o = from + 4 * lane; o < upto; o += 256) {  // one pass: upto - from <= 256
      unsigned v;
      asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(ob + (unsigned)(o & 255)) : "memory");
      *reinterpret_cast<unsigned*>(ops + o) = v;
    }
    flushed = upto;
  };
  const int li = lane >> 3, lj = lane & 7;  // this lane's cell: (i - li, j - lj)

  while (i > sc.stop && j > 0) {
    if (prof) tA = __builtin_amdgcn_s_memtime();
    if (sc.recs && (i & (kRecRows - 1)) == 0 && i != last_rec) {  // arrived on a record row
      last_rec = i;
      // open-addressing table per record row keyed by column: any two
      // segments that reach the same cell of this row find each other
      unsigned long long* rp = sc.recs + (int64_t)kRecSlots * (i / kRecRows);
      int hit = -1;
      unsigned long long v0 = 0;
      if (lane == 0) {
        const unsigned long long mine = rec_pack(j, sc.seg, Lc);
        for (int k = 0; k < kRecSlots; ++k) {
          unsigned long long* sp = rp + ((j + k) & (kRecSlots - 1));
          unsigned long long v = __hip_atomic_load((gu64*)sp, RLX_AGENT);
          if (v == 0) {
            v = atomicCAS((unsigned long long*)sp, 0ull, mine);
            if (v == 0) { hit = 2; break; }  // claimed: this segment owns the cell
          }
          if ((int)((v >> 41) & 0x3fffff) == j) { hit = 1; v0 = v; break; }
        }
      }
      hit = __builtin_amdgcn_readfirstlane(hit);
      if (sc.resolved && __hip_atomic_load((gu32*)sc.resolved, RLX_AGENT) != 0u) {  // not on the final chain
        mseg = -4;
        break;
      }
      if (hit == 1) {  // the owner passed through this very cell: same path from here on
        mseg = __builtin_amdgcn_readfirstlane((int)((v0 >> 27) & 0x3fff));
        midx = __builtin_amdgcn_readfirstlane((int)(v0 & 0x7ffffff));
        break;
      }
    }
    const int w = (i - 1) & (kBandRows - 1);
    const int t = w >> 3;
    {  // ---- make the tile holding the 8x8 block at (i, j) current
      const int b = (i - 1) / kBandRows;
      const int tl = t > 0 ? t - 1 : 0;  // lowest lane of this band the block touches
      const int s = Y::step(t, w & 7, j, Y::hb(b));
      if (b != tb || s < C::TS * tq || tl < tt0 || t >= tt0 + C::TL) {
        const int q = s / C::TS;
        if (sc.resolved && __hip_atomic_load((gu32*)sc.resolved, RLX_AGENT) != 0u) {  // walks along a row
          mseg = -4;                                                                   // cross no record row
          break;
        }
        if (sc.tdone && (b >> sc.task_shift) < task_ok) {  // entering rows of a task not yet seen done
          const int tsk = b >> sc.task_shift;
          const unsigned long long t0w = __builtin_amdgcn_s_memrealtime();
          while (__hip_atomic_load((gu32*)(sc.tdone + tsk), RLX_AGENT) == 0u) {
            __builtin_amdgcn_s_sleep(8);
            if (__builtin_amdgcn_s_memrealtime() - t0w > 400000000ull) {  // ~4 s: a fill task never finished
              if (lane == 0) atomicOr(a.err, 32u);
              return SegOut{Lc, i, j, -2, 0};
            }
          }
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          task_ok = tsk;
        }
        drain();
        n_sw++;
        if (C::NB == 2 && b == pb && q == pq && tl >= pt0 && t < pt0 + C::TL) {
          cur ^= 1;
          tt0 = pt0;
        } else {

          const int nt0 = max(0, t - (C::TL - 3));
          const int nbuf = C::NB == 2 ? (cur ^ 1) : 0;
          issue(nbuf, b, q, nt0);
          drain();
          cur = nbuf;
          tt0 = nt0;
        }
        flush(Lc & ~3);  // issued after the tile landed: the stores drain during this window's walk
        tb = b;
        tq = q;
        yw = C::ywin(q, tt0, Y::hb(b));
        pb = -1;
        if (C::NB == 2 && q > 0) {  // the walk moves down the band: prefetch the next window
          pt0 = max(0, t - (C::TL - 1));
          issue(cur ^ 1, b, q - 1, pt0);
          pb = b;
          pq = q - 1;
        }
      }
    }
    if (prof) { tB = __builtin_amdgcn_s_memtime(); cy_sw += tB - tA; tA = tB; }
    n_blk++;
    const int cbase = C::TC * tq - C::OV;
    const unsigned tbase = lds_addr(&L.tile[cur][0]);
    const unsigned xb = lds_addr(&L.xs[cur][0]), yb = lds_addr(&L.ys[cur][0]);
    // LDS address of staged cell (row ww of band tb, column jj) and its bit shift
    const int hh = Y::hb(tb);
    auto taddr = [&](int ww, int jj, int& sh) -> unsigned {
      const int tt = ww >> 3, rr = ww & 7, ss = Y::step(tt, rr, jj, hh);
      sh = Y::shift(ss, rr, hh);
      return tbase + 4u * (unsigned)(((ss / SPC - cbase) * RPC + Y::slot(rr)) * C::TL + (tt - tt0));
    };
    unsigned vx, vy, vg, vu, vd;
    int shg, shu, shd;
    bool bg, bu, bd;  // border cells (G = 0)
    // Fast path (uniform test): the block and its up/diag neighbours lie in
    // this band, inside the staged window and off the border -> branch-free.
    if (w >= 8 && j >= 9) {
      const int wc = w - li, wu = wc - 1;
      const int jc = j - lj;  // 1-based column of the cell
      const unsigned ag = taddr(wc, jc, shg);
      const unsigned au = taddr(wu, jc, shu);
      const unsigned ad = taddr(wu, jc - 1, shd);
      const unsigned ax = xb + (unsigned)(wc - 8 * tt0);
      const unsigned ay = yb + (unsigned)(jc - 1 - yw);
      asm volatile(
          "ds_read_u8 %0, %5\n\t"
          "ds_read_u8 %1, %6\n\t"
          "ds_read_b32 %2, %7\n\t"
          "ds_read_b32 %3, %8\n\t"
          "ds_read_b32 %4, %9\n\t"
          "s_waitcnt lgkmcnt(0)"
          : "=&v"(vx), "=&v"(vy), "=&v"(vg), "=&v"(vu), "=&v"(vd)
          : "v"(ax), "v"(ay), "v"(ag), "v"(au), "v"(ad)
          : "memory");
      bg = bu = bd = false;
    } else {  // slow path: band top, border, or outside the window
      const int ci = i - li, cj = j - lj;
      const int slo = C::TS * tq - C::OV * SPC, shi = C::TS * tq + C::TS;
      // LDS address of G(ii, jj), ~0u on the border (G = 0), ~1u if not staged
      auto gaddr = [&](int ii, int jj, int& sh) -> unsigned {
        if (ii <= 0 || jj <= 0) { sh = 0; return ~0u; }
        const int ww = ii - 1 - tb * kBandRows;
        const int tt = ww >> 3, rr = ww & 7, ss = Y::step(tt, rr, jj, hh);
        sh = Y::shift(ss, rr, hh);
        if (ww < 0 || tt < tt0 || tt >= tt0 + C::TL || ss < slo || ss >= shi) return ~1u;
        return taddr(ww, jj, sh);
      };
      const unsigned ag = gaddr(ci, cj, shg), au = gaddr(ci - 1, cj, shu), ad = gaddr(ci - 1, cj - 1, shd);
      const int wx = ci - 1 - (tb * kBandRows + 8 * tt0), wy = cj - 1 - yw;
      const bool xin = ci >= 1 && wx >= 0 && wx < 256, yin = cj >= 1 && wy >= 0 && wy < 256;
      const unsigned ax = xin ? xb + (unsigned)wx : xb;
      const unsigned ay = yin ? yb + (unsigned)wy : yb;
      asm volatile(
          "ds_read_u8 %0, %5\n\t"
          "ds_read_u8 %1, %6\n\t"
          "ds_read_b32 %2, %7\n\t"
          "ds_read_b32 %3, %8\n\t"
          "ds_read_b32 %4, %9\n\t"
          "s_waitcnt lgkmcnt(0)"
          : "=&v"(vx), "=&v"(vy), "=&v"(vg), "=&v"(vu), "=&v"(vd)
          : "v"(ax), "v"(ay), "v"(ag < ~1u ? ag : tbase), "v"(au < ~1u ? au : tbase), "v"(ad < ~1u ? ad : tbase)
          : "memory");
      const bool fx = !xin && ci >= 1, fy = !yin && cj >= 1;
      if (fx || fy || ag == ~1u || au == ~1u || ad == ~1u) {
        const Five f = tb_fallback<W, LY>(a.mat, pd, bdw, xg, yg, ci, cj, fx, fy, ag == ~1u, au == ~1u, ad == ~1u,
                                          shg, shu, shd, Five{vx, vy, vg, vu, vd});
        vx = f.v[0]; vy = f.v[1]; vg = f.v[2]; vu = f.v[3]; vd = f.v[4];
      }
      bg = ag == ~0u;
      bu = au == ~0u;
      bd = ad == ~0u;
    }
    const unsigned g = bg ? 0u : (vg >> shg) & MASK;
    const unsigned gu = bu ? 0u : (vu >> shu) & MASK;
    const unsigned gd = bd ? 0u : (vd >> shd) & MASK;
    const bool isD = (vx & 0xffu) == (vy & 0xffu) || ((gd + (unsigned)a.K1 - g) & MASK) == 0u;
    const bool isU = !isD && ((gu - g) & MASK) == 0u;
    // ---- the walk: each lane packs its cell's move (ASCII, low byte: the
    // byte store takes it as is) and successor lane (64 = leaves the block or
    // reaches the border); the walk is a chain of v_readlane with a scalar
    // lane index, one byte store per step.
    const int nli = li + (isD || isU ? 1 : 0), nlj = lj + (isU ? 0 : 1);
    // (segments) also stop on entering a record row
    const bool leaves = nli > 7 || nlj > 7 || i - nli <= sc.stop || j - nlj <= 0 ||
                        (sc.recs && nli > li && ((i - nli) & (kRecRows - 1)) == 0);
    const unsigned code = (isD ? (unsigned)'D' : isU ? (unsigned)'U' : (unsigned)'L') |
                          ((leaves ? 64u : (unsigned)(nli * 8 + nlj)) << 8);
    unsigned long long tW = prof ? __builtin_amdgcn_s_memtime() : 0;
    unsigned curl = 0, last = 0, cw = 0;
    do {
      last = curl;
      cw = __builtin_amdgcn_readlane(code, curl);
      asm volatile("ds_write_b8 %0, %1" ::"v"(ob + (unsigned)(Lc & 255)), "v"(cw) : "memory");
      ++Lc;
      curl = cw >> 8;
    } while (curl < 64u);
    if (prof) cy_walk += __builtin_amdgcn_s_memtime() - tW;
    if (Lc - flushed >= 160) flush(Lc & ~3);  // ring of 256, a block adds <= 15: never overrun
    // the last cell visited and its move give the block's total displacement
    const unsigned op = cw & 0xffu;
    i -= (int)(last >> 3) + (op != 'L' ? 1 : 0);
    j -= (int)(last & 7u) + (op != 'U' ? 1 : 0);
    if (prof) { tB = __builtin_amdgcn_s_memtime(); cy_blk += tB - tA; }
  }
  if (prof && lane == 0) {
    unsigned long long* st = a.stamps + 8 * pd.slot + 2;
    st[0] = cy_sw; st[1] = cy_blk; st[2] = n_blk; st[3] = (n_sw << 32) | (cy_walk & 0xffffffffull);  // diagnostics: walk cycles in the low half
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  flush(Lc);
  drain();
  return SegOut{Lc, i, j, mseg, midx};
}

// Whole-pair trace from (m, n) into the pair's op buffer (nw_align, nw_align_pk).
template <int W, int LY = 0>
__device__ __forceinline__ void trace_whole(const FillArgs& a, const PairDesc& pd, TbLds<W, LY>& L, int lane) {
  const SegOut o = trace_pair<W, LY>(a, pd, L, lane, SegCtx{a.ops + pd.ops_off, pd.m, pd.n, 0, nullptr, nullptr, 0, nullptr});
  if (lane == 0) {
    a.oplen[pd.slot] = o.len;
    a.endij[pd.slot] = make_int2(o.ei, o.ej);
  }
}

template <int MODE, int W>
__global__ __launch_bounds__(256) void nw_align(FillArgs a) {
  constexpr int SPD = 32 / W;
  __shared__ __attribute__((aligned(16))) int ring_all[4][128];
  // E window per super-block: E[64sb-64 .. 64sb+64), two slots per wave
  __shared__ __attribute__((aligned(16))) unsigned ering_all[4][256];
  __shared__ __attribute__((aligned(16))) TbLds<W> tbl[4];
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  int* ring = ring_all[wid];
  unsigned* ering = ering_all[wid];

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
    // linear-space traceback (a.lin_mode): 1 = fill pass keeping only the
    // boundary rows; 2 = recompute of a group of bands from those rows (all
    // already carry this epoch: no waiting, no publishing) into a scratch
    // matrix, then the trace through the group
    const bool store = a.lin_mode != 1;
    const bool to_below = band + 1 < pd.nbands && a.lin_mode != 2;
    const int64_t bstride = (int64_t)pd.nchunks * 64;
    // band 0 has no band above: its (never checked) prefetches read the
    // pair's own boundary area, which is always inside the workspace
    const u64* gin = reinterpret_cast<const u64*>(a.bnd) + pd.bnd_off + (int64_t)(band > 0 ? band - 1 : 0) * bstride + lane;
    const int last_chunk = pd.nchunks > 0 ? pd.nchunks - 1 : 0;
    u64* gout = a.bnd + pd.bnd_off + (int64_t)band * bstride + lane;
    unsigned* mptr = a.mat + pd.mat_off + (int64_t)band * band_dwords(W, pd.sblocks) + lane;

    int h[kRows];
    unsigned acc[kRows];
#pragma unroll
    for (int r = 0; r < kRows; ++r) { h[r] = 0; acc[r] = 0; }
    int Up = 0, stage = 0;
    u64 pend = 0;
    // E window of super-block 0 (columns of steps 0..63 for all lanes):
    // lane t holds E[-64 + t] and E[t]; later windows are loaded one
    // super-block ahead and staged in LDS at their super-block's start.
    const unsigned* Ew = a.E + pd.e_off - 64 + lane;
    unsigned ew0, ew1;
    asm_load_E2(Ew, ew0, ew1);
    asm_load_granule(gin, pend);
    wait_vm_keep<0>(ew0, ew1, pend);
    bool ok = true;
    u64 cyc_wait = 0, cyc_wait0 = 0, n_wait = 0;
    const u64 t_task = a.stamps ? __builtin_amdgcn_s_memtime() : 0;
    // stores one block issues after its prefetch loads (<= 63: vmcnt field)
    constexpr int kBlockStores = (8 / SPD) * kRows > 63 ? 63 : (8 / SPD) * kRows;
    // fill-vs-walk guard: cell (m, n) is lane t's row r of band (m - 1) / 512
    // at step n - 1 + t (the plain fill and the linear-space fill pass)
    int cap_s0 = -1, cap_s = 0, cap_t = 0, cap_r = 0;
    int hs[kRows];
#pragma unroll
    for (int r = 0; r < kRows; ++r) hs[r] = 0;
    if (a.endv && a.lin_mode != 2 && band == (pd.m - 1) / kBandRows) {
      const int wr = (pd.m - 1) % kBandRows;
      cap_t = wr / kRows;
      cap_r = wr % kRows;
      cap_s = pd.n - 1 + cap_t;
      cap_s0 = cap_s & ~7;
    }

    for (int sb = 0; sb < pd.sblocks; ++sb) {
      // --- band-above row for this super-block: B[64sb+1 .. 64sb+64] = chunk sb+1
      int bval = 0;
      if (from_above && sb < pd.nchunks) {
        if (!__all((unsigned)(pend >> 32) == a.epoch)) {
          const u64 tw = a.stamps ? __builtin_amdgcn_s_memtime() : 0;
          pend = wait_granules(gin + 64 * sb, a.epoch, pend, a.err);
          if (a.stamps) {
            const u64 d = __builtin_amdgcn_s_memtime() - tw;
            cyc_wait += d;
            if (sb == 0) cyc_wait0 += d;
            ++n_wait;
          }
          if (!__all((unsigned)(pend >> 32) == a.epoch)) { ok = false; break; }
        }
        bval = (int)(unsigned)pend;
      }
      // prefetch chunk sb+2 (unconditional, clamped: no control flow between
      // this load and the counted wait at the end of block 0 that covers it)
      asm_load_granule(gin + 64 * min(sb + 1, last_chunk), pend);
      int* slot = ring + (sb & 1) * 64;
      slot[lane] = bval;
      unsigned* ewin = ering + (sb & 1) * 128;
      ewin[lane] = ew0;
      ewin[64 + lane] = ew1;
      // next super-block's E window (covered by the counted wait below)
      asm_load_E2(Ew + 64 * (sb + 1), ew0, ew1);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();

      for (int blk = 0; blk < 8; ++blk) {
        const int s0 = sb * 64 + blk * 8;
        // this lane's columns for steps s0..s0+7: E[s0 - lane], E[s0 - lane + 4]
        const unsigned e0 = ewin[blk * 8 + 64 - lane], e1 = ewin[blk * 8 + 68 - lane];
        if (s0 == cap_s0)  // the block of cell (m, n)
          step_block<MODE, W, true, true>(s0, lane, h, Up, stage, acc, xq, e0, e1, slot + blk * 8, mptr, a.K0, a.K1,
                                          store, cap_s & 7, hs);
        else if (sb == 0)
          step_block<MODE, W, true>(s0, lane, h, Up, stage, acc, xq, e0, e1, slot + blk * 8, mptr, a.K0, a.K1, store,
                                    0, hs);
        else
          step_block<MODE, W, false>(s0, lane, h, Up, stage, acc, xq, e0, e1, slot + blk * 8, mptr, a.K0, a.K1, store,
                                     0, hs);
        mptr += (8 / SPD) * kRows * kWave;
        // the window / granule prefetches are older than this block's
        // kBlockStores stores: waiting for the rest leaves those in flight
        // (a no-op after block 0).  The linear-space fill pass stores nothing,
        // so there the count would not cover the prefetches: wait for all.
        wait_vm_keep_or_all<kBlockStores>(!store, ew0, ew1, pend);
      }
      // --- publish chunk sb (columns 64sb-63 .. 64sb of our last row) for band+1
      if (to_below && sb >= 1 && sb <= pd.nchunks) st_granule(gout + 64 * (sb - 1), a.epoch, stage);
      __builtin_amdgcn_wave_barrier();
    }
    if (!ok) return;
    if (cap_s0 >= 0) {  // H(m, n) = G(m, n) + (m + n) pgap
      int v = hs[0];
#pragma unroll
      for (int r = 1; r < kRows; ++r) v = cap_r == r ? hs[r] : v;
      if (lane == cap_t)
        __hip_atomic_fetch_add((gu32*)(a.endv + pd.slot), (unsigned)(v + (pd.m + pd.n) * a.pgap), RLX_AGENT);
    }
    // --- band finished: make its stores visible at agent scope, then count
    // it (MI355X_MICROARCH.md R1: drain -> release fence -> drain -> counter).
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (a.stamps && lane == 0) {  // per pair: band cycles, of which waiting on the band above
      atomicAdd(a.stamps + 8 * pd.slot + 6, (unsigned long long)(__builtin_amdgcn_s_memtime() - t_task));
      atomicAdd(a.stamps + 8 * pd.slot + 7, (unsigned long long)cyc_wait);
      atomicAdd(a.stamps + 8 * a.ntasks_pairs + 3 * pd.slot, (unsigned long long)cyc_wait0);
      atomicAdd(a.stamps + 8 * a.ntasks_pairs + 3 * pd.slot + 1, (unsigned long long)n_wait);
      atomicAdd(a.stamps + 8 * a.ntasks_pairs + 3 * pd.slot + 2, (unsigned long long)pd.sblocks);
    }
    if (a.lin_mode == 1) continue;  // fill pass of the linear-space traceback: no trace
    unsigned prev = 0;
    if (lane == 0) prev = __hip_atomic_fetch_add((gu32*)(a.done + pd.slot), 1u, RLX_AGENT);
    prev = __builtin_amdgcn_readfirstlane(prev);
    // --- the pair's last band: every band wave has released, so acquire and
    // trace the pair here while the other waves keep filling.
    if (prev + 1u == (unsigned)(a.lin_mode == 2 ? pd.lin_nb : pd.nbands)) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (a.stamps && lane == 0) a.stamps[8 * pd.slot] = __builtin_amdgcn_s_memrealtime();
      if (a.lin_mode == 2) {  // one group: from (lin_i, lin_j) up to the group's top row
        SegCtx sc{a.ops + pd.ops_off, pd.lin_i, pd.lin_j, 0, nullptr, nullptr, 0, nullptr};
        sc.stop = pd.lin_stop;
        const SegOut o = trace_pair<W>(a, pd, tbl[wid], lane, sc);
        if (lane == 0) {
          a.oplen[pd.slot] = o.len;
          a.endij[pd.slot] = make_int2(o.ei, o.ej);
        }
      } else {
        trace_whole<W>(a, pd, tbl[wid], lane);
      }
      if (a.stamps && lane == 0) a.stamps[8 * pd.slot + 1] = __builtin_amdgcn_s_memrealtime();
    }
  }
}


// Segmented traceback (nw_align_pk / nw_align_pk2).  Segment ids are
// task * NG + g: g = 0 is traced by the wave that filled the task (the
// pair's last task: from (m, n); every spec_every-th task: speculatively from
// the task's last row), g = 1 .. NG-1 are extra speculative start columns on
// the same row, queued for waves that have no fill task left.  Paths from a
// guessed cell coalesce with the true path only after ~5-15k rows; with
// guesses spread between the diagonal and the proportional column one of
// them is usually close and merges within ~1k rows.
struct SegGeo {  // per kernel: rows per task and band -> task shift
  int RT, task_shift;
};
__device__ __forceinline__ int guess_col(const PairDesc& pd, int R, int g) {
  const int prop = max(1, (int)(((int64_t)pd.n * R) / pd.m));
  if (g == 0 || pd.nguess < 3) return prop;
  // candidates: start diagonal R, proportional, end-anchored diagonal R + n - m
  // (DIAG > UP > LEFT from (m, n) tends to push the surplus gaps to the start)
  const int endd = min(pd.n, max(1, R + pd.n - pd.m));
  const int lo = min(min(R, prop), endd), hi = max(max(R, prop), endd);
  const int mg = (hi - lo) / 4 + R / 16 + 64;
  const int l2 = max(1, lo - mg), h2 = min(pd.n, hi + mg);
  return l2 + (int)((int64_t)(h2 - l2) * (g - 1) / (pd.nguess - 2));
}
// move-buffer offset of segment (boundary k, guess g); the last task's segment is k = K, g = 0
__device__ __forceinline__ int64_t seg_offset(const PairDesc& pd, int RT, int k, int g) {
  const int64_t E = pd.spec_every, NG = pd.nguess;
  return NG * (E * RT * k * (k + 1) / 2 + (int64_t)k * pd.n) + (int64_t)g * ((int64_t)(k + 1) * E * RT + pd.n);
}
template <int W, int LY>
__device__ __forceinline__ void trace_segment(const FillArgs& a, const PairDesc& pd, TbLds<W, LY>& tb, int lane,
                                              int task, int g, int ntp, SegGeo geo) {
  const int E = pd.spec_every, NG = pd.nguess;
  const bool last = task + 1 == ntp;
  const int k = last ? (E > 0 ? (ntp - 1) / E : 0) : (task + 1) / E - 1;
  const int64_t off = seg_offset(pd, geo.RT, k, g);
  const int i0 = last ? pd.m : (task + 1) * geo.RT;
  const int j0 = last ? pd.n : guess_col(pd, i0, g);
  const int seg = task * NG + g;
  // issue priority: fill 3 > the pair's own (last-task) trace 2 > speculation 0,
  // so speculative walks only take cycles the critical-path waves leave idle
  if (last) __builtin_amdgcn_s_setprio(2);
  else __builtin_amdgcn_s_setprio(0);
  if (last && a.stamps && lane == 0) a.stamps[8 * pd.slot] = __builtin_amdgcn_s_memrealtime();
  SegOut o{0, i0, j0, -1, 0};
  if (a.dbg_notrace) {
    o = SegOut{0, pd.m, pd.n, -1, 0};
  } else {
    const SegCtx sc{a.segops + pd.segops_off + off, i0, j0, seg, E > 0 ? a.recs + pd.rec_off : nullptr,
                    a.tdone + pd.task_off, geo.task_shift, last ? nullptr : a.done + pd.slot};
    o = trace_pair<W, LY>(a, pd, tb, lane, sc);
  }
  if (lane == 0) {
    int* si = a.seginfo + 8 * (pd.seg_off + seg);
    si[0] = o.len; si[1] = o.ei; si[2] = o.ej; si[3] = o.mseg; si[4] = o.midx;
    si[5] = (int)(off & 0x7fffffff); si[6] = (int)(off >> 31);
    // finished: publish, then see whether the chain from the pair's last-task
    // segment is now complete (every hop finished, ending at the border)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __hip_atomic_store((gu32*)(si + 7), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (E > 0 && o.mseg != -4) {
      int c = (ntp - 1) * NG;
      for (int hop = 0; hop <= ntp * NG; ++hop) {
        const int* sj = a.seginfo + 8 * (pd.seg_off + c);
        if (__hip_atomic_load((gu32*)(sj + 7), RLX_AGENT) == 0u) break;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        const int nx = __hip_atomic_load((gu32*)(sj + 3), RLX_AGENT);
        if (nx == -1) {
          __hip_atomic_store((gu32*)(a.done + pd.slot), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          break;
        }
        if (nx < 0 || nx >= ntp * NG) break;
        c = nx;
      }
    }
  }
  if (last && a.stamps && lane == 0) a.stamps[8 * pd.slot + 1] = __builtin_amdgcn_s_memrealtime();
  if (a.stamps && lane == 0) {  // per pair: latest end of any segment, and its segment id
    const unsigned long long t = __builtin_amdgcn_s_memrealtime();
    const unsigned long long prev = atomicMax(a.stamps + 11 * a.ntasks_pairs + 1 + 2 * pd.slot, t);
    if (t > prev) a.stamps[11 * a.ntasks_pairs + 2 + 2 * pd.slot] = ((unsigned long long)seg << 32) | (unsigned)o.len;
  }
}
// Task `task` of pair q is filled and its stores released: flag it, queue
// the extra guesses of its boundary, trace segment g = 0.
template <int W, int LY>
__device__ __forceinline__ void run_segments(const FillArgs& a, const PairDesc& pd, int q, TbLds<W, LY>& tb, int lane,
                                             int task, int ntp, SegGeo geo) {
  if (lane == 0) __hip_atomic_store((gu32*)(a.tdone + pd.task_off + task), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const int E = pd.spec_every;
  const bool last = task + 1 == ntp;
  if (!(last || (E > 0 && (task + 1) % E == 0))) return;
  if (!last && pd.nguess > 1) {
    if (lane == 0) {
      const unsigned s0 = atomicAdd(a.tj_tail, (unsigned)(pd.nguess - 1));
      for (int g = 1; g < pd.nguess; ++g) a.tjobs[s0 + g - 1] = make_int2(q, task * pd.nguess + g);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      for (int g = 1; g < pd.nguess; ++g)
        __hip_atomic_store((gu32*)(a.tj_ready + s0 + g - 1), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  trace_segment<W, LY>(a, pd, tb, lane, task, 0, ntp, geo);
}
// A wave with no fill task left traces queued extra guesses until all
// a.ntjobs have been handed out (each is produced by a fill task that
// finishes without waiting on any trace).
template <int W, int LY>
__device__ __forceinline__ void consume_guesses(const FillArgs& a, TbLds<W, LY>& tb, int lane, SegGeo geo) {
  for (;;) {
    unsigned h = 0;
    if (lane == 0) h = atomicAdd(a.tj_head, 1u);
    h = __builtin_amdgcn_readfirstlane(h);
    if (h >= (unsigned)a.ntjobs) return;
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load((gu32*)(a.tj_ready + h), RLX_AGENT) == 0u) {
      __builtin_amdgcn_s_sleep(8);
      if (__hip_atomic_load((gu32*)a.err, RLX_AGENT) != 0u) return;
      if (__builtin_amdgcn_s_memrealtime() - t0 > 400000000ull) {
        if (lane == 0) atomicOr(a.err, 128u);
        return;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    const int2 job = a.tjobs[h];
    const PairDesc pd = a.pairs[job.x];
    const int ntp = (pd.nbands + (1 << geo.task_shift) - 1) >> geo.task_shift;
    trace_segment<W, LY>(a, pd, tb, lane, job.y / pd.nguess, job.y % pd.nguess, ntp, geo);
  }
}

// ===========================================================================
// Packed fill (kPacked): the kProfile recurrence at W = 4 with two cells per
// VGPR as int16 pairs.  On gfx950 v_pk_min_i16 / v_pk_add_u16 / v_perm_b32
// issue at the rate of ONE v_min3 / v_bfe / v_alignbit (profiles/r01/
// valu_probe_gfx950.txt), so per cell the substitution lookup (v_bfe -> half
// a v_perm), the add and the 4-bit packing (v_alignbit -> a quarter v_perm +
// v_bfi) all halve; the two mins stay one instruction-equivalent.
//
// Lane t holds 8 rows as 4 packed registers P[q] = {row q at column
// s-2t+1, row q+4 at column s-2t} (rows 4..7 run one column behind rows 0..3,
// so row q+4 reads row q+3 of the previous step: no same-step dependence
// between halves; lanes are skewed by 2 columns).  Values are G relative to a
// wave-uniform base (a multiple of 16, so G mod 16 is unchanged), re-centred
// every super-block: across one wave G spans < 1400*pgap + 128*pgap, inside
// int16 for the W = 4 range pgap <= 7.  Per cell, with K from the row pair's
// profile bytes selected by the column's SEL word (sign-extended by the 'hi'
// selector byte: both K < 0, or both >= 0):
//     P[q] = pk_min(pk_min(diag + K, left), up)
// Storage (packed layout, see Lay<4, true>): per 4 steps and q, one dword:
// v_perm gathers the low bytes of two steps' P[q] and v_bfi merges two such
// words as nibbles.
// ===========================================================================
typedef short __attribute__((ext_vector_type(2))) s16x2;
__device__ __forceinline__ unsigned pk_min(unsigned a, unsigned b) {
  return __builtin_bit_cast(unsigned, __builtin_elementwise_min(__builtin_bit_cast(s16x2, a), __builtin_bit_cast(s16x2, b)));
}
__device__ __forceinline__ unsigned pk_add(unsigned a, unsigned b) {
  return __builtin_bit_cast(unsigned, __builtin_bit_cast(s16x2, a) + __builtin_bit_cast(s16x2, b));
}
__device__ __forceinline__ unsigned pk_sub(unsigned a, unsigned b) {
  return __builtin_bit_cast(unsigned, __builtin_bit_cast(s16x2, a) - __builtin_bit_cast(s16x2, b));
}
#if NWK_ASM_PREFETCH
__device__ __forceinline__ void asm_load_S3(const unsigned* p, unsigned& a, unsigned& b, unsigned& c) {
  asm volatile(
      "global_load_dword %0, %3, off\n\tglobal_load_dword %1, %3, off offset:256\n\t"
      "global_load_dword %2, %3, off offset:512"
      : "=&v"(a), "=&v"(b), "=&v"(c)
      : "v"(p)
      : "memory");
}
#else
__device__ __forceinline__ void asm_load_S3(const unsigned* p, unsigned& a, unsigned& b, unsigned& c) {
  a = p[0];
  b = p[64];
  c = p[128];
}
#endif
#if NWK_ASM_PREFETCH
template <int N>
__device__ __forceinline__ void wait_vm_keep3(unsigned& a, unsigned& b, unsigned& c, u64& d) {
  static_assert(N >= 0 && N <= 63, "vmcnt is 6 bits");
  asm volatile("s_waitcnt vmcnt(%4)" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "n"(N) : "memory");
}
#else
template <int N>
__device__ __forceinline__ void wait_vm_keep3(unsigned&, unsigned&, unsigned&, u64&) {}
#endif

// Eight wavefront steps s0..s0+7 (s0 % 8 == 0).
//   bslot: LDS ring of (B[s0+1 .. s0+8] - base) << 16 (band-above row)
//   srow:  LDS SEL window at this lane's column for step s0 (8 words)
//   pub:   publish the stage window after the stage shift of step 7
// CAPT: the block of cell (m, n): Ps := every row pair after step s0 + kcap (FillArgs::endv)
template <bool MASK, bool CAPT = false>
__device__ __forceinline__ void step_block_pk(int s0, int lane, unsigned (&P)[4], unsigned& U, unsigned& stage,
                                              const unsigned (&pl)[4], const unsigned (&ph)[4], const unsigned* srow,
                                              const int* bslot, unsigned* mptr, bool pub, u64* gpub, unsigned epoch,
                                              int base, int kcap, unsigned (&Ps)[4]) {
  const int4 bA = *reinterpret_cast<const int4*>(bslot);
  const int4 bB = *reinterpret_cast<const int4*>(bslot + 4);
  const int bv[8] = {bA.x, bA.y, bA.z, bA.w, bB.x, bB.y, bB.z, bB.w};
  const uint2* sp = reinterpret_cast<const uint2*>(srow);
  const uint2 c0 = sp[0], c1 = sp[1], c2 = sp[2], c3 = sp[3];
  const unsigned sel[8] = {c0.x, c0.y, c1.x, c1.y, c2.x, c2.y, c3.x, c3.y};
  unsigned Xa[4];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    // lane 63's {row 3, row 7} of the previous step enters the publish window
    stage = (unsigned)__builtin_amdgcn_update_dpp((int)P[3], (int)stage, 0x130 /*wave_shl:1*/, 0xf, 0xf, false);
    if (k == 7 && pub) st_granule(gpub, epoch, ((int)stage >> 16) + base);
    // up of the first row pair: {lane t-1's row 7 (lane 0: band above), own row 3}, previous step
    const unsigned x = (unsigned)__builtin_amdgcn_update_dpp(bv[k], (int)P[3], 0x138 /*wave_shr:1*/, 0xf, 0xf, false);
    const unsigned up = __builtin_amdgcn_alignbit(P[3], x, 16);
    const unsigned dg0 = U;
    U = up;
    unsigned sk = sel[k];
    asm volatile("" : "+v"(sk));
    unsigned Pn[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const unsigned K = __builtin_amdgcn_perm(ph[q], pl[q], sk);
      const unsigned dg = q ? P[q - 1] : dg0;
      const unsigned uq = q ? Pn[q - 1] : up;
      Pn[q] = pk_min(pk_min(pk_add(dg, K), P[q]), uq);
    }
    if constexpr (MASK) {  // columns <= 0 stay on the border (G = 0; base is 0 here)
      const int s = s0 + k;
      const unsigned M = s > 2 * lane ? 0xffffffffu : (s == 2 * lane ? 0x0000ffffu : 0u);
#pragma unroll
      for (int q = 0; q < 4; ++q) Pn[q] &= M;
    }
    if constexpr (CAPT) {
      if (k == kcap) {
#pragma unroll
        for (int q = 0; q < 4; ++q) Ps[q] = Pn[q];
      }
    }
    if (k & 1) {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        // {row q, row q+4} x {step k-1, step k}: low bytes (nibble + 4 junk bits)
        const unsigned X = __builtin_amdgcn_perm(Pn[q], P[q], 0x06040200u);
        if ((k & 3) == 1) {
          Xa[q] = X;
        } else {
          const unsigned D = (Xa[q] & 0x0f0f0f0fu) | ((X << 4) & 0xf0f0f0f0u);
          __builtin_nontemporal_store(D, mptr + ((k >> 2) * 4 + q) * kWave);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) P[q] = Pn[q];
    __builtin_amdgcn_sched_barrier(0);
  }
}

__global__ __launch_bounds__(256) void nw_align_pk(FillArgs a) {
  constexpr int W = 4;
  __shared__ __attribute__((aligned(16))) int ring_all[4][128];
  // SEL window per super-block: SEL[64sb-128 .. 64sb+64), two slots per wave
  __shared__ __attribute__((aligned(16))) unsigned swin_all[4][384];
  __shared__ __attribute__((aligned(16))) TbLds<W, 1> tbl[4];
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  int* ring = ring_all[wid];
  unsigned* swin = swin_all[wid];
  if (a.stamps && threadIdx.x == 0) atomicMin(a.stamps + 11 * a.ntasks_pairs, (unsigned long long)__builtin_amdgcn_s_memrealtime());

  for (;;) {
    unsigned tk = 0;
    if (lane == 0) tk = atomicAdd(a.counter, 1u);
    tk = __builtin_amdgcn_readfirstlane(tk);
    if (tk >= (unsigned)a.ntasks) {
      if (a.ntjobs > 0) consume_guesses<W, 1>(a, tbl[wid], lane, SegGeo{kBandRows, 0});
      return;
    }
    if (__hip_atomic_load((gu32*)a.err, RLX_AGENT) != 0u) return;
    __builtin_amdgcn_s_setprio(3);
    const int2 task = a.tasks[tk];
    const PairDesc pd = a.pairs[task.x];
    const int band = task.y;
    const int row0 = band * kBandRows + lane * kRows;
    unsigned xq[kRows];
#pragma unroll
    for (int r = 0; r < kRows; ++r) {
      const int row = row0 + r;
      const unsigned cc = row < pd.m ? a.codes[pd.x_off + row] : 0u;
      unsigned p = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) p |= ((unsigned)(cc == (unsigned)q ? a.K0 : a.K1) & 0xffu) << (8 * q);
      xq[r] = p;
    }
    const unsigned pl[4] = {xq[0], xq[1], xq[2], xq[3]};
    const unsigned ph[4] = {xq[4], xq[5], xq[6], xq[7]};

    const bool from_above = band > 0;
    const bool to_below = band + 1 < pd.nbands;
    const int64_t bstride = (int64_t)pd.nchunks * 64;
    const u64* gin = reinterpret_cast<const u64*>(a.bnd) + pd.bnd_off + (int64_t)(band > 0 ? band - 1 : 0) * bstride + lane;
    const int last_chunk = pd.nchunks > 0 ? pd.nchunks - 1 : 0;
    u64* gout = a.bnd + pd.bnd_off + (int64_t)band * bstride + lane;
    unsigned* mptr = a.mat + pd.mat_off + (int64_t)band * band_dwords(W, pd.sblocks) + lane;

    unsigned P[4] = {0u, 0u, 0u, 0u};
    unsigned U = 0, stage = 0;
    int base = 0;
    u64 pend = 0;
    const unsigned* Sg = a.sel + pd.e_off - 128 + lane;
    unsigned sw0, sw1, sw2;
    asm_load_S3(Sg, sw0, sw1, sw2);
    asm_load_granule(gin, pend);
    wait_vm_keep3<0>(sw0, sw1, sw2, pend);
    bool ok = true;
    constexpr int kBlockStores = 8;
    u64 cyc_wait = 0, cyc_wait0 = 0, n_wait = 0;
    const u64 t_task = a.stamps ? __builtin_amdgcn_s_memtime() : 0;
    // fill-vs-walk guard: cell (m, n) is lane t's row r of the last band, held
    // in P[r & 3] (low half r < 4, high half r >= 4) at step n - 1 + 2t + (r >> 2)
    int cap_s0 = -1, cap_s = 0, cap_t = 0, cap_r = 0, cap_base = 0;
    unsigned Ps[4] = {0u, 0u, 0u, 0u};
    if (a.endv && band == pd.nbands - 1) {
      const int wr = (pd.m - 1) - band * kBandRows;
      cap_t = wr / kRows;
      cap_r = wr % kRows;
      cap_s = pd.n - 1 + 2 * cap_t + (cap_r >> 2);
      cap_s0 = cap_s & ~7;
    }

    for (int sb = 0; sb < pd.sblocks; ++sb) {
      // --- band-above row for this super-block: B[64sb+1 .. 64sb+64] = chunk sb
      int bval = 0;
      if (from_above && sb < pd.nchunks) {
        if (!__all((unsigned)(pend >> 32) == a.epoch)) {
          const u64 tw = a.stamps ? __builtin_amdgcn_s_memtime() : 0;
          pend = wait_granules(gin + 64 * sb, a.epoch, pend, a.err);
          if (a.stamps) {
            const u64 d = __builtin_amdgcn_s_memtime() - tw;
            cyc_wait += d;
            if (sb == 0) cyc_wait0 += d;
            ++n_wait;
          }
          if (!__all((unsigned)(pend >> 32) == a.epoch)) { ok = false; break; }
        }
        bval = (int)(unsigned)pend;
      }
      asm_load_granule(gin + 64 * min(sb + 1, last_chunk), pend);
      // --- re-centre the base (after the masked super-blocks 0 and 1)
      if (sb >= 2) {
        const int ref = (int)(short)(__builtin_amdgcn_readlane((int)P[0], 32) & 0xffff);
        const int delta = ref & ~15;
        const unsigned dd = ((unsigned)delta & 0xffffu) * 0x10001u;
#pragma unroll
        for (int q = 0; q < 4; ++q) P[q] = pk_sub(P[q], dd);
        U = pk_sub(U, dd);
        stage -= (unsigned)delta << 16;
        base += delta;
      }
      int* slot = ring + (sb & 1) * 64;
      slot[lane] = (int)((unsigned)(bval - base) << 16);
      unsigned* w = swin + (sb & 1) * 192;
      w[lane] = sw0;
      w[64 + lane] = sw1;
      w[128 + lane] = sw2;
      asm_load_S3(Sg + 64 * (sb + 1), sw0, sw1, sw2);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();

      const bool pub_sb = to_below && sb >= 2 && sb - 2 < pd.nchunks;
      u64* gpub = gout + 64 * (sb >= 2 ? sb - 2 : 0);
      for (int blk = 0; blk < 8; ++blk) {
        const int s0 = sb * 64 + blk * 8;
        const unsigned* srow = w + blk * 8 + 128 - 2 * lane;
        const bool pub = pub_sb && blk == 7;
        if (s0 == cap_s0) {  // the block of cell (m, n)
          step_block_pk<true, true>(s0, lane, P, U, stage, pl, ph, srow, slot + blk * 8, mptr, pub, gpub, a.epoch,
                                    base, cap_s & 7, Ps);
          cap_base = base;
        } else if (sb < 2)
          step_block_pk<true>(s0, lane, P, U, stage, pl, ph, srow, slot + blk * 8, mptr, pub, gpub, a.epoch, base, 0,
                              Ps);
        else
          step_block_pk<false>(s0, lane, P, U, stage, pl, ph, srow, slot + blk * 8, mptr, pub, gpub, a.epoch, base, 0,
                               Ps);
        mptr += 2 * 4 * kWave;
        wait_vm_keep3<kBlockStores>(sw0, sw1, sw2, pend);
      }
      __builtin_amdgcn_wave_barrier();
    }
    if (!ok) return;
    if (cap_s0 >= 0) {  // H(m, n) = G + (m + n) pgap, G = the half (int16) + base
      const int q = cap_r & 3;
      unsigned v = Ps[0];
#pragma unroll
      for (int r = 1; r < 4; ++r) v = q == r ? Ps[r] : v;
      const int g = (int)(short)(cap_r >= 4 ? v >> 16 : v & 0xffffu) + cap_base;
      if (lane == cap_t)
        __hip_atomic_fetch_add((gu32*)(a.endv + pd.slot), (unsigned)(g + (pd.m + pd.n) * a.pgap), RLX_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (a.stamps && lane == 0) {  // per pair: band cycles, of which waiting on the band above
      atomicAdd(a.stamps + 8 * pd.slot + 6, (unsigned long long)(__builtin_amdgcn_s_memtime() - t_task));
      atomicAdd(a.stamps + 8 * pd.slot + 7, (unsigned long long)cyc_wait);
      atomicAdd(a.stamps + 8 * a.ntasks_pairs + 3 * pd.slot, (unsigned long long)cyc_wait0);
      atomicAdd(a.stamps + 8 * a.ntasks_pairs + 3 * pd.slot + 1, (unsigned long long)n_wait);
      atomicAdd(a.stamps + 8 * a.ntasks_pairs + 3 * pd.slot + 2, (unsigned long long)pd.sblocks);
    }
    run_segments<W, 1>(a, pd, task.x, tbl[wid], lane, band, pd.nbands, SegGeo{kBandRows, 0});
  }
}

// ===========================================================================
// Band-pair packed fill (kPacked2): one wave carries bands 2p (low halves)
// and 2p+1 (high halves) of a pair as int16 pairs, the odd band 64 columns
// behind, so lane t holds P[r] = {row r of band 2p at column s-t+1, row r of
// band 2p+1 at column s-t-63} (layout LY 2).  Band 2p+1's first row reads
// band 2p's last row from lane 63 one step earlier through DPP wave_ror:1;
// lanes keep the 1-column skew of nw_align, so a band pair adds 127 steps of
// pipeline lag (nw_align_pk: 190 per single band), the hand-off through HBM
// happens once per 1024 rows, and the per-step overhead is shared by 16
// cells.  Recurrence, base re-centring and 4-bit storage as nw_align_pk
// (across one wave G spans < 2*pgap*1152 + drift: int16 for pgap <= 7).
// ===========================================================================
// Eight wavefront steps s0..s0+7 (s0 % 8 == 0).
//   bslot: LDS ring of B[s0+1 .. s0+8] - base (band-above row, low 16 bits)
//   srow:  LDS SEL64 window at this lane's column for step s0 (8 words)
//   upsel: v_perm selector of up0: lane 0 {B, lane 63's band-2p row}, others identity
// CAPT: the block of cell (m, n): Ps := every row pair after step s0 + kcap (FillArgs::endv)
template <bool MASK, bool CAPT = false>
__device__ __forceinline__ void step_block_pk2(int s0, int lane, unsigned (&P)[kRows], unsigned& U, unsigned& stage,
                                               const unsigned (&pl)[kRows], const unsigned (&ph)[kRows],
                                               const unsigned* srow, const int* bslot, unsigned upsel, unsigned* mptr,
                                               bool pub, u64* gpub, unsigned epoch, int base, int kcap,
                                               unsigned (&Ps)[kRows]) {
  const int4 bA = *reinterpret_cast<const int4*>(bslot);
  const int4 bB = *reinterpret_cast<const int4*>(bslot + 4);
  const int bv[8] = {bA.x, bA.y, bA.z, bA.w, bB.x, bB.y, bB.z, bB.w};
  unsigned sel[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) sel[k] = srow[k];
  unsigned Xa[kRows];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    // lane 63's {row 7 of band 2p, row 7 of band 2p+1} enters the publish window
    stage = (unsigned)__builtin_amdgcn_update_dpp((int)P[kRows - 1], (int)stage, 0x130 /*wave_shl:1*/, 0xf, 0xf, false);
    if (k == 7 && pub) st_granule(gpub, epoch, ((int)stage >> 16) + base);
    // up of row 0: lane t-1's row 7 (both bands); lane 0: {band above, lane 63's band-2p row 7}
    const unsigned x = (unsigned)__builtin_amdgcn_update_dpp(0, (int)P[kRows - 1], 0x13c /*wave_ror:1*/, 0xf, 0xf, false);
    const unsigned up = __builtin_amdgcn_perm(x, (unsigned)bv[k], upsel);
    const unsigned dg0 = U;
    U = up;
    unsigned sk = sel[k];
    asm volatile("" : "+v"(sk));
    unsigned Pn[kRows];
#pragma unroll
    for (int r = 0; r < kRows; ++r) {
      const unsigned K = __builtin_amdgcn_perm(ph[r], pl[r], sk);
      const unsigned dg = r ? P[r - 1] : dg0;
      const unsigned ur = r ? Pn[r - 1] : up;
      Pn[r] = pk_min(pk_min(pk_add(dg, K), P[r]), ur);
    }
    if constexpr (MASK) {  // columns <= 0 stay on the border (G = 0; base is 0 here)
      const int s = s0 + k;
      const unsigned M = s >= lane + 64 ? 0xffffffffu : (s >= lane ? 0x0000ffffu : 0u);
#pragma unroll
      for (int r = 0; r < kRows; ++r) Pn[r] &= M;
    }
    if constexpr (CAPT) {
      if (k == kcap) {
#pragma unroll
        for (int r = 0; r < kRows; ++r) Ps[r] = Pn[r];
      }
    }
    if (k & 1) {
#pragma unroll
      for (int r = 0; r < kRows; ++r) {
        const unsigned X = __builtin_amdgcn_perm(Pn[r], P[r], 0x06040200u);
        if ((k & 3) == 1) {
          Xa[r] = X;
        } else {
          const unsigned D = (Xa[r] & 0x0f0f0f0fu) | ((X << 4) & 0xf0f0f0f0u);
          __builtin_nontemporal_store(D, mptr + ((k >> 2) * kRows + r) * kWave);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < kRows; ++r) P[r] = Pn[r];
    __builtin_amdgcn_sched_barrier(0);
  }
}

#if NWK_ASM_PREFETCH
__device__ __forceinline__ void asm_load_S2(const unsigned* p, unsigned& a, unsigned& b) {
  asm volatile("global_load_dword %0, %2, off\n\tglobal_load_dword %1, %2, off offset:256"
               : "=&v"(a), "=&v"(b)
               : "v"(p)
               : "memory");
}
#else
__device__ __forceinline__ void asm_load_S2(const unsigned* p, unsigned& a, unsigned& b) {
  a = p[0];
  b = p[64];
}
#endif

__global__ __launch_bounds__(256) void nw_align_pk2(FillArgs a) {
  constexpr int W = 4;
  __shared__ __attribute__((aligned(16))) int ring_all[4][128];
  // SEL64 window per super-block: SEL64[64sb-64 .. 64sb+64), two slots per wave
  __shared__ __attribute__((aligned(16))) unsigned swin_all[4][256];
  __shared__ __attribute__((aligned(16))) TbLds<W, 2> tbl[4];
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  int* ring = ring_all[wid];
  unsigned* swin = swin_all[wid];
  const unsigned upsel = lane == 0 ? 0x05040100u : 0x07060504u;
  if (a.stamps && threadIdx.x == 0) atomicMin(a.stamps + 11 * a.ntasks_pairs, (unsigned long long)__builtin_amdgcn_s_memrealtime());

  for (;;) {
    unsigned tk = 0;
    if (lane == 0) tk = atomicAdd(a.counter, 1u);
    tk = __builtin_amdgcn_readfirstlane(tk);
    if (tk >= (unsigned)a.ntasks) {
      if (a.ntjobs > 0) consume_guesses<W, 2>(a, tbl[wid], lane, SegGeo{2 * kBandRows, 1});
      return;
    }
    if (__hip_atomic_load((gu32*)a.err, RLX_AGENT) != 0u) return;
    __builtin_amdgcn_s_setprio(3);
    const int2 task = a.tasks[tk];
    const PairDesc pd = a.pairs[task.x];
    const int bp = task.y;                    // band pair: bands 2bp, 2bp+1
    const int ntp = (pd.nbands + 1) >> 1;     // band pairs of the pair
    const int row0 = 2 * bp * kBandRows + lane * kRows;
    unsigned pl[kRows], ph[kRows];
#pragma unroll
    for (int r = 0; r < kRows; ++r) {
      unsigned p0 = 0, p1 = 0;
      const unsigned c0 = row0 + r < pd.m ? a.codes[pd.x_off + row0 + r] : 0u;
      const unsigned c1 = row0 + kBandRows + r < pd.m ? a.codes[pd.x_off + row0 + kBandRows + r] : 0u;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        p0 |= ((unsigned)(c0 == (unsigned)q ? a.K0 : a.K1) & 0xffu) << (8 * q);
        p1 |= ((unsigned)(c1 == (unsigned)q ? a.K0 : a.K1) & 0xffu) << (8 * q);
      }
      pl[r] = p0;
      ph[r] = p1;
    }

    const bool from_above = bp > 0;
    const bool to_below = bp + 1 < ntp;
    const int64_t bstride = (int64_t)pd.nchunks * 64;
    const u64* gin = reinterpret_cast<const u64*>(a.bnd) + pd.bnd_off + (int64_t)(bp > 0 ? bp - 1 : 0) * bstride + lane;
    const int last_chunk = pd.nchunks > 0 ? pd.nchunks - 1 : 0;
    u64* gout = a.bnd + pd.bnd_off + (int64_t)bp * bstride + lane;
    unsigned* mptr = a.mat + pd.mat_off + (int64_t)bp * 2 * band_dwords(W, pd.sblocks) + lane;

    unsigned P[kRows];
#pragma unroll
    for (int r = 0; r < kRows; ++r) P[r] = 0u;
    unsigned U = 0, stage = 0;
    int base = 0;
    u64 pend = 0;
    const unsigned* Sg = a.sel + pd.e_off - 64 + lane;
    unsigned sw0, sw1;
    asm_load_S2(Sg, sw0, sw1);
    asm_load_granule(gin, pend);
    wait_vm_keep<0>(sw0, sw1, pend);
    bool ok = true;
    constexpr int kBlockStores = 2 * kRows;
    u64 cyc_wait = 0, cyc_wait0 = 0, n_wait = 0;
    const u64 t_task = a.stamps ? __builtin_amdgcn_s_memtime() : 0;
    // fill-vs-walk guard: cell (m, n) is row (m - 1) % 1024 of the last band
    // pair -- half h, lane t, row r -- at step n - 1 + t + 64 h (Lay<4, 2>)
    int cap_s0 = -1, cap_s = 0, cap_t = 0, cap_r = 0, cap_h = 0, cap_base = 0;
    unsigned Ps[kRows];
#pragma unroll
    for (int r = 0; r < kRows; ++r) Ps[r] = 0;
    if (a.endv && bp == ntp - 1) {
      const int wr = (pd.m - 1) - 2 * bp * kBandRows;
      cap_h = wr >= kBandRows ? 1 : 0;
      cap_t = (wr - cap_h * kBandRows) / kRows;
      cap_r = (wr - cap_h * kBandRows) % kRows;
      cap_s = pd.n - 1 + cap_t + 64 * cap_h;
      cap_s0 = cap_s & ~7;
    }

    for (int sb = 0; sb < pd.sblocks; ++sb) {
      // --- band-above row for this super-block: B[64sb+1 .. 64sb+64] = chunk sb
      int bval = 0;
      if (from_above && sb < pd.nchunks) {
        if (!__all((unsigned)(pend >> 32) == a.epoch)) {
          const u64 tw = a.stamps ? __builtin_amdgcn_s_memtime() : 0;
          pend = wait_granules(gin + 64 * sb, a.epoch, pend, a.err);
          if (a.stamps) {
            const u64 d = __builtin_amdgcn_s_memtime() - tw;
            cyc_wait += d;
            if (sb == 0) cyc_wait0 += d;
            ++n_wait;
          }
          if (!__all((unsigned)(pend >> 32) == a.epoch)) { ok = false; break; }
        }
        bval = (int)(unsigned)pend;
      }
      asm_load_granule(gin + 64 * min(sb + 1, last_chunk), pend);
      // --- re-centre the base (after the masked super-blocks 0 and 1)
      if (sb >= 2) {
        const int ref = (int)(short)(__builtin_amdgcn_readlane((int)P[0], 32) & 0xffff);
        const int delta = ref & ~15;
        const unsigned dd = ((unsigned)delta & 0xffffu) * 0x10001u;
#pragma unroll
        for (int r = 0; r < kRows; ++r) P[r] = pk_sub(P[r], dd);
        U = pk_sub(U, dd);
        stage -= (unsigned)delta << 16;
        base += delta;
      }
      int* slot = ring + (sb & 1) * 64;
      slot[lane] = (int)((unsigned)(bval - base) & 0xffffu);
      unsigned* w = swin + (sb & 1) * 128;
      w[lane] = sw0;
      w[64 + lane] = sw1;
      asm_load_S2(Sg + 64 * (sb + 1), sw0, sw1);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();

      const bool pub_sb = to_below && sb >= 2 && sb - 2 < pd.nchunks;
      u64* gpub = gout + 64 * (sb >= 2 ? sb - 2 : 0);
      for (int blk = 0; blk < 8; ++blk) {
        const int s0 = sb * 64 + blk * 8;
        const unsigned* srow = w + blk * 8 + 64 - lane;
        const bool pub = pub_sb && blk == 7;
        if (s0 == cap_s0) {  // the block of cell (m, n)
          step_block_pk2<true, true>(s0, lane, P, U, stage, pl, ph, srow, slot + blk * 8, upsel, mptr, pub, gpub,
                                     a.epoch, base, cap_s & 7, Ps);
          cap_base = base;
        } else if (sb < 2)
          step_block_pk2<true>(s0, lane, P, U, stage, pl, ph, srow, slot + blk * 8, upsel, mptr, pub, gpub, a.epoch,
                               base, 0, Ps);
        else
          step_block_pk2<false>(s0, lane, P, U, stage, pl, ph, srow, slot + blk * 8, upsel, mptr, pub, gpub, a.epoch,
                                base, 0, Ps);
        mptr += 2 * kRows * kWave;
        wait_vm_keep<kBlockStores>(sw0, sw1, pend);
      }
      __builtin_amdgcn_wave_barrier();
    }
    if (!ok) return;
    if (cap_s0 >= 0) {  // H(m, n) = G + (m + n) pgap, G = the half (int16) + base
      unsigned v = Ps[0];
#pragma unroll
      for (int r = 1; r < kRows; ++r) v = cap_r == r ? Ps[r] : v;
      const int g = (int)(short)(cap_h ? v >> 16 : v & 0xffffu) + cap_base;
      if (lane == cap_t)
        __hip_atomic_fetch_add((gu32*)(a.endv + pd.slot), (unsigned)(g + (pd.m + pd.n) * a.pgap), RLX_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (a.stamps && lane == 0) {
      atomicAdd(a.stamps + 8 * pd.slot + 6, (unsigned long long)(__builtin_amdgcn_s_memtime() - t_task));
      atomicAdd(a.stamps + 8 * pd.slot + 7, (unsigned long long)cyc_wait);
      atomicAdd(a.stamps + 8 * a.ntasks_pairs + 3 * pd.slot, (unsigned long long)cyc_wait0);
      atomicAdd(a.stamps + 8 * a.ntasks_pairs + 3 * pd.slot + 1, (unsigned long long)n_wait);
      atomicAdd(a.stamps + 8 * a.ntasks_pairs + 3 * pd.slot + 2, (unsigned long long)pd.sblocks);
    }
    run_segments<W, 2>(a, pd, task.x, tbl[wid], lane, bp, ntp, SegGeo{2 * kBandRows, 1});
  }
}

// Resolves each pair's segment chain (nw_align_pk2): from the last task's
// segment follow the merge links, copying [from, len) of every segment on the
// way into the pair's contiguous op buffer; the end cell comes from the
// segment that ran to the border.  One workgroup per pair.
__global__ __launch_bounds__(256) void nw_gather(FillArgs a, int npairs, int task_shift) {
  __shared__ int c_seg, c_from, c_len, c_done, c_bad, n_seg, n_from, fin_i, fin_j;
  __shared__ long long c_off;
  const int q = blockIdx.x;
  if (q >= npairs) return;
  const PairDesc pd = a.pairs[q];
  const int ntp = (pd.nbands + (1 << task_shift) - 1) >> task_shift;
  const int nseg = ntp * pd.nguess;
  uint8_t* out = a.ops + pd.ops_off;
  if (threadIdx.x == 0) { n_seg = (ntp - 1) * pd.nguess; n_from = 0; }
  int pos = 0;
  for (int hop = 0;; ++hop) {
    __syncthreads();
    if (threadIdx.x == 0) {
      c_seg = n_seg;
      c_from = n_from;
      const int* si = a.seginfo + 8 * (pd.seg_off + c_seg);
      c_len = si[0];
      c_off = (long long)si[5] | ((long long)si[6] << 31);
      c_done = si[3] < 0 ? 1 : 0;
      c_bad = (hop > nseg || si[3] == -2 || c_from < 0 || c_from > c_len) ? 1 : 0;
      fin_i = si[1];
      fin_j = si[2];
      n_seg = si[3];
      n_from = si[4];
      if (!c_done && (n_seg < 0 || n_seg >= nseg)) c_bad = 1;
    }
    __syncthreads();
    if (c_bad) {
      if (threadIdx.x == 0) atomicOr(a.err, 64u);
      return;
    }
    const uint8_t* src = a.segops + pd.segops_off + c_off;
    for (int t = c_from + threadIdx.x; t < c_len; t += blockDim.x) out[pos + t - c_from] = src[t];
    pos += c_len - c_from;
    if (c_done) break;
  }
  if (threadIdx.x == 0) {
    a.oplen[pd.slot] = pos;
    a.endij[pd.slot] = make_int2(fin_i, fin_j);
  }
}

hipError_t launch_gather(const FillArgs& a, int npairs, int task_shift, hipStream_t s) {
  hipLaunchKernelGGL(nw_gather, dim3(npairs), dim3(256), 0, s, a, npairs, task_shift);
  return hipGetLastError();
}

// ===========================================================================
// Affine-gap variant (build-defined, see oracle
// nwo_pair_affine):
//   E = min(E[i][j-1] + ge, H[i][j-1] + go + ge)      F = min(F[i-1][j] + ge, H[i-1][j] + go + ge)
//   H = x == y ? H[i-1][j-1] : min(H[i-1][j-1] + pxy, F, E)
// in plain H-space int32 (no relabelling: three matrices' worth of state).
// Same band / skew / hand-off machinery as nw_align, with two boundary rows
// per band (H and F of its last row) and, per cell, a 4-bit traceback code
// instead of G mod 16:
//   bits 1:0  H's source: 0 diagonal (match, or H[i-1][j-1] + pxy == H),
//             1 F (F == H), 2 E        -- the reference's DIAG > UP > LEFT order
//   bit 2     F opened here (H[i-1][j] + go + ge <= F[i-1][j] + ge: open wins ties)
//   bit 3     E opened here
// The traceback walks these codes with a three-state machine.
// ===========================================================================
constexpr int kAffInf = 0x3fffffff;

// CAPT: the block of cell (m, n): hs := every row's H after step s0 + kcap (FillArgs::endv)
template <bool MASK, bool CAPT = false>
__device__ __forceinline__ void step_block_affine(int s0, int lane, int (&h)[kRows], int (&e)[kRows], int& Up,
                                                  int& f7, int& stH, int& stF, unsigned (&acc)[kRows],
                                                  const unsigned (&xq)[kRows], unsigned e0, unsigned e1,
                                                  const int* bH, const int* bF, unsigned* mptr, int pxy, int goe,
                                                  int ge, int kcap, int (&hs)[kRows]) {
  const int4 hA = *reinterpret_cast<const int4*>(bH), hB = *reinterpret_cast<const int4*>(bH + 4);
  const int4 fA = *reinterpret_cast<const int4*>(bF), fB = *reinterpret_cast<const int4*>(bF + 4);
  const int bh[8] = {hA.x, hA.y, hA.z, hA.w, hB.x, hB.y, hB.z, hB.w};
  const int bf[8] = {fA.x, fA.y, fA.z, fA.w, fB.x, fB.y, fB.z, fB.w};
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    stH = __builtin_amdgcn_update_dpp(h[kRows - 1], stH, 0x130 /*wave_shl:1*/, 0xf, 0xf, false);
    stF = __builtin_amdgcn_update_dpp(f7, stF, 0x130, 0xf, 0xf, false);
    const int uh = __builtin_amdgcn_update_dpp(bh[k], h[kRows - 1], 0x138 /*wave_shr:1*/, 0xf, 0xf, false);
    const int uf = __builtin_amdgcn_update_dpp(bf[k], f7, 0x138, 0xf, 0xf, false);
    const int dg0 = Up;
    Up = uh;
    unsigned ysh = (k < 4 ? e0 : e1) >> (8 * (k & 3));
    asm volatile("" : "+v"(ysh));
    const unsigned yb = ysh & 0xffu;
    int hn[kRows], en[kRows], fprev = uf, hprev = uh;
#pragma unroll
    for (int r = 0; r < kRows; ++r) {
      const int hd = r ? h[r - 1] : dg0;
      const int eo = h[r] + goe, ee = e[r] + ge;
      const int ev = min(eo, ee);
      const int fo = hprev + goe, fe = fprev + ge;
      const int fv = min(fo, fe);
      const bool match = yb == xq[r];
      const int hc = hd + (match ? 0 : pxy);
      const int hv = match ? hd : min(min(hc, fv), ev);
      const unsigned src = hc == hv ? 0u : (fv == hv ? 1u : 2u);
      const unsigned code = src | (fo <= fe ? 4u : 0u) | (eo <= ee ? 8u : 0u);
      acc[r] = __builtin_amdgcn_alignbit(code, acc[r], 4);
      hn[r] = hv;
      en[r] = ev;
      hprev = hv;
      fprev = fv;
    }
    if constexpr (MASK) {  // columns j <= 0 keep the border (H = go + i ge, E = +inf)
      const bool valid = (s0 + k) >= lane;
#pragma unroll
      for (int r = 0; r < kRows; ++r) {
        hn[r] = valid ? hn[r] : h[r];
        en[r] = valid ? en[r] : e[r];
      }
    }
#pragma unroll
    for (int r = 0; r < kRows; ++r) { h[r] = hn[r]; e[r] = en[r]; }
    if constexpr (CAPT) {
      if (k == kcap) {
#pragma unroll
        for (int r = 0; r < kRows; ++r) hs[r] = hn[r];
      }
    }
    f7 = fprev;
    if (k == 7) {
#pragma unroll
      for (int r = 0; r < kRows; ++r) __builtin_nontemporal_store(acc[r], mptr + r * kWave);
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

#if NWK_ASM_PREFETCH
template <int N>
__device__ __forceinline__ void wait_vm_keep4(unsigned& a, unsigned& b, u64& c, u64& d) {
  asm volatile("s_waitcnt vmcnt(%4)" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "n"(N) : "memory");
}
#else
template <int N>
__device__ __forceinline__ void wait_vm_keep4(unsigned&, unsigned&, u64&, u64&) {}
#endif

// Traceback of one affine pair on its 4-bit codes (same LDS tile staging as
// trace_pair).  Per 8x8 block every lane loads its cell's code; the walk is
// a scalar three-state machine over v_readlane.  Moves are emitted reversed:
// 'D', 'U'/'L' (gap extended) and 'u'/'l' (the gap's first column: the host
// charges go + ge there, ge for the others).
// LIN: every code is a fresh move (nw_profile's linear gaps set both "opened"
// bits), so the walk needs no gap state: a cell's two low bits are its move.
template <bool LIN = false, int R = kRows>
__device__ __forceinline__ void trace_pair_affine(const FillArgs& a, const PairDesc& pd, TbLds<4>& L, int lane, unsigned* prog) {
  using C = TbConf<4>;
  constexpr int SPD = C::SPC;
  // R rows per lane (nw_profile: kProfRows): a band is 64 R rows; a tile keeps
  // the same dwords as R = 8's 16 lanes x 8 rows, so it holds TLR = 128 / R lanes
  constexpr int BR = kWave * R, LR = R == 8 ? 3 : 2, TLR = C::TL * kRows / R;
  constexpr int DPC = R * TLR / 64, RPD = 64 / TLR;  // DMAs per column unit, rows per DMA
  static_assert(R == 8 || R == 4, "trace_pair_affine: 4 or 8 rows per lane");
  const int64_t bdw = (int64_t)pd.sblocks * (64 / SPD) * R * kWave;
  const int ncols = 64 * pd.sblocks / SPD;
  const unsigned* mb = a.mat + pd.mat_off;
  const int lane_off = (lane / TLR) * kWave + (lane % TLR);
  unsigned* curt = &L.tile[0][0];  // the tile the walk reads
  auto issue = [&](int b, int q, int t0, unsigned* dst) {
    const unsigned* src = mb + (int64_t)b * bdw + t0 + lane_off;
#pragma unroll
    for (int k = 0; k < C::TILE / 64; ++k) {
      int c = C::TC * q - C::OV + k / DPC;
      c = c < 0 ? 0 : (c >= ncols ? ncols - 1 : c);
      __builtin_amdgcn_global_load_lds((gbl_void*)(src + (int64_t)c * (R * kWave) + (k % DPC) * RPD * kWave),
                                       (lds_void*)(dst + 64 * k), 4, 0, 0);
    }
  };
  // (nwk_msa verbose >= 2) walk cycles: tile switches, code reads, blocks, switches
  const bool wst = LIN && a.stamps != nullptr;
  u64 c_sw = 0, c_rd = 0, n_blk = 0, n_sw = 0;
  const u64 c_w0 = wst ? __builtin_amdgcn_s_memtime() : 0;
  auto drain = []() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); };
  uint8_t* ops = a.ops + pd.ops_off;
  int i = pd.m, j = pd.n, Lc = 0, flushed = 0, tb = -1, tq = 0, tt0 = 0;
  unsigned st = 0;  // 0 = H, 1 = F, 2 = E
  bool bad = false;
  const unsigned ob = lds_addr(&L.obuf[0]);
  auto flush = [&](int upto) {
    const int from = flushed & ~3;
    for (int o = from + 4 * lane; o < upto; o += 256) {
      unsigned v;
      asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(ob + (unsigned)(o & 255)) : "memory");
      *reinterpret_cast<unsigned*>(ops + o) = v;
    }
    flushed = upto;
  };
  const int li = lane >> 3, lj = lane & 7;
  unsigned nit = 0;
  while (i > 0 && j > 0) {
    ++nit;
    if (prog && lane == 0) __hip_atomic_store((gu32*)prog, 0x50000000u | ((nit & 0xff) << 20) | ((unsigned)(i & 0x3ff) << 10) | (unsigned)(j & 0x3ff), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const int w = (i - 1) & (BR - 1);
    const int t = w >> LR;
    const int b = (i - 1) / BR;
    {
      const int tl = max(t - (R + 6) / R, 0);  // the lane of the block's top row
      const int s = j - 1 + t;
      if (b != tb || s < C::TS * tq || tl < tt0 || t >= tt0 + TLR) {
        const u64 cs0 = wst ? __builtin_amdgcn_s_memtime() : 0;
        ++n_sw;
        const int q = s / C::TS;
        drain();
        flush(Lc & ~3);
        const int nt0 = max(0, t - (TLR - 3));
        issue(b, q, nt0, curt);
        drain();
        tb = b; tq = q; tt0 = nt0;
        if (wst) c_sw += __builtin_amdgcn_s_memtime() - cs0;
      }
    }
    // this lane's cell (ci, cj) = (i - li, j - lj)
    ++n_blk;
    const u64 cr0 = wst ? __builtin_amdgcn_s_memtime() : 0;
    const int ci = i - li, cj = j - lj;
    unsigned code = 0;
    if (ci >= 1 && cj >= 1) {
      const int ww = ci - 1 - tb * BR;
      const int tt = ww >> LR, rr = ww & (R - 1), ss = cj - 1 + tt;
      const int slo = C::TS * tq - C::OV * SPD, shi = C::TS * tq + C::TS;
      const int cbase = C::TC * tq - C::OV;
      unsigned v;
      if (ww >= 0 && tt >= tt0 && tt < tt0 + TLR && ss >= slo && ss < shi) {
        const unsigned ad = lds_addr(curt) + 4u * (unsigned)(((ss / SPD - cbase) * R + rr) * TLR + (tt - tt0));
        asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(ad) : "memory");
        code = (v >> (4 * (ss & (SPD - 1)))) & 15u;
      } else {
        if constexpr (R == kRows) {
          code = getG_global<4, 0>(a.mat, pd, bdw, ci, cj);
        } else {  // (same layout, R rows per lane)
          const int w1 = ci - 1, b1 = w1 / BR, t1 = (w1 - b1 * BR) >> LR, r1 = (w1 - b1 * BR) & (R - 1);
          const int s1 = cj - 1 + t1;
          code = (mb[(int64_t)b1 * bdw + ((int64_t)(s1 / SPD) * R + r1) * kWave + t1] >> (4 * (s1 & (SPD - 1)))) & 15u;
        }
      }
    }
    if (wst) {
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      c_rd += __builtin_amdgcn_s_memtime() - cr0;
    }
    if (prog && lane == 0) __hip_atomic_store((gu32*)prog, 0x51000000u | (code & 0xff) << 8 | (nit & 0xff), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    // scalar walk through the block
    int di = 0, dj = 0;
    const int li_lim = min(i, 8), lj_lim = min(j, 8);  // (LIN) leave the block or reach row / column 0
    // (LIN, pd.prio != 0: nwk_msa's merges of few sequences, whose paths seldom leave the
    // diagonal) diagonal runs: when every cell from the block's entry to its edge along the
    // diagonal is a D, the r moves go out at once (one lane-masked LDS write)
    const bool diag_try = LIN && pd.prio != 0;
    const u64 dmask = diag_try ? __ballot((code & 3u) == 0u) : 0ull;
    auto diag_run = [&]() -> bool {
      const int r = min(li_lim - di, lj_lim - dj);  // >= 1 inside the block
      const u64 d8 = 0x8040201008040201ull;
      const u64 m = (r >= 8 ? d8 : d8 & ((1ull << (9 * r - 8)) - 1ull)) << (di * 8 + dj);
      if ((dmask & m) != m) return false;
      if (lane < r) asm volatile("ds_write_b8 %0, %1" ::"v"(ob + (unsigned)((Lc + lane) & 255)), "v"((unsigned)'D') : "memory");
      Lc += r;
      di += r;
      dj += r;
      return true;
    };
    if (diag_try && diag_run()) {
    } else if constexpr (LIN) {
      // Every lane packs its cell's move byte, the lane of the cell the move
      // leads to, whether that cell is still inside the block, and its block
      // coordinates; the scalar walk is then one v_readlane + one s_bfe per move
      // (round 6: ~8 instructions a move, was ~30 -- decode, bounds, index).
      const unsigned src = code & 3u;
      const int nli = li + (int)((3u >> src) & 1u), nlj = lj + (int)((5u >> src) & 1u);
      // (a code the fill never writes, 3, ends the walk: its cell is an exit with bit 17 set)
      const unsigned pk = ((0x6c7544u >> (8 * src)) & 0xffu) | ((unsigned)(nli * 8 + nlj) << 8) |
                          (nli < li_lim && nlj < lj_lim && src != 3u ? 1u << 16 : 0u) | (src == 3u ? 1u << 17 : 0u) |
                          ((unsigned)nli << 20) | ((unsigned)nlj << 24);
      unsigned p;
#if NWK_WALK_JUMP
      // Pointer doubling instead of the serial chain: nx = the next lane on the path
      // (a lane whose move leaves the block points at itself), J2/J4/J8 = nx^2/^4/^8,
      // then lane t finds the path's t-th cell X_t = nx^t(0) (t <= 15: a block path
      // has at most 15 moves) and its packed move. The moves are lanes 0..T, T = the
      // count of in-block X_t; they go out as one lane-masked LDS write.
      {
        const unsigned nx = (pk & (1u << 16)) ? (pk >> 8) & 63u : (unsigned)lane;
#if NWK_WALK_JUMP == 2
        // (five LDS round trips: the path prefix X_0..X_{2k-1} grows by a DPP row
        // shift of X_0..X_{k-1} and one bpermute of J_k, issued with J_2k's)
        unsigned x = lane == 1 ? (unsigned)__builtin_amdgcn_readlane((int)nx, 0) : 0u;
        const unsigned j2 = (unsigned)__builtin_amdgcn_ds_bpermute((int)(nx << 2), (int)nx);
        unsigned y = (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x112 /*row_shr:2*/, 0xf, 0xf, false);
        const unsigned x2 = (unsigned)__builtin_amdgcn_ds_bpermute((int)(y << 2), (int)j2);
        const unsigned j4 = (unsigned)__builtin_amdgcn_ds_bpermute((int)(j2 << 2), (int)j2);
        x = (lane & 14) == 2 ? x2 : x;
        y = (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x114 /*row_shr:4*/, 0xf, 0xf, false);
        const unsigned x4 = (unsigned)__builtin_amdgcn_ds_bpermute((int)(y << 2), (int)j4);
        const unsigned j8 = (unsigned)__builtin_amdgcn_ds_bpermute((int)(j4 << 2), (int)j4);
        x = (lane & 12) == 4 ? x4 : x;
        y = (unsigned)__builtin_amdgcn_update_dpp(0, (int)x, 0x118 /*row_shr:8*/, 0xf, 0xf, false);
        const unsigned x8 = (unsigned)__builtin_amdgcn_ds_bpermute((int)(y << 2), (int)j8);
        x = (lane & 8) ? x8 : x;
#else
        const unsigned j2 = (unsigned)__builtin_amdgcn_ds_bpermute((int)(nx << 2), (int)nx);
        const unsigned j4 = (unsigned)__builtin_amdgcn_ds_bpermute((int)(j2 << 2), (int)j2);
        const unsigned j8 = (unsigned)__builtin_amdgcn_ds_bpermute((int)(j4 << 2), (int)j4);
        unsigned x = (lane & 1) ? (unsigned)__builtin_amdgcn_readlane((int)nx, 0) : 0u;
        const unsigned x2 = (unsigned)__builtin_amdgcn_ds_bpermute((int)(x << 2), (int)j2);
        x = (lane & 2) ? x2 : x;
        const unsigned x4 = (unsigned)__builtin_amdgcn_ds_bpermute((int)(x << 2), (int)j4);
        x = (lane & 4) ? x4 : x;
        const unsigned x8 = (unsigned)__builtin_amdgcn_ds_bpermute((int)(x << 2), (int)j8);
        x = (lane & 8) ? x8 : x;
#endif
        const unsigned px = (unsigned)__builtin_amdgcn_ds_bpermute((int)(x << 2), (int)pk);
        const int T = __popcll(__ballot(lane < 16 && (px & (1u << 16))));
        if (lane <= T) asm volatile("ds_write_b8 %0, %1" ::"v"(ob + (unsigned)((Lc + lane) & 255)), "v"(px & 0xffu) : "memory");  // 'D', 'u', 'l'
        Lc += T + 1;
        p = (unsigned)__builtin_amdgcn_readlane((int)px, T);
      }
#else
      int cur = 0;
      do {  // one exit: the move leaves the block (or reaches row / column 0)
        p = (unsigned)__builtin_amdgcn_readlane((int)pk, cur);
        asm volatile("ds_write_b8 %0, %1" ::"v"(ob + (unsigned)(Lc & 255)), "v"(p & 0xffu) : "memory");  // 'D', 'u', 'l'
        ++Lc;
        cur = (int)((p >> 8) & 63u);
      } while (p & (1u << 16));
#endif
      bad = bad || (p & (1u << 17));  // (the walk fails: err 16 below)
      di = (int)((p >> 20) & 15u);
      dj = (int)((p >> 24) & 15u);
    } else for (;;) {
      const unsigned c = __builtin_amdgcn_readlane(code, di * 8 + dj);
      unsigned op;
      op = 0;
      if (st == 0) {
        const unsigned src = c & 3u;
        if (src == 0) {
          op = 'D';
          ++di; ++dj;
        } else if (src < 3) {
          st = src;  // 1 = F, 2 = E: the gap step below runs from this same cell
        } else {
          bad = true;  // not a code the fill writes
          break;
        }
      }
      if (st == 1) {
        const bool open = (c >> 2) & 1u;
        op = open ? 'u' : 'U';
        st = open ? 0u : 1u;
        ++di;
      } else if (st == 2) {
        const bool open = (c >> 3) & 1u;
        op = open ? 'l' : 'L';
        st = open ? 0u : 2u;
        ++dj;
      }
      asm volatile("ds_write_b8 %0, %1" ::"v"(ob + (unsigned)(Lc & 255)), "v"(op) : "memory");
      ++Lc;
      if (di > 7 || dj > 7 || i - di <= 0 || j - dj <= 0) break;
    }
    i -= di;
    j -= dj;
    if (prog && lane == 0) __hip_atomic_store((gu32*)prog, 0x52000000u | ((unsigned)di << 12) | ((unsigned)dj << 8) | (nit & 0xff), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (Lc - flushed >= 160) flush(Lc & ~3);
    if (bad || Lc > pd.m + pd.n) {
      if (lane == 0) atomicOr(a.err, 16u);
      break;
    }
  }
  if (prog && lane == 0) __hip_atomic_store((gu32*)prog, 0x53000000u | (nit & 0xffff), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  flush(Lc);
  if (prog && lane == 0) __hip_atomic_store((gu32*)prog, 0x54000000u | (nit & 0xffff), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  drain();
  if (prog && lane == 0) __hip_atomic_store((gu32*)prog, 0x55000000u | (nit & 0xffff), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (lane == 0) {
    a.oplen[pd.slot] = Lc;
    a.endij[pd.slot] = make_int2(i, j);
  }
  if (wst && lane == 0) {
    u64* x = a.stamps + 8 * pd.slot;
    x[2] = __builtin_amdgcn_s_memtime() - c_w0;
    x[3] = c_sw;
    x[4] = c_rd;
    x[5] = (n_blk << 32) | n_sw;
    x[6] = (unsigned)Lc;
  }
}

__global__ __launch_bounds__(256) void nw_align_affine(FillArgs a) {
  constexpr int W = 4, SPD = 8;
  __shared__ __attribute__((aligned(16))) int ringH_all[4][128];
  __shared__ __attribute__((aligned(16))) int ringF_all[4][128];
  __shared__ __attribute__((aligned(16))) unsigned ering_all[4][256];
  __shared__ __attribute__((aligned(16))) TbLds<W> tbl[4];
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  int* ringH = ringH_all[wid];
  int* ringF = ringF_all[wid];
  unsigned* ering = ering_all[wid];
  const int pxy = a.K1, go = a.go, ge = a.ge, goe = a.go + a.ge;
  unsigned* prog = a.prog ? a.prog + blockIdx.x * 4 + wid : nullptr;
#define PROG(v) do { if (prog && lane == 0) __hip_atomic_store((gu32*)prog, (unsigned)(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); } while (0)

  for (;;) {
    unsigned tk = 0;
    if (lane == 0) tk = atomicAdd(a.counter, 1u);
    tk = __builtin_amdgcn_readfirstlane(tk);
    PROG(0x10000000u | tk);
    if (tk >= (unsigned)a.ntasks) { PROG(0x60000000u); return; }
    if (__hip_atomic_load((gu32*)a.err, RLX_AGENT) != 0u) return;
    const int2 task = a.tasks[tk];
    const PairDesc pd = a.pairs[task.x];
    const int band = task.y;
    const int row0 = band * kBandRows + lane * kRows;  // 0-based first row of this lane
    unsigned xq[kRows];
    int h[kRows], e[kRows];
    unsigned acc[kRows];
#pragma unroll
    for (int r = 0; r < kRows; ++r) {
      const int row = row0 + r;
      xq[r] = row < pd.m ? a.codes[pd.x_off + row] : 0x100u;
      h[r] = go + (row + 1) * ge;  // H[i][0]
      e[r] = kAffInf;              // E[i][0]
      acc[r] = 0;
    }
    int Up = band == 0 ? 0 : go + band * kBandRows * ge;  // H[row above the band][0]
    int f7 = kAffInf, stH = 0, stF = 0;

    const bool from_above = band > 0;
    const bool to_below = band + 1 < pd.nbands;
    const int64_t bstride = (int64_t)pd.nchunks * 64;
    const int64_t fbase = (int64_t)(pd.nbands - 1) * bstride;  // F rows follow the H rows
    const int bin = band > 0 ? band - 1 : 0;
    const u64* ginH = reinterpret_cast<const u64*>(a.bnd) + pd.bnd_off + (int64_t)bin * bstride + lane;
    const u64* ginF = ginH + fbase;
    const int last_chunk = pd.nchunks > 0 ? pd.nchunks - 1 : 0;
    u64* goutH = a.bnd + pd.bnd_off + (int64_t)band * bstride + lane;
    u64* goutF = goutH + fbase;
    unsigned* mptr = a.mat + pd.mat_off + (int64_t)band * band_dwords(W, pd.sblocks) + lane;
    u64 pH = 0, pF = 0;
    const unsigned* Ew = a.E + pd.e_off - 64 + lane;
    unsigned ew0, ew1;
    asm_load_E2(Ew, ew0, ew1);
    asm_load_granule(ginH, pH);
    asm_load_granule(ginF, pF);
    wait_vm_keep4<0>(ew0, ew1, pH, pF);
    bool ok = true;
    constexpr int kBlockStores = kRows;
    // fill-vs-walk guard: cell (m, n) is lane t's row r of the last band at step n - 1 + t
    int cap_s0 = -1, cap_s = 0, cap_t = 0, cap_r = 0;
    int hs[kRows];
#pragma unroll
    for (int r = 0; r < kRows; ++r) hs[r] = 0;
    if (a.endv && band == pd.nbands - 1) {
      const int wr = (pd.m - 1) - band * kBandRows;
      cap_t = wr / kRows;
      cap_r = wr % kRows;
      cap_s = pd.n - 1 + cap_t;
      cap_s0 = cap_s & ~7;
    }

    for (int sb = 0; sb < pd.sblocks; ++sb) {
      PROG(0x20000000u | sb);
      // --- band-above H and F rows for this super-block's columns 64sb+1 .. 64sb+64
      int bh = go + (64 * sb + lane + 1) * ge, bf = kAffInf;  // band 0: H[0][j], F[0][j]
      if (from_above) {
        bh = 0;
        if (sb < pd.nchunks) {
          if (!__all((unsigned)(pH >> 32) == a.epoch)) pH = wait_granules(ginH + 64 * sb, a.epoch, pH, a.err);
          if (!__all((unsigned)(pF >> 32) == a.epoch)) pF = wait_granules(ginF + 64 * sb, a.epoch, pF, a.err);
          if (!__all((unsigned)(pH >> 32) == a.epoch && (unsigned)(pF >> 32) == a.epoch)) { ok = false; break; }
          bh = (int)(unsigned)pH;
          bf = (int)(unsigned)pF;
        }
      }
      asm_load_granule(ginH + 64 * min(sb + 1, last_chunk), pH);
      asm_load_granule(ginF + 64 * min(sb + 1, last_chunk), pF);
      int* slH = ringH + (sb & 1) * 64;
      int* slF = ringF + (sb & 1) * 64;
      slH[lane] = bh;
      slF[lane] = bf;
      unsigned* ewin = ering + (sb & 1) * 128;
      ewin[lane] = ew0;
      ewin[64 + lane] = ew1;
      asm_load_E2(Ew + 64 * (sb + 1), ew0, ew1);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      for (int blk = 0; blk < 8; ++blk) {
        const int s0 = sb * 64 + blk * 8;
        const unsigned e0 = ewin[blk * 8 + 64 - lane], e1 = ewin[blk * 8 + 68 - lane];
        if (s0 == cap_s0)  // the block of cell (m, n)
          step_block_affine<true, true>(s0, lane, h, e, Up, f7, stH, stF, acc, xq, e0, e1, slH + blk * 8,
                                        slF + blk * 8, mptr, pxy, goe, ge, cap_s & 7, hs);
        else if (sb == 0)
          step_block_affine<true>(s0, lane, h, e, Up, f7, stH, stF, acc, xq, e0, e1, slH + blk * 8, slF + blk * 8, mptr,
                                  pxy, goe, ge, 0, hs);
        else
          step_block_affine<false>(s0, lane, h, e, Up, f7, stH, stF, acc, xq, e0, e1, slH + blk * 8, slF + blk * 8,
                                   mptr, pxy, goe, ge, 0, hs);
        mptr += (8 / SPD) * kRows * kWave;
        wait_vm_keep4<kBlockStores>(ew0, ew1, pH, pF);
      }
      if (to_below && sb >= 1 && sb <= pd.nchunks) {
        st_granule(goutH + 64 * (sb - 1), a.epoch, stH);
        st_granule(goutF + 64 * (sb - 1), a.epoch, stF);
      }
      __builtin_amdgcn_wave_barrier();
    }
    PROG(0x30000000u);
    if (!ok) return;
    if (cap_s0 >= 0) {  // H(m, n) (absolute)
      int v = hs[0];
#pragma unroll
      for (int r = 1; r < kRows; ++r) v = cap_r == r ? hs[r] : v;
      if (lane == cap_t) __hip_atomic_fetch_add((gu32*)(a.endv + pd.slot), (unsigned)v, RLX_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    PROG(0x31000000u);
    unsigned prev = 0;
    if (lane == 0) prev = __hip_atomic_fetch_add((gu32*)(a.done + pd.slot), 1u, RLX_AGENT);
    prev = __builtin_amdgcn_readfirstlane(prev);
    if (prev + 1u == (unsigned)pd.nbands) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      PROG(0x40000000u);
      if (a.dbg_notrace) {
        if (lane == 0) { a.oplen[pd.slot] = 0; a.endij[pd.slot] = make_int2(pd.m, pd.n); }
      } else {
        trace_pair_affine(a, pd, tbl[wid], lane, prog);
        PROG(0x56000000u);
      }
    }
  }
}

// ===========================================================================
// Packed affine fill (kAffinePk, nw_align_pka): the Gotoh recurrence of
// SURVEY §8 a9 on band pairs as int16 pairs -- nw_align_pk2's layout, skew and
// hand-off (bands 2p / 2p+1 in the low / high halves, the odd band 64 columns
// behind, one HBM hand-off per 1024 rows) with nw_align_affine's state: E per
// row in registers, F passed down the rows (across lanes by DPP), two boundary
// rows (H and F) per band pair.
//
// Values are H-space (no relabelling: K = 0 on a match and pxy otherwise, so
// every profile byte is >= 0), scaled by 4 with a 2-bit tag in the low bits,
// relative to a per-half wave-uniform base and biased by kPkaBias so both
// halves stay inside [0, 32767].  Then a 32-bit v_add_u32 adds a packed
// constant (or the profile word) to both halves with no carry between them --
// one full-rate instruction instead of a half-rate v_pk_add_u16 -- and
// v_pk_min_i16 still compares correctly.  The tags make one min yield a value
// and its source, ties going the oracle's way (nwo_pair_affine):
//   E = min(4(H_left + go + ge) | 0, E_left' + 4ge),  E' = E | 3   (open 0 < extend 3)
//   F = min(4(H_up   + go + ge) | 0, F_up'   + 4ge),  F' = F | 1   (open 0 < extend 1)
//   H = min(4(H_diag + K)       | 0, F', E')  ->  tag 0 D, 1 F, 3 E  (D > F > E)
// (for pxy, go, ge >= 0 the reference's match shortcut H = H_diag IS that
// minimum with tag 0: H_diag <= E, F on a match).  The 4-bit
// code stored per cell: bits 1:0 = H's tag, bit 2 = F extended, bit 3 = E
// extended; trace_pair_pka walks it.  The host admits a call only when the
// values provably stay inside the int16 window (pka_admissible, nwk_runtime).
// ===========================================================================
constexpr int kPkaBias = 16000;  // scaled value of a half's base (a multiple of 4)
constexpr int kPkaInf = 32000;   // scaled +inf: E at column 0, F above row 1

__device__ __forceinline__ unsigned pk_or(unsigned a, unsigned m) { return a | m; }

// Eight wavefront steps s0..s0+7 (s0 % 8 == 0).
//   Hc, Ec: per row, H (tag-clean) and E' of the previous step; Nb: its codes
//   F7:     row 7's F' of the previous step (lane t+1's row-0 F-up, publish)
//   bH, bF: LDS rings of the band-above H and F' rows (scaled, low 16 bits)
//   hb0:    packed border H of row 0 (masked steps), + r * ge4 for row r
//   STO:    code stores: 1 always, 0 never (outside the stored window,
//           PairDesc::bits_w), 2 when `sto` (the masked super-blocks)
//   CAPT:   (the block of cell (m, n)) Hs := every row's H after step s0 + kcap
//           (the fill-vs-walk guard's end value, FillArgs::endv)
template <bool MASK, int STO, bool CAPT = false>
__device__ __forceinline__ void step_block_pka(int s0, int lane, bool sto, unsigned (&Hc)[kRows], unsigned (&Ec)[kRows],
                                               unsigned (&Nb)[kRows], unsigned& F7, unsigned& U, unsigned& stH,
                                               unsigned& stF, const unsigned (&pl)[kRows], const unsigned (&ph)[kRows],
                                               const unsigned* srow, const int* bH, const int* bF, unsigned upsel,
                                               unsigned* mptr, bool pub, u64* gpH, u64* gpF, unsigned epoch,
                                               int base_hi, unsigned goe4, unsigned ge4, unsigned hb0, unsigned xfer,
                                               int kcap, unsigned (&Hs)[kRows]) {
  const int4 hA = *reinterpret_cast<const int4*>(bH), hB = *reinterpret_cast<const int4*>(bH + 4);
  const int4 fA = *reinterpret_cast<const int4*>(bF), fB = *reinterpret_cast<const int4*>(bF + 4);
  const int bh[8] = {hA.x, hA.y, hA.z, hA.w, hB.x, hB.y, hB.z, hB.w};
  const int bf[8] = {fA.x, fA.y, fA.z, fA.w, fB.x, fB.y, fB.z, fB.w};
  unsigned sel[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) sel[k] = srow[k];
  unsigned Xa[kRows];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    // lane 63's {row 7 of band 2p, row 7 of band 2p+1} (previous step) enter the publish windows
    stH = (unsigned)__builtin_amdgcn_update_dpp((int)Hc[kRows - 1], (int)stH, 0x130 /*wave_shl:1*/, 0xf, 0xf, false);
    stF = (unsigned)__builtin_amdgcn_update_dpp((int)F7, (int)stF, 0x130, 0xf, 0xf, false);
    if (k == 7 && pub) {
      st_granule(gpH, epoch, (int)((stH >> 16) >> 2) - kPkaBias / 4 + base_hi);
      st_granule(gpF, epoch, (int)((stF >> 16) >> 2) - kPkaBias / 4 + base_hi);
    }
    // row 0's up: lane t-1's row 7 (previous step); lane 0: {band above, lane 63's band-2p row 7}
    const unsigned xH = (unsigned)__builtin_amdgcn_update_dpp(0, (int)Hc[kRows - 1], 0x13c /*wave_ror:1*/, 0xf, 0xf, false);
    const unsigned xF = (unsigned)__builtin_amdgcn_update_dpp(0, (int)F7, 0x13c, 0xf, 0xf, false);
    // lane 0's high half takes lane 63's low-half row: rebase it from base_lo to base_hi (xfer)
    unsigned hup = __builtin_amdgcn_perm(xH, (unsigned)bh[k], upsel) + xfer;
    unsigned fup = __builtin_amdgcn_perm(xF, (unsigned)bf[k], upsel) + xfer;
    unsigned hdg = U;
    U = hup;
    unsigned sk = sel[k];
    asm volatile("" : "+v"(sk));
    unsigned Hn[kRows], En[kRows], Nn[kRows];
#pragma unroll
    for (int r = 0; r < kRows; ++r) {
      const unsigned K = __builtin_amdgcn_perm(ph[r], pl[r], sk);  // {4K(x_lo, y), 4K(x_hi, y')}, K >= 0
      const unsigned dc = hdg + K;                                  // no carry: both halves < 32768
      const unsigned e = pk_min(Hc[r] + goe4, Ec[r] + ge4);
      const unsigned f = pk_min(hup + goe4, fup + ge4);
      const unsigned ec = pk_or(e, 0x00030003u), fc = pk_or(f, 0x00010001u);
      const unsigned g = pk_min(pk_min(dc, ec), fc);
      const unsigned hn = g & 0xfffcfffcu;
      // code: H's tag | F extended << 2 | E extended << 3 (two v_bfi_b32: bit 0 of
      // f's tag is "extended", and so is bit 1 of e's tag 3; bits 4+ are junk)
      const unsigned ext = (f & 0x00010001u) | (e & ~0x00010001u);
      Nn[r] = (g & 0x00030003u) | ((ext << 2) & ~0x00030003u);
      hdg = Hc[r];
      hup = hn;
      fup = fc;
      Hn[r] = hn;
      En[r] = ec;
    }
    if constexpr (MASK) {  // columns <= 0 keep the border: H = go + i ge, E = +inf
      const int s = s0 + k;
      const unsigned M = s >= lane + 64 ? 0xffffffffu : (s >= lane ? 0x0000ffffu : 0u);
#pragma unroll
      for (int r = 0; r < kRows; ++r) {
        const unsigned hb = hb0 + (unsigned)r * ge4;
        Hn[r] = (Hn[r] & M) | (hb & ~M);
        En[r] = (En[r] & M) | ((unsigned)(kPkaInf | 3) * 0x10001u & ~M);
      }
    }
    F7 = fup;
    if constexpr (CAPT) {
      if (k == kcap) {
#pragma unroll
        for (int r = 0; r < kRows; ++r) Hs[r] = Hn[r];
      }
    }
    if (STO == 1 || (STO == 2 && sto)) {
      if (k & 1) {
#pragma unroll
        for (int r = 0; r < kRows; ++r) {
          const unsigned X = __builtin_amdgcn_perm(Nn[r], Nb[r], 0x06040200u);
          if ((k & 3) == 1) {
            Xa[r] = X;
          } else {
            const unsigned D = (Xa[r] & 0x0f0f0f0fu) | ((X << 4) & 0xf0f0f0f0u);
            __builtin_nontemporal_store(D, mptr + ((k >> 2) * kRows + r) * kWave);
          }
        }
      }
    }
#pragma unroll
    for (int r = 0; r < kRows; ++r) {
      Hc[r] = Hn[r];
      Ec[r] = En[r];
      Nb[r] = Nn[r];
    }
    __builtin_amdgcn_sched_barrier(0);
  }
}

// Traceback of one pair on nw_align_pka's codes (layout LY 2), the same LDS
// tile staging as trace_pair and the three-state walk of trace_pair_affine:
// 'D', 'U'/'L' (gap extended) and 'u'/'l' (the gap's first column).
__device__ __forceinline__ void trace_pair_pka(const FillArgs& a, const PairDesc& pd, TbLds<4, 2>& L, int lane,
                                               unsigned* prog) {
  using C = TbConf<4, 2>;
  using Y = Lay<4, 2>;
  constexpr int SPC = Y::SPC, RPC = Y::RPC;
  // windowed storage (PairDesc::bits_w): band pair p holds super-blocks
  // pka_sb_lo(p) .. + nsb - 1; a cell outside them reads as code 16, which
  // ends the walk and flags the pair for a full-storage re-run
  const int nsb = pd.bits_w > 0 ? pd.bits_nblk : pd.sblocks;
  const int64_t bdw = band_dwords(4, nsb);
  const int ncols = 64 * nsb / SPC;
  const unsigned* mb = a.mat + pd.mat_off;
  const int lane_off = (lane >> 4) * kWave + (lane & 15);
  auto sblo_of = [&](int b) { return pka_sb_lo(b >> 1, pd.m, pd.n, pd.bits_w); };
  auto issue = [&](int b, int q, int t0) {
    const unsigned* src = mb + Y::base(b, bdw) + t0 + lane_off;
    const int c0 = 16 * sblo_of(b);
#pragma unroll
    for (int k = 0; k < C::TILE / 64; ++k) {
      int c = C::TC * q - C::OV + k / (RPC / 4) - c0;
      c = c < 0 ? 0 : (c >= ncols ? ncols - 1 : c);
      __builtin_amdgcn_global_load_lds((gbl_void*)(src + (int64_t)c * (RPC * kWave) + 4 * (k % (RPC / 4)) * kWave),
                                       (lds_void*)&L.tile[0][64 * k], 4, 0, 0);
    }
  };
  auto drain = []() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); };
  uint8_t* ops = a.ops + pd.ops_off;
  if (a.dbg_corrupt == pd.slot + 1) {
    // (tests of the fill-vs-walk guard) cell (m, n)'s source tag: D becomes F, F or E becomes D
    const int w1 = pd.m - 1, b1 = w1 / kBandRows, wr = w1 - b1 * kBandRows, t1 = wr / kRows, r1 = wr - t1 * kRows;
    const int h1 = Y::hb(b1), s1 = Y::step(t1, r1, pd.n, h1), sl = sblo_of(b1);
    if (lane == 0 && (unsigned)((s1 >> 6) - sl) < (unsigned)nsb) {
      unsigned* p = const_cast<unsigned*>(mb) + Y::base(b1, bdw) + ((int64_t)(s1 / SPC - 16 * sl) * RPC + r1) * kWave + t1;
      const unsigned sh = Y::shift(s1, r1, h1), d = *p, tag = (d >> sh) & 3u;
      *p = (d & ~(3u << sh)) | ((tag == 0u ? 1u : 0u) << sh);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  int i = pd.m, j = pd.n, Lc = 0, flushed = 0, tb = -1, tq = 0, tt0 = 0, tsb = 0;
  unsigned st = 0;  // 0 = H, 1 = F, 2 = E
  bool bad = false, out = false;
  const unsigned ob = lds_addr(&L.obuf[0]);
  auto flush = [&](int upto) {
    const int from = flushed & ~3;
    for (int o = from + 4 * lane; o < upto; o += 256) {
      unsigned v;
      asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(ob + (unsigned)(o & 255)) : "memory");
      *reinterpret_cast<unsigned*>(ops + o) = v;
    }
    flushed = upto;
  };
  const int li = lane >> 3, lj = lane & 7;
  while (i > 0 && j > 0) {
    if (prog && lane == 0)
      __hip_atomic_store((gu32*)prog, 0x50000000u | ((unsigned)(Lc & 0xff) << 20) | ((unsigned)(i & 0x3ff) << 10) | (unsigned)(j & 0x3ff),
                         __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const int w = (i - 1) & (kBandRows - 1);
    const int t = w >> 3;
    const int b = (i - 1) / kBandRows;
    {
      const int tl = t > 0 ? t - 1 : 0;
      const int s = Y::step(t, w & 7, j, Y::hb(b));
      if (b != tb || s < C::TS * tq || tl < tt0 || t >= tt0 + C::TL) {
        const int q = s / C::TS;
        drain();
        flush(Lc & ~3);
        const int nt0 = max(0, t - (C::TL - 3));
        issue(b, q, nt0);
        drain();
        tb = b; tq = q; tt0 = nt0;
        tsb = sblo_of(b);
      }
    }
    // this lane's cell (ci, cj) = (i - li, j - lj)
    const int ci = i - li, cj = j - lj;
    unsigned code = 0;
    if (ci >= 1 && cj >= 1) {
      const int ww = ci - 1 - tb * kBandRows;
      const int hh = Y::hb(tb);
      const int tt = ww >> 3, rr = ww & 7, ss = Y::step(tt, rr, cj, hh);
      const int slo = C::TS * tq - C::OV * SPC, shi = C::TS * tq + C::TS;
      const int cbase = C::TC * tq - C::OV;
      if (ww >= 0 && tt >= tt0 && tt < tt0 + C::TL && ss >= slo && ss < shi) {
        if ((unsigned)((ss >> 6) - tsb) < (unsigned)nsb) {
          const unsigned ad = lds_addr(&L.tile[0][0]) + 4u * (unsigned)(((ss / SPC - cbase) * RPC + rr) * C::TL + (tt - tt0));
          unsigned v;
          asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(v) : "v"(ad) : "memory");
          code = (v >> Y::shift(ss, rr, hh)) & 15u;
        } else {
          code = 16u;
        }
      } else {
        const int w1 = ci - 1, b1 = w1 / kBandRows, wr = w1 - b1 * kBandRows, t1 = wr / kRows, r1 = wr - t1 * kRows;
        const int h1 = Y::hb(b1), s1 = Y::step(t1, r1, cj, h1), sl = sblo_of(b1);
        if ((unsigned)((s1 >> 6) - sl) < (unsigned)nsb) {
          const unsigned d = mb[Y::base(b1, bdw) + ((int64_t)(s1 / SPC - 16 * sl) * RPC + r1) * kWave + t1];
          code = (d >> Y::shift(s1, r1, h1)) & 15u;
        } else {
          code = 16u;
        }
      }
    }
    // scalar walk through the block
    int di = 0, dj = 0;
    for (;;) {
      const unsigned c = __builtin_amdgcn_readlane(code, di * 8 + dj);
      if (c & 16u) {  // the path left the stored window
        out = true;
        break;
      }
      unsigned op = 0;
      if (st == 0) {
        const unsigned src = c & 3u;
        if (src == 0) {
          op = 'D';
          ++di; ++dj;
        } else if (src == 1) {
          st = 1;  // the gap step below runs from this same cell
        } else if (src == 3) {
          st = 2;
        } else {
          bad = true;  // not a code the fill writes
          break;
        }
      }
      if (st == 1) {
        const bool ext = (c >> 2) & 1u;
        op = ext ? 'U' : 'u';
        st = ext ? 1u : 0u;
        ++di;
      } else if (st == 2) {
        const bool ext = (c >> 3) & 1u;
        op = ext ? 'L' : 'l';
        st = ext ? 2u : 0u;
        ++dj;
      }
      asm volatile("ds_write_b8 %0, %1" ::"v"(ob + (unsigned)(Lc & 255)), "v"(op) : "memory");
      ++Lc;
      if (di > 7 || dj > 7 || i - di <= 0 || j - dj <= 0) break;
    }
    i -= di;
    j -= dj;
    if (out) break;
    if (Lc - flushed >= 160) flush(Lc & ~3);
    if (bad || Lc > pd.m + pd.n) {
      if (lane == 0) atomicOr(a.err, 16u);
      break;
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  flush(Lc);
  drain();
  if (lane == 0) {
    // out of the window: a placeholder result (no moves) and the re-run flag
    a.oplen[pd.slot] = out ? 0 : Lc;
    a.endij[pd.slot] = out ? make_int2(pd.m, pd.n) : make_int2(i, j);
    if (out) a.retry[pd.slot] = 1;
  }
}

// NWK_PKA_WPE > 0: at least that many waves per SIMD (A/B builds)
#ifndef NWK_PKA_WPE
#define NWK_PKA_WPE 0
#endif
#if NWK_PKA_WPE > 0
#define NWK_PKA_OCC __attribute__((amdgpu_waves_per_eu(NWK_PKA_WPE)))
#else
#define NWK_PKA_OCC
#endif
__global__ __launch_bounds__(256) NWK_PKA_OCC void nw_align_pka(FillArgs a) {
  constexpr int W = 4;
  __shared__ __attribute__((aligned(16))) int ringH_all[4][128];
  __shared__ __attribute__((aligned(16))) int ringF_all[4][128];
  // SEL64 window per super-block: SEL64[64sb-64 .. 64sb+64), two slots per wave
  __shared__ __attribute__((aligned(16))) unsigned swin_all[4][256];
  __shared__ __attribute__((aligned(16))) TbLds<W, 2> tbl[4];
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  int* ringH = ringH_all[wid];
  int* ringF = ringF_all[wid];
  unsigned* swin = swin_all[wid];
  const unsigned upsel = lane == 0 ? 0x05040100u : 0x07060504u;
  const int go = a.go, ge = a.ge;
  const unsigned goe4 = (unsigned)(4 * (go + ge)) * 0x10001u, ge4 = (unsigned)(4 * ge) * 0x10001u;
  unsigned* prog = a.prog ? a.prog + blockIdx.x * 4 + wid : nullptr;  // NWK_WATCHDOG progress markers

  for (;;) {
    unsigned tk = 0;
    if (lane == 0) tk = atomicAdd(a.counter, 1u);
    tk = __builtin_amdgcn_readfirstlane(tk);
    PROG(0x10000000u | tk);
    if (tk >= (unsigned)a.ntasks) { PROG(0x60000000u); return; }
    if (__hip_atomic_load((gu32*)a.err, RLX_AGENT) != 0u) return;
    const int2 task = a.tasks[tk];
    const PairDesc pd = a.pairs[task.x];
    const int bp = task.y;                    // band pair: bands 2bp, 2bp+1
    const int ntp = (pd.nbands + 1) >> 1;     // band pairs of the pair
    const int R = 2 * bp * kBandRows;         // rows above band 2bp (0-based first row of the band pair)
    const int row0 = R + lane * kRows;
    unsigned pl[kRows], ph[kRows];
#pragma unroll
    for (int r = 0; r < kRows; ++r) {
      unsigned p0 = 0, p1 = 0;
      const unsigned c0 = row0 + r < pd.m ? a.codes[pd.x_off + row0 + r] : 0u;
      const unsigned c1 = row0 + kBandRows + r < pd.m ? a.codes[pd.x_off + row0 + kBandRows + r] : 0u;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        p0 |= ((unsigned)(c0 == (unsigned)q ? 0 : 4 * a.K1) & 0xffu) << (8 * q);
        p1 |= ((unsigned)(c1 == (unsigned)q ? 0 : 4 * a.K1) & 0xffu) << (8 * q);
      }
      pl[r] = p0;
      ph[r] = p1;
    }

    const bool from_above = bp > 0;
    const bool to_below = bp + 1 < ntp;
    const int64_t bstride = (int64_t)pd.nchunks * 64;
    const int64_t fbase = (int64_t)(ntp - 1) * bstride;  // F rows follow the H rows
    const u64* ginH = reinterpret_cast<const u64*>(a.bnd) + pd.bnd_off + (int64_t)(bp > 0 ? bp - 1 : 0) * bstride + lane;
    const u64* ginF = ginH + fbase;
    const int last_chunk = pd.nchunks > 0 ? pd.nchunks - 1 : 0;
    u64* goutH = a.bnd + pd.bnd_off + (int64_t)bp * bstride + lane;
    u64* goutF = goutH + fbase;
    // windowed storage: this band pair keeps super-blocks sblo .. sblo + nsb - 1
    const int nsb = pd.bits_w > 0 ? pd.bits_nblk : pd.sblocks;
    const int sblo = pka_sb_lo(bp, pd.m, pd.n, pd.bits_w);
    unsigned* mptr = a.mat + pd.mat_off + (int64_t)bp * 2 * band_dwords(W, nsb) + lane;

    // bases: H(first row of the half, column 0) = go + (row + 1) ge, so the
    // border of lane t's row r is kPkaBias + 4 (8t + r) ge in both halves
    int base_lo = go + (R + 1) * ge, base_hi = go + (R + kBandRows + 1) * ge;
    const unsigned hb0 = (unsigned)(kPkaBias + 4 * 8 * lane * ge) * 0x10001u;
    unsigned Hc[kRows], Ec[kRows], Nb[kRows];
#pragma unroll
    for (int r = 0; r < kRows; ++r) {
      Hc[r] = hb0 + (unsigned)r * ge4;
      Ec[r] = (unsigned)(kPkaInf | 3) * 0x10001u;
      Nb[r] = 0;
    }
    // diag of lane 0's first cell: H(R, 0) (= 0 above the first row)
    unsigned U = (unsigned)(kPkaBias + 4 * (8 * lane - 1) * ge) * 0x10001u;
    if (lane == 0 && bp == 0) U = (U & 0xffff0000u) | (unsigned)(kPkaBias - 4 * (go + ge));
    unsigned F7 = (unsigned)(kPkaInf | 1) * 0x10001u, stH = 0, stF = 0;
    u64 pH = 0, pF = 0;
    const unsigned* Sg = a.sel + pd.e_off - 64 + lane;
    unsigned sw0, sw1;
    asm_load_S2(Sg, sw0, sw1);
    asm_load_granule(ginH, pH);
    asm_load_granule(ginF, pF);
    wait_vm_keep4<0>(sw0, sw1, pH, pF);
    bool ok = true;
    constexpr int kBlockStores = 2 * kRows;
    // fill-vs-walk guard: cell (m, n) is row (m - 1) % 1024 of this band pair
    // when it is the last one -- half h, lane t, row r -- at step n - 1 + t + 64 h
    int cap_s0 = -1, cap_s = 0, cap_t = 0, cap_r = 0, cap_h = 0, cap_base = 0;
    unsigned Hs[kRows];
#pragma unroll
    for (int r = 0; r < kRows; ++r) Hs[r] = 0;
    if (a.endv && bp == ntp - 1) {
      const int wr = (pd.m - 1) - R;  // 0 .. 2 kBandRows - 1
      cap_h = wr >= kBandRows ? 1 : 0;
      cap_t = (wr - cap_h * kBandRows) / kRows;
      cap_r = (wr - cap_h * kBandRows) % kRows;
      cap_s = pd.n - 1 + cap_t + 64 * cap_h;
      cap_s0 = cap_s & ~7;
    }

    for (int sb = 0; sb < pd.sblocks; ++sb) {
      PROG(0x20000000u | (unsigned)sb);
      // --- band-above H and F rows for this super-block's columns 64sb+1 .. 64sb+64
      int bh = go + (64 * sb + lane + 1) * ge, bf = 0;  // band pair 0: H[0][j]; F[0][j] = +inf
      if (from_above) {
        bh = 0;
        if (sb < pd.nchunks) {
          if (!__all((unsigned)(pH >> 32) == a.epoch)) pH = wait_granules(ginH + 64 * sb, a.epoch, pH, a.err);
          if (!__all((unsigned)(pF >> 32) == a.epoch)) pF = wait_granules(ginF + 64 * sb, a.epoch, pF, a.err);
          if (!__all((unsigned)(pH >> 32) == a.epoch && (unsigned)(pF >> 32) == a.epoch)) { ok = false; break; }
          bh = (int)(unsigned)pH;
          bf = (int)(unsigned)pF;
        }
      }
      asm_load_granule(ginH + 64 * min(sb + 1, last_chunk), pH);
      asm_load_granule(ginF + 64 * min(sb + 1, last_chunk), pF);
      // --- re-centre each half's base (after the masked super-blocks 0 and 1)
      if (sb >= 2) {
        const unsigned ref = (unsigned)__builtin_amdgcn_readlane((int)Hc[0], 32);
        const int dlo = (int)(ref & 0xffffu) - kPkaBias, dhi = (int)(ref >> 16) - kPkaBias;  // multiples of 4
        const unsigned dd = ((unsigned)dlo & 0xffffu) | ((unsigned)dhi << 16);
#pragma unroll
        for (int r = 0; r < kRows; ++r) {
          Hc[r] = pk_sub(Hc[r], dd);
          Ec[r] = pk_sub(Ec[r], dd);
        }
        U = pk_sub(U, dd);
        F7 = pk_sub(F7, dd);
        stH = pk_sub(stH, dd);
        stF = pk_sub(stF, dd);
        base_lo += dlo / 4;
        base_hi += dhi / 4;
      }
      int* slH = ringH + (sb & 1) * 64;
      int* slF = ringF + (sb & 1) * 64;
      // past the last chunk (columns > n, read by nothing that is kept) the up
      // row is the base itself: every half stays inside [0, 32767] for the
      // carry-free v_add_u32, junk columns included
      const bool real_up = !from_above || sb < pd.nchunks;
      slH[lane] = real_up ? (int)((unsigned)(4 * (bh - base_lo) + kPkaBias) & 0xffffu) : kPkaBias;
      slF[lane] = from_above && sb < pd.nchunks ? (int)(((unsigned)(4 * (bf - base_lo) + kPkaBias) | 1u) & 0xffffu)
                                                : (kPkaInf | 1);
      unsigned* w = swin + (sb & 1) * 128;
      w[lane] = sw0;
      w[64 + lane] = sw1;
      asm_load_S2(Sg + 64 * (sb + 1), sw0, sw1);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();

      const bool pub_sb = to_below && sb >= 2 && sb - 2 < pd.nchunks;
      // scaled base_lo - base_hi in lane 0's high half (multiple of 4: tags kept)
      const unsigned xfer = lane == 0 ? (unsigned)(4 * (base_lo - base_hi)) << 16 : 0u;
      u64* gpH = goutH + 64 * (sb >= 2 ? sb - 2 : 0);
      u64* gpF = goutF + 64 * (sb >= 2 ? sb - 2 : 0);
      const bool sto = (unsigned)(sb - sblo) < (unsigned)nsb;
      for (int blk = 0; blk < 8; ++blk) {
        const int s0 = sb * 64 + blk * 8;
        const unsigned* srow = w + blk * 8 + 64 - lane;
        const bool pub = pub_sb && blk == 7;
        if (s0 == cap_s0) {  // the block of cell (m, n): its H (and the base it is relative to)
          step_block_pka<true, 2, true>(s0, lane, sto, Hc, Ec, Nb, F7, U, stH, stF, pl, ph, srow, slH + blk * 8,
                                        slF + blk * 8, upsel, mptr, pub, gpH, gpF, a.epoch, base_hi, goe4, ge4, hb0,
                                        xfer, cap_s & 7, Hs);
          cap_base = cap_h ? base_hi : base_lo;
        } else if (sb < 2)
          step_block_pka<true, 2>(s0, lane, sto, Hc, Ec, Nb, F7, U, stH, stF, pl, ph, srow, slH + blk * 8,
                                  slF + blk * 8, upsel, mptr, pub, gpH, gpF, a.epoch, base_hi, goe4, ge4, hb0, xfer,
                                  0, Hs);
        else if (sto)
          step_block_pka<false, 1>(s0, lane, sto, Hc, Ec, Nb, F7, U, stH, stF, pl, ph, srow, slH + blk * 8,
                                   slF + blk * 8, upsel, mptr, pub, gpH, gpF, a.epoch, base_hi, goe4, ge4, hb0, xfer,
                                   0, Hs);
        else
          step_block_pka<false, 0>(s0, lane, sto, Hc, Ec, Nb, F7, U, stH, stF, pl, ph, srow, slH + blk * 8,
                                   slF + blk * 8, upsel, mptr, pub, gpH, gpF, a.epoch, base_hi, goe4, ge4, hb0, xfer,
                                   0, Hs);
        // the counted wait keeps this block's stores in flight; a block that
        // stored nothing waits for the prefetches themselves
        if (sto) {
          mptr += 2 * kRows * kWave;
          wait_vm_keep4<kBlockStores>(sw0, sw1, pH, pF);
        } else {
          wait_vm_keep4<0>(sw0, sw1, pH, pF);
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
    PROG(0x30000000u);
    if (!ok) return;
    if (cap_s0 >= 0) {  // H(m, n): lane cap_t's row cap_r, half cap_h (scaled, biased, relative to cap_base)
      unsigned v = Hs[0];
#pragma unroll
      for (int r = 1; r < kRows; ++r) v = cap_r == r ? Hs[r] : v;
      const int hv = (int)((cap_h ? v >> 16 : v & 0xffffu) >> 2) - kPkaBias / 4 + cap_base;
      if (lane == cap_t) __hip_atomic_fetch_add((gu32*)(a.endv + pd.slot), (unsigned)hv, RLX_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned prev = 0;
    if (lane == 0) prev = __hip_atomic_fetch_add((gu32*)(a.done + pd.slot), 1u, RLX_AGENT);
    prev = __builtin_amdgcn_readfirstlane(prev);
    // the pair's last band pair: every task has released, so acquire and trace here
    if (prev + 1u == (unsigned)ntp) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (a.dbg_notrace) {
        if (lane == 0) { a.oplen[pd.slot] = 0; a.endij[pd.slot] = make_int2(pd.m, pd.n); }
      } else {
        PROG(0x40000000u);
        trace_pair_pka(a, pd, tbl[wid], lane, prog);
        PROG(0x56000000u);
      }
    }
  }
}

// ===========================================================================
// Profile-profile fill of the progressive SoP MSA (oracle
// msa_oracle.c nwo_profile_align):
//   H = min(H[i-1][j-1] + sub(i,j), H[i-1][j] + gx(i), H[i][j-1] + gy(j))
//   sub(i,j) = sum_b rc(i)[b] * cnt(j)[b]   (rc(i)[b] = sum_a cntX(i)[a] c(a,b))
// Same band / skew / granule machinery as nw_align_affine, plain H in int32.
// Each cell stores the affine kernels' 4-bit code with both "opened" bits
// set (a linear gap is always a fresh gap), so trace_pair_affine walks it
// unchanged: 'D', 'u' (X column vs a gap column), 'l' (gap column vs Y).
// ===========================================================================
// DOT: how the row / column profiles' six counts are packed (host: nwk_msa,
// per launch): 4 = u8 x 4 in ints 0-1 (v_dot4_u32_u8), 2 = u16 x 2 in ints
// 0-2 (v_dot2_u32_u16), 0 = one int each (v_mad_u32_u24); 5 = rows as 4 with
// single-sequence columns, whose count is one-hot: int 0 is the v_perm
// selector of the column's symbol (one v_perm per cell); the packed forms
// repeat a column's gy right after the counts, so a step reads one 16-byte
// entry.  H is carried as the key 4H (+ the move in bits 0-1 while a cell is
// decided): the three candidates are 4 d, 4 u + 1, 4 l + 2, so one v_min3_u32 gives the cell's
// value and its move with the D < U < L tie order of trace_pair_affine's
// codes, and key | 12 is the stored 4-bit code.  The DP stays below 2^30
// (nwk_msa's admission check), so 4H + 3 fits a u32.
template <int DOT, int N>
__device__ __forceinline__ unsigned prof_sub(const unsigned (&rp)[N], const int4& c0) {
  if constexpr (DOT == 5) {
    return __builtin_amdgcn_perm(rp[1], rp[0], (unsigned)c0.x);  // one-hot column: rc[its symbol]
  } else if constexpr (DOT == 4) {
    return __builtin_amdgcn_udot4(rp[1], (unsigned)c0.y, __builtin_amdgcn_udot4(rp[0], (unsigned)c0.x, 0u, false), false);
  } else if constexpr (DOT == 2) {
    typedef unsigned short us2 __attribute__((ext_vector_type(2)));
    unsigned t = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, rp[0]), __builtin_bit_cast(us2, (unsigned)c0.x), 0u, false);
    t = __builtin_amdgcn_udot2(__builtin_bit_cast(us2, rp[1]), __builtin_bit_cast(us2, (unsigned)c0.y), t, false);
    return __builtin_amdgcn_udot2(__builtin_bit_cast(us2, rp[2]), __builtin_bit_cast(us2, (unsigned)c0.z), t, false);
  } else {
    return 0u;  // (the unpacked form reads both int4s: prof_sub6)
  }
}

template <int DOT, int R = kProfRows>
__global__ __launch_bounds__(256) void nw_profile(FillArgs a) {
  constexpr int W = 4, SPD = 8;
  constexpr int NP = DOT >= 4 ? 2 : DOT == 2 ? 3 : 6;  // packed ints per profile entry
  __shared__ __attribute__((aligned(16))) unsigned ring_all[4][128];
  __shared__ __attribute__((aligned(16))) int4 cwin_all[4][2][256];  // 128 columns x 8 ints, two slots
  __shared__ __attribute__((aligned(16))) TbLds<W> tbl[4];
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  unsigned* ring = ring_all[wid];
  unsigned* prog = a.prog ? a.prog + blockIdx.x * 4 + wid : nullptr;

  for (;;) {
    unsigned tk = 0;
    if (lane == 0) tk = atomicAdd(a.counter, 1u);
    tk = __builtin_amdgcn_readfirstlane(tk);
    PROG(0x10000000u | (tk & 0xffffffu));
    if (tk >= (unsigned)a.ntasks) return;
    if (__hip_atomic_load((gu32*)a.err, RLX_AGENT) != 0u) return;
    const int2 task = a.tasks[tk];
    const PairDesc pd = a.pairs[task.x];
    const int band = task.y;
    const int row0 = band * (R * kWave) + lane * R;  // 0-based first DP row of this lane
    unsigned rp[R][NP], gxk[R], h[R], acc[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int row = min(row0 + r, pd.m - 1);  // rows past m: copies of the last (never traced)
      const int4* pr = reinterpret_cast<const int4*>(a.prow + (pd.x_off + row) * 8);
      const int4 q0 = pr[0], q1 = pr[1];
      const unsigned e[8] = {(unsigned)q0.x, (unsigned)q0.y, (unsigned)q0.z, (unsigned)q0.w,
                             (unsigned)q1.x, (unsigned)q1.y, (unsigned)q1.z, (unsigned)q1.w};
#pragma unroll
      for (int b = 0; b < NP; ++b) rp[r][b] = e[b];
      gxk[r] = 4u * e[6] + 1u;  // up move key increment
      h[r] = 4u * e[7];         // H[i][0]
      acc[r] = 0;
    }
    unsigned Up = band == 0 ? 0u : 4u * (unsigned)a.prow[(pd.x_off + band * (R * kWave) - 1) * 8 + 7];  // H[row above the band][0]
    unsigned stH = 0;
    const bool from_above = band > 0;
    const bool to_below = band + 1 < pd.nbands;
    const int64_t bstride = (int64_t)pd.nchunks * 64;
    const u64* gin = reinterpret_cast<const u64*>(a.bnd) + pd.bnd_off + (int64_t)(band > 0 ? band - 1 : 0) * bstride + lane;
    const int last_chunk = pd.nchunks > 0 ? pd.nchunks - 1 : 0;
    u64* gout = a.bnd + pd.bnd_off + (int64_t)band * bstride + lane;
    unsigned* mptr = a.mat + pd.mat_off + (int64_t)band * prof_band_dwords(pd.sblocks) + lane;
    // column j (1-based; 0 = the H[0][0] entry) is pcol entry y_off + j; window of sb: columns 64sb-63 .. 64sb+64
    const int4* colg = reinterpret_cast<const int4*>(a.pcol) + 2 * (pd.y_off - 63);
    // Granule prefetches are ordinary (compiler-tracked) loads here: this
    // kernel's register pressure makes the compiler move values between
    // registers, and a copy of an asm load's destination taken before its
    // s_waitcnt would read the register before the data landed.
    u64 pend = from_above ? ld_granule(gin) : 0;
    bool ok = true;
    // fill-vs-walk guard: cell (m, n) is lane t's row r of the last band at
    // step n - 1 + t; H = key / 4
    int cap_s = -1, cap_t = 0, cap_r = 0;
    unsigned hs[R];
#pragma unroll
    for (int r = 0; r < R; ++r) hs[r] = 0;
    if (a.endv && band == pd.nbands - 1) {
      const int wr = (pd.m - 1) - band * (R * kWave);
      cap_t = wr / R;
      cap_r = wr % R;
      cap_s = pd.n - 1 + cap_t;
    }

    // one super-block of 64 steps; MASK: super-block 0, whose first 63 steps
    // reach lanes before their column 1 (the border H[i][0] stays)
    auto run_sb = [&](int sb, auto maskc, int capk) {
      constexpr bool MASK = decltype(maskc)::value;
      const unsigned* slot = ring + (sb & 1) * 64;
      const int4* cw = cwin_all[wid][sb & 1];
      // column entries are read one step ahead (the LDS latency hides behind a step)
      auto ld_col = [&](int we, int4& x0, int4& x1) {
        x0 = cw[2 * we];
        if constexpr (DOT == 0) x1 = cw[2 * we + 1];
      };
      int4 n0, n1 = make_int4(0, 0, 0, 0);
      ld_col(64 - lane, n0, n1);
      for (int blk = 0; blk < 8; ++blk) {
        const int s0 = sb * 64 + blk * 8;
        const uint4 bA = *reinterpret_cast<const uint4*>(slot + blk * 8);
        const uint4 bB = *reinterpret_cast<const uint4*>(slot + blk * 8 + 4);
        const unsigned bv[8] = {bA.x, bA.y, bA.z, bA.w, bB.x, bB.y, bB.z, bB.w};
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          stH = __builtin_amdgcn_update_dpp(h[R - 1], stH, 0x130 /*wave_shl:1*/, 0xf, 0xf, false);
          const unsigned uh = __builtin_amdgcn_update_dpp(bv[k], h[R - 1], 0x138 /*wave_shr:1*/, 0xf, 0xf, false);
          const unsigned dg0 = Up;
          Up = uh;
          // this lane's column j = s - lane + 1 -> window entry j - (64sb - 63) = (s - 64sb) - lane + 64
          const int we = blk * 8 + k - lane + 64;
          const int4 c0 = n0, c1 = n1;
          if (k < 7 || blk < 7) ld_col(we + 1, n0, n1);
          // left move key increment: gy follows the packed counts (int 2 / 3), or int 6
          const unsigned lk = 4u * (unsigned)(DOT >= 4 ? c0.z : DOT == 2 ? c0.w : c1.z) + 2u;
          const bool valid = !MASK || (s0 + k) >= lane;
          unsigned hp = uh, nh[R];
#pragma unroll
          for (int r = 0; r < R; ++r) {
            unsigned sub;
            if constexpr (DOT == 0) {
              const unsigned cy[kProfSyms] = {(unsigned)c0.x, (unsigned)c0.y, (unsigned)c0.z,
                                              (unsigned)c0.w, (unsigned)c1.x, (unsigned)c1.y};
              sub = 0;
#pragma unroll
              for (int b = 0; b < kProfSyms; ++b) sub += __umul24(rp[r][b], cy[b]);
            } else {
              sub = prof_sub<DOT>(rp[r], c0);
            }
            const unsigned d = (r ? h[r - 1] : dg0) + 4u * sub;  // diag: row above, previous step
            const unsigned key = min(min(d, h[r] + lk), hp + gxk[r]);
            // (the code nibble is key's low 4 bits with both "opened" bits set: the
            // | 12 of all eight nibbles is one v_or at the store; the empty asm keeps
            // the shift in this step -- sunk to the store, it held 56 keys in
            // registers, with a v_mov each)
            acc[r] = __builtin_amdgcn_alignbit(key, acc[r], 4);
            asm volatile("" : "+v"(acc[r]));
            const unsigned nv = key & ~3u;
            nh[r] = MASK ? (valid ? nv : h[r]) : nv;
            hp = nh[r];
          }
#pragma unroll
          for (int r = 0; r < R; ++r) h[r] = nh[r];  // (d above read the previous step's h[r - 1])
          if (blk * 8 + k == capk) {  // (uniform) the step of cell (m, n): the fill-vs-walk guard's end value
#pragma unroll
            for (int r = 0; r < R; ++r) hs[r] = nh[r];
          }
          if (k == 7) {
#pragma unroll
            for (int r = 0; r < R; ++r) __builtin_nontemporal_store(acc[r] | 0xccccccccu, mptr + r * kWave);
          }
          __builtin_amdgcn_sched_barrier(0);
        }
        mptr += (8 / SPD) * R * kWave;
      }
    };

    for (int sb = 0; sb < pd.sblocks; ++sb) {
      unsigned bval;  // band-above row: H[row above][64sb + 1 + lane] (key form 4H)
      if (from_above) {
        bval = 0;
        if (sb < pd.nchunks) {
          if (!__all((unsigned)(pend >> 32) == a.epoch)) pend = wait_granules(gin + 64 * sb, a.epoch, pend, a.err);
          if (!__all((unsigned)(pend >> 32) == a.epoch)) { ok = false; break; }
          bval = (unsigned)pend;
        }
        pend = ld_granule(gin + 64 * min(sb + 1, last_chunk));  // next chunk, used at the next super-block
      } else {
        bval = 4u * (unsigned)a.pcol[(pd.y_off + 64 * sb + lane + 1) * 8 + 7];  // H[0][j]
      }
      ring[(sb & 1) * 64 + lane] = bval;
      int4* cw = cwin_all[wid][sb & 1];
      // columns 64sb-63 .. 64sb+64: 128 entries of 8 ints = 256 int4
#pragma unroll
      for (int k = 0; k < 4; ++k) cw[lane + 64 * k] = colg[128 * sb + lane + 64 * k];
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
      __builtin_amdgcn_wave_barrier();
      const int capk = cap_s >= 0 && cap_s >> 6 == sb ? cap_s & 63 : -1;
      if (sb == 0)
        run_sb(sb, std::true_type{}, capk);
      else
        run_sb(sb, std::false_type{}, capk);
      if (to_below && sb >= 1 && sb <= pd.nchunks) st_granule(gout + 64 * (sb - 1), a.epoch, (int)stH);
      __builtin_amdgcn_wave_barrier();
      PROG(0x20000000u | ((unsigned)band << 12) | (unsigned)(sb & 0xfff));
    }
    if (!ok) return;
    if (cap_s >= 0) {
      unsigned v = hs[0];
#pragma unroll
      for (int r = 1; r < R; ++r) v = cap_r == r ? hs[r] : v;
      if (lane == cap_t) __hip_atomic_fetch_add((gu32*)(a.endv + pd.slot), v >> 2, RLX_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    PROG(0x30000000u);
    unsigned prev = 0;
    if (lane == 0) prev = __hip_atomic_fetch_add((gu32*)(a.done + pd.slot), 1u, RLX_AGENT);
    prev = __builtin_amdgcn_readfirstlane(prev);
    if (prev + 1u == (unsigned)pd.nbands) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      PROG(0x40000000u);
      // nwk_msa verbose >= 2: per merge 8 u64, {walk start, walk end} (s_memrealtime, 100 MHz), then
      // the walk's cycle counters (trace_pair_affine<true>)
      if (a.stamps && lane == 0) a.stamps[8 * pd.slot] = __builtin_amdgcn_s_memrealtime();
      trace_pair_affine<true, R>(a, pd, tbl[wid], lane, prog);
      if (a.stamps && lane == 0) a.stamps[8 * pd.slot + 1] = __builtin_amdgcn_s_memrealtime();
      PROG(0x60000000u);
    }
  }
}

// ---------------------------------------------------------------------------
template <int MODE, int W>
static hipError_t fill_w(const FillArgs& a, int grid, hipStream_t s) {
  hipLaunchKernelGGL((nw_align<MODE, W>), dim3(grid), dim3(256), 0, s, a);
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
    case kAffine:
      if (bits != 4) return hipErrorInvalidValue;
      hipLaunchKernelGGL(nw_align_affine, dim3(grid), dim3(256), 0, s, a);
      return hipGetLastError();
    case kPacked:
      if (bits != 4) return hipErrorInvalidValue;
      hipLaunchKernelGGL(nw_align_pk, dim3(grid), dim3(256), 0, s, a);
      return hipGetLastError();
    case kPacked2:
      if (bits != 4) return hipErrorInvalidValue;
      hipLaunchKernelGGL(nw_align_pk2, dim3(grid), dim3(256), 0, s, a);
      return hipGetLastError();
    case kProfileDP:
      if (bits != 4) return hipErrorInvalidValue;
      // (kProfileDP passes the profile packing in lin_mode, which only nw_align reads)
      if (a.lin_mode == 5)
        hipLaunchKernelGGL(nw_profile<5>, dim3(grid), dim3(256), 0, s, a);
      else if (a.lin_mode == 4)
        hipLaunchKernelGGL(nw_profile<4>, dim3(grid), dim3(256), 0, s, a);
      else if (a.lin_mode == 2)
        hipLaunchKernelGGL(nw_profile<2>, dim3(grid), dim3(256), 0, s, a);
      else if (a.lin_mode == 0)
        hipLaunchKernelGGL(nw_profile<0>, dim3(grid), dim3(256), 0, s, a);
      else
        return hipErrorInvalidValue;
      return hipGetLastError();
    case kAffinePk:
      if (bits != 4) return hipErrorInvalidValue;
      hipLaunchKernelGGL(nw_align_pka, dim3(grid), dim3(256), 0, s, a);
      return hipGetLastError();
    case kProfile: return fill_m<kProfile>(bits, a, grid, s);
    case kCompare: return fill_m<kCompare>(bits, a, grid, s);
    case kLiteral: return bits == 32 ? fill_w<kLiteral, 32>(a, grid, s) : hipErrorInvalidValue;
  }
  return hipErrorInvalidValue;
}

template <int MODE, int W>
static int occ_w() {
  int n = 0;
  if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, reinterpret_cast<const void*>(&nw_align<MODE, W>), 256, 0) != hipSuccess)
    return 1;
  return n > 0 ? n : 1;
}

int fill_blocks_per_cu(int mode, int bits) {
  if (mode == kLiteral) return occ_w<kLiteral, 32>();
  if (mode == kAffine || mode == kPacked || mode == kPacked2 || mode == kProfileDP || mode == kAffinePk) {
    int n = 0;
    const void* f = mode == kAffine     ? reinterpret_cast<const void*>(&nw_align_affine)
                    : mode == kAffinePk ? reinterpret_cast<const void*>(&nw_align_pka)
                    : mode == kPacked   ? reinterpret_cast<const void*>(&nw_align_pk)
                    : mode == kPacked2  ? reinterpret_cast<const void*>(&nw_align_pk2)
                                        : reinterpret_cast<const void*>(&nw_profile<0>);
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, f, 256, 0) != hipSuccess) return 1;
    return n > 0 ? n : 1;
  }
  const bool p = mode == kProfile;
  switch (bits) {
    case 4: return p ? occ_w<kProfile, 4>() : occ_w<kCompare, 4>();
    case 8: return p ? occ_w<kProfile, 8>() : occ_w<kCompare, 8>();
    case 16: return p ? occ_w<kProfile, 16>() : occ_w<kCompare, 16>();
    default: return p ? occ_w<kProfile, 32>() : occ_w<kCompare, 32>();
  }
}

}  // namespace nwk
