// nwk_bits_dev.h -- device helpers shared by the bit-sliced fill kernels
// (nwk_bits.hip: nw_align_bits / nw_align_strip; nwk_col.hip: nw_align_col):
// coherent reads, the bounded hand-off wait, the bitop3 plane algebra, the
// scalar-walk helpers of the traceback and the fused pair finalize.
#pragma once
#include "nwk_internal.h"
#include "nwk_sha_dev.h"

namespace nwk {
namespace {

typedef unsigned long long u64;
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned gu32;
#define BITS_RLX __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT

constexpr int kBR = kBitsRows;  // rows per band (64 lanes x 32 bits)

__device__ __forceinline__ unsigned long long bits_opaque_zero() {
  unsigned long long z = 0;
  asm volatile("" : "+v"(z));
  return z;
}

// Reads at the coherence point (an atomic add of 0): a plain load can hit a
// stale line in this XCD's L2 when another XCD wrote the word during the launch
__device__ __forceinline__ unsigned ld_fresh(const unsigned* p) {
  return __hip_atomic_fetch_add((gu32*)p, (unsigned)bits_opaque_zero(), BITS_RLX);
}
__device__ __forceinline__ u64 ld_fresh64(const u64* p) {
  return __hip_atomic_fetch_add((gu64*)p, bits_opaque_zero(), BITS_RLX);
}

// Polls the granules lanes 0..n-1 hold until every one carries `epoch`
// (bounded: ~4 s of wall time, or another wave's failure).
__device__ __noinline__ u64 bits_wait(const u64* p, bool mine, unsigned epoch, u64 v, unsigned* err) {
  const u64 t0 = __builtin_amdgcn_s_memrealtime();
  for (;;) {
    if (__all(!mine || (unsigned)(v >> 32) == epoch)) return v;
    __builtin_amdgcn_s_sleep(4);
    if (__builtin_amdgcn_readfirstlane(__hip_atomic_load((gu32*)err, BITS_RLX)) != 0u) return 0;
    if (__builtin_amdgcn_s_memrealtime() - t0 > 400000000ull) {
      if ((threadIdx.x & 63) == 0) atomicOr(err, 1u);
      return 0;
    }
    // a read-modify-write is performed at the coherence point (no stale L2 copy)
    if (mine) v = __hip_atomic_fetch_add((gu64*)p, bits_opaque_zero(), BITS_RLX);
  }
}

// The plane update with explicit v_bitop3_b32 (any 3-input boolean function,
// full rate on gfx950: 2.7 cycles per wave-instruction against 4.4 for
// v_or3 / v_and_or, profiles/r02/valu_probe_gfx950.txt).  Truth-table
// immediates are built from the operand masks kA = S0, kB = S1, kC = S2.
#ifndef NWK_BITS_BOP3
#define NWK_BITS_BOP3 1
#endif
constexpr unsigned kA = 0xF0u, kB = 0xCCu, kC = 0xAAu;
#define BOP3(a, b, c, f) __builtin_amdgcn_bitop3_b32((a), (b), (c), (unsigned)((f) & 0xFFu))

// acc | OR_{j >= J, j + K < NP} (~X_j & D_{j+K});  D_i is all ones for i < SR
template <int NP, int SR, int K, int J>
__device__ __forceinline__ unsigned bits_conv(unsigned acc, const unsigned (&X)[NP], const unsigned (&D)[NP]) {
  if constexpr (J + K >= NP) {
    return acc;
  } else {
    if constexpr (J + K < SR) acc = BOP3(acc, X[J], X[J], kA | ~kB);
    else acc = BOP3(acc, X[J], D[J + K], kA | (~kB & kC));
    return bits_conv<NP, SR, K, J + 1>(acc, X, D);
  }
}

// plane K of the difference D - X:  OR_j (~X_j & D_{j+K})
template <int NP, int SR, int K>
__device__ __forceinline__ unsigned bits_diff(const unsigned (&X)[NP], const unsigned (&D)[NP]) {
  constexpr bool ones0 = K < SR;  // D_K all ones
  if constexpr (K + 1 >= NP) {
    if constexpr (ones0) return ~X[0];
    else return BOP3(X[0], D[K], D[K], ~kA & kB);
  } else {
    constexpr bool ones1 = K + 1 < SR;
    unsigned acc;
    if constexpr (ones0 && ones1) {
      acc = BOP3(X[0], X[1], X[1], ~kA | ~kB);
    } else if constexpr (ones0) {
      acc = BOP3(X[0], X[1], D[K + 1], ~kA | (~kB & kC));
    } else {
      acc = BOP3(X[0], D[K], D[K], ~kA & kB);
      acc = BOP3(acc, X[1], D[K + 1], kA | (~kB & kC));
    }
    return bits_conv<NP, SR, K, 2>(acc, X, D);
  }
}

template <int NP, int SR>
__device__ __forceinline__ void bits_diffs(const unsigned (&X)[NP], const unsigned (&D)[NP], unsigned (&out)[NP]) {
  out[0] = bits_diff<NP, SR, 0>(X, D);
  out[1] = bits_diff<NP, SR, 1>(X, D);
  if constexpr (NP == 4) {
    out[2] = bits_diff<NP, SR, 2>(X, D);
    out[3] = bits_diff<NP, SR, 3>(X, D);
  }
}


#define BITS_PROG(v)                                                                                         \
  do {                                                                                                       \
    if (prog && lane == 0) __hip_atomic_store((gu32*)prog, (unsigned)(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); \
  } while (0)

// scalar min (the compiler would take v_min3 and a readfirstlane round trip)
__device__ __forceinline__ int smin(int a, int b) {
  int r;
  asm("s_min_i32 %0, %1, %2" : "=s"(r) : "s"(__builtin_amdgcn_readfirstlane(a)), "s"(__builtin_amdgcn_readfirstlane(b)) : "scc");
  return r;
}

__device__ __forceinline__ int sminu(int a, int b) {
  int r;
  asm("s_min_u32 %0, %1, %2" : "=s"(r) : "s"(__builtin_amdgcn_readfirstlane(a)), "s"(__builtin_amdgcn_readfirstlane(b)) : "scc");
  return r;
}
// first set bit of a 64-bit mask, -1 when none
__device__ __forceinline__ int sff1(u64 m) {
  int r;
  asm("s_ff1_i32_b64 %0, %1" : "=s"(r) : "s"(m) : "scc");
  return r;
}

#ifndef NWK_TRACE_PROF
#define NWK_TRACE_PROF 0  // 1: the timeline's trace columns become a cycle breakdown (A/B only)
#endif
constexpr int kTraceRing = 1024;  // bytes of LDS per wave for the trace's move ring
#ifndef NWK_TRACE_NB
#define NWK_TRACE_NB 3  // step-tiles per prefetched batch
#endif
constexpr int kNB = NWK_TRACE_NB;
// s_waitcnt immediate for vmcnt(n) leaving expcnt / lgkmcnt alone (gfx9 encoding)
constexpr int waitcnt_vm(int n) { return (n & 15) | ((n >> 4) << 14) | 0x0F70; }

// NWK_TRACE_PRIO 1: the traceback wave raises its issue priority (s_setprio 3)
#ifndef NWK_TRACE_PRIO
#define NWK_TRACE_PRIO 0
#endif

// ---- Fused pair finalize (FillArgs::fuse_fin) ------------------------------
// The same work as nw_rows + nw_hash (nwk_hash.hip), done inside the fill
// launch so results leave the GPU as pairs finish.  The rows are built by the
// wave that traced the pair (all 64 lanes busy); the SHA-512 -- sequential
// within a row -- runs one row per lane on waves that claim 32 traced pairs at
// a time from a queue, so every hashing instruction works for 64 rows (hashing
// in the tracing wave itself, two lanes of 64, cost ~32x the issue and slowed
// C3 by 3%, profiles/r03/ab/fused_finalize_not_kept.txt).

// align1 / align2 (skel:263-272 prefix, then the moves in forward order: 64
// per iteration, a wave scan of the packed x / y advances) and the path cost
// (= dp[m][n], the reference's penalty) -> fin_len[slot], fin_len[np + slot].
// Returns false when the walk or its moves are inconsistent (error word set):
// the pair is then not queued, so no record with stale rows is ever published.
__device__ __forceinline__ bool fin_rows(const FillArgs& a, const PairDesc& pd, int lane, int nops, int2 e) {
  using namespace shadev;
  const int pre = e.x > 0 ? e.x : e.y;
  if (e.x < 0 || e.y < 0 || e.x > pd.m || e.y > pd.n || nops < 0 || pre + nops > pd.m + pd.n) {
    if (lane == 0) atomicOr(a.err, 128u);  // (a walk that did not end on the border)
    return false;
  }
  const uint8_t* ops = a.ops + pd.ops_off;
  const uint8_t* x = a.raw + pd.x_off;
  const uint8_t* y = a.raw + pd.y_off;
  uint8_t* r1 = a.rows1 + (pd.ops_off - a.ops_base);
  uint8_t* r2 = a.rows2 + (pd.ops_off - a.ops_base);
  for (int t = lane; t < pre; t += 64) {  // prefix run
    r1[t] = e.x > 0 ? x[t] : (uint8_t)'_';
    r2[t] = e.x > 0 ? (uint8_t)'_' : y[t];
  }
  int ix = e.x, iy = e.y;
  int pen = 0;
  bool off = false;  // a move left the matrix
  for (int base = 0; base < nops; base += 64) {
    const int f = base + lane;
    const bool live = f < nops;
    const unsigned op = live ? ops[nops - 1 - f] : 0u;
    const bool d = op == 'D', up = op == 'U';
    const bool ax = live && (d || up), ay = live && (d || !up);
    const unsigned adv = (ax ? 1u : 0u) | (ay ? 0x10000u : 0u);
    const unsigned inc = wave_incl_scan(adv, lane);
    const unsigned exc = inc - adv;
    if (live) {
      const int xi = ix + (int)(exc & 0xffffu), yi = iy + (int)(exc >> 16);
      if ((ax && xi >= pd.m) || (ay && yi >= pd.n)) {
        atomicOr(a.err, 256u);  // (moves that leave the matrix)
        off = true;
      } else {
        const unsigned chx = ax ? x[xi] : (unsigned)'_';
        const unsigned chy = ay ? y[yi] : (unsigned)'_';
        r1[pre + f] = (uint8_t)chx;
        r2[pre + f] = (uint8_t)chy;
        pen += d ? (chx == chy ? 0 : a.pxy) : a.pgap;
      }
    }
    const unsigned tot = (unsigned)__shfl((int)inc, 63);
    ix += (int)(tot & 0xffffu);
    iy += (int)(tot >> 16);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) pen += __shfl_xor(pen, o);
  pen += pre * a.pgap;
  if (lane == 0) {
    a.fin_len[pd.slot] = pre + nops;  // both rows have this length
    a.fin_len[a.ntasks_pairs + pd.slot] = pen;
  }
  // the fill-vs-walk guard (skel:274): the walked path must cost the fill's
  // H(m, n); a pair that disagrees is not queued (no record) and re-runs
  if (a.endv && !__any(off)) {
    const int ev = (int)__hip_atomic_load((gu32*)(a.endv + pd.slot), BITS_RLX);
    if (__builtin_amdgcn_readfirstlane(pen) != ev) {
      if (lane == 0) a.retry[pd.slot] = 2;
      return false;
    }
  }
  return !__any(off);
}

// After fin_rows: publish the rows (a hashing wave may run on another XCD)
// and queue the pair.  Every traced pair (also one that left its storage
// window and re-runs later) is counted in hq_ctl[2].
__device__ __forceinline__ void hq_push(const FillArgs& a, const PairDesc& pd, int lane, bool queue) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  if (lane == 0) {
    if (queue) {
      const unsigned pos = __hip_atomic_fetch_add(a.hq_ctl, 1u, BITS_RLX);
      __hip_atomic_store((gu64*)(a.hq + pos), ((u64)a.epoch << 32) | (unsigned)pd.slot, BITS_RLX);
    }
    __hip_atomic_fetch_add(a.hq_ctl + 2, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// Claims up to 32 queued pairs (at least 32 unless `drain`) and hashes them:
// lane 2q + s runs SHA-512 over row s of pair q, the even lane then hashes the
// two digests' hex (skel:155-157) and writes the host-mapped record and its
// flag.  Returns whether it hashed anything.
__device__ __forceinline__ bool hq_hash(const FillArgs& a, int lane, bool drain) {
  using namespace shadev;
  unsigned tail = 0, head = 0;
  if (lane == 0) {
    tail = ld_fresh(a.hq_ctl);
    head = ld_fresh(a.hq_ctl + 1);
  }
  tail = __builtin_amdgcn_readfirstlane(tail);
  head = __builtin_amdgcn_readfirstlane(head);
  const unsigned avail = tail - head;
  if (avail == 0 || avail > 0x7fffffffu || (!drain && avail < 32)) return false;
  const unsigned want = avail < 32 ? avail : 32;
  unsigned ok = 0;
  if (lane == 0)
    ok = __hip_atomic_compare_exchange_strong(a.hq_ctl + 1, &head, head + want, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_AGENT) ? 1u : 0u;
  if (!__builtin_amdgcn_readfirstlane(ok)) return false;  // another wave took them: the caller retries
  head = __builtin_amdgcn_readfirstlane(head);
  const int q = lane >> 1, side = lane & 1;
  const bool live = q < (int)want;
  u64 ent = 0;
  if (live) {  // the producer reserved the entry just before writing it
    const u64 t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
      ent = ld_fresh64(a.hq + head + q);
      if ((unsigned)(ent >> 32) == a.epoch) break;
      if (__builtin_amdgcn_s_memrealtime() - t0 > 400000000ull) break;
    }
  }
  const bool ok_ent = !live || (unsigned)(ent >> 32) == a.epoch;
  if (!__all(ok_ent)) {
    if (lane == 0) atomicOr(a.err, 32u);
    return true;
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // the producers' rows
  const int slot = live ? (int)(unsigned)ent : 0;
  // (row length and penalty were written on the producer's XCD: fresh reads)
  int64_t L = live ? (int)ld_fresh(reinterpret_cast<const unsigned*>(a.fin_len + slot)) : 0;
  // (a queue entry or row length outside its pair: report, hash nothing)
  const bool sane = !live || ((unsigned)slot < (unsigned)a.ntasks_pairs && L >= 0 &&
                              L <= (int64_t)a.pairs[slot].m + a.pairs[slot].n);
  if (!__all(sane)) {
    if (lane == 0) atomicOr(a.err, 64u);
    return true;
  }
  const uint4* row = reinterpret_cast<const uint4*>((side ? a.rows2 : a.rows1) + (a.pairs[slot].ops_off - a.ops_base));
  Sha sh;
  sh.init();
  const int64_t nblk = live ? (L + 17 + 127) / 128 : 0, ndata = (L + 127) / 128;
  int64_t wblk = nblk;  // per wave: as many blocks as its longest row
  for (int o = 32; o > 0; o >>= 1) wblk = max(wblk, (int64_t)__shfl_xor(wblk, o));
  uint4 cur[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) cur[k] = ndata > 0 ? row[k] : make_uint4(0, 0, 0, 0);
  for (int64_t bk = 0; bk < wblk; ++bk) {
    uint64_t w[16];
#pragma unroll
    for (int k = 0; k < 8; ++k) {  // little-endian dwords -> big-endian 64-bit words
      w[2 * k] = ((uint64_t)__builtin_bswap32(cur[k].x) << 32) | __builtin_bswap32(cur[k].y);
      w[2 * k + 1] = ((uint64_t)__builtin_bswap32(cur[k].z) << 32) | __builtin_bswap32(cur[k].w);
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) cur[k] = bk + 1 < ndata ? row[8 * (bk + 1) + k] : make_uint4(0, 0, 0, 0);
    const int64_t b0 = 128 * bk;  // message bytes [b0, b0 + 128)
#pragma unroll
    for (int k = 0; k < 16; ++k) {  // clear bytes past L, place the 0x80 terminator
      const int64_t s0 = b0 + 8 * k;
      if (s0 + 8 > L) {
        const int keep = (int)max((int64_t)0, min((int64_t)8, L - s0));
        uint64_t v = keep > 0 ? w[k] & (~0ull << (64 - 8 * keep)) : 0ull;
        if (L >= s0 && L < s0 + 8) v |= 0x80ull << (56 - 8 * (L - s0));
        w[k] = v;
      }
    }
    if (bk == nblk - 1) w[15] = (uint64_t)L * 8u;
    if (bk < nblk) sh.block_rolled(w);
  }
  uint64_t other[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) other[k] = __shfl_xor(sh.s[k], 1);
  if (live && side == 0) {
    Sha p;
    p.init();
    uint64_t w[16];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      w[2 * k] = hex16((uint32_t)(sh.s[k] >> 32));
      w[2 * k + 1] = hex16((uint32_t)sh.s[k]);
    }
    p.block_rolled(w);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      w[2 * k] = hex16((uint32_t)(other[k] >> 32));
      w[2 * k + 1] = hex16((uint32_t)other[k]);
    }
    p.block_rolled(w);
#pragma unroll
    for (int k = 0; k < 16; ++k) w[k] = 0;
    w[0] = 0x8000000000000000ULL;
    w[15] = 256 * 8;
    p.block_rolled(w);
    uint64_t* out = reinterpret_cast<uint64_t*>(a.fin_hash + 64 * (int64_t)slot);
#pragma unroll
    for (int k = 0; k < 8; ++k) out[k] = __builtin_bswap64(p.s[k]);
    a.fin_pen[slot] = (int)ld_fresh(reinterpret_cast<const unsigned*>(a.fin_len + a.ntasks_pairs + slot));
    __threadfence_system();  // the record, then its flag (the host polls it during the launch)
    __hip_atomic_store(a.fin_flag + slot, a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  return true;
}

// Out of fill tasks: at most kDrainWaves waves stay to hash what is left
// until every pair of the launch is traced and claimed (bounded like the
// hand-off waits: ~4 s without progress, or another wave's failure).
constexpr unsigned kDrainWaves = 64;
__device__ __forceinline__ void hq_drain(const FillArgs& a, int lane) {
  unsigned w = 0;
  if (lane == 0) w = __hip_atomic_fetch_add(a.hq_ctl + 3, 1u, BITS_RLX);
  if (__builtin_amdgcn_readfirstlane(w) >= kDrainWaves) return;
  u64 t0 = __builtin_amdgcn_s_memrealtime();
  for (;;) {
    if (hq_hash(a, lane, true)) {
      t0 = __builtin_amdgcn_s_memrealtime();
      continue;
    }
    unsigned traced = 0, tail = 0, head = 0;
    if (lane == 0) {
      traced = ld_fresh(a.hq_ctl + 2);
      tail = ld_fresh(a.hq_ctl);
      head = ld_fresh(a.hq_ctl + 1);
    }
    traced = __builtin_amdgcn_readfirstlane(traced);
    tail = __builtin_amdgcn_readfirstlane(tail);
    head = __builtin_amdgcn_readfirstlane(head);
    if (traced >= (unsigned)a.ntasks_pairs && head == tail) return;
    if (__builtin_amdgcn_readfirstlane(__hip_atomic_load((gu32*)a.err, BITS_RLX)) != 0u) return;
    if (__builtin_amdgcn_s_memrealtime() - t0 > 400000000ull) {
      if (lane == 0) atomicOr(a.err, 32u);
      return;
    }
    __builtin_amdgcn_s_sleep(32);
  }
}

// At least NWK_BITS_WPE waves per SIMD: 4 (<= 128 VGPRs, a few spills outside
// the step loop) beat the compiler's 3 (143 VGPRs) by 2% on C3, 6% on C4.
#ifndef NWK_BITS_WPE
#define NWK_BITS_WPE 4
#endif
#if NWK_BITS_WPE > 0
#define NWK_BITS_OCC __attribute__((amdgpu_waves_per_eu(NWK_BITS_WPE)))
#else
#define NWK_BITS_OCC
#endif

// FUSE: the instantiation with the fused finalize (FillArgs::fuse_fin); the
// plain one carries none of its code, so the hashing's registers never touch
// the fill and trace (one instantiation with both: lone C3 trace 4.7 -> 5.8 ms)
}  // namespace
}  // namespace nwk
