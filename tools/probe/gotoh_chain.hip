// gotoh_chain.hip -- the bit-sliced Gotoh step (gotoh_bits.h) with band
// hand-off: pairs of any height, 2048-row bands in a chain, one wave per band.
//
// Layout as gotoh_gpu.hip (bit b of lane t = row R0 + 32 t + b + 1, at column
// s - 32 t - b at step s).  A band's last row (lane 63, bit 31: column
// s - 2047) goes to an LDS ring each step; at the end of every 32-step segment
// the next complete 32 columns are packed by ballot into 11 plane words (8 of
// h, 3 of f) and published as self-tagged granules {epoch:32 | word:32}.  The
// band below polls them with atomic reads (the coherence point, as
// nw_align_bits' bits_wait) and stages one word per plane into LDS, bit 31 per
// column, as the DPP fill-in of lane 0.  Tasks are dequeued from one counter
// in dependency order (band-major), so a band's producer is always running.
//
//   gotoh_chain check < pairs    "x y" per line, any |x|: H[m][n] per pair
//   gotoh_chain trace < pairs    the same with every cell's four words stored, then
//                                nwo_pair_affine's walk over them on the host: "H a1 a2"
//   gotoh_chain dtrace < pairs   the same walk on the device (gotoh_walk; pairs of
//                                equal m + n)
//   gotoh_chain dtrate [pairs] [m] [n] [window]
//                                fill + windowed store, then the device walk, timed
//   gotoh_chain rate [pairs] [m] [n] [window]
//                                pairs random m x n pairs, prints GCUPS; window >= 0
//                                stores the four traceback words of every 4-step
//                                block within `window` columns of the diagonal
//                                (4-step blocks of 4 KB), else fill only
//
// C5's scoring (pxy 3, go 3, ge 1).  A probe: not part of libnwk.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <string>
#include <type_traits>
#include <vector>

#include "../../multiple-sequence-alignment-openmp-openmpi_amd/csrc/nwk_gotoh_planes.h"

using namespace gotoh_bits;
using C5 = Cfg<3, 1, 3>;
constexpr int kGO = 3;
constexpr int NQ1 = C5::NQ > 0 ? C5::NQ : 1;
constexpr int kPl = C5::NV + NQ1;  // planes handed down: h then f (11)
constexpr int kPs = 12;            // LDS / granule stride per column / chunk

typedef unsigned long long u64;
typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned gu32;
#define RLX __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT

#define HIPCHK(x)                                                                  \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

struct Pair {
  const unsigned* xp;  // [nb * 64][2] row code planes
  const unsigned* yr;  // [(n >> 5) + 4][2] reversed column chunks (gotoh_gpu.hip)
  u64* hand;           // [nb][nw][kPs] granules of each band's last row
  long long* out;      // sum of v over column n, all rows (atomic)
  unsigned* mat;       // (STORE) [nb][nblk][1024] traceback words, 4-step blocks
  int m, n, nb, nw;    // nw = (n >> 5) + 1 chunks of 32 columns
  int w, nblk;         // (STORE) window: steps within w columns of the diagonal j = i n / m
};

__device__ __forceinline__ u64 opaque_zero() {
  u64 z = 0;
  asm volatile("" : "+v"(z));
  return z;
}

template <bool CHECK, bool STORE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4, 4))) void gotoh_chain(
    const Pair* pairs, const int2* tasks, int ntasks, unsigned* counter, unsigned* err, unsigned epoch,
    unsigned* sink) {
  __shared__ __attribute__((aligned(16))) unsigned cons_all[4][32 * kPs];
  __shared__ __attribute__((aligned(16))) unsigned ring_all[4][64 * kPs];
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  unsigned* cons = cons_all[wid];
  unsigned* ring = ring_all[wid];
  unsigned sk = 0;
  for (;;) {
    unsigned tk = 0;
    if (lane == 0) tk = atomicAdd(counter, 1u);
    tk = __builtin_amdgcn_readfirstlane(tk);
    if (tk >= (unsigned)ntasks) break;
    if (__builtin_amdgcn_readfirstlane(__hip_atomic_load((gu32*)err, RLX)) != 0u) break;
    const int2 task = tasks[tk];
    const Pair P = pairs[task.x];
    const int band = task.y;
    const int R0 = band * 2048;
    const unsigned x0 = P.xp[2 * (band * 64 + lane)], x1 = P.xp[2 * (band * 64 + lane) + 1];
    const u64* gin = P.hand + ((size_t)(band > 0 ? band - 1 : 0) * P.nw) * kPs;
    u64* gout = P.hand + ((size_t)band * P.nw) * kPs;
    const bool to_below = band + 1 < P.nb;
    const int kmax = P.n >> 5;  // last chunk holding a real column
    uint32_t v[C5::NV], e[NQ1], h[C5::NV], f[NQ1];
    const uint32_t row1 = (band == 0 && lane == 0) ? 1u : 0u;  // v(1, 0) = -go
#pragma unroll
    for (int p = 0; p < C5::NV; ++p) {
      v[p] = p < kGO ? ~row1 : 0u;
      h[p] = 0u;
    }
#pragma unroll
    for (int q = 0; q < NQ1; ++q) e[q] = f[q] = ~0u;
    const int nsteps = P.n + 2048 + 32;
    // (STORE) the band's stored 4-step blocks: its diagonal cells lie at steps
    // R0 n / m .. + 2048 (1 + n / m); keep w columns either side
    const int blo = STORE ? (int)std::max(0ll, ((long long)R0 * P.n / P.m - P.w) >> 2) : 0;
    // block layout: word w of step s at w * 256 + (s & 2) * 64 + 2 lane + (s & 1)
    unsigned* mb = STORE ? P.mat + (size_t)band * P.nblk * 1024 + lane * 2 : nullptr;
    unsigned dq[4][2];
    long long acc = 0;
    bool ok = true;
    for (int s0 = 0; s0 < nsteps && ok; s0 += 32) {
      const int j = s0 >> 5;
      // --- the row above for lane 0's columns 32 j .. 32 j + 31 -> cons (bit 31)
      {
        unsigned w = 0;  // lane p < kPl: plane p's word (bit r = column 32 j + r)
        if (band == 0) {  // row 0: h(0, 1) = -go (no plane), h(0, c > 1) = 0 (planes < go), f = +inf
          const unsigned h0 = j == 0 ? ~3u : ~0u;  // columns 0 and 1 cleared in chunk 0
          w = lane < kGO ? h0 : (lane < C5::NV ? 0u : ~0u);
        } else if (j <= kmax) {
          u64 g = lane < kPl ? __hip_atomic_fetch_add((gu64*)(gin + (size_t)j * kPs + lane), opaque_zero(), RLX) : 0;
          const u64 t0 = __builtin_amdgcn_s_memrealtime();
          while (!__all(lane >= kPl || (unsigned)(g >> 32) == epoch)) {
            __builtin_amdgcn_s_sleep(2);
            if (__builtin_amdgcn_s_memrealtime() - t0 > 400000000ull ||
                __builtin_amdgcn_readfirstlane(__hip_atomic_load((gu32*)err, RLX)) != 0u) {
              if (lane == 0) atomicOr(err, 1u);
              ok = false;
              break;
            }
            if (lane < kPl) g = __hip_atomic_fetch_add((gu64*)(gin + (size_t)j * kPs + lane), opaque_zero(), RLX);
          }
          w = (unsigned)g;
        }
        // lane r < 32 writes column 32 j + r's entry: plane p's bit at bit 31
#pragma unroll
        for (int p = 0; p < kPl; ++p) {
          const unsigned wp = (unsigned)__builtin_amdgcn_readlane((int)w, p);
          if (lane < 32) cons[lane * kPs + p] = ((wp >> lane) & 1u) << 31;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
      }
      const int q = j - lane;
      const int qi = q < -1 ? -1 : (q > kmax + 1 ? kmax + 1 : q);
      const unsigned lo0 = P.yr[2 * (qi + 2)], lo1 = P.yr[2 * (qi + 2) + 1];
      const unsigned hi0 = P.yr[2 * (qi + 1)], hi1 = P.yr[2 * (qi + 1) + 1];
      auto seg = [&](auto mask_t) {
        constexpr bool mask = decltype(mask_t)::value;
#pragma unroll 4
        for (int r = 0; r < 32; ++r) {
          const int s = s0 + r;
          const unsigned sh = 31u - (unsigned)r;
          const unsigned y0 = __builtin_amdgcn_alignbit(hi0, lo0, sh);
          const unsigned y1 = __builtin_amdgcn_alignbit(hi1, lo1, sh);
          const uint32_t match = ~((x0 ^ y0) | (x1 ^ y1));
          const uint4 ca = *reinterpret_cast<const uint4*>(cons + r * kPs);
          const uint4 cb = *reinterpret_cast<const uint4*>(cons + r * kPs + 4);
          const uint4 cc = *reinterpret_cast<const uint4*>(cons + r * kPs + 8);
          const unsigned inj[12] = {ca.x, ca.y, ca.z, ca.w, cb.x, cb.y, cb.z, cb.w, cc.x, cc.y, cc.z, cc.w};
          uint32_t U[C5::NV], fU[NQ1];
#pragma unroll
          for (int p = 0; p < C5::NV; ++p) {
            const unsigned T = (unsigned)__builtin_amdgcn_update_dpp((int)inj[p], (int)h[p], 0x138, 0xf, 0xf, false);
            U[p] = __builtin_amdgcn_alignbit(h[p], T, 31);
          }
#pragma unroll
          for (int p = 0; p < NQ1; ++p) {
            const unsigned T =
                (unsigned)__builtin_amdgcn_update_dpp((int)inj[C5::NV + p], (int)f[p], 0x138, 0xf, 0xf, false);
            fU[p] = __builtin_amdgcn_alignbit(f[p], T, 31);
          }
          uint32_t D, Fs, Ee, Fe, vn[C5::NV], en[NQ1];
          step<C5>(match, v, e, U, fU, vn, en, h, f, D, Fs, Ee, Fe);
#pragma unroll
          for (int p = 0; p < C5::NV; ++p) v[p] = vn[p];
#pragma unroll
          for (int qq = 0; qq < NQ1; ++qq) e[qq] = en[qq];
          if constexpr (mask) {  // columns <= 0 keep the left border
            const int lim = s - 32 * lane;
            const uint32_t M = lim <= 0 ? ~0u : (lim >= 32 ? 0u : ~((1u << lim) - 1u));
#pragma unroll
            for (int p = 0; p < C5::NV; ++p) v[p] = (v[p] & ~M) | ((p < kGO ? ~row1 : 0u) & M);
#pragma unroll
            for (int qq = 0; qq < NQ1; ++qq) e[qq] |= M;
          }
          if (to_below && lane == 63) {  // the band's last row at column s - 2047
            unsigned* en_ = ring + ((s - 2047) & 63) * kPs;
            *reinterpret_cast<uint4*>(en_) = make_uint4(h[0], h[1], h[2], h[3]);
            *reinterpret_cast<uint4*>(en_ + 4) = make_uint4(h[4], h[5], h[6], h[7]);
            *reinterpret_cast<uint4*>(en_ + 8) = make_uint4(f[0], f[1], f[2], 0u);
          }
          if constexpr (CHECK) {
            const int b = s - P.n - 32 * lane;
            if (b >= 0 && b < 32 && R0 + 32 * lane + b < P.m) {
              int vv = C5::VLO;
#pragma unroll
              for (int p = 0; p < C5::NV; ++p) vv += (int)((v[p] >> b) & 1u);
              acc += vv;
            }
          }
          sk ^= D;
          if constexpr (STORE) {  // four words per lane and step; every 2 steps one 8-byte
                                  // store per word, 512 B contiguous across the wave
            dq[0][r & 1] = D;
            dq[1][r & 1] = Fs;
            dq[2][r & 1] = Ee;
            dq[3][r & 1] = Fe;
            if ((r & 1) == 1) {
              const int rel = (s >> 2) - blo;
              if ((unsigned)rel < (unsigned)P.nblk) {
                typedef unsigned u2 __attribute__((ext_vector_type(2)));
#pragma unroll
                for (int w4 = 0; w4 < 4; ++w4)
                  __builtin_nontemporal_store(u2{dq[w4][0], dq[w4][1]},
                                              reinterpret_cast<u2*>(mb + (size_t)rel * 1024 + w4 * 256 + (s & 2) * 64));
              }
            }
          }
        }
      };
      if (s0 < 2048 + 32) seg(std::true_type{});
      else seg(std::false_type{});
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
        if (lane < kPl) __hip_atomic_store((gu64*)(gout + (size_t)k * kPs + lane), ((u64)epoch << 32) | word, RLX);
      }
    }
    if (CHECK && ok) {
      for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
      if (lane == 0) atomicAdd((unsigned long long*)P.out, (unsigned long long)acc);
    }
  }
  sink[(blockIdx.x * 4 + wid) * 64 + lane] = sk;
}

// Device walk (probe): one wave per pair walks nwo_pair_affine's traceback
// over the stored words.  Tiles of 64 steps x 2 row-lanes (t0 - 1, t0) of one
// band are staged in LDS by the whole wave (lane L: step s_hi - L, 8 loads),
// then every lane runs the same (uniform) walk over the tile; lane 0 writes
// the moves ('D', 'U', 'L' from the end) and the walk's last cell.
__global__ __launch_bounds__(64) void gotoh_walk(const Pair* pairs, int np, char* moves, int* nmoves, int2* ends,
                                                 unsigned* err) {
  __shared__ unsigned tile[4][2][64];
  const int pi = blockIdx.x;
  if (pi >= np) return;
  const int lane = threadIdx.x;
  const Pair P = pairs[pi];
  char* mv = moves + (size_t)pi * (P.m + P.n);
  int i = P.m, j = P.n, st = 0, k = 0;
  int tb = -1, t0 = -1, shi = -1;  // the staged tile
  long long tblo = 0;                // its band's first stored block
  while (i > 0 && j > 0) {
    const int r = i - 1, band = r >> 11, t = (r & 2047) >> 5, b = r & 31, s = j + 32 * t + b;
    if (band != tb || (t != t0 && t != t0 - 1) || s > shi || s < shi - 63) {
      tb = band;
      t0 = t;
      shi = s;
      const long long blo = std::max(0ll, ((long long)band * 2048 * P.n / P.m - P.w) >> 2);
      tblo = blo;
      const int ss = shi - lane;
      const long long rel = ss >= 0 ? (ss >> 2) - blo : -1;
      const bool in = rel >= 0 && rel < P.nblk;
#pragma unroll
      for (int w = 0; w < 4; ++w)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int tl = t0 - 1 + h;
          unsigned val = 0;
          if (in && tl >= 0)
            val = P.mat[((size_t)band * P.nblk + rel) * 1024 + w * 256 + (ss & 2) * 64 + 2 * tl + (ss & 1)];
          tile[w][h][lane] = val;
        }
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __syncthreads();
    }
    {  // a cell outside the stored blocks (the path left the window) fails the walk
      const long long rel0 = (s >> 2) - tblo;
      if (rel0 < 0 || rel0 >= P.nblk) {
        if (lane == 0) atomicOr(err, 2u);
        break;
      }
    }
    const int h = t == t0 ? 1 : 0, q = shi - s;
    const unsigned c = ((tile[0][h][q] >> b) & 1u) | ((tile[1][h][q] >> b) & 1u) << 1 |
                       ((tile[2][h][q] >> b) & 1u) << 2 | ((tile[3][h][q] >> b) & 1u) << 3;
    char m;
    if (st == 0 && (c & 1u)) {
      m = 'D';
      --i;
      --j;
    } else {
      if (st == 0) st = (c & 2u) ? 1 : 2;
      if (st == 1) {
        st = (c & 8u) ? 1 : 0;
        m = 'U';
        --i;
      } else {
        st = (c & 4u) ? 2 : 0;
        m = 'L';
        --j;
      }
    }
    if (lane == 0) mv[k] = m;
    ++k;
  }
  if (lane == 0) {
    nmoves[pi] = k;
    ends[pi] = make_int2(i, j);
  }
}

static int code(char c) { return c == 'A' ? 0 : c == 'C' ? 1 : c == 'G' ? 2 : 3; }

struct HostPair {
  std::vector<unsigned> xp, yr;
  int m, n, nb;
};

static HostPair build_pair(const std::string& x, const std::string& y) {
  HostPair H;
  H.m = (int)x.size();
  H.n = (int)y.size();
  H.nb = (H.m + 2047) / 2048;
  for (int t = 0; t < 64 * H.nb; ++t) {
    unsigned p0 = 0, p1 = 0;
    for (int b = 0; b < 32; ++b) {
      const int i = 32 * t + b;
      const int c = i < H.m ? code(x[i]) : 0;
      p0 |= (unsigned)(c & 1) << b;
      p1 |= (unsigned)(c >> 1) << b;
    }
    H.xp.push_back(p0);
    H.xp.push_back(p1);
  }
  const int nq = (H.n >> 5) + 1;
  for (int q = -2; q <= nq; ++q) {
    unsigned w0 = 0, w1 = 0;
    for (int r = 0; r < 32; ++r) {
      const int col = 32 * q + r;
      const int c = (col >= 1 && col <= H.n) ? code(y[col - 1]) : 0;
      w0 |= (unsigned)(c & 1) << (31 - r);
      w1 |= (unsigned)(c >> 1) << (31 - r);
    }
    H.yr.push_back(w0);
    H.yr.push_back(w1);
  }
  return H;
}

// uploads `hp` (shared device copies for identical pairs when `same`), runs
// `reps` timed launches after one warm-up; returns ms per launch
struct Walks {
  std::vector<std::string> moves;  // from the end of the alignment
  std::vector<int> n;
  std::vector<int2> end;
  float ms = 0;
};

static double run(const std::vector<HostPair>& hp, bool check, int reps, std::vector<long long>& out, bool same,
                  int win = -1, std::vector<std::vector<unsigned>>* mats = nullptr, std::vector<int>* nblks = nullptr,
                  Walks* walks = nullptr) {
  const int np = (int)hp.size();
  std::vector<Pair> P(np);
  std::vector<void*> allocs;
  int maxb = 0;
  for (int i = 0; i < np; ++i) {
    const HostPair& H = hp[i];
    unsigned *dx, *dy;
    if (!same || i == 0) {
      HIPCHK(hipMalloc(&dx, H.xp.size() * 4));
      HIPCHK(hipMalloc(&dy, H.yr.size() * 4));
      HIPCHK(hipMemcpy(dx, H.xp.data(), H.xp.size() * 4, hipMemcpyHostToDevice));
      HIPCHK(hipMemcpy(dy, H.yr.data(), H.yr.size() * 4, hipMemcpyHostToDevice));
      allocs.push_back(dx);
      allocs.push_back(dy);
    } else {
      dx = const_cast<unsigned*>(P[0].xp);
      dy = const_cast<unsigned*>(P[0].yr);
    }
    const int nw = (H.n >> 5) + 1;
    u64* hand;
    HIPCHK(hipMalloc(&hand, (size_t)H.nb * nw * kPs * 8));
    HIPCHK(hipMemset(hand, 0, (size_t)H.nb * nw * kPs * 8));
    allocs.push_back(hand);
    unsigned* mat = nullptr;
    int nblk = 0;
    if (win >= 0) {  // blocks covering 2048 (1 + n / m) + 2 win steps, + 2 for rounding
      nblk = (int)((2048ll * (H.m + H.n) / H.m + 2ll * win) / 4) + 2;
      HIPCHK(hipMalloc(&mat, (size_t)H.nb * nblk * 1024 * 4));
      allocs.push_back(mat);
    }
    P[i] = Pair{dx, dy, hand, nullptr, mat, H.m, H.n, H.nb, nw, win, nblk};
    maxb = std::max(maxb, H.nb);
  }
  long long* dout;
  HIPCHK(hipMalloc(&dout, 8 * np));
  for (int i = 0; i < np; ++i) P[i].out = dout + i;
  std::vector<int2> tk;  // band-major: every band's producer is dequeued before it
  for (int b = 0; b < maxb; ++b)
    for (int i = 0; i < np; ++i)
      if (b < hp[i].nb) tk.push_back(make_int2(i, b));
  Pair* dp;
  int2* dt;
  unsigned *dctr, *derr, *dsink;
  HIPCHK(hipMalloc(&dp, sizeof(Pair) * np));
  HIPCHK(hipMemcpy(dp, P.data(), sizeof(Pair) * np, hipMemcpyHostToDevice));
  HIPCHK(hipMalloc(&dt, sizeof(int2) * tk.size()));
  HIPCHK(hipMemcpy(dt, tk.data(), sizeof(int2) * tk.size(), hipMemcpyHostToDevice));
  HIPCHK(hipMalloc(&dctr, 4));
  HIPCHK(hipMalloc(&derr, 4));
  HIPCHK(hipMemset(derr, 0, 4));
  int dev = 0, cus = 0;
  HIPCHK(hipGetDevice(&dev));
  HIPCHK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  const int grid = cus * 4;  // 4 waves per SIMD, persistent
  HIPCHK(hipMalloc(&dsink, (size_t)grid * 256 * 4));
  hipEvent_t a, b;
  HIPCHK(hipEventCreate(&a));
  HIPCHK(hipEventCreate(&b));
  double ms_sum = 0;
  for (int r = 0; r <= reps; ++r) {  // launch 0 is the warm-up; every launch has a fresh epoch
    HIPCHK(hipMemset(dctr, 0, 4));
    HIPCHK(hipMemset(dout, 0, 8 * np));
    HIPCHK(hipEventRecord(a));
    if (check && win >= 0) hipLaunchKernelGGL((gotoh_chain<true, true>), dim3(grid), dim3(256), 0, 0, dp, dt, (int)tk.size(), dctr, derr, 1u + r, dsink);
    else if (check) hipLaunchKernelGGL((gotoh_chain<true, false>), dim3(grid), dim3(256), 0, 0, dp, dt, (int)tk.size(), dctr, derr, 1u + r, dsink);
    else if (win >= 0) hipLaunchKernelGGL((gotoh_chain<false, true>), dim3(grid), dim3(256), 0, 0, dp, dt, (int)tk.size(), dctr, derr, 1u + r, dsink);
    else hipLaunchKernelGGL((gotoh_chain<false, false>), dim3(grid), dim3(256), 0, 0, dp, dt, (int)tk.size(), dctr, derr, 1u + r, dsink);
    HIPCHK(hipEventRecord(b));
    HIPCHK(hipEventSynchronize(b));
    HIPCHK(hipGetLastError());
    float ms = 0;
    HIPCHK(hipEventElapsedTime(&ms, a, b));
    if (r > 0) ms_sum += ms;
  }
  unsigned herr = 0;
  HIPCHK(hipMemcpy(&herr, derr, 4, hipMemcpyDeviceToHost));
  if (herr) { std::fprintf(stderr, "gotoh_chain: wait timed out (err %u)\n", herr); std::exit(4); }
  out.resize(np);
  HIPCHK(hipMemcpy(out.data(), dout, 8 * np, hipMemcpyDeviceToHost));
  if (walks && win >= 0) {  // device walk over the stored words, one wave per pair
    char* dmv;
    int* dnm;
    int2* den;
    size_t tot = 0;
    for (const HostPair& H : hp) tot += (size_t)H.m + H.n;
    HIPCHK(hipMalloc(&dmv, tot));
    HIPCHK(hipMalloc(&dnm, 4 * np));
    HIPCHK(hipMalloc(&den, 8 * np));
    std::vector<size_t> off(np + 1, 0);
    for (int i = 0; i < np; ++i) off[i + 1] = off[i] + (size_t)hp[i].m + hp[i].n;
    // (the kernel indexes moves by pi * (m + n): equal-size pairs only, checked here)
    for (int i = 0; i < np; ++i)
      if (off[i] != (size_t)i * ((size_t)hp[i].m + hp[i].n)) { std::fprintf(stderr, "dtrace: pairs must share m + n\n"); std::exit(2); }
    HIPCHK(hipEventRecord(a));
    hipLaunchKernelGGL(gotoh_walk, dim3(np), dim3(64), 0, 0, dp, np, dmv, dnm, den, derr);
    HIPCHK(hipEventRecord(b));
    HIPCHK(hipEventSynchronize(b));
    HIPCHK(hipGetLastError());
    float wms = 0;
    HIPCHK(hipEventElapsedTime(&wms, a, b));
    walks->ms = wms;
    HIPCHK(hipMemcpy(&herr, derr, 4, hipMemcpyDeviceToHost));
    if (herr) { std::fprintf(stderr, "gotoh_walk: left the stored window (err %u)\n", herr); std::exit(5); }
    std::vector<char> mv(tot);
    walks->n.resize(np);
    walks->end.resize(np);
    HIPCHK(hipMemcpy(mv.data(), dmv, tot, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(walks->n.data(), dnm, 4 * np, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(walks->end.data(), den, 8 * np, hipMemcpyDeviceToHost));
    walks->moves.resize(np);
    for (int i = 0; i < np; ++i) walks->moves[i].assign(mv.data() + off[i], mv.data() + off[i] + walks->n[i]);
    (void)hipFree(dmv); (void)hipFree(dnm); (void)hipFree(den);
  }
  if (mats && win >= 0) {  // the stored words, per pair
    mats->resize(np);
    nblks->resize(np);
    for (int i = 0; i < np; ++i) {
      (*nblks)[i] = P[i].nblk;
      (*mats)[i].resize((size_t)hp[i].nb * P[i].nblk * 1024);
      HIPCHK(hipMemcpy((*mats)[i].data(), P[i].mat, (*mats)[i].size() * 4, hipMemcpyDeviceToHost));
    }
  }
  for (void* p : allocs) (void)hipFree(p);
  (void)hipFree(dout); (void)hipFree(dp); (void)hipFree(dt); (void)hipFree(dctr); (void)hipFree(derr); (void)hipFree(dsink);
  return reps > 0 ? ms_sum / reps : 0.0;
}

// nwo_pair_affine's walk (oracle/nw_oracle.c:240-270) over the words the GPU
// stored: cell (i, j) is row r = i - 1 of band r / 2048 (lane t, bit b), step
// s = j + 32 t + b, word w at block (s >> 2) - blo, w * 256 + (s & 2) * 64 + 2 t + (s & 1)
static void walk_stored(const std::string& x, const std::string& y, const std::vector<unsigned>& mat, int nblk,
                        int win, std::string& a1, std::string& a2) {
  const int m = (int)x.size(), n = (int)y.size(), l = m + n;
  auto bits = [&](int i, int j) {
    const int r = i - 1, band = r / 2048, t = (r % 2048) / 32, b = r % 32, s = j + 32 * t + b;
    const long long blo = std::max(0ll, ((long long)band * 2048 * n / m - win) >> 2);
    const long long rel = (s >> 2) - blo;
    if (rel < 0 || rel >= nblk) { std::fprintf(stderr, "walk left the stored blocks\n"); std::exit(5); }
    const size_t base = ((size_t)band * nblk + rel) * 1024 + (s & 2) * 64 + 2 * t + (s & 1);
    unsigned o = 0;
    for (int w = 0; w < 4; ++w) o |= ((mat[base + w * 256] >> b) & 1u) << w;
    return o;  // bit 0 D, 1 F-source, 2 E-extend, 3 F-extend
  };
  std::string xa(l + 1, ' '), ya(l + 1, ' ');
  int i = m, j = n, xp = l, yp = l, st = 0;
  while (!(i == 0 || j == 0)) {
    const unsigned c = bits(i, j);
    if (st == 0) {
      if (c & 1u) { xa[xp--] = x[i - 1]; ya[yp--] = y[j - 1]; --i; --j; continue; }
      st = (c & 2u) ? 1 : 2;
    }
    if (st == 1) { st = (c & 8u) ? 1 : 0; xa[xp--] = x[i - 1]; ya[yp--] = '_'; --i; }
    else { st = (c & 4u) ? 2 : 0; xa[xp--] = '_'; ya[yp--] = y[j - 1]; --j; }
  }
  while (xp > 0) xa[xp--] = i > 0 ? x[--i] : '_';
  while (yp > 0) ya[yp--] = j > 0 ? y[--j] : '_';
  int id = 1;
  for (int a = l; a >= 1; --a)
    if (ya[a] == '_' && xa[a] == '_') { id = a + 1; break; }
  a1 = xa.substr(id);
  a2 = ya.substr(id);
}

int main(int argc, char** argv) {
  const std::string mode = argc > 1 ? argv[1] : "rate";
  std::vector<HostPair> hp;
  std::vector<long long> sums;
  if (mode == "dtrace" || mode == "dtrate") {
    // dtrace: stdin pairs (equal m + n), every step stored, walked on the device
    // dtrate [pairs] [m] [n] [window]: C5-shaped random pairs, fill + store, then
    // the device walk; prints both times
    std::vector<std::pair<std::string, std::string>> seqs;
    int win;
    if (mode == "dtrace") {
      std::string x, y;
      int maxlen = 0;
      while (std::cin >> x >> y) {
        hp.push_back(build_pair(x, y));
        seqs.emplace_back(x, y);
        maxlen = std::max(maxlen, (int)y.size());
      }
      if (hp.empty()) return 2;
      win = maxlen + 2048;
    } else {
      const int np = argc > 2 ? std::atoi(argv[2]) : 16;
      const int m = argc > 3 ? std::atoi(argv[3]) : 200000;
      const int n = argc > 4 ? std::atoi(argv[4]) : 200000;
      win = argc > 5 ? std::atoi(argv[5]) : 8192;
      if (np < 1 || np > 512 || m < 2048 || m > 1 << 20 || n < 32 || n > 1 << 20 || win < 0) return 2;
      srand(3);
      for (int q = 0; q < np; ++q) {  // related pairs: a mutated copy (the path stays near the diagonal)
        std::string x(m, 'A'), y;
        for (auto& c : x) c = "ACGT"[rand() & 3];
        y = x.substr(0, std::min(m, n));
        for (auto& c : y) if ((rand() & 7) == 0) c = "ACGT"[rand() & 3];
        while ((int)y.size() < n) y.push_back("ACGT"[rand() & 3]);
        hp.push_back(build_pair(x, y));
      }
    }
    Walks wk;
    const double ms = run(hp, mode == "dtrace", mode == "dtrace" ? 0 : 1, sums, false, win, nullptr, nullptr, &wk);
    if (mode == "dtrate") {
      long long mv = 0;
      for (int v : wk.n) mv += v;
      std::printf("{\"pairs\": %d, \"m\": %d, \"n\": %d, \"window\": %d, \"fill_store_ms\": %.2f, \"walk_ms\": %.2f, "
                  "\"moves\": %lld, \"ns_per_move_per_pair\": %.1f}\n",
                  (int)hp.size(), hp[0].m, hp[0].n, win, ms, wk.ms, mv, wk.ms * 1e6 / (mv / (double)hp.size()));
      return 0;
    }
    for (size_t q = 0; q < hp.size(); ++q) {
      const std::string &x = seqs[q].first, &y = seqs[q].second;
      const int m = (int)x.size(), n = (int)y.size(), l = m + n;
      std::string xa(l + 1, ' '), ya(l + 1, ' ');
      int i = m, j = n, xp = l, yp = l;
      for (char c : wk.moves[q]) {
        if (c == 'D') { xa[xp--] = x[i - 1]; ya[yp--] = y[j - 1]; --i; --j; }
        else if (c == 'U') { xa[xp--] = x[i - 1]; ya[yp--] = '_'; --i; }
        else { xa[xp--] = '_'; ya[yp--] = y[j - 1]; --j; }
      }
      if (i != wk.end[q].x || j != wk.end[q].y) { std::fprintf(stderr, "dtrace: end cell mismatch\n"); return 6; }
      while (xp > 0) xa[xp--] = i > 0 ? x[--i] : '_';
      while (yp > 0) ya[yp--] = j > 0 ? y[--j] : '_';
      int id = 1;
      for (int a = l; a >= 1; --a)
        if (ya[a] == '_' && xa[a] == '_') { id = a + 1; break; }
      const long long H = kGO - sums[q] + (long long)(m + n);
      std::printf("%lld %s %s\n", H, xa.substr(id).empty() ? "-" : xa.substr(id).c_str(),
                  ya.substr(id).empty() ? "-" : ya.substr(id).c_str());
    }
    return 0;
  }
  if (mode == "check" || mode == "trace") {
    std::vector<std::pair<std::string, std::string>> seqs;
    std::string x, y;
    int maxlen = 0;
    while (std::cin >> x >> y) {
      if (x.empty() || y.empty() || x.size() > (1u << 20) || y.size() > (1u << 20)) { std::fprintf(stderr, "bad pair\n"); return 2; }
      hp.push_back(build_pair(x, y));
      seqs.emplace_back(x, y);
      maxlen = std::max(maxlen, (int)y.size());
    }
    // trace: every step stored (window wider than any pair), walked on the host
    const int win = mode == "trace" ? maxlen + 2048 : -1;
    std::vector<std::vector<unsigned>> mats;
    std::vector<int> nblks;
    run(hp, true, 0, sums, false, win, &mats, &nblks);
    for (size_t i = 0; i < hp.size(); ++i) {  // H = G(0, n) - sum v + (m + n) ge
      const long long H = kGO - sums[i] + (long long)(hp[i].m + hp[i].n);
      if (mode == "check") { std::printf("%lld\n", H); continue; }
      std::string a1, a2;
      walk_stored(seqs[i].first, seqs[i].second, mats[i], nblks[i], win, a1, a2);
      std::printf("%lld %s %s\n", H, a1.empty() ? "-" : a1.c_str(), a2.empty() ? "-" : a2.c_str());
    }
    return 0;
  }
  const int np = argc > 2 ? std::atoi(argv[2]) : 42;
  const int m = argc > 3 ? std::atoi(argv[3]) : 200000;
  const int n = argc > 4 ? std::atoi(argv[4]) : 200000;
  const int win = argc > 5 ? std::atoi(argv[5]) : -1;  // >= 0: store the traceback words within win columns
  if (np < 1 || np > 4096 || m < 1 || m > 1 << 20 || n < 32 || n > 1 << 20) { std::fprintf(stderr, "bad size\n"); return 2; }
  srand(1);
  std::string x(m, 'A'), y(n, 'A');
  for (auto& c : x) c = "ACGT"[rand() & 3];
  for (auto& c : y) c = "ACGT"[rand() & 3];
  const HostPair H = build_pair(x, y);
  for (int i = 0; i < np; ++i) hp.push_back(H);
  const double ms = run(hp, false, 2, sums, true, win);
  const double cells = (double)np * m * n;
  std::printf("{\"pairs\": %d, \"m\": %d, \"n\": %d, \"bands\": %d, \"window\": %d, \"ms\": %.2f, \"gcups\": %.1f}\n", np, m, n,
              H.nb, win, ms, cells / ms / 1e6);
  return 0;
}
