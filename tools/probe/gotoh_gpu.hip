// gotoh_gpu.hip -- chain-free rate of the bit-sliced Gotoh step
// (gotoh_bits.h) on gfx950, in nw_align_bits' anti-diagonal band layout.
//
// One wave = one independent 2048-row band of one pair (no band above: row 0
// is the border), n columns: bit b of lane t is row 32 t + b + 1, and at step
// s it is at column s - 32 t - b.  Left inputs (v, e) stay in the bit; upper
// inputs (h, f) come from bit b - 1 of the previous step (bit 0: lane t - 1's
// bit 31 over DPP, lane 0: the border row).  Columns <= 0 are held at the
// left border (v(i, 0), e = +inf).
//
//   gotoh_gpu check < pairs      rows of stdin "x y" (|x| <= 2048): prints H[m][n]
//                                per pair (tests/test_gotoh_bits_probe.py checks
//                                it against the oracle)
//   gotoh_gpu rate [waves] [n] [store] [occ]
//                                random pairs, 2048 x n cells per wave, prints
//                                GCUPS; store = 1 writes the four traceback words
//                                of every step (0.5 B per cell, no window)
//
// C5's scoring only (pxy 3, go 3, ge 1).
#include <hip/hip_runtime.h>

#include <chrono>
#include <type_traits>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <iostream>
#include <string>
#include <vector>

#include "../../multiple-sequence-alignment-openmp-openmpi_amd/csrc/nwk_gotoh_planes.h"

using namespace gotoh_bits;
using C5 = Cfg<3, 1, 3>;
constexpr int kGO = 3;
constexpr int NQ1 = C5::NQ > 0 ? C5::NQ : 1;

#define HIPCHK(x)                                                                  \
  do {                                                                             \
    hipError_t e_ = (x);                                                           \
    if (e_ != hipSuccess) {                                                        \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                \
    }                                                                              \
  } while (0)

// per task: x code planes (64 lanes x 2 words), y reversed chunk words
// yr[2 * (q + 2)] .. (plane 0, 1) for chunks q = -2 .. nq (bit 31 - r of chunk
// q = code of column 32 q + r; columns outside 1..n are code 0)
struct Task {
  const unsigned* xp;  // [64][2]
  const unsigned* yr;  // [(nq + 3)][2]
  int m, n;
};

template <bool CHECK, bool STORE, int OCC>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(OCC, OCC))) void gotoh_band(
    const Task* tasks, int ntasks, long long* out, unsigned* sink, unsigned* st) {
  const int lane = threadIdx.x & 63;
  const int wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (wave >= ntasks) return;
  const Task tk = tasks[wave];
  const unsigned x0 = tk.xp[2 * lane], x1 = tk.xp[2 * lane + 1];
  uint32_t v[C5::NV], e[NQ1], h[C5::NV], f[NQ1];
  // every bit starts at a column <= 0: the left border
  const uint32_t row1 = lane == 0 ? 1u : 0u;  // bit 0 of lane 0 is row 1: v(1, 0) = -go
#pragma unroll
  for (int p = 0; p < C5::NV; ++p) {
    v[p] = p < kGO ? ~row1 : 0u;
    h[p] = 0u;
  }
#pragma unroll
  for (int q = 0; q < NQ1; ++q) e[q] = f[q] = ~0u;
  // lane 0's DPP fill-ins: row 0's h (0 past column 1: planes p < go set) and f (+inf)
  uint32_t Th[C5::NV], Tf[NQ1];
#pragma unroll
  for (int p = 0; p < C5::NV; ++p) Th[p] = p < kGO ? 0x80000000u : 0u;
#pragma unroll
  for (int q = 0; q < NQ1; ++q) Tf[q] = 0x80000000u;
  const int nsteps = tk.n + 2048 + 32;  // the last bit (lane 63, bit 31) reaches column n
  long long acc = 0;                     // CHECK: sum of v over column n
  unsigned sk = 0;
  unsigned* stp = st + (size_t)wave * 4 * 64 * 32 + lane;  // (STORE) a 32-step ring per wave
  for (int s0 = 0; s0 < nsteps; s0 += 32) {
    // y window of this 32-step segment: chunks k - t and k - t - 1 (k = s0 / 32)
    const int q = (s0 >> 5) - lane;
    const int qi = q < -1 ? -1 : (q > (tk.n >> 5) + 1 ? (tk.n >> 5) + 1 : q);
    const unsigned lo0 = tk.yr[2 * (qi + 2)], lo1 = tk.yr[2 * (qi + 2) + 1];
    const unsigned hi0 = tk.yr[2 * (qi + 1)], hi1 = tk.yr[2 * (qi + 1) + 1];
    auto seg = [&](auto mask_t) {
    constexpr bool mask = decltype(mask_t)::value;
#pragma unroll 4
    for (int r = 0; r < 32; ++r) {
      const int s = s0 + r;
      const unsigned sh = 31u - (unsigned)r;
      const unsigned y0 = __builtin_amdgcn_alignbit(hi0, lo0, sh);
      const unsigned y1 = __builtin_amdgcn_alignbit(hi1, lo1, sh);
      const uint32_t match = ~((x0 ^ y0) | (x1 ^ y1));
      // upper inputs: h, f of bit b - 1 (previous step); lane 0 bit 0: row 0 at
      // column s: h(0, s) = -go at s = 1, else 0 (columns <= 0 are masked); f = +inf
      // (the DPP leaves lane 0's old value in place: Th / Tf carry the border
      // bit from step to step with no re-initialisation; s = 1, in the masked
      // segments only, clears it for h(0, 1) = -go)
      uint32_t U[C5::NV], fU[NQ1];
#pragma unroll
      for (int p = 0; p < C5::NV; ++p) {
        unsigned old = Th[p];
        if constexpr (mask) old = (p < kGO && s != 1) ? 0x80000000u : 0u;
        Th[p] = (unsigned)__builtin_amdgcn_update_dpp((int)old, (int)h[p], 0x138 /*wave_shr:1*/, 0xf, 0xf, false);
        U[p] = __builtin_amdgcn_alignbit(h[p], Th[p], 31);
      }
#pragma unroll
      for (int p = 0; p < NQ1; ++p) {
        Tf[p] = (unsigned)__builtin_amdgcn_update_dpp((int)Tf[p], (int)f[p], 0x138, 0xf, 0xf, false);
        fU[p] = __builtin_amdgcn_alignbit(f[p], Tf[p], 31);
      }
      uint32_t D, Fs, Ee, Fe, vn[C5::NV], en[NQ1];
      step<C5>(match, v, e, U, fU, vn, en, h, f, D, Fs, Ee, Fe);  // (h, f: their old values are in U, fU)
#pragma unroll
      for (int p = 0; p < C5::NV; ++p) v[p] = vn[p];
#pragma unroll
      for (int qq = 0; qq < NQ1; ++qq) e[qq] = en[qq];
      if constexpr (mask) {  // bits at columns <= 0 (b >= s - 32 t) keep the left border
        const int lim = s - 32 * lane;
        const uint32_t M = lim <= 0 ? ~0u : (lim >= 32 ? 0u : ~((1u << lim) - 1u));
#pragma unroll
        for (int p = 0; p < C5::NV; ++p) v[p] = (v[p] & ~M) | ((p < kGO ? ~row1 : 0u) & M);
#pragma unroll
        for (int qq = 0; qq < NQ1; ++qq) e[qq] |= M;
      }
      if constexpr (CHECK) {  // bit b of lane t is at column n when b = s - n - 32 t
        const int b = s - tk.n - 32 * lane;
        if (b >= 0 && b < 32 && 32 * lane + b < tk.m) {
          int vv = C5::VLO;
#pragma unroll
          for (int p = 0; p < C5::NV; ++p) vv += (int)((v[p] >> b) & 1u);
          acc += vv;
        }
      }
      if constexpr (STORE) {
        unsigned* w = stp + (size_t)(r & 31) * 4 * 64;
        __builtin_nontemporal_store(D, w);
        __builtin_nontemporal_store(Fs, w + 64);
        __builtin_nontemporal_store(Ee, w + 128);
        __builtin_nontemporal_store(Fe, w + 192);
      }
      sk ^= D;
    }
    };
    if (s0 < 2048 + 32) seg(std::true_type{});
    else seg(std::false_type{});
  }
  if constexpr (CHECK) {
    // G(m, n) = G(0, n) - sum_i v(i, n), G(0, n) = go; H = G + (m + n) ge
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
    if (lane == 0) out[wave] = kGO - acc + (long long)(tk.m + tk.n);
  }
  sink[wave * 64 + lane] = sk;
}

static int code(char c) {
  switch (c) {
    case 'A': return 0;
    case 'C': return 1;
    case 'G': return 2;
    default: return 3;
  }
}

struct Host {
  std::vector<unsigned> xp, yr;
  std::vector<Task> tasks;  // pointers are offsets until upload
  std::vector<size_t> xo, yo;
};

static void add_pair(Host& H, const std::string& x, const std::string& y) {
  const int m = (int)x.size(), n = (int)y.size();
  H.xo.push_back(H.xp.size());
  for (int t = 0; t < 64; ++t) {
    unsigned p0 = 0, p1 = 0;
    for (int b = 0; b < 32; ++b) {
      const int i = 32 * t + b;
      // rows past m: a code no column has (never read: 2048-row bands only here)
      const int c = i < m ? code(x[i]) : 0;
      p0 |= (unsigned)(c & 1) << b;
      p1 |= (unsigned)(c >> 1) << b;
    }
    H.xp.push_back(p0);
    H.xp.push_back(p1);
  }
  const int nq = (n >> 5) + 1;
  H.yo.push_back(H.yr.size());
  for (int q = -2; q <= nq; ++q) {
    unsigned w0 = 0, w1 = 0;
    for (int r = 0; r < 32; ++r) {
      const int col = 32 * q + r;  // 1-based column
      const int c = (col >= 1 && col <= n) ? code(y[col - 1]) : 0;
      w0 |= (unsigned)(c & 1) << (31 - r);
      w1 |= (unsigned)(c >> 1) << (31 - r);
    }
    H.yr.push_back(w0);
    H.yr.push_back(w1);
  }
  H.tasks.push_back(Task{nullptr, nullptr, m, n});
}

template <bool CHECK, bool STORE, int OCC = 4>
static double run(Host& H, std::vector<long long>& res, int reps) {
  unsigned *dx, *dy, *dsink, *dst = nullptr;
  Task* dt;
  long long* dout;
  const int nt = (int)H.tasks.size();
  HIPCHK(hipMalloc(&dx, H.xp.size() * 4));
  HIPCHK(hipMalloc(&dy, H.yr.size() * 4));
  HIPCHK(hipMemcpy(dx, H.xp.data(), H.xp.size() * 4, hipMemcpyHostToDevice));
  HIPCHK(hipMemcpy(dy, H.yr.data(), H.yr.size() * 4, hipMemcpyHostToDevice));
  std::vector<Task> t = H.tasks;
  for (int i = 0; i < nt; ++i) {
    t[i].xp = dx + H.xo[i];
    t[i].yr = dy + H.yo[i];
  }
  HIPCHK(hipMalloc(&dt, sizeof(Task) * nt));
  HIPCHK(hipMemcpy(dt, t.data(), sizeof(Task) * nt, hipMemcpyHostToDevice));
  HIPCHK(hipMalloc(&dout, 8 * nt));
  HIPCHK(hipMalloc(&dsink, 4 * 64 * (size_t)nt));
  if (STORE) HIPCHK(hipMalloc(&dst, (size_t)nt * 4 * 64 * 32 * 4));
  const int grid = (nt + 3) / 4;
  hipEvent_t a, b;
  HIPCHK(hipEventCreate(&a));
  HIPCHK(hipEventCreate(&b));
  hipLaunchKernelGGL((gotoh_band<CHECK, STORE, OCC>), dim3(grid), dim3(256), 0, 0, dt, nt, dout, dsink, dst);  // warm-up
  HIPCHK(hipDeviceSynchronize());
  HIPCHK(hipEventRecord(a));
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((gotoh_band<CHECK, STORE, OCC>), dim3(grid), dim3(256), 0, 0, dt, nt, dout, dsink, dst);
  HIPCHK(hipEventRecord(b));
  HIPCHK(hipEventSynchronize(b));
  HIPCHK(hipGetLastError());
  float ms = 0;
  HIPCHK(hipEventElapsedTime(&ms, a, b));
  res.resize(nt);
  HIPCHK(hipMemcpy(res.data(), dout, 8 * nt, hipMemcpyDeviceToHost));
  hipFree(dx); hipFree(dy); hipFree(dt); hipFree(dout); hipFree(dsink);
  if (dst) hipFree(dst);
  return ms / reps;
}

int main(int argc, char** argv) {
  const std::string mode = argc > 1 ? argv[1] : "rate";
  Host H;
  std::vector<long long> res;
  if (mode == "check") {
    std::string x, y;
    while (std::cin >> x >> y) {
      if (x.size() > 2048 || y.empty() || x.empty()) { std::fprintf(stderr, "pair out of range\n"); return 2; }
      add_pair(H, x, y);
    }
    run<true, false>(H, res, 1);
    for (long long v : res) std::printf("%lld\n", v);
    return 0;
  }
  const int waves = argc > 2 ? std::atoi(argv[2]) : 8192;
  const int n = argc > 3 ? std::atoi(argv[3]) : 4096;
  const bool store = argc > 4 && std::atoi(argv[4]) != 0;
  const int occ = argc > 5 ? std::atoi(argv[5]) : 4;  // waves per SIMD the register budget is cut for (4 or 5)
  if (waves < 1 || waves > 65536 || n < 32 || n > 1 << 20) { std::fprintf(stderr, "bad size\n"); return 2; }
  srand(1);
  std::string x(2048, 'A'), y(n, 'A');
  for (auto& c : x) c = "ACGT"[rand() & 3];
  for (auto& c : y) c = "ACGT"[rand() & 3];
  for (int w = 0; w < waves; ++w) add_pair(H, x, y);  // one pair's data, many waves (rate only)
  const double ms = occ == 5 ? (store ? run<false, true, 5>(H, res, 3) : run<false, false, 5>(H, res, 3))
                             : (store ? run<false, true, 4>(H, res, 3) : run<false, false, 4>(H, res, 3));
  const double cells = (double)waves * 2048.0 * n;
  const double steps = (double)n + 2048 + 32;
  std::printf("{\"waves\": %d, \"n\": %d, \"store\": %d, \"occ\": %d, \"ms\": %.3f, \"gcups\": %.1f, \"ns_per_wave_step\": %.2f}\n",
              waves, n, (int)store, occ, ms, cells / ms / 1e6, ms * 1e6 / steps);
  return 0;
}
