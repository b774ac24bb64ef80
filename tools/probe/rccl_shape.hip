// rccl_shape.hip -- a kernel with the resource shape of RCCL's collective
// kernel on gfx950 (ncclDevKernel_Generic_*: 248-256 VGPRs, 37,664 B of LDS,
// 256 threads per block; read from librccl's gfx950 code object notes), for
// tools/overlap_probe.py: can such a block start while a persistent fill
// launch (4 waves/SIMD x 128 VGPRs on every CU) runs, and how late?
//   rs_init()            side stream + host-mapped timestamps
//   rs_launch(blocks, spin)  launch on the side stream, return at once (spin < 0: a one-wave tiny kernel)
//   rs_poll(out[4])      {first block's start, last block's end (s_memrealtime,
//                        100 MHz), blocks started, blocks ended}
//   rs_sync()            wait for the side stream
//   rs_now()             the device clock now (one tiny launch, synchronous)
#include <hip/hip_runtime.h>

namespace {
hipStream_t g_stream = nullptr;
unsigned long long* g_ts = nullptr;  // host-mapped: [0] min start, [1] max end, [2] started, [3] ended

__global__ __launch_bounds__(256) void rccl_shape(unsigned long long* ts, int spin) {
  __shared__ unsigned lds[37664 / 4];
  asm volatile("" ::: "v255");  // allocate 256 VGPRs, as ncclDevKernel_Generic does
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    atomicMin(ts, t0);
    atomicAdd(ts + 2, 1ull);
    __threadfence_system();
  }
  for (int q = threadIdx.x; q < 37664 / 4; q += 256) lds[q] = q;
  __syncthreads();
  unsigned acc = 0;
  while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)spin) acc += lds[(acc + threadIdx.x) % (37664 / 4)];
  if (threadIdx.x == 0) {
    atomicMax(ts + 1, __builtin_amdgcn_s_memrealtime() + (acc == 0xffffffffu ? 1 : 0));
    atomicAdd(ts + 3, 1ull);
    __threadfence_system();
  }
}

// one wave, few registers: does anything at all start on a free CU?
__global__ __launch_bounds__(64) void tiny(unsigned long long* ts) {
  if (threadIdx.x == 0) {
    atomicMin(ts, __builtin_amdgcn_s_memrealtime());
    atomicAdd(ts + 2, 1ull);
    atomicMax(ts + 1, __builtin_amdgcn_s_memrealtime());
    atomicAdd(ts + 3, 1ull);
    __threadfence_system();
  }
}

__global__ void clock_now(unsigned long long* out) { *out = __builtin_amdgcn_s_memrealtime(); }

// where a block runs: {XCC_ID, HW_ID} (gfx9 HW_ID: wave [3:0], simd [5:4], cu [11:8], sh [12], se [15:13])
__global__ void where(unsigned* out) {
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = __builtin_amdgcn_s_getreg((20 << 0) | (0 << 6) | (31 << 11));  // HW_REG_XCC_ID
    out[2 * blockIdx.x + 1] = __builtin_amdgcn_s_getreg((4 << 0) | (0 << 6) | (31 << 11));  // HW_REG_HW_ID
  }
}
}  // namespace

// mask[nwords]: launches `blocks` one-wave blocks of `where` on a stream with
// that CU mask and returns their {XCC_ID, HW_ID} pairs in out[2 blocks]
extern "C" int rs_where(const unsigned* mask, int nwords, int blocks, unsigned* out) {
  hipStream_t s;
  if (hipExtStreamCreateWithCUMask(&s, (uint32_t)nwords, mask) != hipSuccess) return -1;
  unsigned* d = nullptr;
  if (hipMalloc(&d, 8 * (size_t)blocks) != hipSuccess) return -2;
  hipLaunchKernelGGL(where, dim3(blocks), dim3(64), 0, s, d);
  if (hipStreamSynchronize(s) != hipSuccess) return -3;
  (void)hipMemcpy(out, d, 8 * (size_t)blocks, hipMemcpyDeviceToHost);
  (void)hipFree(d);
  (void)hipStreamDestroy(s);
  return 0;
}

extern "C" int rs_init() {
  if (hipStreamCreateWithFlags(&g_stream, hipStreamNonBlocking) != hipSuccess) return -1;
  if (hipHostMalloc((void**)&g_ts, 64, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return -2;
  return 0;
}

extern "C" int rs_launch(int blocks, int spin_ticks) {
  g_ts[0] = ~0ull;
  g_ts[1] = g_ts[2] = g_ts[3] = 0;
  void* d = nullptr;
  if (hipHostGetDevicePointer(&d, g_ts, 0) != hipSuccess) return -1;
  if (spin_ticks < 0) hipLaunchKernelGGL(tiny, dim3(blocks), dim3(64), 0, g_stream, (unsigned long long*)d);
  else hipLaunchKernelGGL(rccl_shape, dim3(blocks), dim3(256), 0, g_stream, (unsigned long long*)d, spin_ticks);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

extern "C" void rs_poll(unsigned long long* out) {
  for (int q = 0; q < 4; ++q) out[q] = __atomic_load_n(g_ts + q, __ATOMIC_ACQUIRE);
}

extern "C" int rs_sync() { return hipStreamSynchronize(g_stream) == hipSuccess ? 0 : -1; }

extern "C" unsigned long long rs_now() {
  void* d = nullptr;
  unsigned long long* h = nullptr;
  if (hipHostMalloc((void**)&h, 8, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) return 0;
  (void)hipHostGetDevicePointer(&d, h, 0);
  hipLaunchKernelGGL(clock_now, dim3(1), dim3(1), 0, g_stream, (unsigned long long*)d);
  (void)hipStreamSynchronize(g_stream);
  const unsigned long long v = *h;
  (void)hipHostFree(h);
  return v;
}
