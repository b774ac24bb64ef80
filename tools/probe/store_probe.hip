// WRITE_SIZE per stored byte for the store forms the fill kernels use
// (rocprofv3 --pmc WRITE_SIZE): 64 lanes x 8 B contiguous per instruction as
//   mode 0: relaxed agent-scope atomic store (the granule publish, st_granule)
//   mode 1: plain store
//   mode 2: non-temporal store
//   mode 3: 64 lanes x 4 B non-temporal (the code stores)
// build: hipcc -O3 --offload-arch=gfx950 store_probe.hip -o store_probe
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef unsigned long long u64;
typedef __attribute__((address_space(1))) unsigned long long gu64;

__global__ void store_kernel(u64* buf, size_t n_inst, int mode) {
  const int lane = threadIdx.x & 63;
  const size_t wave = (blockIdx.x * (size_t)blockDim.x + threadIdx.x) >> 6;
  const size_t nw = (gridDim.x * (size_t)blockDim.x) >> 6;
  for (size_t i = wave; i < n_inst; i += nw) {
    if (mode == 3) {
      unsigned* p = reinterpret_cast<unsigned*>(buf) + i * 64 + lane;
      __builtin_nontemporal_store((unsigned)(i + lane), p);
    } else {
      u64* p = buf + i * 64 + lane;
      const u64 v = ((u64)7 << 32) | (unsigned)(i + lane);
      if (mode == 0) __hip_atomic_store((gu64*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else if (mode == 1) *p = v;
      else __builtin_nontemporal_store(v, p);
    }
  }
}

int main(int argc, char** argv) {
  const int mode = argc > 1 ? atoi(argv[1]) : 0;
  const size_t bytes = (size_t)4 << 30;
  u64* buf;
  if (hipMalloc(&buf, bytes) != hipSuccess) return 1;
  const size_t per_inst = mode == 3 ? 256 : 512;
  const size_t n_inst = bytes / 512;  // (mode 3 writes half the buffer)
  hipLaunchKernelGGL(store_kernel, dim3(1024), dim3(256), 0, 0, buf, n_inst, mode);
  hipDeviceSynchronize();
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  hipEventRecord(a);
  hipLaunchKernelGGL(store_kernel, dim3(1024), dim3(256), 0, 0, buf, n_inst, mode);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  printf("mode %d: %.3f GB stored in %.3f ms (%.1f GB/s)\n", mode, n_inst * per_inst / 1e9, ms, n_inst * per_inst / 1e6 / ms);
  return 0;
}
