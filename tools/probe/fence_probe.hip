// Probe: does an agent-scope release fence (buffer_wbl2) in one kernel stall
// while another kernel's waves spin on atomics?  Bounded spins (2 s).
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((address_space(1))) unsigned gu32;
#define RLX __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT
__device__ unsigned opaque0() { unsigned z = 0; asm volatile("" : "+v"(z)); return z; }

__global__ void waiter(unsigned* flag, unsigned* out, int sleep) {
  __shared__ unsigned big[10000];
  unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  unsigned polls = 0, v = 0;
  for (;;) {
    if (threadIdx.x == 0) v = __hip_atomic_fetch_add((gu32*)flag, opaque0(), RLX);
    v = __builtin_amdgcn_readfirstlane(v);
    ++polls;
    if (v != 0) break;
    if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) break;
    if (sleep) __builtin_amdgcn_s_sleep(32);
  }
  big[threadIdx.x] = v;
  if (threadIdx.x == 0) { out[blockIdx.x * 4] = v + big[0] * 0; out[blockIdx.x * 4 + 1] = polls; out[blockIdx.x * 4 + 2] = (unsigned)((__builtin_amdgcn_s_memrealtime() - t0) / 100); }
}
__global__ void setter(unsigned* flag, unsigned* data, int fence) {
  data[threadIdx.x + blockIdx.x * 256] = 7;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (fence) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (threadIdx.x == 0) __hip_atomic_fetch_add((gu32*)flag, 1u, RLX);
}
int main() {
  unsigned *flag, *out, *data;
  hipMalloc(&flag, 256); hipMalloc(&out, 4096); hipMalloc(&data, 1 << 20);
  hipStream_t s1, s2;
  hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
  hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
  // warm both kernels
  hipLaunchKernelGGL(setter, dim3(1), dim3(256), 0, s1, flag, data, 1);
  hipLaunchKernelGGL(waiter, dim3(1), dim3(64), 0, s1, flag, out, 1);
  hipDeviceSynchronize();
  const int cfg[][4] = {{1, 1, 1, 1}, {1, 36, 1, 1}, {0, 36, 1, 1}, {1, 36, 0, 1}, {1, 36, 1, 9}, {1, 36, 1, 0}};
  for (auto& c : cfg) {
    int fence = c[0], nw = c[1], sleep = c[2], order = c[3];
    hipEvent_t ev; hipEventCreate(&ev);
    hipMemsetAsync(flag, 0, 256, s1); hipMemsetAsync(out, 0, 4096, s1);
    hipEventRecord(ev, s1);
    hipStreamWaitEvent(s2, ev, 0);
    unsigned long long t0 = 0;
    if (order) {
      hipLaunchKernelGGL(setter, dim3(order), dim3(256), 0, s1, flag, data, fence);
      hipLaunchKernelGGL(waiter, dim3(nw), dim3(64), 0, s2, flag, out, sleep);
    } else {
      hipLaunchKernelGGL(waiter, dim3(nw), dim3(64), 0, s2, flag, out, sleep);
      hipLaunchKernelGGL(setter, dim3(1), dim3(256), 0, s1, flag, data, fence);
    }
    hipDeviceSynchronize();
    unsigned h[4 * 36]; hipMemcpy(h, out, sizeof h, hipMemcpyDeviceToHost);
    unsigned mx = 0, seen = 0;
    for (int b = 0; b < nw; ++b) { mx = h[4 * b + 2] > mx ? h[4 * b + 2] : mx; seen += h[4 * b] != 0; }
    printf("fence=%d waiters=%d sleep=%d setter_blocks=%d: seen %u/%d max_us=%u\n", fence, nw, sleep, order, seen, nw, mx);
    hipEventDestroy(ev);
  }
  return 0;
}
