// Probe: do two kernels on two streams run concurrently, and is an atomic
// counter written by one visible to the other's atomic poll?  Bounded spins.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((address_space(1))) unsigned gu32;
#define RLX __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT
__device__ unsigned opaque0() { unsigned z = 0; asm volatile("" : "+v"(z)); return z; }

__global__ void waiter(unsigned* flag, unsigned* out, int mode) {
  unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  unsigned polls = 0, v = 0;
  for (;;) {
    if (mode == 0) v = __hip_atomic_load((gu32*)flag, RLX);
    else v = __hip_atomic_fetch_add((gu32*)flag, opaque0(), RLX);
    ++polls;
    if (v != 0) break;
    if (__builtin_amdgcn_s_memrealtime() - t0 > 200000000ull) break;  // 2 s
    __builtin_amdgcn_s_sleep(8);
  }
  unsigned xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  if (threadIdx.x == 0) { out[0] = v; out[1] = polls; out[2] = (unsigned)((__builtin_amdgcn_s_memrealtime() - t0) / 100); out[3] = xcc & 0xf; }
}
__global__ void setter(unsigned* flag, unsigned* out) {
  unsigned xcc;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
  if (threadIdx.x == 0) { __hip_atomic_fetch_add((gu32*)flag, 1u, RLX); out[4] = xcc & 0xf; }
}
int main() {
  unsigned *flag, *out;
  hipMalloc(&flag, 256); hipMalloc(&out, 256);
  hipStream_t s1, s2;
  hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
  hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
  for (int mode = 0; mode < 2; ++mode)
    for (int order = 0; order < 2; ++order) {
      hipMemset(flag, 0, 256); hipMemset(out, 0, 256); hipDeviceSynchronize();
      if (order == 0) {
        hipLaunchKernelGGL(waiter, dim3(1), dim3(64), 0, s2, flag, out, mode);
        hipLaunchKernelGGL(setter, dim3(1), dim3(64), 0, s1, flag, out);
      } else {
        hipLaunchKernelGGL(setter, dim3(1), dim3(64), 0, s1, flag, out);
        hipLaunchKernelGGL(waiter, dim3(1), dim3(64), 0, s2, flag, out, mode);
      }
      hipDeviceSynchronize();
      unsigned h[8]; hipMemcpy(h, out, 32, hipMemcpyDeviceToHost);
      printf("mode=%s order=%s: seen=%u polls=%u us=%u waiter_xcc=%u setter_xcc=%u\n", mode ? "atomic-rmw" : "sc1-load",
             order ? "setter-first" : "waiter-first", h[0], h[1], h[2], h[3], h[4]);
    }
  // nwk's launch sequence: memset on s1, event on s1, s2 waits on it,
  // "fill" (setter) on s1 first, then "traceback" (waiter) on s2.
  for (int variant = 0; variant < 3; ++variant) {
    hipEvent_t ev; hipEventCreate(&ev);
    hipMemsetAsync(flag, 0, 256, s1); hipMemsetAsync(out, 0, 256, s1);
    hipEventRecord(ev, s1);
    if (variant != 1) hipStreamWaitEvent(s2, ev, 0);
    if (variant == 2) {
      hipLaunchKernelGGL(waiter, dim3(1), dim3(64), 0, s2, flag, out, 1);
      hipLaunchKernelGGL(setter, dim3(1), dim3(64), 0, s1, flag, out);
    } else {
      hipLaunchKernelGGL(setter, dim3(1), dim3(64), 0, s1, flag, out);
      hipLaunchKernelGGL(waiter, dim3(1), dim3(64), 0, s2, flag, out, 1);
    }
    hipDeviceSynchronize();
    unsigned h[8]; hipMemcpy(h, out, 32, hipMemcpyDeviceToHost);
    printf("nwk-sequence variant %d: seen=%u polls=%u us=%u\n", variant, h[0], h[1], h[2]);
    hipEventDestroy(ev);
  }
  return 0;
}
