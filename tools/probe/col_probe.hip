// Issue-rate probe for the column-wise bit-parallel fill:
// cycles per wave-instruction of the carry-chain instructions and of the
// scalar lane-mask shifts that move carries between lanes, at 2 and 4 waves
// per SIMD (grid = CUs * wps blocks of 4 waves).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define REP16(X) X X X X X X X X X X X X X X X X
typedef unsigned long long u64;

template <int OP>
__global__ __launch_bounds__(256) void probe(unsigned* out, int iters, u64* cyc) {
  unsigned a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 ^ 9, a5 = a0 ^ 11, a6 = a0 + 13, a7 = a0 + 17;
  unsigned b = blockIdx.x | 1, c = b * 77;
  u64 s0 = 1, s1 = 2, s2 = 3, s3 = 4, s4 = 5, s5 = 6, s6 = 7, s7 = 8;
  u64 t0s = 3; unsigned t1s = 5;
  const u64 t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#define ADDC8(INS)                                                                                           \
  asm volatile(INS " %0, %8, %0, %16, %8\n\t" INS " %1, %9, %1, %16, %9\n\t" INS " %2, %10, %2, %16, %10\n\t" \
               INS " %3, %11, %3, %16, %11\n\t" INS " %4, %12, %4, %16, %12\n\t" INS " %5, %13, %5, %16, %13\n\t" \
               INS " %6, %14, %6, %16, %14\n\t" INS " %7, %15, %7, %16, %15"                                  \
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7), "+s"(s0),     \
                 "+s"(s1), "+s"(s2), "+s"(s3), "+s"(s4), "+s"(s5), "+s"(s6), "+s"(s7)                          \
               : "v"(b));
// one v_addc per carry chain + the scalar shift that feeds the next lane: s_lshl_b64 + s_or_b32
#define MIX8()                                                                                                   \
  asm volatile("v_addc_co_u32 %0, %8, %0, %16, %8\n\ts_lshl_b64 %8, %8, 1\n\ts_or_b64 %8, %8, %17\n\t"             \
               "v_addc_co_u32 %1, %9, %1, %16, %9\n\ts_lshl_b64 %9, %9, 1\n\ts_or_b64 %9, %9, %17\n\t"             \
               "v_addc_co_u32 %2, %10, %2, %16, %10\n\ts_lshl_b64 %10, %10, 1\n\ts_or_b64 %10, %10, %17\n\t"       \
               "v_addc_co_u32 %3, %11, %3, %16, %11\n\ts_lshl_b64 %11, %11, 1\n\ts_or_b64 %11, %11, %17\n\t"       \
               "v_addc_co_u32 %4, %12, %4, %16, %12\n\ts_lshl_b64 %12, %12, 1\n\ts_or_b64 %12, %12, %17\n\t"       \
               "v_addc_co_u32 %5, %13, %5, %16, %13\n\ts_lshl_b64 %13, %13, 1\n\ts_or_b64 %13, %13, %17\n\t"       \
               "v_addc_co_u32 %6, %14, %6, %16, %14\n\ts_lshl_b64 %14, %14, 1\n\ts_or_b64 %14, %14, %17\n\t"       \
               "v_addc_co_u32 %7, %15, %7, %16, %15\n\ts_lshl_b64 %15, %15, 1\n\ts_or_b64 %15, %15, %17"           \
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7), "+s"(s0),         \
                 "+s"(s1), "+s"(s2), "+s"(s3), "+s"(s4), "+s"(s5), "+s"(s6), "+s"(s7)                              \
               : "v"(b), "s"(t0s) : "scc");
// the same VALU with 3 bitop3 between addcs (the kernel's mix: ~1 carry op in 4-5)
#define MIXB8()                                                                                                  \
  asm volatile("v_addc_co_u32 %0, %8, %0, %16, %8\n\ts_lshl_b64 %8, %8, 1\n\ts_or_b64 %8, %8, %17\n\t"             \
               "v_bitop3_b32 %1, %1, %16, %2 bitop3:0xde\n\tv_bitop3_b32 %2, %2, %16, %3 bitop3:0xde\n\t"          \
               "v_bitop3_b32 %3, %3, %16, %4 bitop3:0xde\n\t"                                                      \
               "v_addc_co_u32 %4, %9, %4, %16, %9\n\ts_lshl_b64 %9, %9, 1\n\ts_or_b64 %9, %9, %17\n\t"             \
               "v_bitop3_b32 %5, %5, %16, %6 bitop3:0xde\n\tv_bitop3_b32 %6, %6, %16, %7 bitop3:0xde\n\t"          \
               "v_bitop3_b32 %7, %7, %16, %0 bitop3:0xde"                                                          \
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7), "+s"(s0),         \
                 "+s"(s1), "+s"(s2), "+s"(s3), "+s"(s4), "+s"(s5), "+s"(s6), "+s"(s7)                              \
               : "v"(b), "s"(t0s) : "scc");
#define CND8()                                                                                                   \
  asm volatile("v_cndmask_b32 %0, %0, %16, %8\n\tv_cndmask_b32 %1, %1, %16, %9\n\tv_cndmask_b32 %2, %2, %16, %10\n\t" \
               "v_cndmask_b32 %3, %3, %16, %11\n\tv_cndmask_b32 %4, %4, %16, %12\n\tv_cndmask_b32 %5, %5, %16, %13\n\t" \
               "v_cndmask_b32 %6, %6, %16, %14\n\tv_cndmask_b32 %7, %7, %16, %15"                                   \
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)                   \
               : "s"(s0), "s"(s1), "s"(s2), "s"(s3), "s"(s4), "s"(s5), "s"(s6), "s"(s7), "v"(b));
#define BOP8()                                                                                                   \
  asm volatile("v_bitop3_b32 %0, %0, %8, %1 bitop3:0xde\n\tv_bitop3_b32 %1, %1, %8, %2 bitop3:0xde\n\t"             \
               "v_bitop3_b32 %2, %2, %8, %3 bitop3:0xde\n\tv_bitop3_b32 %3, %3, %8, %4 bitop3:0xde\n\t"             \
               "v_bitop3_b32 %4, %4, %8, %5 bitop3:0xde\n\tv_bitop3_b32 %5, %5, %8, %6 bitop3:0xde\n\t"             \
               "v_bitop3_b32 %6, %6, %8, %7 bitop3:0xde\n\tv_bitop3_b32 %7, %7, %8, %0 bitop3:0xde"                 \
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) : "v"(b));
#define SALU8()                                                                                                  \
  asm volatile("s_lshl_b64 %0, %0, 1\n\ts_lshl_b64 %1, %1, 1\n\ts_lshl_b64 %2, %2, 1\n\ts_lshl_b64 %3, %3, 1\n\t"   \
               "s_lshl_b64 %4, %4, 1\n\ts_lshl_b64 %5, %5, 1\n\ts_lshl_b64 %6, %6, 1\n\ts_lshl_b64 %7, %7, 1"       \
               : "+s"(s0), "+s"(s1), "+s"(s2), "+s"(s3), "+s"(s4), "+s"(s5), "+s"(s6), "+s"(s7) : : "scc");
    if constexpr (OP == 0) { REP16(ADDC8("v_addc_co_u32")) }
    if constexpr (OP == 1) { REP16(MIX8()) }
    if constexpr (OP == 2) { REP16(MIXB8()) }
    if constexpr (OP == 3) { REP16(CND8()) }
    if constexpr (OP == 4) { REP16(BOP8()) }
    if constexpr (OP == 5) { REP16(SALU8()) }
  }
  const u64 t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
  out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + (unsigned)(s0 + s1 + s2 + s3 + s4 + s5 + s6 + s7) + c + t1s;
}

template <int OP>
void run(const char* name, int cus, int per_rep) {
  const int iters = 2000;
  for (int wps = 1; wps <= 4; wps *= 2) {
    const int blocks = cus * wps;
    unsigned* out;
    u64* cyc;
    hipMalloc(&out, blocks * 256 * 4);
    hipMalloc(&cyc, blocks * 4 * 8);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipLaunchKernelGGL(probe<OP>, dim3(blocks), dim3(256), 0, 0, out, 10, cyc);
    hipEventRecord(e0);
    hipLaunchKernelGGL(probe<OP>, dim3(blocks), dim3(256), 0, 0, out, iters, cyc);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double ninst = (double)iters * 16 * per_rep;  // counted instructions per wave
    printf("%-40s wps=%d  %.2f ns per counted instr per SIMD (= %.2f cyc @2.4GHz)\n", name, wps,
           ms * 1e6 / (ninst * wps), ms * 1e6 / (ninst * wps) * 2.4);
    hipFree(out);
    hipFree(cyc);
  }
}

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  printf("CUs %d\n", cus);
  run<4>("v_bitop3_b32 (per VALU)", cus, 8);
  run<0>("v_addc_co_u32 sgpr carry (per VALU)", cus, 8);
  run<3>("v_cndmask_b32 sgpr mask (per VALU)", cus, 8);
  run<5>("s_lshl_b64 (per SALU)", cus, 8);
  run<1>("addc + lshl_b64 + or_b32 (per addc)", cus, 8);
  run<2>("addc+2 SALU, 3 bitop3 (per VALU)", cus, 8);
  return 0;
}
