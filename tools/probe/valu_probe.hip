// VALU issue-rate probe: cycles per wave-instruction for the fill kernel's
// integer ops, with 1..4 waves per SIMD (grid = CUs * 4 * wps waves).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define REP16(X) X X X X X X X X X X X X X X X X

template <int OP>
__global__ __launch_bounds__(256) void probe(unsigned* out, int iters, unsigned long long* cyc) {
  unsigned a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 ^ 9, a5 = a0 ^ 11, a6 = a0 + 13, a7 = a0 + 17;
  unsigned b = blockIdx.x | 1, c = b * 77;
  unsigned long long p0 = a0, p1 = a1, p2 = a2, p3 = a3, pb = b;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#define BODY(INS)                                                                                  \
  asm volatile(INS " %0, %0, %8, %9\n\t" INS " %1, %1, %8, %9\n\t" INS " %2, %2, %8, %9\n\t" INS       \
               " %3, %3, %8, %9\n\t" INS " %4, %4, %8, %9\n\t" INS " %5, %5, %8, %9\n\t" INS           \
               " %6, %6, %8, %9\n\t" INS " %7, %7, %8, %9"                                           \
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)       \
               : "v"(b), "v"(c));
#define BODY2(INS)                                                                                 \
  asm volatile(INS " %0, %0, %8\n\t" INS " %1, %1, %8\n\t" INS " %2, %2, %8\n\t" INS " %3, %3, %8\n\t" \
               INS " %4, %4, %8\n\t" INS " %5, %5, %8\n\t" INS " %6, %6, %8\n\t" INS " %7, %7, %8"      \
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)       \
               : "v"(b));
#define BODYPK(INS)                                                                                \
  asm volatile(INS " %0, %0, %4\n\t" INS " %1, %1, %4\n\t" INS " %2, %2, %4\n\t" INS " %3, %3, %4\n\t"    \
               INS " %0, %0, %4\n\t" INS " %1, %1, %4\n\t" INS " %2, %2, %4\n\t" INS " %3, %3, %4"        \
               : "+v"(p0), "+v"(p1), "+v"(p2), "+v"(p3) : "v"(pb));
    if constexpr (OP == 0) { REP16(BODY("v_min3_i32")) }
    if constexpr (OP == 1) { REP16(BODY("v_bfe_i32")) }
    if constexpr (OP == 2) { REP16(BODY("v_alignbit_b32")) }
    if constexpr (OP == 3) { REP16(BODY2("v_add_u32")) }
    if constexpr (OP == 4) { REP16(BODY2("v_pk_min_i16")) }
    if constexpr (OP == 5) { REP16(BODY2("v_pk_add_u16")) }
    if constexpr (OP == 6) { REP16(BODY("v_perm_b32")) }
    if constexpr (OP == 7) { REP16(BODY("v_add3_u32")) }
    if constexpr (OP == 8) { REP16(BODY2("v_min_i32")) }
    if constexpr (OP == 9) { REP16(BODY("v_pk_min3_i16")) }
    if constexpr (OP == 10) { REP16(BODY("v_med3_i32")) }
    if constexpr (OP == 11) { REP16(BODY2("v_pk_sub_u16")) }
    if constexpr (OP == 12) { REP16(BODY2("v_add_f32")) }
    if constexpr (OP == 13) { REP16(BODY2("v_min_f32")) }
    if constexpr (OP == 14) { REP16(BODY("v_min3_f32")) }
    if constexpr (OP == 15) { REP16(BODY2("v_sub_u32")) }
    if constexpr (OP == 16) { REP16(BODY2("v_and_b32")) }
    if constexpr (OP == 17) { REP16(BODY2("v_lshrrev_b32")) }
    if constexpr (OP == 18) { REP16(BODY2("v_max_i32")) }
    if constexpr (OP == 19) { REP16(BODY2("v_mul_f32")) }
    if constexpr (OP == 20) { REP16(BODY("v_fma_f32")) }
    if constexpr (OP == 21) { REP16(BODYPK("v_pk_add_f32")) }
    if constexpr (OP == 22) { REP16(BODY2("v_or_b32")) }
    if constexpr (OP == 23) { REP16(BODY2("v_max_f32")) }
    if constexpr (OP == 24) { REP16(BODY2("v_min_u32")) }
    if constexpr (OP == 25) { REP16(BODY2("v_xor_b32")) }
    if constexpr (OP == 26) { REP16(BODY2("v_sub_f32")) }
    if constexpr (OP == 27) { REP16(BODYPK("v_pk_mul_f32")) }
#define BODYX(INS, SUF)                                                                              \
  asm volatile(INS " %0, %0, %8, %9 " SUF "\n\t" INS " %1, %1, %8, %9 " SUF "\n\t" INS " %2, %2, %8, %9 " SUF \
               "\n\t" INS " %3, %3, %8, %9 " SUF "\n\t" INS " %4, %4, %8, %9 " SUF "\n\t" INS " %5, %5, %8, %9 " \
               SUF "\n\t" INS " %6, %6, %8, %9 " SUF "\n\t" INS " %7, %7, %8, %9 " SUF                             \
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)       \
               : "v"(b), "v"(c));
#define BODYDPP(CTL)                                                                               \
  asm volatile("v_mov_b32_dpp %0, %8 " CTL "\n\tv_mov_b32_dpp %1, %8 " CTL "\n\tv_mov_b32_dpp %2, %8 " CTL       \
               "\n\tv_mov_b32_dpp %3, %8 " CTL "\n\tv_mov_b32_dpp %4, %8 " CTL "\n\tv_mov_b32_dpp %5, %8 " CTL      \
               "\n\tv_mov_b32_dpp %6, %8 " CTL "\n\tv_mov_b32_dpp %7, %8 " CTL                                       \
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)       \
               : "v"(b));
    if constexpr (OP == 28) { REP16(BODYX("v_bitop3_b32", "bitop3:0xde")) }
    if constexpr (OP == 29) { REP16(BODY("v_or3_b32")) }
    if constexpr (OP == 30) { REP16(BODY("v_and_or_b32")) }
    if constexpr (OP == 31) { REP16(BODYDPP("wave_shr:1 row_mask:0xf bank_mask:0xf")) }
    if constexpr (OP == 32) { REP16(BODY("v_lshl_or_b32")) }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if ((threadIdx.x & 63) == 0) cyc[blockIdx.x * 4 + (threadIdx.x >> 6)] = t1 - t0;
  out[blockIdx.x * 256 + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + (unsigned)(p0 + p1 + p2 + p3);
}

template <int OP>
void run(const char* name, int cus) {
  const int iters = 2000;
  for (int wps = 2; wps <= 2; wps *= 2) {
    const int blocks = cus * wps;  // 4 waves per block -> wps waves per SIMD
    unsigned* out; unsigned long long* cyc;
    hipMalloc(&out, blocks * 256 * 4);
    hipMalloc(&cyc, blocks * 4 * 8);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipLaunchKernelGGL(probe<OP>, dim3(blocks), dim3(256), 0, 0, out, 10, cyc);
    hipEventRecord(e0);
    hipLaunchKernelGGL(probe<OP>, dim3(blocks), dim3(256), 0, 0, out, iters, cyc);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    std::vector<unsigned long long> c(blocks * 4);
    hipMemcpy(c.data(), cyc, c.size() * 8, hipMemcpyDeviceToHost);
    double avg = 0; for (auto v : c) avg += v; avg /= c.size();
    const double ninst = (double)iters * 128;
    // wall: SIMD cycles per wave-instruction assuming 2.4 GHz; memtime: per-wave cycles (shader clock) / instr * wps
    printf("%-16s wps=%d  wall %.2f ns/instr/SIMD (=%.2f cyc@2.4GHz)  memtime per wave %.2f cyc/instr\n", name, wps,
           ms * 1e6 / (ninst * wps), ms * 1e6 / (ninst * wps) * 2.4, avg / ninst);
    hipFree(out); hipFree(cyc);
  }
}

int main() {
  hipDeviceProp_t p; hipGetDeviceProperties(&p, 0);
  const int cus = p.multiProcessorCount;
  printf("CUs %d, clock %d kHz\n", cus, p.clockRate);
  run<12>("v_add_f32", cus);
  run<13>("v_min_f32", cus);
  run<14>("v_min3_f32", cus);
  run<15>("v_sub_u32", cus);
  run<16>("v_and_b32", cus);
  run<17>("v_lshrrev_b32", cus);
  run<18>("v_max_i32", cus);
  run<19>("v_mul_f32", cus);
  run<20>("v_fma_f32", cus);
  run<21>("v_pk_add_f32", cus);
  run<22>("v_or_b32", cus);
  run<23>("v_max_f32", cus);
  run<24>("v_min_u32", cus);
  run<25>("v_xor_b32", cus);
  run<26>("v_sub_f32", cus);
  run<27>("v_pk_mul_f32", cus);
  run<0>("v_min3_i32", cus);
  run<1>("v_bfe_i32", cus);
  run<2>("v_alignbit_b32", cus);
  run<3>("v_add_u32", cus);
  run<4>("v_pk_min_i16", cus);
  run<5>("v_pk_add_u16", cus);
  run<6>("v_perm_b32", cus);
  run<7>("v_add3_u32", cus);
  run<8>("v_min_i32", cus);
  run<10>("v_med3_i32", cus);
  run<11>("v_pk_sub_u16", cus);
  run<28>("v_bitop3_b32", cus);
  run<29>("v_or3_b32", cus);
  run<30>("v_and_or_b32", cus);
  run<31>("v_mov_b32_dpp wave_shr:1", cus);
  run<32>("v_lshl_or_b32", cus);
  return 0;
}
