// valu_rate.hip — issue cost of the VALU instructions the K2/K3 inner loops use,
// measured on gfx950 with s_memtime inside the kernel.
//   hipcc -O3 --offload-arch=gfx950 valu_rate.hip -o valu_rate && ./valu_rate
// For each op: 8 independent chains per wave (throughput) and 1 chain (latency),
// at 1 and 4 waves per SIMD. Prints cycles per instruction per SIMD.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

constexpr int kIters = 32768;

#define OP8(INS) OP8T(INS, "")
#define OP8T(INS, T)                                                                 \
  asm volatile(INS " %0, %0, %8" T "\n\t" INS " %1, %1, %8" T "\n\t" INS " %2, %2, %8" T "\n\t" \
               INS " %3, %3, %8" T "\n\t" INS " %4, %4, %8" T "\n\t" INS " %5, %5, %8" T "\n\t" \
               INS " %6, %6, %8" T "\n\t" INS " %7, %7, %8" T                        \
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) \
               : "v"(b))
#define OP8_3(INS, TAIL)                                                             \
  asm volatile(INS " %0, %0, %8, %8" TAIL "\n\t" INS " %1, %1, %8, %8" TAIL "\n\t"    \
               INS " %2, %2, %8, %8" TAIL "\n\t" INS " %3, %3, %8, %8" TAIL "\n\t"    \
               INS " %4, %4, %8, %8" TAIL "\n\t" INS " %5, %5, %8, %8" TAIL "\n\t"    \
               INS " %6, %6, %8, %8" TAIL "\n\t" INS " %7, %7, %8, %8" TAIL           \
               : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7) \
               : "v"(b))
#define DEP8(INS) DEP8T(INS, "")
#define DEP8T(INS, T)                                                                \
  asm volatile(INS " %0, %0, %1" T "\n\t" INS " %0, %0, %1" T "\n\t" INS " %0, %0, %1" T "\n\t" \
               INS " %0, %0, %1" T "\n\t" INS " %0, %0, %1" T "\n\t" INS " %0, %0, %1" T "\n\t" \
               INS " %0, %0, %1" T "\n\t" INS " %0, %0, %1" T : "+v"(a0) : "v"(b))

template <int OP>
__global__ void k(uint64_t *cyc, uint32_t *sink) {
  uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5,
           a6 = a0 + 6, a7 = a0 + 7, b = blockIdx.x | 0x10001;
  uint64_t t0 = __builtin_readcyclecounter();
  for (int it = 0; it < kIters; ++it) {
    if constexpr (OP == 0) OP8("v_pk_max_i16");
    if constexpr (OP == 1) OP8T("v_pk_sub_u16", " clamp");
    if constexpr (OP == 2) OP8("v_pk_add_u16");
    if constexpr (OP == 3) OP8("v_max_i32");
    if constexpr (OP == 4) OP8("v_add_u32");
    if constexpr (OP == 5) OP8_3("v_perm_b32", "");
    if constexpr (OP == 6) OP8_3("v_max3_i32", "");
    if constexpr (OP == 7) OP8_3("v_bitop3_b32", " bitop3:0x80");
    if constexpr (OP == 8) OP8("v_pk_max_u16");
    if constexpr (OP == 9) {  // DPP row shift (wave_shr:1 is a VALU mov with DPP)
      asm volatile(
          "v_mov_b32_dpp %0, %8 wave_shr:1 row_mask:0xf bank_mask:0xf\n\t"
          "v_mov_b32_dpp %1, %8 wave_shr:1 row_mask:0xf bank_mask:0xf\n\t"
          "v_mov_b32_dpp %2, %8 wave_shr:1 row_mask:0xf bank_mask:0xf\n\t"
          "v_mov_b32_dpp %3, %8 wave_shr:1 row_mask:0xf bank_mask:0xf\n\t"
          "v_mov_b32_dpp %4, %8 wave_shr:1 row_mask:0xf bank_mask:0xf\n\t"
          "v_mov_b32_dpp %5, %8 wave_shr:1 row_mask:0xf bank_mask:0xf\n\t"
          "v_mov_b32_dpp %6, %8 wave_shr:1 row_mask:0xf bank_mask:0xf\n\t"
          "v_mov_b32_dpp %7, %8 wave_shr:1 row_mask:0xf bank_mask:0xf"
          : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
          : "v"(b));
    }
    if constexpr (OP == 10) DEP8("v_pk_max_i16");
    if constexpr (OP == 11) DEP8("v_max_i32");
    if constexpr (OP == 12) DEP8T("v_pk_sub_u16", " clamp");
    // float forms: does the f32 datapath issue wave64 in 2 cycles (SIMD-32)?
    if constexpr (OP == 13) OP8("v_add_f32");
    if constexpr (OP == 14) OP8("v_max_f32");
    if constexpr (OP == 15) OP8_3("v_max3_f32", "");
    if constexpr (OP == 16) OP8_3("v_fma_f32", "");
    if constexpr (OP == 17) OP8("v_pk_add_f16");
    if constexpr (OP == 18) OP8_3("v_pk_maximum3_f16", "");
    if constexpr (OP == 19) OP8_3("v_pk_fma_f16", "");
    if constexpr (OP == 20) OP8("v_add_u32");
    if constexpr (OP == 21) OP8_3("v_max3_u32", "");
    if constexpr (OP == 23) OP8("v_mul_f32");
    if constexpr (OP == 25) DEP8("v_add_f32");
    if constexpr (OP == 26) OP8_3("v_med3_f32", "");
    if constexpr (OP == 27) OP8_3("v_max3_i16", "");
    if constexpr (OP == 28) OP8("v_max_f16");
  }
  uint64_t t1 = __builtin_readcyclecounter();
  if (threadIdx.x % 64 == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
  sink[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

template <int OP>
int run(const char *name, int instr_per_iter, int waves_per_simd) {
  hipDeviceProp_t p;
  CHECK(hipGetDeviceProperties(&p, 0));
  const int cus = p.multiProcessorCount;
  const int blocks = cus * waves_per_simd;  // 256-thread blocks: one wave per SIMD each
  uint64_t *cyc;
  uint32_t *sink;
  CHECK(hipMalloc(&cyc, blocks * 4 * sizeof(uint64_t)));
  CHECK(hipMalloc(&sink, blocks * 256 * sizeof(uint32_t)));
  hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, cyc, sink);
  CHECK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL(k<OP>, dim3(blocks), dim3(256), 0, 0, cyc, sink);
  CHECK(hipEventRecord(e1));
  CHECK(hipDeviceSynchronize());
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  uint64_t *h = new uint64_t[blocks * 4];
  CHECK(hipMemcpy(h, cyc, blocks * 4 * sizeof(uint64_t), hipMemcpyDeviceToHost));
  double avg = 0;
  for (int i = 0; i < blocks * 4; ++i) avg += h[i];
  avg /= blocks * 4;
  const double instr = (double)kIters * instr_per_iter;  // per wave
  // cycles per instruction per SIMD: a wave's cycles / (its instructions x waves sharing the SIMD)
  printf("%-28s waves/SIMD=%d  wave-cycles/instr=%.2f  SIMD-cycles/instr=%.2f  (%.3f ms, clk~%.2f GHz)\n",
         name, waves_per_simd, avg / instr, avg / instr / waves_per_simd, ms,
         avg / (ms * 1e6));
  delete[] h;
  CHECK(hipFree(cyc));
  CHECK(hipFree(sink));
  return 0;
}

int main(int argc, char **argv) {
  if (argc > 1) {  // float set only
    for (int w : {1, 2, 4, 8}) {
      run<13>("v_add_f32 x8", 8, w);
      run<23>("v_mul_f32 x8", 8, w);
      run<14>("v_max_f32 x8", 8, w);
      run<15>("v_max3_f32 x8", 8, w);
      run<26>("v_med3_f32 x8", 8, w);
      run<16>("v_fma_f32 x8", 8, w);
      run<17>("v_pk_add_f16 x8", 8, w);
      run<18>("v_pk_maximum3_f16 x8", 8, w);
      run<19>("v_pk_fma_f16 x8", 8, w);
      run<28>("v_max_f16 x8", 8, w);
      run<27>("v_max3_i16 x8", 8, w);
      run<20>("v_add_u32 x8", 8, w);
      run<21>("v_max3_u32 x8", 8, w);
      run<25>("v_add_f32 dep chain", 8, w);
    }
    return 0;
  }
  for (int w : {1, 4, 6, 8}) {
    run<0>("v_pk_max_i16 x8 indep", 8, w);
    run<1>("v_pk_sub_u16 clamp x8", 8, w);
    run<2>("v_pk_add_u16 x8", 8, w);
    run<8>("v_pk_max_u16 x8", 8, w);
    run<3>("v_max_i32 x8", 8, w);
    run<4>("v_add_u32 x8", 8, w);
    run<5>("v_perm_b32 x8", 8, w);
    run<6>("v_max3_i32 x8", 8, w);
    run<7>("v_bitop3_b32 x8", 8, w);
    run<9>("v_mov_b32_dpp wave_shr x8", 8, w);
    run<10>("v_pk_max_i16 dep chain", 8, w);
    run<11>("v_max_i32 dep chain", 8, w);
    run<12>("v_pk_sub_u16 dep chain", 8, w);
  }
  return 0;
}
