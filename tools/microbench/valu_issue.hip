// valu_issue.hip — chip-wide issue rate of single VALU instructions on gfx950, by
// opcode and encoding (VOP1/VOP2 4-byte, VOP3/VOP3P 8-byte, DPP, SDWA), from wall
// time: 8 independent chains per wave, 8 waves per SIMD, 256 CUs.
//   hipcc -O3 --offload-arch=gfx950 valu_issue.hip -o valu_issue && ./valu_issue
// Prints G wave-instructions/s (wall time) and s_memtime ticks per instruction.
// s_memtime does not tick at the shader clock on gfx950 (it reads ~1.4 GHz
// where GRBM_GUI_ACTIVE shows ~2.4 GHz), so cycles per instruction come from a
// rocprofv3 PMC pass instead: tools/valu_pmc_summary.py.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s\n", hipGetErrorString(e)); return 1; } } while (0)

constexpr int kIters = 16384;

// Operand patterns: D = dst (+v), B = second source (v), S = an SGPR
#define R8(I) I(0) I(1) I(2) I(3) I(4) I(5) I(6) I(7)
#define ASM8(TXT)                                                                     \
  asm volatile(TXT : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), \
               "+v"(a7) : "v"(b), "s"(sb), "s"(mask) : "vcc", "s20", "s21", "s22", "s23", "s24", "s25", "s26", "s27", "s28", "s29", "s30", "s31", "s32", "s33", "s34", "s35")
#define L2(OP, T) OP " %0, %0, %8" T "\n\t" OP " %1, %1, %8" T "\n\t" OP " %2, %2, %8" T "\n\t" OP " %3, %3, %8" T "\n\t" \
                  OP " %4, %4, %8" T "\n\t" OP " %5, %5, %8" T "\n\t" OP " %6, %6, %8" T "\n\t" OP " %7, %7, %8" T
#define L1(OP, T) OP " %0, %8" T "\n\t" OP " %1, %8" T "\n\t" OP " %2, %8" T "\n\t" OP " %3, %8" T "\n\t" \
                  OP " %4, %8" T "\n\t" OP " %5, %8" T "\n\t" OP " %6, %8" T "\n\t" OP " %7, %8" T
#define L3(OP, T) OP " %0, %0, %8, %8" T "\n\t" OP " %1, %1, %8, %8" T "\n\t" OP " %2, %2, %8, %8" T "\n\t" \
                  OP " %3, %3, %8, %8" T "\n\t" OP " %4, %4, %8, %8" T "\n\t" OP " %5, %5, %8, %8" T "\n\t" \
                  OP " %6, %6, %8, %8" T "\n\t" OP " %7, %7, %8, %8" T
#define L3S(OP, T) OP " %0, %0, %8, %9" T "\n\t" OP " %1, %1, %8, %9" T "\n\t" OP " %2, %2, %8, %9" T "\n\t" \
                  OP " %3, %3, %8, %9" T "\n\t" OP " %4, %4, %8, %9" T "\n\t" OP " %5, %5, %8, %9" T "\n\t" \
                  OP " %6, %6, %8, %9" T "\n\t" OP " %7, %7, %8, %9" T
#define L2S(OP, T) OP " %0, %9, %0" T "\n\t" OP " %1, %9, %1" T "\n\t" OP " %2, %9, %2" T "\n\t" OP " %3, %9, %3" T "\n\t" \
                  OP " %4, %9, %4" T "\n\t" OP " %5, %9, %5" T "\n\t" OP " %6, %9, %6" T "\n\t" OP " %7, %9, %7" T

#define L3M(OP, T) OP " %0, %0, %8, %10" T "\n\t" OP " %1, %1, %8, %10" T "\n\t" OP " %2, %2, %8, %10" T "\n\t" \
                  OP " %3, %3, %8, %10" T "\n\t" OP " %4, %4, %8, %10" T "\n\t" OP " %5, %5, %8, %10" T "\n\t" \
                  OP " %6, %6, %8, %10" T "\n\t" OP " %7, %7, %8, %10" T
#define LC(OP, T) OP " s[20:21], %0, %8\n\t" OP " s[22:23], %1, %8\n\t" OP " s[24:25], %2, %8\n\t" OP " s[26:27], %3, %8\n\t" \
                  OP " s[28:29], %4, %8\n\t" OP " s[30:31], %5, %8\n\t" OP " s[32:33], %6, %8\n\t" OP " s[34:35], %7, %8"
#define LCV(OP, T) OP " vcc, %0, %8\n\t" OP " vcc, %1, %8\n\t" OP " vcc, %2, %8\n\t" OP " vcc, %3, %8\n\t" \
                  OP " vcc, %4, %8\n\t" OP " vcc, %5, %8\n\t" OP " vcc, %6, %8\n\t" OP " vcc, %7, %8"
#define L2Z(OP, T) OP " %0, 1.0, %0" T "\n\t" OP " %1, 1.0, %1" T "\n\t" OP " %2, 1.0, %2" T "\n\t" OP " %3, 1.0, %3" T "\n\t" \
                  OP " %4, 1.0, %4" T "\n\t" OP " %5, 1.0, %5" T "\n\t" OP " %6, 1.0, %6" T "\n\t" OP " %7, 1.0, %7" T
#define L2K(OP, T) OP " %0, 0x12345, %0" T "\n\t" OP " %1, 0x12345, %1" T "\n\t" OP " %2, 0x12345, %2" T "\n\t" OP " %3, 0x12345, %3" T "\n\t" \
                  OP " %4, 0x12345, %4" T "\n\t" OP " %5, 0x12345, %5" T "\n\t" OP " %6, 0x12345, %6" T "\n\t" OP " %7, 0x12345, %7" T
#define L1S(OP, T) OP " %0, %9" T "\n\t" OP " %1, %9" T "\n\t" OP " %2, %9" T "\n\t" OP " %3, %9" T "\n\t" \
                  OP " %4, %9" T "\n\t" OP " %5, %9" T "\n\t" OP " %6, %9" T "\n\t" OP " %7, %9" T

struct Op { const char *name; int id; };

#define OPS(X)                                         \
  X(0, "v_add_f32_e32", L2("v_add_f32_e32", ""))        \
  X(1, "v_add_f32_e64", L2("v_add_f32_e64", ""))        \
  X(2, "v_max_f32_e32", L2("v_max_f32_e32", ""))        \
  X(3, "v_max_f32_e64", L2("v_max_f32_e64", ""))        \
  X(4, "v_min_f32_e32", L2("v_min_f32_e32", ""))        \
  X(5, "v_mul_f32_e32", L2("v_mul_f32_e32", ""))        \
  X(6, "v_sub_f32_e32", L2("v_sub_f32_e32", ""))        \
  X(7, "v_fmac_f32_e32", L2("v_fmac_f32_e32", ""))      \
  X(8, "v_fma_f32", L3("v_fma_f32", ""))                \
  X(9, "v_max3_f32", L3("v_max3_f32", ""))              \
  X(10, "v_add_u32_e32", L2("v_add_u32_e32", ""))       \
  X(11, "v_add_u32_e64", L2("v_add_u32_e64", ""))       \
  X(12, "v_sub_u32_e32", L2("v_sub_u32_e32", ""))       \
  X(13, "v_max_i32_e32", L2("v_max_i32_e32", ""))       \
  X(14, "v_max_u32_e32", L2("v_max_u32_e32", ""))       \
  X(15, "v_min_i32_e32", L2("v_min_i32_e32", ""))       \
  X(16, "v_and_b32_e32", L2("v_and_b32_e32", ""))       \
  X(17, "v_or_b32_e32", L2("v_or_b32_e32", ""))         \
  X(18, "v_xor_b32_e32", L2("v_xor_b32_e32", ""))       \
  X(19, "v_lshlrev_b32_e32", L2("v_lshlrev_b32_e32", ""))  \
  X(20, "v_mov_b32_e32", L1("v_mov_b32_e32", ""))       \
  X(21, "v_add_f16_e32", L2("v_add_f16_e32", ""))       \
  X(22, "v_max_f16_e32", L2("v_max_f16_e32", ""))       \
  X(23, "v_max_i16_e32", L2("v_max_i16_e32", ""))       \
  X(24, "v_max_u16_e32", L2("v_max_u16_e32", ""))       \
  X(25, "v_add_u16_e32", L2("v_add_u16_e32", ""))       \
  X(26, "v_add3_u32", L3("v_add3_u32", ""))             \
  X(27, "v_max3_i32", L3("v_max3_i32", ""))             \
  X(28, "v_max3_u32", L3("v_max3_u32", ""))             \
  X(29, "v_bfi_b32", L3("v_bfi_b32", ""))               \
  X(30, "v_perm_b32", L3("v_perm_b32", ""))             \
  X(31, "v_xad_u32", L3("v_xad_u32", ""))               \
  X(32, "v_lshl_add_u32", L3("v_lshl_add_u32", ""))     \
  X(33, "v_pk_add_f16", L2("v_pk_add_f16", ""))         \
  X(34, "v_pk_max_f16", L2("v_pk_max_f16", ""))         \
  X(35, "v_pk_add_u16", L2("v_pk_add_u16", ""))         \
  X(36, "v_pk_max_i16", L2("v_pk_max_i16", ""))         \
  X(37, "v_pk_fma_f16", L3("v_pk_fma_f16", ""))         \
  X(38, "v_pk_maximum3_f16", L3("v_pk_maximum3_f16", "")) \
  X(39, "v_max3_f16", L3("v_max3_f16", ""))             \
  X(40, "v_max3_i16", L3("v_max3_i16", ""))             \
  X(41, "v_add_f32 dpp row_shr:1", L2("v_add_f32_dpp", " row_shr:1 row_mask:0xf bank_mask:0xf")) \
  X(42, "v_max_f32 dpp row_shr:1", L2("v_max_f32_dpp", " row_shr:1 row_mask:0xf bank_mask:0xf")) \
  X(43, "v_mov_b32 dpp wave_shr:1", L1("v_mov_b32_dpp", " wave_shr:1 row_mask:0xf bank_mask:0xf")) \
  X(44, "v_max_f32 sdwa", L2("v_max_f32_sdwa", " dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD")) \
  X(45, "v_cndmask_b32_e32 (vcc)", L2("v_cndmask_b32_e32", ", vcc")) \
  X(46, "v_max_f32_e32 sgpr src0", L2S("v_max_f32_e32", ""))  \
  X(47, "v_add_f32_e32 sgpr src0", L2S("v_add_f32_e32", ""))  \
  X(48, "v_fma_f32 sgpr src2", L3S("v_fma_f32", ""))    \
  X(49, "v_max3_f32 sgpr src2", L3S("v_max3_f32", ""))  \
  X(50, "v_pk_add_f16 op_sel", L2("v_pk_add_f16", " op_sel:[1,0] op_sel_hi:[0,1]")) \
  X(51, "v_min_f16_e32", L2("v_min_f16_e32", ""))       \
  X(52, "v_sub_f16_e32", L2("v_sub_f16_e32", ""))       \
  X(53, "v_mul_f16_e32", L2("v_mul_f16_e32", ""))       \
  \
  X(55, "v_max_u16 sdwa hi", L2("v_max_u16_sdwa", " dst_sel:WORD_1 dst_unused:UNUSED_PRESERVE src0_sel:WORD_1 src1_sel:WORD_1")) \
  X(56, "v_med3_f32", L3("v_med3_f32", ""))             \
  X(57, "v_maximum3_f32", L3("v_maximum3_f32", ""))     \
  X(58, "v_cvt_f32_f16", L1("v_cvt_f32_f16_e32", ""))   \
  X(59, "v_cndmask_b32_e64 s[] mask", L3M("v_cndmask_b32_e64", ""))  \
  X(60, "v_cmp_gt_u32_e64 -> s[]", LC("v_cmp_gt_u32_e64", ""))  \
  X(61, "v_cmp_gt_u32_e32 -> vcc", LCV("v_cmp_gt_u32_e32", ""))  \
  X(62, "v_mul_u32_u24_e32", L2("v_mul_u32_u24_e32", ""))  \
  X(63, "v_mul_lo_u32", L2("v_mul_lo_u32", ""))  \
  X(64, "v_lshrrev_b32_e32", L2("v_lshrrev_b32_e32", ""))  \
  X(65, "v_bfe_u32", L3("v_bfe_u32", ""))  \
  X(66, "v_mad_u32_u24", L3("v_mad_u32_u24", ""))  \
  X(67, "v_max_f32 inline 0", L2Z("v_max_f32_e32", ""))  \
  X(68, "v_add_f16 inline -1.0", L2Z("v_add_f16_e32", ""))  \
  X(69, "v_max_f16 inline 0", L2Z("v_max_f16_e32", ""))  \
  X(70, "v_add_u32 inline 1", L2Z("v_add_u32_e32", ""))  \
  X(71, "v_and_b32 literal", L2K("v_and_b32_e32", ""))  \
  X(72, "v_cndmask_b32_e32 vcc (set)", L2("v_cndmask_b32_e32", ", vcc"))  \
  X(73, "v_sub_u16_e32", L2("v_sub_u16_e32", ""))  \
  X(74, "v_subrev_f16_e32", L2("v_subrev_f16_e32", ""))  \
  X(75, "v_min_u16_e32", L2("v_min_u16_e32", ""))  \
  X(76, "v_min_u32_e32", L2("v_min_u32_e32", ""))  \
  X(77, "v_add_co_u32_e32", L2("v_add_co_u32_e32", ""))  \
  X(78, "v_fmac_f32 dpp", L2("v_fmac_f32_dpp", " row_shr:1 row_mask:0xf bank_mask:0xf"))  \
  X(79, "v_mov_b32_e32 from sgpr", L1S("v_mov_b32_e32", ""))  \
  X(80, "v_ashrrev_i32_e32", L2("v_ashrrev_i32_e32", ""))  \
  X(81, "mix 1 pkmax3 : 1 add_u32", L3("v_pk_maximum3_f16", "") "\n\t" L2("v_add_u32_e32", ""))  \
  X(82, "mix 1 pkmax3 : 2 add_u32", L3("v_pk_maximum3_f16", "") "\n\t" L2("v_add_u32_e32", "") "\n\t" L2("v_xor_b32_e32", ""))  \
  X(83, "mix 1 pkadd : 1 add_u32", L2("v_pk_add_f16", "") "\n\t" L2("v_add_u32_e32", ""))  \
  X(84, "mix 2 pkmax3 : 1 add_u32", L3("v_pk_maximum3_f16", "") "\n\t" L2("v_add_u32_e32", "") "\n\t" L3("v_pk_maximum3_f16", ""))  \
  X(85, "mix 1 perm : 1 and", L3("v_perm_b32", "") "\n\t" L2("v_and_b32_e32", ""))  \
  X(86, "v_pk_maximum3_f16 x16", L3("v_pk_maximum3_f16", "") "\n\t" L3("v_pk_maximum3_f16", ""))  \
  X(87, "v_add_u32 x16", L2("v_add_u32_e32", "") "\n\t" L2("v_xor_b32_e32", ""))

template <int OP>
__global__ void k(uint64_t *cyc, uint32_t *sink) {
  // normal floats in f32 and in both f16 halves (no denormals): 0x3F80_3C00 + t
  uint32_t a0 = 0x3F803C00u + (threadIdx.x & 7), a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,
           a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7, b = 0x3F813C01u + (blockIdx.x & 3);
  uint32_t sb = 0x3F823C02u;
  const uint64_t mask = __builtin_amdgcn_read_exec() & (0x5555555555555555ull << (blockIdx.x & 1));
  asm volatile("s_mov_b64 vcc, %0" ::"s"(mask) : "vcc");
  uint64_t t0 = __builtin_readcyclecounter();
  for (int it = 0; it < kIters; ++it) {
#define X(ID, NAME, TXT) if constexpr (OP == ID) ASM8(TXT);
    OPS(X)
#undef X
  }
  uint64_t t1 = __builtin_readcyclecounter();
  if (threadIdx.x % 64 == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
  sink[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
}

constexpr int InstrPerIter(int op) { return op == 82 || op == 84 ? 24 : (op >= 81 && op <= 87 && op != 80) ? 16 : 8; }

template <int OP>
int run(const char *name, int waves_per_simd) {
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
  const double per_wave = (double)kIters * InstrPerIter(OP);
  const double total = per_wave * blocks * 4;
  const double clk = avg / (ms * 1e6);  // GHz
  printf("%-28s w=%d  %7.1f G wave-instr/s   %.2f s_memtime ticks/instr (%.2f G ticks/s)\n", name, waves_per_simd,
         total / (ms * 1e6), avg / per_wave / waves_per_simd, clk);
  delete[] h;
  CHECK(hipFree(cyc));
  CHECK(hipFree(sink));
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
  return 0;
}

int main() {
  for (int w : {4, 8}) {
#define X(ID, NAME, TXT) if (ID >= 79 || w == 8) run<ID>(NAME, w);
    OPS(X)
#undef X
  }
  return 0;
}
