/*
 * gpu_trap.c — TEST INFRASTRUCTURE ONLY.
 *
 * The reference's aligner.cpp always references its ten GPU plugin symbols
 * (reference common.h:37 defines NUMBER_GPUS; the declarations are
 * aligner_gpu.h:33-114). oracle/_ref/ghostm_ref, the reference CPU program used
 * as the parity oracle, links this file instead of any plugin: every symbol
 * exits with status 2, so an oracle run that ever reached the GPU path would fail
 * loudly instead of silently running product code. The signatures follow this
 * repo's include/ghostm_hip.h Part 1 (same C ABI).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

static void trap(const char *name) {
  fprintf(stderr, "oracle/_ref: GPU plugin symbol %s called in the CPU oracle build\n", name);
  exit(2);
}

int InitGpu(void) { trap("InitGpu"); return 1; }

size_t GetNeededGPUMemorySize(uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t e,
                              uint32_t f) {
  (void)a; (void)b; (void)c; (void)d; (void)e; (void)f;
  trap("GetNeededGPUMemorySize");
  return 0;
}

int CheckGpuMemory(uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t e, uint32_t f) {
  (void)a; (void)b; (void)c; (void)d; (void)e; (void)f;
  trap("CheckGpuMemory");
  return 1;
}

int SetOptionGpu(uint32_t max_list_length, int score_matrix[], int device) {
  (void)max_list_length; (void)score_matrix; (void)device;
  trap("SetOptionGpu");
  return 1;
}

void printGpuInfo(int device) { (void)device; trap("printGpuInfo"); }

int SetQueryGpu(uint8_t sequences[], uint32_t n, uint32_t len) {
  (void)sequences; (void)n; (void)len;
  trap("SetQueryGpu");
  return 1;
}

int SetDbGpu(uint8_t sequences[], uint32_t len, uint32_t keys_count[], uint32_t kcl,
             uint32_t positions[], uint32_t npos) {
  (void)sequences; (void)len; (void)keys_count; (void)kcl; (void)positions; (void)npos;
  trap("SetDbGpu");
  return 1;
}

uint32_t SearchNextGpu(uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t e, uint32_t f,
                       uint32_t g, uint32_t h, uint32_t *counts, uint32_t *starts) {
  (void)a; (void)b; (void)c; (void)d; (void)e; (void)f; (void)g; (void)h;
  (void)counts; (void)starts;
  trap("SearchNextGpu");
  return 0;
}

void CalculateScoreGpu(uint32_t a, uint32_t b, uint32_t c, uint32_t scores[], uint32_t ends[],
                       uint32_t d, uint32_t e, int open_gap, int extend_gap) {
  (void)a; (void)b; (void)c; (void)scores; (void)ends; (void)d; (void)e;
  (void)open_gap; (void)extend_gap;
  trap("CalculateScoreGpu");
}

int FreeGpu(void) { trap("FreeGpu"); return 1; }
