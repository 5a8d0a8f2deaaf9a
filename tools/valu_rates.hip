// Issue cost of single VALU instructions on gfx950 (measurement tool, not product code): each
// kernel runs 8 independent chains per lane of one instruction kind (inline asm, so exactly
// that instruction), 64 per chain per loop trip; 8 waves per SIMD on every CU.  Cost per
// wave-instruction per SIMD = elapsed cycles x SIMDs / wave-instructions.
// build: hipcc --offload-arch=gfx950 -O2 -o tools/valu_rates tools/valu_rates.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CH8(S) S(0) S(1) S(2) S(3) S(4) S(5) S(6) S(7)

#define KERNEL(NAME, STMT)                                                                  \
  __global__ void __launch_bounds__(256) NAME(uint32_t *out, int iters, uint32_t y, uint32_t z) { \
    uint32_t x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4,            \
             x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;                                         \
    uint64_t q0 = x0, q1 = x1, q2 = x2, q3 = x3, q4 = x4, q5 = x5, q6 = x6, q7 = x7;        \
    for (int it = 0; it < iters; it++) {                                                    \
      _Pragma("unroll") for (int r = 0; r < 64; r++) { CH8(STMT) }                          \
    }                                                                                       \
    out[blockIdx.x * 256 + threadIdx.x] = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7 ^           \
        (uint32_t)(q0 ^ q1 ^ q2 ^ q3 ^ q4 ^ q5 ^ q6 ^ q7);                                  \
  }

#define S_XOR(i) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(x##i) : "v"(y));
#define S_ALIGN(i) asm volatile("v_alignbit_b32 %0, %0, %1, %2" : "+v"(x##i) : "v"(y), "v"(z));
#define S_SHL64(i) asm volatile("v_lshlrev_b64 %0, 3, %0" : "+v"(q##i));
#define S_ADD3(i) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x##i) : "v"(y), "v"(z));
#define S_MAX3(i) asm volatile("v_max3_i32 %0, %0, %1, %2" : "+v"(x##i) : "v"(y), "v"(z));
#define S_LSHLADD(i) asm volatile("v_lshl_add_u32 %0, %0, 1, %1" : "+v"(x##i) : "v"(y));
#define S_XOR_E64(i) asm volatile("v_xor_b32_e64 %0, %1, %0" : "+v"(x##i) : "v"(y));
#define S_FFBL(i) asm volatile("v_ffbl_b32 %0, %0" : "+v"(x##i));
#define S_DPP(i) asm volatile("v_mov_b32_dpp %0, %0 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(x##i));
#define S_ASHR(i) asm volatile("v_ashrrev_i32 %0, 5, %0" : "+v"(x##i));
#define S_MIN(i) asm volatile("v_min_i32 %0, %1, %0" : "+v"(x##i) : "v"(y));
#define S_SHR32(i) asm volatile("v_lshrrev_b32 %0, 3, %0" : "+v"(x##i));

KERNEL(k_xor, S_XOR)
KERNEL(k_align, S_ALIGN)
KERNEL(k_shl64, S_SHL64)
KERNEL(k_add3, S_ADD3)
KERNEL(k_max3, S_MAX3)
KERNEL(k_lshladd, S_LSHLADD)
KERNEL(k_xor_e64, S_XOR_E64)
KERNEL(k_ffbl, S_FFBL)
KERNEL(k_dpp, S_DPP)
KERNEL(k_ashr, S_ASHR)
KERNEL(k_min, S_MIN)
KERNEL(k_shr32, S_SHR32)

typedef void (*kfn)(uint32_t *, int, uint32_t, uint32_t);

int main() {
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int ncu = p.multiProcessorCount;
  const int blocks = ncu * 8;                  // 8 blocks of 4 waves per CU: 8 waves per SIMD
  uint32_t *out;
  hipMalloc(&out, (size_t)blocks * 256 * 4);
  const int iters = 2000;
  struct { const char *name; kfn f; } ks[] = {
      {"v_xor_b32 (VOP2)", k_xor}, {"v_xor_b32_e64 (VOP3)", k_xor_e64},
      {"v_alignbit_b32", k_align}, {"v_lshlrev_b64", k_shl64}, {"v_add3_u32", k_add3},
      {"v_max3_i32", k_max3}, {"v_lshl_add_u32", k_lshladd}, {"v_ffbl_b32", k_ffbl},
      {"v_mov_b32_dpp", k_dpp}, {"v_ashrrev_i32", k_ashr}, {"v_min_i32", k_min},
      {"v_lshrrev_b32", k_shr32}};
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  int clk_khz = 0;
  hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0);
  const double ghz = 2.4;                      // MI355X_MICROARCH.md; reported: clk_khz
  for (auto &k : ks) {
    hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, 10, 1u, 2u);   // warm-up
    hipDeviceSynchronize();
    hipEventRecord(a, 0);
    hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, iters, 1u, 2u);
    hipEventRecord(b, 0);
    hipEventSynchronize(b);
    float ms = 0;
    hipEventElapsedTime(&ms, a, b);
    const double winst = (double)blocks * 4 * iters * 64 * 8;     // wave-instructions
    const double simd_cycles = ms * 1e-3 * ghz * 1e9 * ncu * 4;
    printf("%-22s %8.3f ms  %.2f cycles per wave-instruction per SIMD  (clock attr %d kHz)\n",
           k.name, ms, simd_cycles / winst, clk_khz);
  }
  hipFree(out);
  return 0;
}
