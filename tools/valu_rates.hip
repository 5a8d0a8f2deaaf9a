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
#define S_ADD(i) asm volatile("v_add_u32 %0, %1, %0" : "+v"(x##i) : "v"(y));
#define S_SUB(i) asm volatile("v_sub_u32 %0, %0, %1" : "+v"(x##i) : "v"(y));
#define S_AND(i) asm volatile("v_and_b32 %0, %1, %0" : "+v"(x##i) : "v"(y));
#define S_OR(i) asm volatile("v_or_b32 %0, %1, %0" : "+v"(x##i) : "v"(y));
#define S_MAX(i) asm volatile("v_max_i32 %0, %1, %0" : "+v"(x##i) : "v"(y));
#define S_MINU(i) asm volatile("v_min_u32 %0, %1, %0" : "+v"(x##i) : "v"(y));
#define S_MED3(i) asm volatile("v_med3_i32 %0, %0, %1, %2" : "+v"(x##i) : "v"(y), "v"(z));
#define S_CND(i) asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(x##i) : "v"(y));
#define S_ADDDPP(i) asm volatile("v_add_u32_dpp %0, %0, %1 row_shr:1 row_mask:0xf bank_mask:0xf" : "+v"(x##i) : "v"(y));
#define S_BFE(i) asm volatile("v_bfe_u32 %0, %0, 3, 7" : "+v"(x##i));
#define S_PERM(i) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(x##i) : "v"(y), "v"(z));
#define S_LSHL32(i) asm volatile("v_lshlrev_b32 %0, 3, %0" : "+v"(x##i));
#define S_NOT(i) asm volatile("v_not_b32 %0, %0" : "+v"(x##i));
#define S_MUL24(i) asm volatile("v_mul_u32_u24 %0, %1, %0" : "+v"(x##i) : "v"(y));
#define S_LSHLOR(i) asm volatile("v_lshl_or_b32 %0, %0, 2, %1" : "+v"(x##i) : "v"(y));
#define S_BFI(i) asm volatile("v_bfi_b32 %0, %1, %0, %2" : "+v"(x##i) : "v"(y), "v"(z));
#define S_XAD(i) asm volatile("v_xad_u32 %0, %0, %1, %2" : "+v"(x##i) : "v"(y), "v"(z));
#define S_ADDCO(i) asm volatile("v_add_co_u32 %0, vcc, %1, %0" : "+v"(x##i) : "v"(y) : "vcc");
// selects: with a mask made once before the loop (sgpr pair), and a compare + select pair per
// step with its own mask register per chain (the pattern compiled code uses)
#define S_CNDS(i) asm volatile("v_cndmask_b32_e64 %0, %0, %1, %2" : "+v"(x##i) : "v"(y), "s"(msk));
#define S_CMPCND(i) asm volatile("v_cmp_lt_i32_e64 %1, %0, %2\n\tv_cndmask_b32_e64 %0, %0, %2, %1" : "+v"(x##i), "=s"(m##i) : "v"(y));
#define S_CMP(i) asm volatile("v_cmp_lt_i32_e64 %1, %0, %2" : "+v"(x##i), "=s"(m##i) : "v"(y));
#define S_CMPCNDV(i) asm volatile("v_cmp_lt_i32_e32 vcc, %0, %1\n\tv_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(x##i) : "v"(y) : "vcc");
#define S_CNDV(i) asm volatile("v_cndmask_b32_e32 %0, %0, %1, vcc" : "+v"(x##i) : "v"(y));

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
KERNEL(k_add, S_ADD)
KERNEL(k_sub, S_SUB)
KERNEL(k_and, S_AND)
KERNEL(k_or, S_OR)
KERNEL(k_max, S_MAX)
KERNEL(k_minu, S_MINU)
KERNEL(k_med3, S_MED3)
KERNEL(k_cnd, S_CND)
KERNEL(k_adddpp, S_ADDDPP)
KERNEL(k_bfe, S_BFE)
KERNEL(k_perm, S_PERM)
KERNEL(k_lshl32, S_LSHL32)
KERNEL(k_not, S_NOT)
KERNEL(k_mul24, S_MUL24)
KERNEL(k_lshlor, S_LSHLOR)
KERNEL(k_bfi, S_BFI)
KERNEL(k_xad, S_XAD)
KERNEL(k_addco, S_ADDCO)

#define KERNELM(NAME, STMT)                                                                 \
  __global__ void __launch_bounds__(256) NAME(uint32_t *out, int iters, uint32_t y, uint32_t z) { \
    uint32_t x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4,            \
             x5 = x0 + 5, x6 = x0 + 6, x7 = x0 + 7;                                         \
    uint64_t msk = __builtin_amdgcn_ballot_w64(threadIdx.x & 1);                            \
    uint64_t m0, m1, m2, m3, m4, m5, m6, m7;                                                \
    for (int it = 0; it < iters; it++) {                                                    \
      _Pragma("unroll") for (int r = 0; r < 64; r++) { CH8(STMT) }                          \
    }                                                                                       \
    out[blockIdx.x * 256 + threadIdx.x] = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7 ^ (uint32_t)msk; \
  }
KERNELM(k_cnds, S_CNDS)
KERNELM(k_cmpcnd, S_CMPCND)
KERNELM(k_cmp, S_CMP)
KERNELM(k_cmpcndv, S_CMPCNDV)
// VCC written once before the loop, then only read by the selects
__global__ void __launch_bounds__(256) k_cndv(uint32_t *out, int iters, uint32_t y, uint32_t z) {
  uint32_t x0 = threadIdx.x, x1 = x0 + 1, x2 = x0 + 2, x3 = x0 + 3, x4 = x0 + 4, x5 = x0 + 5,
           x6 = x0 + 6, x7 = x0 + 7;
  asm volatile("v_cmp_gt_u32_e32 vcc, %0, %1" :: "v"(x0), "v"(z) : "vcc");
  for (int it = 0; it < iters; it++) {
    _Pragma("unroll") for (int r = 0; r < 64; r++) { CH8(S_CNDV) }
  }
  out[blockIdx.x * 256 + threadIdx.x] = x0 ^ x1 ^ x2 ^ x3 ^ x4 ^ x5 ^ x6 ^ x7;
}

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
      {"v_lshrrev_b32", k_shr32}, {"v_add_u32", k_add}, {"v_sub_u32", k_sub},
      {"v_and_b32", k_and}, {"v_or_b32", k_or}, {"v_max_i32", k_max}, {"v_min_u32", k_minu},
      {"v_med3_i32", k_med3}, {"v_cndmask_b32 (vcc)", k_cnd}, {"v_add_u32_dpp", k_adddpp},
      {"v_bfe_u32", k_bfe}, {"v_perm_b32", k_perm}, {"v_lshlrev_b32", k_lshl32},
      {"v_not_b32", k_not}, {"v_mul_u32_u24", k_mul24}, {"v_lshl_or_b32", k_lshlor},
      {"v_bfi_b32", k_bfi}, {"v_xad_u32", k_xad}, {"v_add_co_u32", k_addco},
      {"v_cndmask_b32_e64 (sgpr mask)", k_cnds}, {"v_cmp_e64 + v_cndmask (2 instr)", k_cmpcnd},
      {"v_cmp_lt_i32_e64", k_cmp}, {"v_cmp_e32 vcc + v_cndmask_e32 vcc", k_cmpcndv},
      {"v_cndmask_b32_e32 (vcc set once)", k_cndv}};
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
