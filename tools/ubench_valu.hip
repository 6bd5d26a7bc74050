// ubench_valu.hip -- VALU issue throughput per instruction type on gfx950
// (standalone microbenchmark, tools/, not part of libdsx).  Each kernel runs
// ITER iterations of 8 independent inline-asm instructions per lane; prints
// wave64 instructions per SIMD per cycle (from wall time and the clock).
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_valu.hip -o tools/ubench_valu
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

constexpr int ITER = 4096;

#define BODY8(INS)                                                                  \
  asm volatile(INS : "+v"(a0) : "v"(b), "v"(c)); asm volatile(INS : "+v"(a1) : "v"(b), "v"(c)); \
  asm volatile(INS : "+v"(a2) : "v"(b), "v"(c)); asm volatile(INS : "+v"(a3) : "v"(b), "v"(c)); \
  asm volatile(INS : "+v"(a4) : "v"(b), "v"(c)); asm volatile(INS : "+v"(a5) : "v"(b), "v"(c)); \
  asm volatile(INS : "+v"(a6) : "v"(b), "v"(c)); asm volatile(INS : "+v"(a7) : "v"(b), "v"(c));

#define KERNEL(NAME, INS)                                                            \
  __global__ void NAME(uint32_t* out, uint32_t seed) {                              \
    uint32_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, \
             a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;                                  \
    uint32_t b = seed * 3u + 1u, c = seed * 5u + 7u;                                 \
    for (int i = 0; i < ITER; ++i) { BODY8(INS) }                                   \
    uint32_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;                              \
    if (r == 0x12345679u) out[0] = r;                                               \
  }

KERNEL(k_xor, "v_xor_b32 %0, %0, %1")
KERNEL(k_add, "v_add_u32 %0, %0, %1")
KERNEL(k_alignbit, "v_alignbit_b32 %0, %0, %0, 31")
KERNEL(k_perm, "v_perm_b32 %0, %0, %1, %2")
KERNEL(k_cvt, "v_cvt_f32_u32 %0, %0")
KERNEL(k_fma, "v_fma_f32 %0, %0, %1, %2")
KERNEL(k_mul_f32, "v_mul_f32 %0, %0, %1")
KERNEL(k_mad24, "v_mad_u32_u24 %0, %0, %1, %2")
KERNEL(k_mul24, "v_mul_u32_u24 %0, %0, %1")
KERNEL(k_xad, "v_xad_u32 %0, %0, %1, %2")
KERNEL(k_or3, "v_or3_b32 %0, %0, %1, %2")
KERNEL(k_lshl_or, "v_lshl_or_b32 %0, %0, 1, %1")
KERNEL(k_bfi, "v_bfi_b32 %0, %0, %1, %2")
KERNEL(k_min3, "v_min3_u32 %0, %0, %1, %2")
KERNEL(k_sad, "v_sad_u32 %0, %0, %1, %2")
KERNEL(k_mullo, "v_mul_lo_u32 %0, %0, %1")
KERNEL(k_mulhi, "v_mul_hi_u32 %0, %0, %1")
KERNEL(k_xor_e64, "v_xor_b32_e64 %0, %0, %1")
KERNEL(k_sdwa_mov, "v_mov_b32_sdwa %0, %1 dst_sel:BYTE_1 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_2")
KERNEL(k_sdwa_or, "v_or_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2")
KERNEL(k_min, "v_min_u32 %0, %0, %1")
KERNEL(k_sub, "v_sub_u32 %0, %0, %1")
KERNEL(k_lshr, "v_lshrrev_b32 %0, 3, %0")
KERNEL(k_and, "v_and_b32 %0, %0, %1")
KERNEL(k_cvt_ubyte, "v_cvt_f32_ubyte1 %0, %0")


KERNEL(k_min3f_abs, "v_min3_f32 %0, |%0|, |%1|, |%2|")
KERNEL(k_minf_abs, "v_min_f32_e64 %0, |%0|, |%1|")
KERNEL(k_pk_min_u16, "v_pk_min_u16 %0, %0, %1")
KERNEL(k_max3u, "v_max3_u32 %0, %0, %1, %2")
KERNEL(k_bitop3, "v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96")
KERNEL(k_add3, "v_add3_u32 %0, %0, %1, %2")
KERNEL(k_or, "v_or_b32 %0, %0, %1")
KERNEL(k_lshl, "v_lshlrev_b32 %0, 3, %0")
KERNEL(k_mov, "v_mov_b32 %0, %1")
KERNEL(k_dot2u16, "v_dot2_u32_u16 %0, %0, %1, %2")
KERNEL(k_madu16, "v_mad_u32_u16 %0, %0, %1, %2")
KERNEL(k_alignbyte, "v_alignbyte_b32 %0, %0, %1, 1")
KERNEL(k_mulhi24, "v_mul_hi_u32_u24 %0, %0, %1")
KERNEL(k_min_u16, "v_min_u16 %0, %0, %1")
KERNEL(k_pk_mad_u16, "v_pk_mad_u16 %0, %0, %1, %2")
KERNEL(k_med3u, "v_med3_u32 %0, %0, %1, %2")
KERNEL(k_minimum3f, "v_minimum3_f32 %0, %0, %1, %2")
KERNEL(k_min3i, "v_min3_i32 %0, %0, %1, %2")
KERNEL(k_maxf, "v_max_f32 %0, %0, %1")
KERNEL(k_addf, "v_add_f32 %0, %0, %1")
KERNEL(k_sub_f32, "v_sub_f32 %0, %0, %1")
KERNEL(k_xor_sdwa, "v_xor_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2")
KERNEL(k_lshl_sdwa, "v_lshlrev_b32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2")
KERNEL(k_and_or, "v_and_or_b32 %0, %0, %1, %2")
KERNEL(k_lshl_add, "v_lshl_add_u32 %0, %0, 1, %1")
KERNEL(k_bfe, "v_bfe_u32 %0, %0, 8, 8")

// compare into SGPR pairs + s_or accumulate (ballot pattern)
__global__ void k_cmp(uint32_t* out, uint32_t seed) {
  uint32_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3;
  uint32_t b = seed * 3u + 1u;
  uint64_t acc = 0;
  for (int i = 0; i < ITER; ++i) {
    uint64_t m0, m1, m2, m3;
    asm volatile("v_cmp_eq_u32_e64 %0, %1, %2" : "=s"(m0) : "v"(a0), "v"(b));
    asm volatile("v_cmp_eq_u32_e64 %0, %1, %2" : "=s"(m1) : "v"(a1), "v"(b));
    asm volatile("v_cmp_eq_u32_e64 %0, %1, %2" : "=s"(m2) : "v"(a2), "v"(b));
    asm volatile("v_cmp_eq_u32_e64 %0, %1, %2" : "=s"(m3) : "v"(a3), "v"(b));
    asm volatile("v_cmp_eq_u32_e64 %0, %1, %2" : "=s"(m0) : "v"(a0), "v"(a1));
    asm volatile("v_cmp_eq_u32_e64 %0, %1, %2" : "=s"(m1) : "v"(a1), "v"(a2));
    asm volatile("v_cmp_eq_u32_e64 %0, %1, %2" : "=s"(m2) : "v"(a2), "v"(a3));
    asm volatile("v_cmp_eq_u32_e64 %0, %1, %2" : "=s"(m3) : "v"(a3), "v"(a0));
    acc |= m0 | m1 | m2 | m3;
  }
  if (acc == 0x12345679u) out[0] = (uint32_t)acc;
}

// packed f32 fma (2 lanes of work per instruction)
__global__ void k_pkfma(uint32_t* out, uint32_t seed) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 a0 = {(float)threadIdx.x, 1.f}, a1 = a0 + 1.f, a2 = a0 + 2.f, a3 = a0 + 3.f, a4 = a0 + 4.f,
     a5 = a0 + 5.f, a6 = a0 + 6.f, a7 = a0 + 7.f;
  f2 b = {1.0001f, 0.9999f}, c = {0.5f, 0.25f};
  for (int i = 0; i < ITER; ++i) { BODY8("v_pk_fma_f32 %0, %0, %1, %2") }
  f2 r = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
  if (r.x == 1234.5f) out[0] = 1;
}

// dependent chain: alignbit -> xor (the hash recurrence), 8 chains interleaved
__global__ void k_chain(uint32_t* out, uint32_t seed) {
  uint32_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4,
           a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t b = seed * 3u + 1u, c = 0;
  for (int i = 0; i < ITER / 2; ++i) {
    BODY8("v_alignbit_b32 %0, %0, %0, 31")
    BODY8("v_xor_b32 %0, %0, %1")
  }
  uint32_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (r == 0x12345679u + c) out[0] = r;
}

// N independent dependent chains (alignbit -> xor per step), 8 steps per iteration
template <int N>
__global__ void k_chainN(uint32_t* out, uint32_t seed) {
  uint32_t a[N];
#pragma unroll
  for (int j = 0; j < N; ++j) a[j] = threadIdx.x ^ (seed + j);
  uint32_t b = seed * 3u + 1u;
  for (int i = 0; i < ITER / N; ++i) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
#pragma unroll
      for (int j = 0; j < N; ++j) asm volatile("v_alignbit_b32 %0, %0, %0, 31" : "+v"(a[j]));
#pragma unroll
      for (int j = 0; j < N; ++j) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(a[j]) : "v"(b));
    }
  }
  uint32_t r = 0;
#pragma unroll
  for (int j = 0; j < N; ++j) r ^= a[j];
  if (r == 0x12345679u) out[0] = r;
}

// v_mad_u64_u32 (64-bit result; the low half is h*inv + c)
__global__ void k_mad64(uint32_t* out, uint32_t seed) {
  uint64_t a0 = threadIdx.x ^ seed, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint32_t b = seed * 3u + 1u;
  uint64_t c = seed * 5u + 7u;
  for (int i = 0; i < ITER; ++i) {
#define M64(x) asm volatile("v_mad_u64_u32 %0, vcc, %1, %2, %3" : "=v"(x) : "v"((uint32_t)x), "v"(b), "v"(c) : "vcc");
    M64(a0) M64(a1) M64(a2) M64(a3) M64(a4) M64(a5) M64(a6) M64(a7)
  }
  uint64_t r = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;
  if (r == 0x12345679u) out[0] = (uint32_t)r;
}

int main() {
  uint32_t* o;
  CHK(hipMalloc(&o, 64));
  int clk_khz = 0;
  CHK(hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeClockRate, 0));
  const int ncu = 256;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  struct K { const char* name; void (*f)(uint32_t*, uint32_t); int per_iter; };
  K ks[] = {{"v_xor_b32", k_xor, 8},       {"v_xor_b32_e64", k_xor_e64, 8}, {"v_add_u32", k_add, 8},
            {"v_alignbit_b32", k_alignbit, 8}, {"v_perm_b32", k_perm, 8},   {"v_cvt_f32_u32", k_cvt, 8},
            {"v_fma_f32", k_fma, 8},       {"v_mul_f32", k_mul_f32, 8},     {"v_mad_u32_u24", k_mad24, 8},
            {"v_mul_u32_u24", k_mul24, 8}, {"v_xad_u32", k_xad, 8},         {"v_or3_b32", k_or3, 8},
            {"v_lshl_or_b32", k_lshl_or, 8}, {"v_bfi_b32", k_bfi, 8},       {"v_min3_u32", k_min3, 8},
            {"v_sad_u32", k_sad, 8},       {"v_mul_lo_u32", k_mullo, 8},    {"v_mul_hi_u32", k_mulhi, 8},
            {"v_cmp_e64+s_or", k_cmp, 8},  {"v_mov_b32_sdwa", k_sdwa_mov, 8}, {"v_or_b32_sdwa", k_sdwa_or, 8},
            {"v_min_u32", k_min, 8},       {"v_sub_u32", k_sub, 8},         {"v_lshrrev_b32", k_lshr, 8},
            {"v_and_b32", k_and, 8},       {"v_cvt_f32_ubyte1", k_cvt_ubyte, 8},  {"v_pk_fma_f32", k_pkfma, 8},    {"chain alignbit+xor", k_chain, 8},
            {"v_lshl_add_u32", k_lshl_add, 8}, {"v_bfe_u32", k_bfe, 8},
            {"chain1 (alignbit,xor)", k_chainN<1>, 8}, {"chain2", k_chainN<2>, 8}, {"chain4", k_chainN<4>, 8},
            {"chain8", k_chainN<8>, 8}, {"v_mad_u64_u32", k_mad64, 8},
            {"v_min3_f32 abs", k_min3f_abs, 8}, {"v_min_f32 abs", k_minf_abs, 8}, {"v_pk_min_u16", k_pk_min_u16, 8},
            {"v_max3_u32", k_max3u, 8}, {"v_bitop3_b32", k_bitop3, 8}, {"v_add3_u32", k_add3, 8}, {"v_or_b32", k_or, 8},
            {"v_lshlrev_b32", k_lshl, 8}, {"v_mov_b32", k_mov, 8}, {"v_dot2_u32_u16", k_dot2u16, 8},
            {"v_mad_u32_u16", k_madu16, 8}, {"v_alignbyte_b32", k_alignbyte, 8}, {"v_mul_hi_u32_u24", k_mulhi24, 8},
            {"v_min_u16", k_min_u16, 8}, {"v_pk_mad_u16", k_pk_mad_u16, 8}, {"v_med3_u32", k_med3u, 8},
            {"v_minimum3_f32", k_minimum3f, 8}, {"v_min3_i32", k_min3i, 8}, {"v_max_f32", k_maxf, 8},
            {"v_add_f32", k_addf, 8}, {"v_sub_f32", k_sub_f32, 8}, {"v_xor_b32_sdwa", k_xor_sdwa, 8},
            {"v_lshlrev_b32_sdwa", k_lshl_sdwa, 8}, {"v_and_or_b32", k_and_or, 8}};
  printf("clock attr %d kHz\n", clk_khz);
  for (int wps : {2, 4}) {
    for (auto& k : ks) {
      const int threads = 64 * 4 * wps;  // one block per CU, wps waves per SIMD
      hipLaunchKernelGGL(k.f, dim3(ncu), dim3(threads), 0, 0, o, 1u);
      hipEventRecord(e0);
      const int reps = 5;
      for (int r = 0; r < reps; ++r) hipLaunchKernelGGL(k.f, dim3(ncu), dim3(threads), 0, 0, o, 1u);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      ms /= reps;
      // wave64 instructions per SIMD: wps waves x ITER x per_iter
      const double inst = (double)wps * ITER * k.per_iter;
      const double cyc = ms * 1e-3 * clk_khz * 1e3;
      printf("wps=%d %-22s %8.3f ms  %.3f cyc/inst/SIMD\n", wps, k.name, ms, cyc / inst);
    }
  }
  return 0;
}
