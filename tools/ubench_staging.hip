// ubench_staging.hip -- how fast can each lane stream its own contiguous
// segment (the scan kernel's access pattern) into registers?  Standalone
// microbenchmark (tools/, not part of libdsx).  Each kernel XORs the words it
// receives so the loads stay live; prints GB/s per variant.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_staging.hip -o /tmp/ubench
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void dma16(const u32x4& rsrc, uint32_t voff, uint32_t lds_addr) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %1, %3, 0 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(lds_addr), "s"(rsrc) : "memory");
}

// plain coalesced streaming read (HBM ceiling)
__global__ void k_copy(const uint4* p, uint64_t n16, uint32_t* out) {
  uint32_t acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += (uint64_t)gridDim.x * blockDim.x) {
    uint4 v = p[i];
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678) out[0] = acc;
}

// per-lane segments of S bytes, register loads, DEPTH rounds of 48 B in flight
template <int DEPTH>
__global__ __launch_bounds__(1024) void k_reg(const uint8_t* base, uint32_t S, uint32_t nregions, uint32_t* out) {
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const uint32_t waves = blockDim.x >> 6;
  uint32_t acc = 0;
  const uint32_t R = S / 48;
  for (uint32_t region = blockIdx.x * waves + wave; region < nregions; region += gridDim.x * waves) {
    const u32x4* p = (const u32x4*)(base + ((uint64_t)region * 64 + lane) * S);
    u32x4 buf[DEPTH][3];
#pragma unroll
    for (int d = 0; d < DEPTH; ++d)
#pragma unroll
      for (int c = 0; c < 3; ++c) buf[d][c] = __builtin_nontemporal_load(p + d * 3 + c);
    for (uint32_t r = 0; r < R; r += DEPTH) {
#pragma unroll
      for (int d = 0; d < DEPTH; ++d) {
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          acc ^= buf[d][c].x ^ buf[d][c].y ^ buf[d][c].z ^ buf[d][c].w;
          const uint32_t nr = r + d + DEPTH;
          if (nr < R) buf[d][c] = __builtin_nontemporal_load(p + nr * 3 + c);
        }
      }
    }
  }
  if (acc == 0x12345678) out[0] = acc;
}

// per-lane segments, LDS-DMA rows of ROWB bytes (multiple of 48), NB buffers
template <int ROWB, int NB, int WAVES>
__global__ __launch_bounds__(WAVES * 64) void k_dma(const uint8_t* base, uint32_t S, uint32_t nregions, uint64_t len, uint32_t* out) {
  constexpr int BUF = 64 * ROWB;
  constexpr int NI = BUF / 1024;  // DMA instructions per batch
  __shared__ __attribute__((aligned(16))) uint8_t lds[WAVES * NB * BUF];
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  uint8_t* stage = lds + wave * NB * BUF;
  const uint32_t stage_lds = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)stage);
  uint32_t acc = 0;
  const uint32_t B = S / ROWB;  // batches per lane segment
  uint32_t roff[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const uint32_t u = i * 64 + lane;
    roff[i] = (u / (ROWB / 16)) * S + (u % (ROWB / 16)) * 16;
  }
  for (uint32_t region = blockIdx.x * WAVES + wave; region < nregions; region += gridDim.x * WAVES) {
    const uint64_t rp = (uint64_t)(uintptr_t)(base + (uint64_t)region * 64 * S);
    u32x4 rs;
    rs.x = __builtin_amdgcn_readfirstlane((uint32_t)rp);
    rs.y = __builtin_amdgcn_readfirstlane((uint32_t)(rp >> 32) & 0xFFFF);
    rs.z = 64u * S;
    rs.w = 0x00020000u;
    auto issue = [&](uint32_t b) {
      const uint32_t dst = stage_lds + (b % NB) * BUF;
#pragma unroll
      for (int i = 0; i < NI; ++i) dma16(rs, b < B ? roff[i] + b * ROWB : 0xFFFFFFF0u, dst + i * 1024);
    };
    for (int b = 0; b < NB - 1; ++b) issue(b);
    for (uint32_t b = 0; b < B; ++b) {
      if constexpr (NB == 8) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NI * 6) : "memory");
      else if constexpr (NB == 4) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NI * 2) : "memory");
      else if constexpr (NB == 3) asm volatile("s_waitcnt vmcnt(%0)" :: "n"(NI) : "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const uint4* src = (const uint4*)(stage + (b % NB) * BUF + lane * ROWB);
#pragma unroll
      for (int c = 0; c < ROWB / 16; ++c) { uint4 v = src[c]; acc ^= v.x ^ v.y ^ v.z ^ v.w; }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      issue(b + NB - 1);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  if (acc == 0x12345678) out[0] = acc;
}

// k_dma + a contiguous L2 prefetch: every PFB batches the wave touches, with
// one buffer_load_dword per lane into a dummy LDS slot, the next PFK KiB of
// 64/(PFK*16) lane segments per instruction (one dword per 64 B half-line), so
// DRAM sees PFK KiB contiguous bursts instead of 64 interleaved ROWB-byte rows.
template <int ROWB, int NB, int WAVES, int PFK, int AHEAD>
__global__ __launch_bounds__(WAVES * 64) void k_dma_pf(const uint8_t* base, uint32_t S, uint32_t nregions, uint64_t len, uint32_t* out) {
  constexpr int BUF = 64 * ROWB;
  constexpr int NI = BUF / 1024;
  constexpr int LPS = PFK * 16;          // lanes per segment chunk (one per 64 B)
  constexpr int SPI = 64 / LPS;          // segments per prefetch instruction
  constexpr int NPI = 64 / SPI;          // prefetch instructions per PFK KiB of all 64 segments
  __shared__ __attribute__((aligned(16))) uint8_t lds[WAVES * NB * BUF + WAVES * 256];
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  uint8_t* stage = lds + wave * NB * BUF;
  const uint32_t stage_lds = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)stage);
  const uint32_t dummy_lds = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)(lds + WAVES * NB * BUF + wave * 256));
  uint32_t acc = 0;
  const uint32_t B = S / ROWB;
  uint32_t roff[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const uint32_t u = i * 64 + lane;
    roff[i] = (u / (ROWB / 16)) * S + (u % (ROWB / 16)) * 16;
  }
  const uint32_t pf_seg = lane / LPS, pf_off = (lane % LPS) * 64;
  for (uint32_t region = blockIdx.x * WAVES + wave; region < nregions; region += gridDim.x * WAVES) {
    const uint64_t rp = (uint64_t)(uintptr_t)(base + (uint64_t)region * 64 * S);
    u32x4 rs;
    rs.x = __builtin_amdgcn_readfirstlane((uint32_t)rp);
    rs.y = __builtin_amdgcn_readfirstlane((uint32_t)(rp >> 32) & 0xFFFF);
    rs.z = 64u * S;
    rs.w = 0x00020000u;
    auto issue = [&](uint32_t b) {
      const uint32_t dst = stage_lds + (b % NB) * BUF;
#pragma unroll
      for (int i = 0; i < NI; ++i) dma16(rs, b < B ? roff[i] + b * ROWB : 0xFFFFFFF0u, dst + i * 1024);
    };
    // prefetch instruction pi: chunk pi / NPI (PFK KiB of SPI segments); issued
    // as Q per batch (a dummy out-of-range load once AHEAD chunks ahead) so
    // that vmcnt counting stays exact
    constexpr int Q = (NPI * ROWB + PFK * 1024 - 1) / (PFK * 1024) + 1;
    uint32_t pi = 0;
    auto prefetch1 = [&](uint32_t cur_chunk) {
      const uint32_t c = pi / NPI, i = pi % NPI;
      uint32_t vo = 0xFFFFFFF0u;
      if (c <= cur_chunk + AHEAD) {
        const uint32_t o = c * PFK * 1024u + pf_off;
        if (o < S) vo = (i * SPI + pf_seg) * S + o;
        ++pi;
      }
      uint32_t keep;
      asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dword %1, %3, 0 offen lds\n\ts_mov_b32 m0, %0"
                   : "=&s"(keep) : "v"(vo), "s"(dummy_lds), "s"(rs) : "memory");
    };
    for (int b = 0; b < NB - 1; ++b) {
      issue(b);
#pragma unroll
      for (int q = 0; q < Q; ++q) prefetch1(0);
    }
    for (uint32_t b = 0; b < B; ++b) {
      asm volatile("s_waitcnt vmcnt(%0)" :: "n"((NB - 2) * (NI + Q) + Q) : "memory");
      const uint4* src = (const uint4*)(stage + (b % NB) * BUF + lane * ROWB);
#pragma unroll
      for (int c = 0; c < ROWB / 16; ++c) { uint4 v = src[c]; acc ^= v.x ^ v.y ^ v.z ^ v.w; }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      issue(b + NB - 1);
#pragma unroll
      for (int q = 0; q < Q; ++q) prefetch1((b * ROWB) / (PFK * 1024u));
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  if (acc == 0x12345678) out[0] = acc;
}

int main(int argc, char** argv) {
  const uint64_t len = (argc > 1 ? strtoull(argv[1], nullptr, 10) : 4ull) << 30;
  uint8_t* d; uint32_t* o;
  CHK(hipMalloc(&d, len + 4096)); CHK(hipMalloc(&o, 64));
  CHK(hipMemset(d, 7, len));
  int ncu = 256;
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  auto timeit = [&](const char* name, auto launch) {
    for (int i = 0; i < 3; ++i) launch();
    hipEventRecord(e0);
    const int it = 10;
    for (int i = 0; i < it; ++i) launch();
    hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    printf("%-44s %8.3f ms  %7.0f GB/s  %s\n", name, ms / it, len / (ms / it * 1e-3) / 1e9, hipGetErrorString(hipGetLastError()));
  };
  timeit("coalesced copy-read", [&] { k_copy<<<ncu * 8, 256>>>((const uint4*)d, len / 16, o); });
  for (uint32_t S : {8448u, 33024u, 2304u}) {
    const uint32_t nreg = (uint32_t)(len / (64ull * S));
    char nm[96];
#define RUN(ROWB, NB, W, label) snprintf(nm, sizeof nm, "S=%u " label, S); \
    timeit(nm, [&] { k_dma<ROWB, NB, W><<<ncu, W * 64>>>(d, S, nreg, len, o); });
    RUN(128, 2, 8, "rows128 1-ahead 8w")
    RUN(128, 3, 6, "rows128 2-ahead 6w")
    RUN(128, 4, 4, "rows128 3-ahead 4w")
    RUN(256, 2, 4, "rows256 1-ahead 4w")
    RUN(128, 1, 16, "rows128 0-ahead 16w")
    RUN(64, 2, 16, "rows64 1-ahead 16w")
    RUN(96, 3, 8, "rows96 2-ahead 8w (old)")
#undef RUN
#define RUNPF(ROWB, NB, W, PFK, AH, label) snprintf(nm, sizeof nm, "S=%u " label, S); \
    timeit(nm, [&] { k_dma_pf<ROWB, NB, W, PFK, AH><<<ncu, W * 64>>>(d, S, nreg, len, o); });
    RUNPF(128, 2, 8, 1, 1, "pf rows128 1-ahead 8w pfk1 a1")
    RUNPF(128, 2, 8, 1, 2, "pf rows128 1-ahead 8w pfk1 a2")
    RUNPF(128, 2, 8, 2, 1, "pf rows128 1-ahead 8w pfk2 a1")
    RUNPF(128, 2, 8, 4, 1, "pf rows128 1-ahead 8w pfk4 a1")
#undef RUNPF
  }
  return 0;
}
