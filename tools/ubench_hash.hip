// ubench_hash.hip -- issue rate of the scan's per-byte instruction mix on
// gfx950 at 1..4 waves per SIMD (standalone microbenchmark, tools/, not part
// of libdsx).  Each lane hashes NB synthetic bytes held in registers:
//   chain : h = bitop3(alignbit(h), x, y)              (the recurrence alone)
//   mix   : + v_perm address, v_mul_lo prefilter, v_min3 every 2 bytes
//   lds   : mix + the ds_read_b64 table lookup 8 bytes ahead (scanl's layout)
//   lds32 : mix + two ds_read_b32 per lookup (scanm's layout)
// Prints ns per byte-step per SIMD and VALU cycles per byte per SIMD.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_hash.hip -o tools/ubench_hash
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

constexpr int TRIPS = 512;  // trips of 64 bytes

template <int KIND>
__device__ __forceinline__ void k_hash(uint32_t* out, uint32_t seed) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[65536];
  for (int i = threadIdx.x; i < 65536 / 4; i += blockDim.x)
    reinterpret_cast<uint32_t*>(lds)[i] = (uint32_t)i * 2654435761u ^ seed;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t slot8 = (lane & 31u) * 8u, slot4 = (lane & 31u) * 4u;
  uint32_t w[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) w[k] = (threadIdx.x + k) * 0x9E3779B9u ^ seed;
  uint32_t h = seed, ring[48];
#pragma unroll
  for (int k = 0; k < 48; ++k) ring[k] = k * seed;
  uint32_t acc = 0;
  const uint32_t ninv = seed | 1u, thr = 7u;
  uint64_t L[2][8];
  uint64_t L3[3][8];
  uint32_t LT[2][8], LR[2][8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    L[0][q] = L[1][q] = q;
    L3[0][q] = L3[1][q] = L3[2][q] = q;
    LT[0][q] = LT[1][q] = LR[0][q] = LR[1][q] = q;
  }
  for (int t = 0; t < TRIPS; ++t) {
#pragma unroll
    for (int g = 0; g < 8; ++g) {  // 8 subgroups of 8 bytes
      uint32_t tv[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int k = ((g + 1) % 8) * 8 + q;
        const uint32_t sel = 0x0C0C0000u | ((4u + (uint32_t)(k & 3)) << 8);
        uint32_t x, y;
        if constexpr (KIND == 0) {
          x = w[k >> 2];
          y = ring[(g * 8 + q) % 48];
        } else if constexpr (KIND == 1) {
          x = __builtin_amdgcn_perm(w[k >> 2], slot8, sel);
          y = ring[(g * 8 + q) % 48];
          ring[(g * 8 + q) % 48] = x;
        } else if constexpr (KIND == 2) {
          const uint32_t addr = __builtin_amdgcn_perm(w[k >> 2], slot8, sel);
          const uint64_t v = L[g & 1][q];
          L[(g + 1) & 1][q] = *reinterpret_cast<const uint64_t*>(lds + addr);
          x = (uint32_t)v;
          y = ring[(g * 8 + q) % 48];
          ring[(g * 8 + q) % 48] = (uint32_t)(v >> 32);
        } else if constexpr (KIND == 4) {  // lookups two subgroups ahead
          const int k2 = ((g + 2) % 8) * 8 + q;
          const uint32_t sel2 = 0x0C0C0000u | ((4u + (uint32_t)(k2 & 3)) << 8);
          const uint32_t addr = __builtin_amdgcn_perm(w[k2 >> 2], slot8, sel2);
          const uint64_t v = L3[g % 3][q];
          L3[(g + 2) % 3][q] = *reinterpret_cast<const uint64_t*>(lds + addr);
          x = (uint32_t)v;
          y = ring[(g * 8 + q) % 48];
          ring[(g * 8 + q) % 48] = (uint32_t)(v >> 32);
        } else {
          const uint32_t addr = __builtin_amdgcn_perm(w[k >> 2], slot4, sel);
          x = LT[g & 1][q];
          y = ring[(g * 8 + q) % 48];
          ring[(g * 8 + q) % 48] = LR[g & 1][q];
          LT[(g + 1) & 1][q] = *reinterpret_cast<const uint32_t*>(lds + addr);
          LR[(g + 1) & 1][q] = *reinterpret_cast<const uint32_t*>(lds + addr + 128u);
        }
        h = __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_alignbit(h, h, 31), x, y, 0x96);
        tv[q] = h * ninv;
      }
      if constexpr (KIND != 0) {
        uint32_t mn = tv[0];
#pragma unroll
        for (int q = 1; q < 8; ++q) mn = __builtin_elementwise_min(mn, tv[q]);
        if (__builtin_expect(__ballot(mn < thr) != 0, 0)) acc += mn;
      }
      w[g * 2] ^= h;  // keep the row live and changing
    }
  }
  if ((h ^ acc) == 0x12345679u) out[0] = h;
}

template <int KIND, int WPS>
__global__ __launch_bounds__(256 * WPS, 1) void k_run(uint32_t* out, uint32_t seed) {
  k_hash<KIND>(out, seed);
}

template <int KIND, int WPS>
int run(const char* name, uint32_t* d, int ncu) {
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  for (int rep = 0; rep < 2; ++rep) {
    CHK(hipEventRecord(a));
    hipLaunchKernelGGL((k_run<KIND, WPS>), dim3(ncu), dim3(256 * WPS), 0, 0, d, 12345u);
    CHK(hipEventRecord(b));
    CHK(hipEventSynchronize(b));
  }
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, a, b));
  // byte-steps per SIMD: WPS waves x TRIPS x 64 bytes
  const double steps = (double)WPS * TRIPS * 64;
  printf("%-6s wps=%d  %.3f ms  %.3f ns/byte-step/SIMD  (%.2f cycles at 2.1 GHz)\n", name, WPS,
         ms, ms * 1e6 / steps, ms * 1e6 / steps * 2.1);
  return 0;
}

int main() {
  hipDeviceProp_t p;
  CHK(hipGetDeviceProperties(&p, 0));
  const int ncu = p.multiProcessorCount;
  uint32_t* d;
  CHK(hipMalloc(&d, 64));
  run<0, 1>("chain", d, ncu); run<0, 2>("chain", d, ncu); run<0, 3>("chain", d, ncu); run<0, 4>("chain", d, ncu);
  run<1, 1>("mix", d, ncu);   run<1, 2>("mix", d, ncu);   run<1, 3>("mix", d, ncu);   run<1, 4>("mix", d, ncu);
  run<2, 1>("lds", d, ncu);   run<2, 2>("lds", d, ncu);   run<2, 3>("lds", d, ncu);   run<2, 4>("lds", d, ncu);
  run<3, 1>("lds32", d, ncu); run<3, 2>("lds32", d, ncu); run<3, 3>("lds32", d, ncu); run<3, 4>("lds32", d, ncu);
  run<4, 1>("lds_d2", d, ncu); run<4, 2>("lds_d2", d, ncu); run<4, 3>("lds_d2", d, ncu);
  return 0;
}
