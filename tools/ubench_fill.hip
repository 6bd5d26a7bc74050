// ubench_fill.hip -- what scanl_kernel's prologue costs (standalone, tools/):
// the launch of 256 workgroups x 512 threads holding 128 KiB of LDS each,
// (a) empty, (b) + the 64 KiB table fill as scanl_kernel does it (one
// constant-memory load per thread, 16 ds_write_b64), (c) + one line DMA per
// lane and its wait.  Prints the mean of 50 launches each (HIP events).
//   hipcc --offload-arch=gfx950 -O3 -I include tools/ubench_fill.hip -o tools/ubench_fill
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

#include "dsx_buzhash_table.h"

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__constant__ uint32_t cT[256] = DSX_BUZHASH_TABLE_INIT;

template <int KIND>
__global__ __launch_bounds__(512, 1) void k_pro(uint32_t* out, const uint8_t* src) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[65536 + 8 * 8192];
  if constexpr (KIND >= 1) {
    const uint32_t v = threadIdx.x & 255u;
    const uint32_t tv = cT[v];
    uint2 t;
    t.x = tv;
    t.y = __builtin_amdgcn_alignbit(tv, tv, 16);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const uint32_t slot = (threadIdx.x >> 8) + (uint32_t)(k * 2);
      *reinterpret_cast<uint2*>(lds + v * 256u + slot * 8u) = t;
    }
  }
  if constexpr (KIND >= 2) {  // one 128-B line per lane through registers
    const uint4* p = reinterpret_cast<const uint4*>(src + ((uint64_t)blockIdx.x * 512 + threadIdx.x) * 128);
    uint4 acc = p[0];
#pragma unroll
    for (int i = 1; i < 8; ++i) {
      const uint4 q = p[i];
      acc.x ^= q.x; acc.y ^= q.y; acc.z ^= q.z; acc.w ^= q.w;
    }
    *reinterpret_cast<uint4*>(lds + 65536 + (threadIdx.x & 511u) * 16) = acc;
  }
  __syncthreads();
  if (threadIdx.x == 0 && lds[blockIdx.x & 65535] == 0x5A && lds[(blockIdx.x * 7) & 65535] == 0xA5)
    out[blockIdx.x] = 1u;
}

template <int KIND>
int run(const char* name, uint32_t* d, const uint8_t* src, int ncu) {
  hipEvent_t a, b;
  CHK(hipEventCreate(&a));
  CHK(hipEventCreate(&b));
  for (int w = 0; w < 5; ++w) hipLaunchKernelGGL((k_pro<KIND>), dim3(ncu), dim3(512), 0, 0, d, src);
  CHK(hipEventRecord(a));
  for (int i = 0; i < 50; ++i) hipLaunchKernelGGL((k_pro<KIND>), dim3(ncu), dim3(512), 0, 0, d, src);
  CHK(hipEventRecord(b));
  CHK(hipEventSynchronize(b));
  float ms = 0;
  CHK(hipEventElapsedTime(&ms, a, b));
  printf("%-28s %.2f us per launch\n", name, ms * 1000.0f / 50);
  return 0;
}

int main() {
  hipDeviceProp_t p;
  CHK(hipGetDeviceProperties(&p, 0));
  const int ncu = p.multiProcessorCount;
  uint32_t* d;
  uint8_t* src;
  CHK(hipMalloc(&d, 4 * ncu));
  CHK(hipMalloc(&src, (size_t)ncu * 512 * 128));
  CHK(hipMemset(src, 1, (size_t)ncu * 512 * 128));
  run<0>("empty (LDS 128 KiB)", d, src, ncu);
  run<1>("+ table fill", d, src, ncu);
  run<2>("+ table fill + one line/lane", d, src, ncu);
  return 0;
}
