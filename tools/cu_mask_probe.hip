// Which physical CUs does a CU-masked stream use?  For each mask variant, a
// spinning probe kernel (many small workgroups) records XCC_ID and HW_ID
// (SE / SH / CU) of every workgroup; the host prints the CUs each XCC gets.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <set>
#include <tuple>
#include <vector>

__global__ void probe(unsigned* out, unsigned long long spin) {
  unsigned xcc, hwid;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < spin) __builtin_amdgcn_s_sleep(2);
  if (threadIdx.x == 0) {
    out[2 * blockIdx.x] = xcc;
    out[2 * blockIdx.x + 1] = hwid;
  }
}

int main(int argc, char** argv) {
  hipDeviceProp_t prop;
  hipGetDeviceProperties(&prop, 0);
  const int ncu = prop.multiProcessorCount;
  const int nb = 8192;
  unsigned* d;
  hipMalloc(&d, 2 * nb * sizeof(unsigned));
  std::vector<unsigned> h(2 * nb);
  // variants: all bits; the last 8 bits cleared; bits {0..7} cleared; every
  // 32nd bit cleared; single bits 0..15 cleared
  std::vector<std::pair<const char*, std::vector<int>>> variants = {
      {"all", {}}, {"clear 248..255", {248, 249, 250, 251, 252, 253, 254, 255}},
      {"clear 0..7", {0, 1, 2, 3, 4, 5, 6, 7}}, {"clear k*32+31", {31, 63, 95, 127, 159, 191, 223, 255}}};
  for (int b = 0; b < 16; ++b) variants.push_back({"single", {b}});
  for (auto& v : variants) {
    std::vector<unsigned> mask((ncu + 31) / 32, 0u);
    for (int i = 0; i < ncu; ++i) mask[i / 32] |= 1u << (i % 32);
    for (int b : v.second) mask[b / 32] &= ~(1u << (b % 32));
    hipStream_t s;
    if (hipExtStreamCreateWithCUMask(&s, (unsigned)mask.size(), mask.data()) != hipSuccess) {
      printf("mask create failed\n");
      return 1;
    }
    hipMemsetAsync(d, 0xFF, 2 * nb * sizeof(unsigned), s);
    hipLaunchKernelGGL(probe, dim3(nb), dim3(64), 0, s, d, 2000ull);  // 20 us each
    hipStreamSynchronize(s);
    hipMemcpy(h.data(), d, 2 * nb * sizeof(unsigned), hipMemcpyDeviceToHost);
    std::set<std::tuple<unsigned, unsigned, unsigned, unsigned>> cus;  // xcc, se, sh, cu
    for (int i = 0; i < nb; ++i) {
      const unsigned x = h[2 * i], w = h[2 * i + 1];
      cus.insert({x, (w >> 13) & 7u, (w >> 12) & 1u, (w >> 8) & 15u});
    }
    int per[8] = {};
    for (auto& t : cus) per[std::get<0>(t) & 7]++;
    printf("%-16s", v.first);
    if (!v.second.empty() && v.second.size() == 1) printf(" bit %3d:", v.second[0]);
    else printf("        :");
    printf(" total %3zu  per-XCC", cus.size());
    for (int x = 0; x < 8; ++x) printf(" %2d", per[x]);
    if (v.second.size() == 1) {  // which CU vanished
      static std::set<std::tuple<unsigned, unsigned, unsigned, unsigned>> all;
      if (all.empty()) {
        // recompute the full set once
      }
    }
    printf("\n");
    if (std::string(v.first) == "all") {
      printf("  (xcc,se,sh,cu) sample:");
      int k = 0;
      for (auto& t : cus) {
        if (k++ >= 40) break;
        printf(" (%u,%u,%u,%u)", std::get<0>(t), std::get<1>(t), std::get<2>(t), std::get<3>(t));
      }
      printf("\n");
    }
    hipStreamDestroy(s);
  }
  return 0;
}
