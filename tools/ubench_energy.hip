// ubench_energy.hip -- energy per GiB of the scan's staging alternatives
// (VERDICT r03 item 3).  Standalone microbenchmark (tools/, not part of libdsx).
//
// Every variant reads a device buffer with the scan's geometry -- one
// workgroup of 8 waves per CU, a wave owns 64 lane segments of S = 8448 B and
// lane l consumes its own segment in 128-B lines -- and XORs what it receives
// so the loads stay live.  Each variant runs back to back for ~1.5 s while a
// host thread samples board power (hwmon power1_input) every ~4 ms; the line
// printed is time per GiB, median board power, and J/GiB (median power x
// time), idle power subtracted too.
//   A dma_copy    scanl's staging: 8 LDS-DMA (nt) per line into the wave's
//                 8 KiB line buffer, wait, 8 ds_read_b128 of the lane's row;
//   B dma_only    A without the ds_read (the HBM -> L2 -> LDS path alone);
//   C reg_lane    each lane loads its own line, 8 x global_load_dwordx4 nt
//                 straight to VGPRs, the next line in flight (no LDS);
//   D coalesced   a plain coalesced stream (each wave instruction 1 KiB
//                 contiguous), the HBM read floor;
//   A with the other cache policies of the line loads (none, sc1, sc0 sc1 nt).
//   hipcc --offload-arch=gfx950 -O3 tools/ubench_energy.hip -o tools/ubench_energy
//   ./tools/ubench_energy [GiB=8] [seconds=1.5]
#include <hip/hip_runtime.h>
#include <dirent.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <ctype.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <string>
#include <thread>
#include <vector>

#define CHK(x)                                                                   \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      printf("%s: %s\n", #x, hipGetErrorString(e_));                             \
      exit(1);                                                                   \
    }                                                                            \
  } while (0)
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr uint32_t kS = 8448;  // lane segment (scanl's default at 1 GiB)

// 8 LDS-DMA wave instructions, 1 KiB each, M0 stepped by 1 KiB (scanl's DMA8);
// POL: 1 nt (scanl's default), 0 none, 2 sc1, 3 sc0 sc1 nt
#define DMA8(POLSTR)                                                                        \
  asm volatile(                                                                             \
      "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %9\n\ts_nop 0\n\t"                                  \
      "buffer_load_dwordx4 %1, %10, 0 offen " POLSTR "lds\n\ts_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t" \
      "buffer_load_dwordx4 %2, %10, 0 offen " POLSTR "lds\n\ts_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t" \
      "buffer_load_dwordx4 %3, %10, 0 offen " POLSTR "lds\n\ts_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t" \
      "buffer_load_dwordx4 %4, %10, 0 offen " POLSTR "lds\n\ts_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t" \
      "buffer_load_dwordx4 %5, %10, 0 offen " POLSTR "lds\n\ts_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t" \
      "buffer_load_dwordx4 %6, %10, 0 offen " POLSTR "lds\n\ts_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t" \
      "buffer_load_dwordx4 %7, %10, 0 offen " POLSTR "lds\n\ts_add_u32 m0, m0, 0x400\n\ts_nop 0\n\t" \
      "buffer_load_dwordx4 %8, %10, 0 offen " POLSTR "lds\n\ts_mov_b32 m0, %0"               \
      : "=&s"(keep)                                                                         \
      : "v"(vo[0]), "v"(vo[1]), "v"(vo[2]), "v"(vo[3]), "v"(vo[4]), "v"(vo[5]), "v"(vo[6]),  \
        "v"(vo[7]), "s"(lds), "s"(rsrc)                                                     \
      : "memory", "scc")
template <int POL>
__device__ __forceinline__ void dma8(const u32x4& rsrc, const uint32_t (&vo)[8], uint32_t lds) {
  uint32_t keep;
  if constexpr (POL == 1) DMA8("nt ");
  else if constexpr (POL == 2) DMA8("sc1 ");
  else if constexpr (POL == 3) DMA8("sc0 sc1 nt ");
  else DMA8("");
}
#undef DMA8

template <bool COPY, int POL>
__global__ __launch_bounds__(512, 1) void k_dma(const uint8_t* base, uint32_t nregions, uint32_t* out) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[8 * 8192];
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const uint32_t stage = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(__attribute__((address_space(3))) void*)(lds + wave * 8192));
  // instruction i, lane j: 16-B unit u = 64i + j of the 64 x 128 B image: row u/8, chunk u%8
  uint32_t dbase[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint32_t u = i * 64u + lane;
    dbase[i] = (u >> 3) * kS + (u & 7u) * 16u;
  }
  uint32_t acc = 0;
  for (uint32_t region = blockIdx.x * 8 + wave; region < nregions; region += gridDim.x * 8) {
    const uint64_t rp = (uint64_t)(uintptr_t)(base + (uint64_t)region * 64 * kS);
    u32x4 rs;
    rs.x = __builtin_amdgcn_readfirstlane((uint32_t)rp);
    rs.y = __builtin_amdgcn_readfirstlane((uint32_t)(rp >> 32) & 0xFFFFu);
    rs.z = 64u * kS;
    rs.w = 0x00020000u;
    uint32_t vo[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) vo[i] = dbase[i];
    dma8<POL>(rs, vo, stage);
    for (uint32_t b = 0; b < kS / 128; ++b) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if constexpr (COPY) {
        const uint8_t* row = lds + wave * 8192 + lane * 128;
#pragma unroll
        for (int c = 0; c < 8; ++c) {
          const uint4 q = *reinterpret_cast<const uint4*>(row + ((c + (lane >> 1)) & 7) * 16);
          acc ^= q.x ^ q.y ^ q.z ^ q.w;
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
      if (b + 1 < kS / 128) {
#pragma unroll
        for (int i = 0; i < 8; ++i) vo[i] = dbase[i] + (b + 1) * 128u;
        dma8<POL>(rs, vo, stage);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ __launch_bounds__(512, 1) void k_reg(const uint8_t* base, uint32_t nregions, uint32_t* out) {
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  uint32_t acc = 0;
  for (uint32_t region = blockIdx.x * 8 + wave; region < nregions; region += gridDim.x * 8) {
    const u32x4* p = (const u32x4*)(base + ((uint64_t)region * 64 + lane) * kS);
    u32x4 cur[8], nxt[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) cur[c] = __builtin_nontemporal_load(p + c);
    for (uint32_t b = 0; b < kS / 128; ++b) {
      if (b + 1 < kS / 128) {
#pragma unroll
        for (int c = 0; c < 8; ++c) nxt[c] = __builtin_nontemporal_load(p + (b + 1) * 8 + c);
      }
#pragma unroll
      for (int c = 0; c < 8; ++c) acc ^= cur[c].x ^ cur[c].y ^ cur[c].z ^ cur[c].w;
#pragma unroll
      for (int c = 0; c < 8; ++c) cur[c] = nxt[c];
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ void k_coalesced(const u32x4* p, uint64_t n16, uint32_t* out) {
  uint32_t acc = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16;
       i += (uint64_t)gridDim.x * blockDim.x) {
    const u32x4 v = __builtin_nontemporal_load(p + i);
    acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// ---- board power of THIS GPU: the hwmon of HIP device 0's PCI function (the
// box's other GPUs run other jobs: the busiest hwmon is not ours) ----------
struct Sampler {
  std::vector<std::string> files;
  std::vector<std::vector<double>> w;  // per file, watts
  std::atomic<bool> run{false};
  std::thread th;
  Sampler() {
    char bus[64] = {0};
    if (hipDeviceGetPCIBusId(bus, sizeof bus, 0) != hipSuccess) return;
    for (char* p = bus; *p; ++p) *p = (char)tolower(*p);
    std::string hw = std::string("/sys/bus/pci/devices/") + bus + "/hwmon";
    DIR* h = opendir(hw.c_str());
    if (!h) return;
    while (dirent* f = readdir(h))
      if (!strncmp(f->d_name, "hwmon", 5)) files.push_back(hw + "/" + f->d_name + "/power1_input");
    closedir(h);
    printf("power: %s\n", files.empty() ? "(no hwmon)" : files[0].c_str());
  }
  static double read1(const std::string& f) {
    FILE* fp = fopen(f.c_str(), "r");
    if (!fp) return -1;
    double v = -1;
    if (fscanf(fp, "%lf", &v) != 1) v = -1;
    fclose(fp);
    return v / 1e6;
  }
  void start() {
    w.assign(files.size(), {});
    run = true;
    th = std::thread([this] {
      while (run) {
        for (size_t i = 0; i < files.size(); ++i) w[i].push_back(read1(files[i]));
        std::this_thread::sleep_for(std::chrono::milliseconds(4));
      }
    });
  }
  // median of the file with the highest median
  double stop() {
    run = false;
    if (th.joinable()) th.join();
    double best = -1;
    for (auto& v : w) {
      if (v.empty()) continue;
      std::vector<double> s = v;
      std::sort(s.begin(), s.end());
      best = std::max(best, s[s.size() / 2]);
    }
    return best;
  }
};

int main(int argc, char** argv) {
  const uint64_t gib = argc > 1 ? strtoull(argv[1], nullptr, 10) : 8;
  const double secs = argc > 2 ? atof(argv[2]) : 1.5;
  const uint32_t nregions = (uint32_t)((gib << 30) / (64ull * kS));
  const uint64_t len = (uint64_t)nregions * 64 * kS;
  uint8_t* d;
  uint32_t* o;
  CHK(hipMalloc(&d, len + 4096));
  CHK(hipMalloc(&o, 64));
  CHK(hipMemset(d, 0x5A, len));
  // random-ish bytes (a constant buffer could compress on some paths)
  {
    std::vector<uint64_t> h(1 << 20);
    uint64_t x = 88172645463325252ull;
    for (auto& v : h) {
      x ^= x << 13; x ^= x >> 7; x ^= x << 17;
      v = x;
    }
    for (uint64_t off = 0; off < len; off += h.size() * 8)
      CHK(hipMemcpy(d + off, h.data(), std::min<uint64_t>(h.size() * 8, len - off), hipMemcpyHostToDevice));
  }
  CHK(hipDeviceSynchronize());
  Sampler smp;
  std::this_thread::sleep_for(std::chrono::milliseconds(1500));
  smp.start();
  std::this_thread::sleep_for(std::chrono::milliseconds(600));
  const double idle = smp.stop();
  printf("buffer %.2f GiB, lane segment %u B, hwmon files %zu, idle %.1f W\n", len / 1073741824.0, kS,
         smp.files.size(), idle);
  printf("%-16s %9s %9s %8s %8s %9s\n", "variant", "ms/GiB", "TB/s", "W(med)", "J/GiB", "dJ/GiB");
  hipEvent_t e0, e1;
  CHK(hipEventCreate(&e0));
  CHK(hipEventCreate(&e1));
  auto run = [&](const char* name, auto launch) {
    for (int i = 0; i < 3; ++i) launch();
    CHK(hipDeviceSynchronize());
    CHK(hipEventRecord(e0));
    launch();
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms1;
    CHK(hipEventElapsedTime(&ms1, e0, e1));
    const int reps = std::max(4, (int)(secs * 1e3 / ms1));
    smp.start();
    CHK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) launch();
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    const double pw = smp.stop();
    float ms;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    CHK(hipGetLastError());
    const double per_gib = ms / reps / (len / 1073741824.0);
    printf("%-16s %9.4f %9.3f %8.1f %8.3f %9.3f\n", name, per_gib, 1.073741824 / per_gib, pw,
           pw * per_gib / 1e3, (pw - idle) * per_gib / 1e3);
    fflush(stdout);
    std::this_thread::sleep_for(std::chrono::milliseconds(1000));  // cool down between variants
  };
  const int ncu = 256;
  run("dma_copy", [&] { k_dma<true, 1><<<ncu, 512>>>(d, nregions, o); });
  run("dma_only", [&] { k_dma<false, 1><<<ncu, 512>>>(d, nregions, o); });
  run("reg_lane", [&] { k_reg<<<ncu, 512>>>(d, nregions, o); });
  run("coalesced", [&] { k_coalesced<<<ncu * 8, 256>>>((const u32x4*)d, len / 16, o); });
  run("dma_copy_pol0", [&] { k_dma<true, 0><<<ncu, 512>>>(d, nregions, o); });
  run("dma_copy_sc1", [&] { k_dma<true, 2><<<ncu, 512>>>(d, nregions, o); });
  run("dma_copy_sc01nt", [&] { k_dma<true, 3><<<ncu, 512>>>(d, nregions, o); });
  run("dma_copy", [&] { k_dma<true, 1><<<ncu, 512>>>(d, nregions, o); });
  return 0;
}
