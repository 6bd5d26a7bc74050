// Do streams share hardware queues in the IndexFromFile call's shape?
// The library's context touches the null stream at creation (hipMemset), then
// uses its scan stream and copy stream; a one-window IndexFromFile call adds
// the feeder's stream and the window-digest stream.  With GPU_MAX_HW_QUEUES=4
// (the box's setting) a fifth stream must share an HSA queue with another one,
// and a kernel on a shared queue waits for the kernel ahead of it (in-order
// packets with the barrier bit).  Here: a 20 ms one-workgroup spin on the
// last stream created, then 20 short kernels on each other stream; the host
// prints how long each stream's short kernels took to drain.  A stream that
// drains in ~20 ms sits on the spinning stream's queue.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

__global__ void spin(unsigned* out, unsigned long long ticks) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < ticks) __builtin_amdgcn_s_sleep(8);
  if (threadIdx.x == 0) out[blockIdx.x] = 1u;
}

__global__ void tick(unsigned* out) {
  if (threadIdx.x == 0) out[blockIdx.x] += 1u;
}

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e_ = (x);                                               \
    if (e_ != hipSuccess) {                                            \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));          \
      return 1;                                                        \
    }                                                                  \
  } while (0)

int main(int argc, char** argv) {
  const int nstreams = argc > 1 ? atoi(argv[1]) : 4;
  const bool touch_null = argc > 2 ? atoi(argv[2]) != 0 : true;
  const char* q = getenv("GPU_MAX_HW_QUEUES");
  unsigned* d;
  CK(hipMalloc(&d, 4096 * sizeof(unsigned)));
  if (touch_null) CK(hipMemset(d, 0, 4096 * sizeof(unsigned)));  // as dsx_create does
  // prio 1: the last stream at the lowest priority; 2: also the first at the
  // highest (ROCclr keeps a queue pool per priority)
  const int prio = argc > 3 ? atoi(argv[3]) : 0;
  // idle: streams created first (at the default priority) and never used, as
  // torch's stream pool creates 32 at once; do they take queues?
  const int idle = argc > 4 ? atoi(argv[4]) : 0;
  // prio 3: every measured stream at the highest priority
  std::vector<hipStream_t> pool(idle);
  for (auto& x : pool) CK(hipStreamCreateWithFlags(&x, hipStreamNonBlocking));
  int least = 0, greatest = 0;
  CK(hipDeviceGetStreamPriorityRange(&least, &greatest));
  std::vector<hipStream_t> s(nstreams);
  for (int i = 0; i < nstreams; ++i) {
    if (prio == 3)
      CK(hipStreamCreateWithPriority(&s[i], hipStreamNonBlocking, greatest));
    else if (prio >= 1 && i == nstreams - 1)
      CK(hipStreamCreateWithPriority(&s[i], hipStreamNonBlocking, least));
    else if (prio >= 2 && i == 0)
      CK(hipStreamCreateWithPriority(&s[i], hipStreamNonBlocking, greatest));
    else
      CK(hipStreamCreateWithFlags(&s[i], hipStreamNonBlocking));
  }
  // first use of every stream, in creation order (queues are taken at first use)
  for (auto& x : s) hipLaunchKernelGGL(tick, dim3(1), dim3(64), 0, x, d);
  CK(hipDeviceSynchronize());
  // memrealtime runs at 100 MHz: 20 ms = 2,000,000 ticks
  const unsigned long long ticks = 2000000ull;
  printf("{\"GPU_MAX_HW_QUEUES\": \"%s\", \"streams\": %d, \"null_touched\": %d, \"prio\": %d, \"idle\": %d, \"drain_ms\": [",
         q ? q : "", nstreams, (int)touch_null, prio, idle);
  for (int victim = 0; victim < nstreams; ++victim) {
    // spin on the victim stream, then short kernels on each other stream
    hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, s[victim], d + 1024, ticks);
    const double t0 = now_ms();
    std::vector<double> drain(nstreams, 0.0);
    for (int i = 0; i < nstreams; ++i) {
      if (i == victim) continue;
      for (int k = 0; k < 20; ++k) hipLaunchKernelGGL(tick, dim3(1), dim3(64), 0, s[i], d + 64 * i);
    }
    for (int left = nstreams - 1; left > 0;) {  // poll: each stream's own drain time
      for (int i = 0; i < nstreams; ++i) {
        if (i == victim || drain[i] > 0) continue;
        const hipError_t e = hipStreamQuery(s[i]);
        if (e == hipSuccess) {
          drain[i] = now_ms() - t0;
          --left;
        } else if (e != hipErrorNotReady) {
          CK(e);
        }
      }
      if (now_ms() - t0 > 5000) {
        fprintf(stderr, "probe: streams did not drain in 5 s\n");
        return 1;
      }
    }
    CK(hipStreamSynchronize(s[victim]));
    printf("%s[", victim ? ", " : "");
    for (int i = 0; i < nstreams; ++i) printf("%s%.2f", i ? ", " : "", drain[i]);
    printf("]");
  }
  printf("]}\n");
  for (auto& x : s) CK(hipStreamDestroy(x));
  for (auto& x : pool) CK(hipStreamDestroy(x));
  CK(hipFree(d));
  return 0;
}
