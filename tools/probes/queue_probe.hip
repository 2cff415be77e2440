// tools/probes/queue_probe.hip -- development probe (not product code): does a long-running
// kernel on one stream delay work on other streams (streams share GPU_MAX_HW_QUEUES hardware
// queues, whose packets run in order)?  Compared for a plain stream, a high-priority stream and
// a CU-masked stream (hipExtStreamCreateWithCUMask) as the parked kernel's stream.
// The parked kernel is bounded: it spins on the 100 MHz wall clock for a fixed time.
//   hipcc -O2 --offload-arch=gfx950 -o build/queue_probe tools/probes/queue_probe.hip
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <vector>

#define CK(x)                                                                     \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s: %s (line %d)\n", #x, hipGetErrorString(e_), __LINE__); \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

__global__ void k_park(unsigned long long ticks) {  // wall_clock64 runs at 100 MHz
  const unsigned long long t0 = wall_clock64();
  while (wall_clock64() - t0 < ticks) __builtin_amdgcn_s_sleep(10);
}
__global__ void k_empty() {}

static double now_ms() {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void trial(const char *name, hipStream_t parked) {
  std::vector<hipStream_t> others(12);
  for (auto &s : others) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipLaunchKernelGGL(k_park, 1, 64, 0, parked, 20000000ull);  // 200 ms
  const double t0 = now_ms();
  int blocked = 0;
  printf("%-22s", name);
  for (size_t i = 0; i < others.size(); ++i) {
    const double a = now_ms();
    hipLaunchKernelGGL(k_empty, 1, 64, 0, others[i]);
    CK(hipStreamSynchronize(others[i]));
    const double dt = now_ms() - a;
    blocked += dt > 50;
    printf(" %6.1f", dt);
  }
  CK(hipStreamSynchronize(parked));
  printf("  | blocked %d of %zu, park took %.1f ms\n", blocked, others.size(), now_ms() - t0);
  for (auto &s : others) CK(hipStreamDestroy(s));
}

int main() {
  CK(hipSetDevice(0));
  hipLaunchKernelGGL(k_empty, 1, 64, 0, nullptr);
  CK(hipDeviceSynchronize());
  hipStream_t plain, hi, masked, masked_all;
  CK(hipStreamCreateWithFlags(&plain, hipStreamNonBlocking));
  trial("plain stream", plain);
  int lo = 0, hip_hi = 0;
  CK(hipDeviceGetStreamPriorityRange(&lo, &hip_hi));
  CK(hipStreamCreateWithPriority(&hi, hipStreamNonBlocking, hip_hi));
  trial("high-priority stream", hi);
  std::vector<uint32_t> mask(8, 0u);  // 256 CUs: 8 words
  mask[0] = 0x0000FFFFu;              // CUs 0..15
  CK(hipExtStreamCreateWithCUMask(&masked, static_cast<uint32_t>(mask.size()), mask.data()));
  trial("CU-masked (16 CUs)", masked);
  std::vector<uint32_t> all(8, 0xFFFFFFFFu);
  CK(hipExtStreamCreateWithCUMask(&masked_all, static_cast<uint32_t>(all.size()), all.data()));
  trial("CU-masked (all CUs)", masked_all);
  printf("probe ok\n");
  return 0;
}
