// Development probe (the two-thread per-stripe limit): hipHostUnregister waits
// until the whole device is idle.  Do the other ways of moving a 7 MiB pageable range to the GPU
// wait for another thread's work too?  Thread B keeps 256 MiB H2D copies running on its stream
// (or idles); thread A, per round, moves a fresh 7 MiB range of a touched 1 GiB arena by
//   register:  hipHostRegister, hipMemcpyAsync, hipStreamSynchronize, hipHostUnregister
//   pageable:  hipMemcpyAsync straight from the pageable range (the runtime stages or pins it)
//   hsa_lock:  hsa_amd_memory_lock, hipMemcpyAsync, hipStreamSynchronize, hsa_amd_memory_unlock
// timing the pin, the copy and the release.  No kernel touches host memory.  One JSON line per
// (method, B mode); A stops after 150 rounds or 2 s.
// Build: hipcc -O2 -o build/hsa_lock_probe tools/probes/hsa_lock_probe.cpp -lhsa-runtime64 -lpthread
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      fprintf(stderr, "%s: %s line %d\n", #x, hipGetErrorString(e), __LINE__); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)
#define HK(x)                                                      \
  do {                                                             \
    hsa_status_t s = (x);                                          \
    if (s != HSA_STATUS_SUCCESS) {                                 \
      fprintf(stderr, "%s: status %d line %d\n", #x, s, __LINE__); \
      exit(1);                                                     \
    }                                                              \
  } while (0)

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
static double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v.empty() ? 0 : v[v.size() / 2];
}
static double pct(std::vector<double> v, double q) {
  std::sort(v.begin(), v.end());
  return v.empty() ? 0 : v[std::min(v.size() - 1, static_cast<size_t>(q * v.size()))];
}

static hsa_status_t find_gpu(hsa_agent_t agent, void *data) {
  hsa_device_type_t t;
  if (hsa_agent_get_info(agent, HSA_AGENT_INFO_DEVICE, &t) == HSA_STATUS_SUCCESS && t == HSA_DEVICE_TYPE_GPU) {
    *static_cast<hsa_agent_t *>(data) = agent;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}

int main() {
  const size_t big = 256ull << 20, small = 7ull << 20, arena = 1ull << 30;
  CK(hipSetDevice(0));
  char *hb, *db, *ds;
  CK(hipHostMalloc(reinterpret_cast<void **>(&hb), big, hipHostMallocDefault));
  CK(hipMalloc(&db, big));
  CK(hipMalloc(&ds, small));
  char *a = static_cast<char *>(aligned_alloc(4096, arena));
  memset(a, 3, arena);
  HK(hsa_init());  // the runtime HIP already opened: one more reference
  hsa_agent_t gpu{};
  hsa_iterate_agents(find_gpu, &gpu);
  if (!gpu.handle) {
    fprintf(stderr, "no GPU agent\n");
    return 1;
  }
  hipStream_t sa, sb;
  CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
  const char *methods[] = {"register", "pageable", "hsa_lock"};
  size_t round = 0;
  for (int method = 0; method < 3; ++method)
    for (int busy = 0; busy < 2; ++busy) {
      std::atomic<bool> stop{false};
      std::thread tb;
      if (busy)
        tb = std::thread([&] {
          CK(hipSetDevice(0));
          while (!stop.load()) {
            CK(hipMemcpyAsync(db, hb, big, hipMemcpyHostToDevice, sb));
            CK(hipStreamSynchronize(sb));
          }
        });
      std::vector<double> pin, cp, rel, total;
      const double start = now();
      for (int i = 0; i < 150 && now() - start < 2.0; ++i, ++round) {
        char *p = a + (round * small) % (arena - small);
        p = reinterpret_cast<char *>(reinterpret_cast<uintptr_t>(p) & ~uintptr_t(4095));
        const double t0 = now();
        if (method == 0) CK(hipHostRegister(p, small, hipHostRegisterDefault));
        void *agent_ptr = nullptr;
        if (method == 2) HK(hsa_amd_memory_lock(p, small, &gpu, 1, &agent_ptr));
        const double t1 = now();
        CK(hipMemcpyAsync(ds, p, small, hipMemcpyHostToDevice, sa));
        CK(hipStreamSynchronize(sa));
        const double t2 = now();
        if (method == 0) CK(hipHostUnregister(p));
        if (method == 2) HK(hsa_amd_memory_unlock(p));
        const double t3 = now();
        pin.push_back((t1 - t0) * 1e6);
        cp.push_back((t2 - t1) * 1e6);
        rel.push_back((t3 - t2) * 1e6);
        total.push_back((t3 - t0) * 1e6);
      }
      stop = true;
      if (tb.joinable()) tb.join();
      printf("{\"method\": \"%s\", \"other_thread\": \"%s\", \"rounds\": %zu, \"pin_us_p50\": %.1f, \"copy_us_p50\": %.1f, "
             "\"copy_GBps_p50\": %.1f, \"release_us_p50\": %.1f, \"release_us_p90\": %.1f, \"total_us_p50\": %.1f, "
             "\"total_us_p90\": %.1f}\n",
             methods[method], busy ? "256 MiB H2D copies" : "idle", pin.size(), median(pin), median(cp),
             small / (median(cp) * 1e-6) / 1e9, median(rel), pct(rel, 0.9), median(total), pct(total, 0.9));
      fflush(stdout);
    }
  return 0;
}
