// Development probe: does hipHostUnregister (or hipHostRegister) wait for
// work another thread has in flight on its own stream?  Thread B keeps a 256 MiB H2D copy (about
// 4.7 ms) running on its stream; thread A registers a 7 MiB pageable range, copies it H2D on its
// stream, synchronises that stream and unregisters, timing each step.  Then the same with B idle.
// A stops after 200 rounds or 3 s.  One JSON line per case; per-round times on stderr.
// Build: hipcc -O2 -o build/unregister_wait_probe tools/probes/unregister_wait_probe.cpp -lpthread
#include <hip/hip_runtime.h>

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

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v.empty() ? 0 : v[v.size() / 2];
}

int main() {
  const size_t big = 256ull << 20, small = 7ull << 20;
  const int iters = 200;
  char *hb;
  CK(hipHostMalloc(reinterpret_cast<void **>(&hb), big, hipHostMallocDefault));
  char *db, *ds;
  CK(hipMalloc(&db, big));
  CK(hipMalloc(&ds, small));
  // A's ranges: a 1 GiB pageable arena walked 7 MiB at a time, every page touched
  const size_t arena = 1ull << 30;
  char *a = static_cast<char *>(aligned_alloc(4096, arena));
  memset(a, 3, arena);
  hipStream_t sa, sb;
  CK(hipStreamCreateWithFlags(&sa, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&sb, hipStreamNonBlocking));
  // B's modes: 0 idle; 1 copy + hipStreamSynchronize; 2 copy + spin on hipStreamQuery;
  // 3 copy + hipEventSynchronize on an event recorded after it
  const char *names[] = {"idle", "copies, hipStreamSynchronize", "copies, spin on hipStreamQuery",
                         "copies, hipEventSynchronize"};
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  for (int mode = 0; mode < 4; ++mode) {
    std::atomic<bool> stop{false};
    std::thread tb;
    if (mode)
      tb = std::thread([&] {
        CK(hipSetDevice(0));
        while (!stop.load()) {
          CK(hipMemcpyAsync(db, hb, big, hipMemcpyHostToDevice, sb));
          if (mode == 1) CK(hipStreamSynchronize(sb));
          if (mode == 2)
            while (hipStreamQuery(sb) == hipErrorNotReady) {
            }
          if (mode == 3) {
            CK(hipEventRecord(ev, sb));
            CK(hipEventSynchronize(ev));
          }
        }
      });
    std::vector<double> reg, cp, unreg;
    const double start = now();
    for (int i = 0; i < iters && now() - start < 3.0; ++i) {
      char *p = a + (static_cast<size_t>(i) * small) % (arena - small);
      p = reinterpret_cast<char *>(reinterpret_cast<uintptr_t>(p) & ~uintptr_t(4095));
      const double t0 = now();
      CK(hipHostRegister(p, small, hipHostRegisterDefault));
      const double t1 = now();
      CK(hipMemcpyAsync(ds, p, small, hipMemcpyHostToDevice, sa));
      CK(hipStreamSynchronize(sa));
      const double t2 = now();
      CK(hipHostUnregister(p));
      const double t3 = now();
      reg.push_back((t1 - t0) * 1e6);
      cp.push_back((t2 - t1) * 1e6);
      unreg.push_back((t3 - t2) * 1e6);
      fprintf(stderr, "mode %d iter %d reg %.0f copy %.0f unreg %.0f us\n", mode, i, (t1 - t0) * 1e6, (t2 - t1) * 1e6,
              (t3 - t2) * 1e6);
    }
    stop = true;
    if (tb.joinable()) tb.join();
    printf("{\"other_thread\": \"%s\", \"iters\": %zu, \"register_us_p50\": %.1f, \"copy_sync_us_p50\": %.1f, "
           "\"unregister_us_p50\": %.1f, \"register_us_max\": %.1f, \"unregister_us_max\": %.1f}\n",
           names[mode], reg.size(), median(reg), median(cp), median(unreg),
           reg.empty() ? 0 : *std::max_element(reg.begin(), reg.end()),
           unreg.empty() ? 0 : *std::max_element(unreg.begin(), unreg.end()));
    fflush(stdout);
  }
  return 0;
}
