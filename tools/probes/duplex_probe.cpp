// Development probe: does PCIe carry H2D and D2H at full rate at the same time? (VERDICT r04 item 4:
// host-path encodes move k*C in while the previous batch's m*C come out.)  hipMemcpyAsync of
// `bytes` on two non-blocking streams, one direction each, alone and together, from hipHostMalloc
// memory and from a hipHostRegister'ed malloc arena; one JSON line per case.
// Build: hipcc -O2 -o build/duplex_probe tools/probes/duplex_probe.cpp
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

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

int main(int argc, char **argv) {
  const size_t bytes = (argc > 1 ? strtoull(argv[1], nullptr, 10) : 512) << 20;
  const int reps = 5;
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  char *d1, *d2;
  CK(hipMalloc(&d1, bytes));
  CK(hipMalloc(&d2, bytes));
  for (int kind = 0; kind < 2; ++kind) {
    char *h1, *h2;
    void *raw1 = nullptr, *raw2 = nullptr;
    if (kind == 0) {
      CK(hipHostMalloc(reinterpret_cast<void **>(&h1), bytes, hipHostMallocDefault));
      CK(hipHostMalloc(reinterpret_cast<void **>(&h2), bytes, hipHostMallocDefault));
    } else {
      raw1 = aligned_alloc(4096, bytes);
      raw2 = aligned_alloc(4096, bytes);
      h1 = static_cast<char *>(raw1);
      h2 = static_cast<char *>(raw2);
      memset(h1, 1, bytes);
      memset(h2, 2, bytes);
      CK(hipHostRegister(h1, bytes, hipHostRegisterDefault));
      CK(hipHostRegister(h2, bytes, hipHostRegisterDefault));
    }
    double best[3] = {1e9, 1e9, 1e9};
    for (int r = 0; r <= reps; ++r) {
      for (int mode = 0; mode < 3; ++mode) {  // 0 H2D alone, 1 D2H alone, 2 both
        CK(hipDeviceSynchronize());
        const double t0 = now();
        if (mode != 1) CK(hipMemcpyAsync(d1, h1, bytes, hipMemcpyHostToDevice, s1));
        if (mode != 0) CK(hipMemcpyAsync(h2, d2, bytes, hipMemcpyDeviceToHost, s2));
        CK(hipStreamSynchronize(s1));
        CK(hipStreamSynchronize(s2));
        const double t = now() - t0;
        if (r > 0) best[mode] = std::min(best[mode], t);
      }
    }
    printf("{\"host\": \"%s\", \"bytes\": %zu, \"h2d_alone_GBps\": %.2f, \"d2h_alone_GBps\": %.2f, "
           "\"both_each_GBps\": %.2f, \"both_total_GBps\": %.2f}\n",
           kind == 0 ? "hipHostMalloc" : "hipHostRegister", bytes, bytes / best[0] / 1e9, bytes / best[1] / 1e9,
           bytes / best[2] / 1e9, 2 * bytes / best[2] / 1e9);
    fflush(stdout);
    if (kind == 0) {
      CK(hipHostFree(h1));
      CK(hipHostFree(h2));
    } else {
      CK(hipHostUnregister(h1));
      CK(hipHostUnregister(h2));
      free(raw1);
      free(raw2);
    }
  }
  return 0;
}
