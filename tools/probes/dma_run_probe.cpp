// Development probe: what does a single-stripe host decode pay to move its chunks by DMA instead
// of packing them?  For pageable caller memory registered per call
// (InPlacePin's mechanism) and for hipHostMalloc memory:
//   register / unregister cost of a run, H2D and D2H time of runs of 256 KiB .. 6 MiB on one
//   stream, and six 1 MiB H2D runs issued back to back (a 1 MiB RS(6+3) stripe's survivors).
// Prints one JSON line per measurement (median of reps, microseconds).
// Build: hipcc -O2 -o build/dma_run_probe tools/probes/dma_run_probe.cpp
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static double median(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return v[v.size() / 2];
}

int main() {
  const size_t kMax = 8u << 20;
  const int reps = 40;
  hipStream_t st;
  hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
  char *dev = nullptr;
  hipMalloc(reinterpret_cast<void **>(&dev), kMax);
  // pageable arena, 4x the LLC-ish working set so runs are not cache-hot
  const size_t arena = 512u << 20;
  char *pg = static_cast<char *>(aligned_alloc(4096, arena));
  std::memset(pg, 7, arena);
  char *pinned = nullptr;
  hipHostMalloc(reinterpret_cast<void **>(&pinned), kMax, hipHostMallocDefault);
  std::memset(pinned, 7, kMax);
  const size_t sizes[] = {256u << 10, 1u << 20, 5u << 20, 6u << 20};
  size_t at = 0;
  auto next = [&](size_t n) {
    if (at + n > arena) at = 0;
    char *p = pg + at;
    at += (n + 4095) & ~size_t(4095);
    return p;
  };
  for (size_t n : sizes) {
    std::vector<double> reg, unreg, h2d, d2h, h2d_pin, d2h_pin;
    for (int r = 0; r < reps; ++r) {
      char *p = next(n);
      double t0 = now_us();
      if (hipHostRegister(p, n, hipHostRegisterPortable | hipHostRegisterMapped) != hipSuccess) {
        printf("{\"error\": \"register\"}\n");
        return 1;
      }
      double t1 = now_us();
      hipMemcpyAsync(dev, p, n, hipMemcpyHostToDevice, st);
      hipStreamSynchronize(st);
      double t2 = now_us();
      hipMemcpyAsync(p, dev, n, hipMemcpyDeviceToHost, st);
      hipStreamSynchronize(st);
      double t3 = now_us();
      hipHostUnregister(p);
      double t4 = now_us();
      reg.push_back(t1 - t0);
      h2d.push_back(t2 - t1);
      d2h.push_back(t3 - t2);
      unreg.push_back(t4 - t3);
      t0 = now_us();
      hipMemcpyAsync(dev, pinned, n, hipMemcpyHostToDevice, st);
      hipStreamSynchronize(st);
      t1 = now_us();
      hipMemcpyAsync(pinned, dev, n, hipMemcpyDeviceToHost, st);
      hipStreamSynchronize(st);
      t2 = now_us();
      h2d_pin.push_back(t1 - t0);
      d2h_pin.push_back(t2 - t1);
    }
    printf("{\"bytes\": %zu, \"register_us\": %.1f, \"unregister_us\": %.1f, \"h2d_registered_us\": %.1f, "
           "\"d2h_registered_us\": %.1f, \"h2d_hostmalloc_us\": %.1f, \"d2h_hostmalloc_us\": %.1f, "
           "\"h2d_registered_gbps\": %.1f, \"h2d_hostmalloc_gbps\": %.1f}\n",
           n, median(reg), median(unreg), median(h2d), median(d2h), median(h2d_pin), median(d2h_pin),
           n / median(h2d) / 1e3, n / median(h2d_pin) / 1e3);
    fflush(stdout);
  }
  {  // a 1 MiB stripe's survivors: register one 5 MiB run + one 1 MiB run, six 1 MiB DMAs, one kernel-free D2H
    std::vector<double> tot, dma_only;
    for (int r = 0; r < reps; ++r) {
      char *d5 = next(6u << 20);
      char *p1 = next(1u << 20);
      char *o1 = next(1u << 20);
      double t0 = now_us();
      hipHostRegister(d5, 5u << 20, hipHostRegisterPortable | hipHostRegisterMapped);
      hipHostRegister(p1, 1u << 20, hipHostRegisterPortable | hipHostRegisterMapped);
      hipHostRegister(o1, 1u << 20, hipHostRegisterPortable | hipHostRegisterMapped);
      double t1 = now_us();
      for (int j = 0; j < 5; ++j) hipMemcpyAsync(dev + (size_t(j) << 20), d5 + (size_t(j) << 20), 1u << 20, hipMemcpyHostToDevice, st);
      hipMemcpyAsync(dev + (5u << 20), p1, 1u << 20, hipMemcpyHostToDevice, st);
      hipMemcpyAsync(o1, dev + (6u << 20), 1u << 20, hipMemcpyDeviceToHost, st);
      hipStreamSynchronize(st);
      double t2 = now_us();
      hipHostUnregister(d5);
      hipHostUnregister(p1);
      hipHostUnregister(o1);
      double t3 = now_us();
      tot.push_back(t3 - t0);
      dma_only.push_back(t2 - t1);
    }
    printf("{\"case\": \"1MiB RS(6+3) decode transfers: 3 registrations, 6 x 1 MiB H2D + 1 MiB D2H\", \"total_us\": %.1f, "
           "\"dma_us\": %.1f, \"data_gibps_if_total\": %.1f}\n",
           median(tot), median(dma_only), (6.0 * (1 << 20)) / median(tot) * 1e6 / (1 << 30));
  }
  return 0;
}
