// Development probe: can the host path verify, per chunk, that a caller's buffer is page-locked
// and find its device alias cheaply?  (needed before caller-pinned small runs may move by kernel)
// Build: hipcc -O2 -o tools/probes/pinned_attr_probe tools/probes/pinned_attr_probe.cpp
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

int main() {
  const size_t n = 1ull << 30, chunk = 64 << 10, count = n / chunk;
  char *h = nullptr;
  if (hipHostMalloc(reinterpret_cast<void **>(&h), n, hipHostMallocDefault) != hipSuccess) return 1;
  char *pg = static_cast<char *>(malloc(n));
  size_t identity = 0, pinned = 0;
  auto t0 = std::chrono::steady_clock::now();
  for (size_t i = 0; i < count; ++i) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, h + i * chunk) != hipSuccess) continue;
    pinned += a.type == hipMemoryTypeHost;
    identity += a.devicePointer == h + i * chunk;
  }
  auto t1 = std::chrono::steady_clock::now();
  size_t pg_pinned = 0;
  for (size_t i = 0; i < count; ++i) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, pg + i * chunk) != hipSuccess) {
      (void)hipGetLastError();
      continue;
    }
    pg_pinned += a.type == hipMemoryTypeHost;
  }
  auto t2 = std::chrono::steady_clock::now();
  hipDeviceptr_t base = 0;
  size_t size = 0;
  const hipError_t r = hipMemGetAddressRange(&base, &size, reinterpret_cast<hipDeviceptr_t>(h + 12345 * 16));
  const double us1 = std::chrono::duration<double, std::micro>(t1 - t0).count() / count;
  const double us2 = std::chrono::duration<double, std::micro>(t2 - t1).count() / count;
  printf("hipHostMalloc 1 GiB, %zu interior 64 KiB chunk pointers: %.3f us/query, host-typed %zu, devicePointer==host %zu\n",
         count, us1, pinned, identity);
  printf("pageable malloc, same count: %.3f us/query, host-typed %zu (must be 0)\n", us2, pg_pinned);
  printf("hipMemGetAddressRange(interior pinned ptr): rc %d, base==h %d, size %zu\n", static_cast<int>(r),
         reinterpret_cast<char *>(base) == h, size);
  (void)hipHostFree(h);
  free(pg);
  return 0;
}
