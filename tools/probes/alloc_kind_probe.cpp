// Development probe: what tells a caller's hipHostMalloc allocation from a range the caller
// hipHostRegister'ed?  (the engine keeps kernel transport for the first and moves the second by
// DMA only, DESIGN.md "Caller page-locked memory")  Prints one JSON line per allocation kind with
// every attribute the runtime answers for an interior pointer.
// Build: hipcc -O2 -o build/alloc_kind_probe tools/probes/alloc_kind_probe.cpp
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

static void report(const char *kind, char *base, size_t bytes) {
  char *p = base + bytes / 2 + 4096 + 16;  // an interior pointer, as a chunk of a cache page
  hipPointerAttribute_t a;
  std::memset(&a, 0, sizeof(a));
  const hipError_t ra = hipPointerGetAttributes(&a, p);
  if (ra != hipSuccess) (void)hipGetLastError();
  unsigned flags = 0xFFFFFFFFu;
  const hipError_t rf = hipHostGetFlags(&flags, p);
  if (rf != hipSuccess) (void)hipGetLastError();
  unsigned flags_base = 0xFFFFFFFFu;
  const hipError_t rfb = hipHostGetFlags(&flags_base, base);
  if (rfb != hipSuccess) (void)hipGetLastError();
  void *dptr = nullptr;
  const hipError_t rd = hipHostGetDevicePointer(&dptr, p, 0);
  if (rd != hipSuccess) (void)hipGetLastError();
  hipDeviceptr_t rbase = nullptr;
  size_t rsize = 0;
  const hipError_t rr = hipMemGetAddressRange(&rbase, &rsize, reinterpret_cast<hipDeviceptr_t>(p));
  if (rr != hipSuccess) (void)hipGetLastError();
  unsigned long long buffer_id = 0;
  const hipError_t rb = hipPointerGetAttribute(&buffer_id, HIP_POINTER_ATTRIBUTE_BUFFER_ID, reinterpret_cast<hipDeviceptr_t>(p));
  if (rb != hipSuccess) (void)hipGetLastError();
  int mapped = -1;
  const hipError_t rm = hipPointerGetAttribute(&mapped, HIP_POINTER_ATTRIBUTE_MAPPED, reinterpret_cast<hipDeviceptr_t>(p));
  if (rm != hipSuccess) (void)hipGetLastError();
  unsigned access = 0;
  const hipError_t rac = hipPointerGetAttribute(&access, HIP_POINTER_ATTRIBUTE_ACCESS_FLAGS, reinterpret_cast<hipDeviceptr_t>(p));
  if (rac != hipSuccess) (void)hipGetLastError();
  // cost of the candidate queries (the per-chunk check runs them on the per-stripe path)
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < 10000; ++i) {
    unsigned f = 0;
    if (hipHostGetFlags(&f, p) != hipSuccess) (void)hipGetLastError();
  }
  const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / 1e4;
  printf("{\"kind\": \"%s\", \"attr_rc\": %d, \"type\": %d, \"device\": %d, \"dev_eq_host\": %d, \"hostPointer_eq\": %d, "
         "\"isManaged\": %d, \"allocationFlags\": \"0x%x\", \"getflags_rc\": %d, \"getflags\": \"0x%x\", "
         "\"getflags_base_rc\": %d, \"getflags_base\": \"0x%x\", \"getdevptr_rc\": %d, \"getdevptr_eq_host\": %d, "
         "\"range_rc\": %d, \"range_base_eq\": %d, \"range_size\": %zu, \"buffer_id_rc\": %d, \"buffer_id\": %llu, "
         "\"mapped_rc\": %d, \"mapped\": %d, \"access_rc\": %d, \"access\": %u, \"getflags_us\": %.3f}\n",
         kind, static_cast<int>(ra), static_cast<int>(a.type), a.device, a.devicePointer == p,
         a.hostPointer == p, a.isManaged, a.allocationFlags, static_cast<int>(rf), flags, static_cast<int>(rfb), flags_base,
         static_cast<int>(rd), dptr == p, static_cast<int>(rr), reinterpret_cast<char *>(rbase) == base, rsize,
         static_cast<int>(rb), buffer_id, static_cast<int>(rm), mapped, static_cast<int>(rac), access, us);
  fflush(stdout);
}

int main() {
  const size_t n = 8u << 20;
  struct HM {
    const char *name;
    unsigned flags;
  } hm[] = {{"hostmalloc_default", hipHostMallocDefault},
            {"hostmalloc_coherent", hipHostMallocCoherent},
            {"hostmalloc_noncoherent", hipHostMallocNonCoherent},
            {"hostmalloc_portable_mapped", hipHostMallocPortable | hipHostMallocMapped},
            {"hostmalloc_writecombined", hipHostMallocWriteCombined}};
  for (const HM &k : hm) {
    char *h = nullptr;
    if (hipHostMalloc(reinterpret_cast<void **>(&h), n, k.flags) != hipSuccess) {
      (void)hipGetLastError();
      printf("{\"kind\": \"%s\", \"alloc\": \"failed\"}\n", k.name);
      continue;
    }
    report(k.name, h, n);
    (void)hipHostFree(h);
  }
  struct HR {
    const char *name;
    unsigned flags;
  } hr[] = {{"register_default", hipHostRegisterDefault},
            {"register_mapped", hipHostRegisterMapped},
            {"register_portable_mapped", hipHostRegisterPortable | hipHostRegisterMapped}};
  for (const HR &k : hr) {
    char *h = static_cast<char *>(mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0));
    std::memset(h, 1, n);
    if (hipHostRegister(h, n, k.flags) != hipSuccess) {
      (void)hipGetLastError();
      printf("{\"kind\": \"%s\", \"register\": \"failed\"}\n", k.name);
      munmap(h, n);
      continue;
    }
    report(k.name, h, n);
    (void)hipHostUnregister(h);
    munmap(h, n);
  }
  {  // a malloc'd (heap) buffer registered at an unaligned start, as numpy arrays are
    char *raw = static_cast<char *>(malloc(n + 4096));
    char *h = raw + 64;
    std::memset(raw, 1, n + 4096);
    if (hipHostRegister(h, n, 0) == hipSuccess) {
      report("register_malloc_unaligned", h, n);
      (void)hipHostUnregister(h);
    } else {
      (void)hipGetLastError();
      printf("{\"kind\": \"register_malloc_unaligned\", \"register\": \"failed\"}\n");
    }
    free(raw);
  }
  {  // pageable, for reference
    char *h = static_cast<char *>(malloc(n));
    std::memset(h, 1, n);
    report("pageable", h, n);
    free(h);
  }
  {
    char *d = nullptr;
    if (hipMalloc(reinterpret_cast<void **>(&d), n) == hipSuccess) {
      report("device", d, n);
      (void)hipFree(d);
    }
  }
  return 0;
}
