// Does a GPU kernel reading host memory through a hipHostRegister device alias see the pages the
// process has NOW, after the same virtual range was registered, unregistered, unmapped and mapped
// again (new physical pages)?  A stale registration would show the old contents.
//   hipcc --offload-arch=gfx950 -O2 -o build/reg_reuse_probe tools/probes/reg_reuse_probe.hip
#include <hip/hip_runtime.h>
#include <sys/mman.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>

__global__ void k_sum(const unsigned *p, size_t n, unsigned long long *out) {
  unsigned long long s = 0;
  for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) s += p[i];
  atomicAdd(out, s);
}
__global__ void k_fill(unsigned *p, size_t n, unsigned v) {
  for (size_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) p[i] = v;
}

int main(int argc, char **argv) {
  const size_t bytes = (argc > 1 ? atol(argv[1]) : 8) << 20, n = bytes / 4;
  const int iters = argc > 2 ? atoi(argv[2]) : 50;
  unsigned long long *dsum;
  hipMalloc(&dsum, 8);
  int bad_read = 0, bad_write = 0;
  void *fixed = nullptr;
  for (int it = 0; it < iters; ++it) {
    // map (at the same address every time after the first), fill on the CPU, register, read on the GPU
    void *h = mmap(fixed, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | (fixed ? MAP_FIXED : 0), -1, 0);
    if (h == MAP_FAILED) { perror("mmap"); return 1; }
    fixed = h;
    unsigned *u = static_cast<unsigned *>(h);
    const unsigned v = 1000u + it;
    for (size_t i = 0; i < n; ++i) u[i] = v;
    if (hipHostRegister(h, bytes, hipHostRegisterPortable | hipHostRegisterMapped) != hipSuccess) { printf("register failed\n"); return 1; }
    void *d = nullptr;
    hipHostGetDevicePointer(&d, h, 0);
    hipMemset(dsum, 0, 8);
    k_sum<<<256, 256>>>(static_cast<unsigned *>(d), n, dsum);
    // and a GPU write of the next value, read back on the CPU
    k_fill<<<256, 256>>>(static_cast<unsigned *>(d), n, v + 1000000u);
    hipDeviceSynchronize();
    unsigned long long s = 0;
    hipMemcpy(&s, dsum, 8, hipMemcpyDeviceToHost);
    if (s != static_cast<unsigned long long>(v) * n) ++bad_read;
    size_t wrong = 0;
    for (size_t i = 0; i < n; ++i) wrong += u[i] != v + 1000000u;
    if (wrong) ++bad_write;
    if ((s != static_cast<unsigned long long>(v) * n || wrong) && bad_read + bad_write < 6)
      printf("iter %d: gpu read sum %llu (want %llu, device ptr %p host %p), %zu words not written\n", it, s,
             static_cast<unsigned long long>(v) * n, d, h, wrong);
    hipHostUnregister(h);
    munmap(h, bytes);  // the next iteration maps new pages at the same address
  }
  printf("{\"bytes\": %zu, \"iters\": %d, \"stale_reads\": %d, \"lost_writes\": %d}\n", bytes, iters, bad_read, bad_write);
  return 0;
}
