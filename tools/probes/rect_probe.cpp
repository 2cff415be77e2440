// Development probe: per-copy cost of the pinned-DMA host path (round 5, c5 host lows).  The
// engine moves a hipHostRegister'ed batch laid out [stripe][k+m][C] as one hipMemcpyAsync per
// stripe (k*C in, m*C out).  Compare, for H2D of the k data chunks and D2H of the m parity chunks
// of n stripes: one copy per stripe, one hipMemcpy2DAsync over all stripes, and one contiguous copy
// of the same byte count (the link's ceiling).  Also both directions at once (stripe copies on two
// streams, as the pipeline runs them).  One JSON line per case.
// Build: hipcc -O2 -o build/rect_probe tools/probes/rect_probe.cpp
// Run:   build/rect_probe k m chunk_bytes n
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
  const size_t k = argc > 1 ? atoi(argv[1]) : 8, m = argc > 2 ? atoi(argv[2]) : 3;
  const size_t C = argc > 3 ? strtoull(argv[3], nullptr, 10) : (512 << 10);
  const size_t n = argc > 4 ? atoi(argv[4]) : 256;
  const size_t pitch = (k + m) * C, hbytes = n * pitch;
  char *h = static_cast<char *>(aligned_alloc(4096, hbytes));
  memset(h, 7, hbytes);
  CK(hipHostRegister(h, hbytes, hipHostRegisterDefault));
  char *din, *dout;
  CK(hipMalloc(&din, n * k * C));
  CK(hipMalloc(&dout, n * m * C));
  hipStream_t s1, s2;
  CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
  CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  const int reps = 5;
  const char *names[] = {"h2d per-stripe", "h2d 2d", "h2d contiguous", "d2h per-stripe", "d2h 2d",
                         "d2h contiguous", "both per-stripe", "both 2d"};
  for (int mode = 0; mode < 8; ++mode) {
    double best = 1e9;
    for (int r = 0; r <= reps; ++r) {
      CK(hipDeviceSynchronize());
      const double t0 = now();
      const bool in = mode < 3 || mode >= 6, out = (mode >= 3 && mode < 6) || mode >= 6;
      const int kind = mode >= 6 ? mode - 6 : mode % 3;  // 0 per-stripe, 1 2d, 2 contiguous
      if (in) {
        if (kind == 0)
          for (size_t s = 0; s < n; ++s) CK(hipMemcpyAsync(din + s * k * C, h + s * pitch, k * C, hipMemcpyHostToDevice, s1));
        else if (kind == 1)
          CK(hipMemcpy2DAsync(din, k * C, h, pitch, k * C, n, hipMemcpyHostToDevice, s1));
        else
          CK(hipMemcpyAsync(din, h, n * k * C, hipMemcpyHostToDevice, s1));
      }
      if (out) {
        if (kind == 0)
          for (size_t s = 0; s < n; ++s)
            CK(hipMemcpyAsync(h + s * pitch + k * C, dout + s * m * C, m * C, hipMemcpyDeviceToHost, s2));
        else if (kind == 1)
          CK(hipMemcpy2DAsync(h + k * C, pitch, dout, m * C, m * C, n, hipMemcpyDeviceToHost, s2));
        else
          CK(hipMemcpyAsync(h, dout, n * m * C, hipMemcpyDeviceToHost, s2));
      }
      CK(hipStreamSynchronize(s1));
      CK(hipStreamSynchronize(s2));
      const double t = now() - t0;
      if (r > 0) best = std::min(best, t);
    }
    const bool in = mode < 3 || mode >= 6, out = (mode >= 3 && mode < 6) || mode >= 6;
    const double inb = in ? double(n * k * C) : 0, outb = out ? double(n * m * C) : 0;
    printf("{\"case\": \"%s\", \"k\": %zu, \"m\": %zu, \"chunk\": %zu, \"stripes\": %zu, \"ms\": %.3f, "
           "\"h2d_GBps\": %.2f, \"d2h_GBps\": %.2f}\n",
           names[mode], k, m, C, n, best * 1e3, inb / best / 1e9, outb / best / 1e9);
    fflush(stdout);
  }
  CK(hipHostUnregister(h));
  free(h);
  return 0;
}
