// tools/probes/xcd_balance.hip -- do the 8 XCDs finish the headline's tiles together?
// (the RS(6+3) 1 MiB encode runs at 0.76 of 8 TB/s on some fresh allocations,
// 0.80-0.83 on others, and the slow ones show more DRAM credit stalls.)
//
// The engine's bytewise kernel deals each XCD a contiguous eighth of the tiles (xcd_remap).  If
// the physical pages behind one eighth are slower, that XCD finishes last and the others idle.
// This probe runs the encode's memory shape (6 data shards in, 3 parity shards out per stripe,
// 8 KiB tiles, non-temporal, XOR instead of GF arithmetic) over fresh allocations and records
// every workgroup's end time (s_memrealtime, 100 MHz), then reports per XCD when its last
// workgroup ended.  Modes 1 and 2 run the same tiles from persistent workgroups that take tiles
// from their own XCD's eighth through a per-XCD atomic counter; in mode 2 they then help the other
// XCDs, so a slow eighth is shared out; its time on the same allocations is the A/B.
// Build: hipcc -O3 --offload-arch=gfx950 -o build/xcd_balance tools/probes/xcd_balance.hip
// Run:   build/xcd_balance [trials=8] [stripes=4096]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define G __attribute__((address_space(1)))

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      fprintf(stderr, "%s: %s line %d\n", #x, hipGetErrorString(e), __LINE__); \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

constexpr int K = 6, R = 3, BS = 256, IT = 2;
constexpr int64_t TILE = (int64_t)BS * 16 * IT;  // 8 KiB per shard

struct Args {
  uint64_t in, out;  // data [N][K][C], parity [N][R][C]
  int64_t C;
  uint32_t ntiles, per_xcd;  // tiles, tiles in each XCD's eighth (the last may hold fewer)
  unsigned long long *stamp;  // per workgroup (static) / per tile (dynamic): end time
  unsigned *ctr;              // dynamic: next tile of each eighth, one 128-B line each
};

__device__ __forceinline__ void do_tile(const Args &a, uint32_t t) {
  const uint32_t tps = (uint32_t)(a.C / TILE);
  const uint32_t s = t / tps;
  const int64_t off = (int64_t)(t - s * tps) * TILE + threadIdx.x * 16;
  u32x4 v[K][IT];
#pragma unroll
  for (int j = 0; j < K; ++j)
#pragma unroll
    for (int it = 0; it < IT; ++it)
      v[j][it] = __builtin_nontemporal_load((const G u32x4 *)(a.in + ((int64_t)s * K + j) * a.C + off + it * BS * 16));
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int it = 0; it < IT; ++it) {
      u32x4 acc = v[r][it];
#pragma unroll
      for (int j = 0; j < K; ++j)
        if (j != r) acc ^= v[j][it];
      __builtin_nontemporal_store(acc, (G u32x4 *)(a.out + ((int64_t)s * R + r) * a.C + off + it * BS * 16));
    }
}

// static: one tile per workgroup, each XCD's blocks (b, b+8, ...) on a contiguous eighth
__global__ __launch_bounds__(BS) void k_static(Args a) {
  const uint32_t b = blockIdx.x, xcd = b & 7;
  const uint32_t t = xcd * a.per_xcd + (b >> 3);
  if (t < a.ntiles && (b >> 3) < a.per_xcd) do_tile(a, t);
  __syncthreads();
  if (threadIdx.x == 0) a.stamp[b] = __builtin_amdgcn_s_memrealtime();
}

// dynamic: persistent workgroups; own eighth first, then (steal = 1) the others'
__global__ __launch_bounds__(BS) void k_dynamic(Args a, int steal) {
  __shared__ uint32_t next;
  const uint32_t xcd = blockIdx.x & 7;
  for (uint32_t k = 0; k < (steal ? 8u : 1u); ++k) {
    const uint32_t e = (xcd + k) & 7;
    const uint32_t lo = e * a.per_xcd, hi = min(a.ntiles, lo + a.per_xcd);
    for (;;) {
      if (threadIdx.x == 0) next = lo + atomicAdd(a.ctr + 32 * e, 1u);
      __syncthreads();
      // readfirstlane: the tile index, and so the loop's exit, is wave-uniform
      const uint32_t t = __builtin_amdgcn_readfirstlane(next);
      if (t >= hi) break;
      do_tile(a, t);
      if (threadIdx.x == 0) a.stamp[t] = __builtin_amdgcn_s_memrealtime() | ((unsigned long long)xcd << 60);
      // every wave has read `next` before thread 0 overwrites it; the barrier also closes the
      // divergent stores above before the back edge (with the barriers placed around the read
      // instead, the structurizer put one on a path thread 0 skipped, and the launch hung)
      __syncthreads();
    }
  }
}

int main(int argc, char **argv) {
  const int trials = argc > 1 ? atoi(argv[1]) : 8;
  const int N = argc > 2 ? atoi(argv[2]) : 4096;
  const int64_t C = 1 << 20;
  const uint32_t tps = (uint32_t)(C / TILE), ntiles = tps * N, per = (ntiles + 7) / 8;
  hipDeviceProp_t prop;
  CK(hipGetDeviceProperties(&prop, 0));
  const int nwg_dyn = prop.multiProcessorCount * 8;  // 8 x 256-thread workgroups per CU
  unsigned long long *stamp;
  unsigned *ctr;
  CK(hipMalloc(&stamp, sizeof(unsigned long long) * ntiles));
  CK(hipMalloc(&ctr, 8 * 128));
  std::vector<unsigned long long> h(ntiles);
  for (int trial = 0; trial < trials; ++trial) {
    void *spacer = nullptr;
    CK(hipMalloc(&spacer, (size_t)((trial * 37) % 11 + 1) << 28));
    void *din, *dout;
    CK(hipMalloc(&din, (size_t)N * K * C));
    CK(hipMalloc(&dout, (size_t)N * R * C));
    CK(hipFree(spacer));
    CK(hipMemset(din, 0x5a, (size_t)N * K * C));
    Args a{(uint64_t)din, (uint64_t)dout, C, ntiles, per, stamp, ctr};
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    for (int mode = 0; mode < 3; ++mode) {
      fprintf(stderr, "trial %d mode %d\n", trial, mode);
      float best = 1e9f, sum = 0.f;
      const int reps = 5;
      for (int rep = 0; rep <= reps; ++rep) {
        CK(hipMemset(ctr, 0, 8 * 128));
        unsigned long long t0 = 0;
        CK(hipEventRecord(e0, 0));
        if (mode == 0)
          k_static<<<per * 8, BS>>>(a);
        else
          k_dynamic<<<nwg_dyn, BS>>>(a, mode == 2);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (rep == 0) continue;  // first launch: cold parity pages
        best = std::min(best, ms);
        sum += ms;
        if (rep == reps) {
          // per-XCD finish, relative to the earliest end of any workgroup
          const size_t n = mode == 0 ? (size_t)per * 8 : ntiles;
          CK(hipMemcpy(h.data(), stamp, sizeof(unsigned long long) * n, hipMemcpyDeviceToHost));
          unsigned long long first = ~0ull, last[8] = {0}, tiles[8] = {0};
          for (size_t i = 0; i < n; ++i) {
            const unsigned long long v = h[i] & ((1ull << 60) - 1);
            const int x = mode == 0 ? (int)(i & 7) : (int)(h[i] >> 60);
            first = std::min(first, v);
            last[x] = std::max(last[x], v);
            ++tiles[x];
          }
          (void)t0;
          printf("{\"trial\": %d, \"mode\": \"%s\", \"din_mib\": %llu, \"ms_mean\": %.4f, \"ms_best\": %.4f, \"frac\": %.4f, "
                 "\"xcd_last_end_us\": [",
                 trial, mode == 0 ? "static" : mode == 1 ? "own-eighth" : "stealing", (unsigned long long)((uintptr_t)din >> 20), sum / reps, best,
                 (double)N * (K + R) * C / (sum / reps / 1e3) / 8e12);
          for (int x = 0; x < 8; ++x) printf("%s%.1f", x ? ", " : "", (last[x] - first) / 100.0);
          printf("], \"xcd_tiles\": [");
          for (int x = 0; x < 8; ++x) printf("%s%llu", x ? ", " : "", tiles[x]);
          printf("]}\n");
          fflush(stdout);
        }
      }
    }
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    CK(hipFree(din));
    CK(hipFree(dout));
  }
  return 0;
}
