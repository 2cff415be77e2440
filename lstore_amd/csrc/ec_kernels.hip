// ec_kernels.hip -- host-side launch policy for the gfx950 erasure kernels
// (device code: ec_kernels_impl.h, instantiated per R in ec_kernels_inst.hip).
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <type_traits>

#include "ec_hiperr.h"
#include "ec_kernels_impl.h"

namespace lsec {

namespace {

int g_bw_variant = 0, g_bs_variant = 0;

int default_grid(uint64_t ntiles) {
  // One tile per block: on this streaming pattern a full grid beat every grid-stride
  // size from 2 to 16 blocks per CU by 5-7% (tools/kprobe.hip).
  return static_cast<int>(std::min<uint64_t>(std::max<uint64_t>(ntiles, 1), (1ull << 31) - 1));
}

constexpr int kQueueDevs = 64;
std::once_flag g_queue_once[kQueueDevs];
unsigned *g_queue[kQueueDevs];
std::atomic<uint32_t> g_queue_next[kQueueDevs];
struct SlotState {
  std::atomic<int> busy{0};  // taken by a launch that has not recorded its event yet
  hipEvent_t ev = nullptr;   // recorded after the slot's last launch
};
SlotState *g_slots[kQueueDevs];
int g_cus[kQueueDevs];

// tile mode: 0 static eighths, 1 all tiles shared, 2 a static prefix and a shared tail
std::atomic<int> g_tiles_mode{-1};  // -1: not read from LSEC_TILES yet

int tiles_mode() {
  int v = g_tiles_mode.load(std::memory_order_relaxed);
  if (v < 0) {
    const char *e = getenv("LSEC_TILES");
    const int want = !e ? 2 : std::strcmp(e, "static") == 0 ? 0 : std::strcmp(e, "shared") == 0 ? 1 : 2;
    g_tiles_mode.compare_exchange_strong(v, want);
    v = g_tiles_mode.load(std::memory_order_relaxed);
  }
  return v;
}

bool tiles_shared() { return tiles_mode() != 0; }

// the static prefix's share of each eighth, in 1/64ths (LSEC_TILES_PRE_64THS, A/B runs)
uint32_t prefix_64ths() {
  static const uint32_t v = [] {
    const char *e = getenv("LSEC_TILES_PRE_64THS");
    const long x = e ? atol(e) : 56;
    return static_cast<uint32_t>(std::max(0L, std::min(64L, x)));
  }();
  return v;
}

template <typename F>
hipError_t by_r(int R, F f) {
  switch (R) {
    case 1: return f(std::integral_constant<int, 1>());
    case 2: return f(std::integral_constant<int, 2>());
    case 3: return f(std::integral_constant<int, 3>());
    case 4: return f(std::integral_constant<int, 4>());
    case 5: return f(std::integral_constant<int, 5>());
    case 6: return f(std::integral_constant<int, 6>());
    case 7: return f(std::integral_constant<int, 7>());
    case 8: return f(std::integral_constant<int, 8>());
    default: return hipErrorInvalidValue;
  }
}

// Launch shape for a K x R bytewise launch (codes in ec_kernels_impl.h).  variant 0 = the
// automatic policy measured with tools/kbench.py (profiles/r01_v6_kbench_branchfree.txt,
// r01_v10_kbench_xorrow.txt):
//   R == 1 (single-erasure decode: XOR-heavy, read-bound)  8 B per lane, branchy cells
//   K >= 16 (VALU-bound wide codes)                          16 B per lane, branch-free: 2 x 16 B
//                                                            needs 256 VGPRs there (1 wave/SIMD);
//                                                            RS 20+6 67 %, 16+4 79 % vs 51 / 63 %
//   otherwise                                                2 x 16 B per lane, branch-free
int bytewise_shape(int K, int R) {
  if (g_bw_variant > 0) return (g_bw_variant - 1) % kBwShapes;
  if (R == 1) return 4;
  return K >= 16 ? 1 : 0;
}

// the device of stream st (the current device for the null stream), or -1
int stream_device(hipStream_t st) {
  int dev = -1;
  if (quiet([&] { return st ? hipStreamGetDevice(st, &dev) : hipGetDevice(&dev); }) != hipSuccess) return -1;
  return dev;
}

}  // namespace

namespace {
std::atomic<unsigned long long *> g_stamps{nullptr};
std::atomic<uint32_t> g_nstamps{0};
}  // namespace

unsigned long long *launch_stamps(uint32_t *n) {
  *n = g_nstamps.load(std::memory_order_relaxed);
  return g_stamps.load(std::memory_order_relaxed);
}

void set_launch_stamps(unsigned long long *p, uint32_t n) {
  g_nstamps.store(p ? n : 0, std::memory_order_relaxed);
  g_stamps.store(p, std::memory_order_relaxed);
}

unsigned *tile_queue_slot(hipStream_t st, uint64_t ntiles) {
  // small launches (a stripe or a few) keep the static eighths: one tile per block, no counters
  if (!tiles_shared() || ntiles < kTileQueueMinTiles) return nullptr;
  const int dev = stream_device(st);
  if (dev < 0 || dev >= kQueueDevs) return nullptr;
  std::call_once(g_queue_once[dev], [dev] {
    const size_t bytes = sizeof(unsigned) * kTileQueueWords * kTileQueueRing;
    void *p = nullptr;
    int cus = 0;
    // On st's device, which need not be the calling thread's current one.  One quiet() call does
    // the switch, the allocation, the clear and the switch back, so all of it runs on one thread:
    // with a caller's error pending quiet() runs its call on the helper thread, and a device
    // switched there would not be the one a later quiet() call allocates on.
    const hipError_t e = quiet([&] {
      int cur = -1;
      hipError_t r = hipGetDevice(&cur);
      if (r != hipSuccess) return r;
      if (cur != dev && (r = hipSetDevice(dev)) != hipSuccess) return r;
      r = hipMalloc(&p, bytes);
      if (r == hipSuccess) r = hipMemset(p, 0, bytes);
      if (r == hipSuccess) r = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
      if (r != hipSuccess && p) {
        (void)hipFree(p);
        p = nullptr;
      }
      if (cur != dev) {
        const hipError_t back = hipSetDevice(cur);
        if (r == hipSuccess) r = back;
      }
      return r;
    });
    if (e != hipSuccess || cus <= 0 || !p) {
      if (p) (void)quiet([&] { return hipFree(p); });
      return;
    }
    g_cus[dev] = cus;
    g_slots[dev] = new SlotState[kTileQueueRing];  // kept for the process's life, as the queue
    g_queue[dev] = static_cast<unsigned *>(p);
  });
  if (!g_queue[dev]) return nullptr;
  // a slot no launch still holds: not one between its taking and its event (busy), and not one
  // whose last launch has yet to finish (its event; normally long done, a ring later)
  SlotState *slots = g_slots[dev];
  for (int tries = 0; tries < kTileQueueRing; ++tries) {
    const uint32_t i = g_queue_next[dev].fetch_add(1, std::memory_order_relaxed) % kTileQueueRing;
    if (slots[i].busy.exchange(1, std::memory_order_acquire) != 0) continue;
    if (slots[i].ev && quiet([&] { return hipEventSynchronize(slots[i].ev); }) != hipSuccess) {
      slots[i].busy.store(0, std::memory_order_release);
      return nullptr;
    }
    return g_queue[dev] + static_cast<size_t>(i) * kTileQueueWords;
  }
  return nullptr;
}

void tile_queue_release(hipStream_t st, unsigned *slot) {
  if (!slot) return;
  const int dev = stream_device(st);
  if (dev < 0 || dev >= kQueueDevs || !g_queue[dev]) return;
  SlotState &ss = g_slots[dev][(slot - g_queue[dev]) / kTileQueueWords];
  if (!ss.ev && quiet([&] { return hipEventCreateWithFlags(&ss.ev, hipEventDisableTiming); }) != hipSuccess) ss.ev = nullptr;
  // (an event that failed to record keeps its earlier state; the slot's launch was queued on st)
  if (ss.ev && quiet([&] { return hipEventRecord(ss.ev, st); }) != hipSuccess) {
    (void)quiet([&] { return hipStreamSynchronize(st); });
  }
  ss.busy.store(0, std::memory_order_release);
}

namespace {
// bit 0: the tile loops of launch_tiled's kernels, bit 1: the compiled networks; -1: not read from
// LSEC_TILE_PHASE yet (unset: 1, the measured default -- RS(8+4) at 4-8 MiB +1.1-1.7 %, every other
// shape level, the networks level or -0.6 %: profiles/r06_v7_tile_phase_ab.txt,
// r06_v10_tile_phase_mem_mode_ab.txt)
std::atomic<int> g_tile_phase{-1};

int tile_phase_mode() {
  int v = g_tile_phase.load(std::memory_order_relaxed);
  if (v < 0) {
    const char *e = getenv("LSEC_TILE_PHASE");
    v = e && *e ? (atoi(e) & 3) : 1;
    int expect = -1;
    if (!g_tile_phase.compare_exchange_strong(expect, v)) v = expect;
  }
  return v;
}
}  // namespace

bool tile_phase_on() { return (tile_phase_mode() & 1) != 0; }
bool tile_phase_net_on() { return (tile_phase_mode() & 2) != 0; }

void set_tile_phase(int mode) { g_tile_phase.store(mode & 3, std::memory_order_relaxed); }

size_t occupancy_lds_bytes(int64_t shard_bytes) {
  static const int cap = [] {
    const char *e = getenv("LSEC_WGS_CAP");
    return e ? std::max(0, atoi(e)) : 0;
  }();
  static const int64_t min_bytes = [] {
    const char *e = getenv("LSEC_WGS_CAP_MIN_KB");
    return e ? static_cast<int64_t>(atoll(e)) << 10 : 0;
  }();
  if (cap <= 0 || shard_bytes < min_bytes) return 0;
  // 160 KiB of LDS per CU; 2 KiB left for the kernels' own static LDS
  const size_t per = (160u << 10) / static_cast<size_t>(cap);
  return per > (2u << 10) ? (per - (2u << 10)) & ~static_cast<size_t>(255) : 0;
}

int persistent_grid(const void *kernel, int grid, hipStream_t st) {
  const int dev = stream_device(st);
  if (dev < 0 || dev >= kQueueDevs || g_cus[dev] <= 0) return 0;
  static std::mutex mu;
  static std::map<const void *, int> per_cu;  // resident workgroups per CU, by kernel
  int n = 0;
  {
    std::lock_guard<std::mutex> lk(mu);
    auto it = per_cu.find(kernel);
    if (it != per_cu.end()) {
      n = it->second;
    } else {
      if (quiet([&] { return hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, kernel, kBlock, 0); }) != hipSuccess) n = 0;
      per_cu[kernel] = n;
    }
  }
  // LSEC_TILES_WGS overrides the workgroups per CU (A/B runs)
  static const int force = [] {
    const char *e = getenv("LSEC_TILES_WGS");
    return e ? atoi(e) : 0;
  }();
  if (force > 0) n = force;
  static const int cap = [] {  // LSEC_WGS_CAP (occupancy_lds_bytes): no more persistent blocks than fit
    const char *e = getenv("LSEC_WGS_CAP");
    return e ? std::max(0, atoi(e)) : 0;
  }();
  if (cap > 0 && n > cap) n = cap;
  if (n <= 0) return 0;
  // a multiple of 8: every XCD the same number of workgroups (blocks are dealt round-robin)
  const int full = n * g_cus[dev];
  const int pg = std::max(8, std::min(grid, full) & ~7);
  static const bool trace = getenv("LSEC_TRACE") != nullptr;
  if (trace) fprintf(stderr, "[lsec tiles] kernel %p: %d workgroups per CU x %d CUs -> grid %d (of %d tiles)\n", kernel, n, g_cus[dev], pg, grid);
  return pg;
}

void set_tile_mode(int mode) { g_tiles_mode.store(std::max(0, std::min(2, mode)), std::memory_order_relaxed); }

int tile_mode() { return tiles_mode(); }

uint32_t tiles_prefix(uint32_t ntiles) {
  if (tiles_mode() != 2) return 0;
  const uint64_t per = (static_cast<uint64_t>(ntiles) + 7) / 8;
  return static_cast<uint32_t>(per * prefix_64ths() / 64);
}

void set_kernel_variant(int bw, int bs) {
  g_bw_variant = bw;
  g_bs_variant = bs;
}

int bytewise_variant() { return g_bw_variant; }
int bitsliced_variant() { return g_bs_variant; }

hipError_t launch_bytewise(const ApplyArgs &a, hipStream_t st, int grid_blocks) {
  if (a.K < 1 || a.K > kMaxK || a.R < 1 || a.R > 8 || a.size % 8 != 0) return hipErrorInvalidValue;
  if (a.nstripes <= 0 || a.size == 0) return hipSuccess;
  const int shape = a.accumulate ? 1 : bytewise_shape(a.K, a.R);  // as dispatch_bytewise's accumulate launch
  const uint64_t tile = static_cast<uint64_t>(kBlock) * 4 * bw_shape_vw(shape) * bw_shape_it(shape);
  const uint64_t ntiles = ((a.size + tile - 1) / tile) * static_cast<uint64_t>(a.nstripes);
  if (ntiles >= (1ull << 31)) return hipErrorInvalidValue;
  const int grid = grid_blocks > 0 ? grid_blocks : default_grid(ntiles);
  return by_r(a.R, [&](auto r) { return dispatch_bytewise<decltype(r)::value>(a, st, grid, shape); });
}

hipError_t launch_bytewise_magic(const ApplyArgs &a, hipStream_t st, int grid_blocks) {
  if (a.K < 1 || a.K > kMaxK || a.R < 1 || a.R > 8 || a.size % 8 != 0 || !a.magic_acc) return hipErrorInvalidValue;
  if (a.nstripes <= 0 || a.size == 0) return hipSuccess;
  const uint64_t tile = static_cast<uint64_t>(kBlock) * 16 * (a.K >= 16 ? 1 : 2);  // dispatch_bytewise_magic's IT
  const uint64_t ntiles = ((a.size + tile - 1) / tile) * static_cast<uint64_t>(a.nstripes);
  if (ntiles >= (1ull << 31)) return hipErrorInvalidValue;
  const int grid = grid_blocks > 0 ? grid_blocks : default_grid(ntiles);
  return by_r(a.R, [&](auto r) { return dispatch_bytewise_magic<decltype(r)::value>(a, st, grid); });
}

hipError_t launch_bitsliced(const ApplyArgs &a, hipStream_t st, int grid_blocks, int dw_pref) {
  if (a.K < 1 || a.K > kMaxK || a.R < 1 || a.R > 8 || a.packet <= 0 || a.packet % 4 != 0 ||
      a.size % (8LL * a.packet) != 0)
    return hipErrorInvalidValue;
  if (a.nstripes <= 0 || a.size == 0) return hipSuccess;
  // dwords per lane: the A/B variant when one is set, else the caller's preference (1, 2, 4), else 1
  const int want = g_bs_variant != 0 ? g_bs_variant : dw_pref;
  int dw = (want == 2 || want == 4) && !a.magic_acc && !a.accumulate ? want : 1;
  while (dw > 1 && a.packet % (4 * dw) != 0) dw >>= 1;
  const uint64_t col_bytes = a.size / 8;
  const uint64_t tile = kBlock * 4ull * dw;
  const uint64_t ntiles = ((col_bytes + tile - 1) / tile) * static_cast<uint64_t>(a.nstripes);
  if (ntiles >= (1ull << 31)) return hipErrorInvalidValue;
  const int grid = grid_blocks > 0 ? grid_blocks : default_grid(ntiles);
  return by_r(a.R, [&](auto r) { return dispatch_bitsliced<decltype(r)::value>(a, st, grid, dw); });
}

bool bitmatrix_w_supported(int w) {
  switch (w) {
#define LSEC_BM_CASE(WW) case WW:
    LSEC_BITMATRIX_W(LSEC_BM_CASE)
#undef LSEC_BM_CASE
    return true;
    default:
      return false;
  }
}

hipError_t launch_bitmatrix(const ApplyArgs &a, hipStream_t st, int grid_blocks) {
  if (a.K < 1 || a.K > kMaxK || a.R < 1 || a.R > 2 || a.w < 2 || a.w > kMaxW || !a.masks ||
      a.packet <= 0 || a.packet % 4 != 0 || a.size % (static_cast<int64_t>(a.w) * a.packet) != 0)
    return hipErrorInvalidValue;
  if (a.nstripes <= 0 || a.size == 0) return hipSuccess;
  const uint64_t col_bytes = a.size / a.w;
  const uint64_t ntiles = ((col_bytes + kBlock * 4 - 1) / (kBlock * 4)) * static_cast<uint64_t>(a.nstripes);
  if (ntiles >= (1ull << 31)) return hipErrorInvalidValue;
  const int grid = grid_blocks > 0 ? grid_blocks : default_grid(ntiles);
  return by_r(a.R, [&](auto r) { return dispatch_bitmatrix<decltype(r)::value>(a, st, grid); });
}

hipError_t launch_wordwise(const ApplyArgs &a, hipStream_t st, int grid_blocks) {
  if (a.K < 1 || a.K > kMaxK || a.R < 1 || a.R > 8 || (a.w != 16 && a.w != 32) || !a.masks || a.size % 8 != 0)
    return hipErrorInvalidValue;
  if (a.nstripes <= 0 || a.size == 0) return hipSuccess;
  // transposed bit-sliced kernel (4*w bytes per lane) up to 8 rows at w = 16 and 4 at w = 32;
  // the mask-per-bit kernel (16 / 8 bytes per lane) beyond that
  // (lsec_set_kernel_variant's second argument 10 selects the mask-per-bit kernel: A/B runs)
  const bool transposed = g_bs_variant != 10 && (a.w == 16 || a.R <= 4);
  const uint64_t tile = kBlock * (transposed ? 4ull * a.w : a.w == 16 ? 16ull : 8ull);
  const uint64_t ntiles = ((a.size + tile - 1) / tile) * static_cast<uint64_t>(a.nstripes);
  if (ntiles >= (1ull << 31)) return hipErrorInvalidValue;
  const int grid = grid_blocks > 0 ? grid_blocks : default_grid(ntiles);
  if (transposed) return by_r(a.R, [&](auto r) { return dispatch_gfw_transposed<decltype(r)::value>(a, st, grid); });
  return by_r(a.R, [&](auto r) { return dispatch_wordwise<decltype(r)::value>(a, st, grid); });
}

hipError_t launch_gfw_bitsliced(const ApplyArgs &a, hipStream_t st, int grid_blocks) {
  if (a.K < 1 || a.K > kMaxK || a.R < 1 || a.R > (a.w == 32 ? 4 : 8) || (a.w != 16 && a.w != 32) || !a.masks ||
      a.packet <= 0 || a.packet % 4 != 0 || a.size % (static_cast<int64_t>(a.w) * a.packet) != 0)
    return hipErrorInvalidValue;
  if (a.nstripes <= 0 || a.size == 0) return hipSuccess;
  const uint64_t col_bytes = a.size / a.w;
  const uint64_t ntiles = ((col_bytes + kBlock * 4 - 1) / (kBlock * 4)) * static_cast<uint64_t>(a.nstripes);
  if (ntiles >= (1ull << 31)) return hipErrorInvalidValue;
  const int grid = grid_blocks > 0 ? grid_blocks : default_grid(ntiles);
  return by_r(a.R, [&](auto r) { return dispatch_gfw_bitsliced<decltype(r)::value>(a, st, grid); });
}

// ------------------------------------------------------------------ stripe magic (adler32)
namespace {

// one block per (stripe, 8 KiB column tile); each lane reads 16 B x 2 of every shard
__global__ __launch_bounds__(kBlock) void k_stripe_magic(MagicArgs a) {
  __shared__ uint32_t red[kBlock / 64];
  constexpr int kIt = 2, kTile = kBlock * 16 * kIt;
  const int64_t C = a.size;
  const uint32_t tps = static_cast<uint32_t>((C + kTile - 1) / kTile);
  const uint32_t ntiles = tps * static_cast<uint32_t>(a.nstripes);
  const uint64_t L = static_cast<uint64_t>(a.total_shards ? a.total_shards : a.nshards) * a.chunk;
  for (uint32_t t = xcd_remap(blockIdx.x, gridDim.x); t < ntiles; t += gridDim.x) {
    const uint32_t s = t / tps;
    const int64_t off0 = static_cast<int64_t>(t - s * tps) * kTile + threadIdx.x * 16;
    uint64_t as = 0, bs = 0;
    for (int i = 0; i < a.nshards; ++i) {
      const uint64_t base = a.sh[i].base + s * a.sh[i].stride;
#pragma unroll
      for (int it = 0; it < kIt; ++it) {
        const int64_t o = off0 + it * kBlock * 16;
        u32x4 v = 0u;
        if (o + 16 <= C) {
          v = __builtin_nontemporal_load(gptr<u32x4>(base + o));
        } else if (o < C) {
          const u32x2 h = *gptr<u32x2>(base + o);
          v.x = h.x;
          v.y = h.y;
        }
        adler_add(v, L - static_cast<uint64_t>(static_cast<int64_t>(a.shard0 + i) * a.chunk + a.col0 + o), as, bs);
      }
    }
    const uint32_t am = block_sum(static_cast<uint32_t>(as % kAdlerMod), red);
    const uint32_t bm = block_sum(static_cast<uint32_t>(bs % kAdlerMod), red);
    if (threadIdx.x == 0) {
      atomicAdd(a.acc + 2 * s, static_cast<unsigned long long>(am));
      atomicAdd(a.acc + 2 * s + 1, static_cast<unsigned long long>(bm));
    }
  }
}

__global__ void k_magic_finalize(const unsigned long long *acc, int nstripes, uint64_t total_len, uint8_t *magic) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s >= nstripes) return;
  const uint32_t A = static_cast<uint32_t>((1 + acc[2 * s]) % kAdlerMod);
  const uint32_t B = static_cast<uint32_t>((total_len % kAdlerMod + acc[2 * s + 1]) % kAdlerMod);
  const uint32_t m = (B << 16) | A;
  magic[4 * s + 0] = m & 255;
  magic[4 * s + 1] = (m >> 8) & 255;
  magic[4 * s + 2] = (m >> 16) & 255;
  magic[4 * s + 3] = m >> 24;
}

// one block per (stripe, 8 KiB column tile): OR of a^b over every pair, one flag store per
// differing wave
__global__ __launch_bounds__(kBlock) void k_chunk_diff(DiffArgs a) {
  constexpr int kIt = 2, kTile = kBlock * 16 * kIt;
  const int64_t C = a.size;
  const uint32_t tps = static_cast<uint32_t>((C + kTile - 1) / kTile);
  const uint32_t ntiles = tps * static_cast<uint32_t>(a.nstripes);
  for (uint32_t t = xcd_remap(blockIdx.x, gridDim.x); t < ntiles; t += gridDim.x) {
    const uint32_t s = t / tps;
    const int64_t off0 = static_cast<int64_t>(t - s * tps) * kTile + threadIdx.x * 16;
    uint32_t d = 0;
    for (int p = 0; p < a.npairs; ++p) {
      const uint64_t pa = a.a[p].base + s * a.a[p].stride, pb = a.b[p].base + s * a.b[p].stride;
#pragma unroll
      for (int it = 0; it < kIt; ++it) {
        const int64_t o = off0 + it * kBlock * 16;
        if (o + 16 <= C) {
          const u32x4 x = __builtin_nontemporal_load(gptr<u32x4>(pa + o));
          const u32x4 y = __builtin_nontemporal_load(gptr<u32x4>(pb + o));
          const u32x4 z = x ^ y;
          d |= z.x | z.y | z.z | z.w;
        } else if (o < C) {
          const u32x2 x = *gptr<u32x2>(pa + o), y = *gptr<u32x2>(pb + o);
          d |= (x.x ^ y.x) | (x.y ^ y.y);
        }
      }
    }
    if (__any(d != 0) && (threadIdx.x & 63) == 0) a.flags[s] = 1;
  }
}

__global__ __launch_bounds__(kBlock) void k_gather(const GatherPiece *list, char *dst) {
  const GatherPiece g = list[blockIdx.x];
  const LSEC_GLOBAL u32x2 *src = gptr<u32x2>(g.src);
  LSEC_GLOBAL u32x2 *out = gptr_w<u32x2>(reinterpret_cast<uint64_t>(dst) + g.dst_off);
  for (uint64_t i = threadIdx.x; i < g.bytes / 8; i += kBlock) out[i] = __builtin_nontemporal_load(src + i);
}

// HBM probe: a plain streaming copy with the coding kernels' memory shape (one 8 KiB tile
// per block, XCD-contiguous block order, 2 x 16 B non-temporal loads and stores per lane).
// bench.py times it beside the encode as this box's practical read+write ceiling.
__global__ __launch_bounds__(kBlock) void k_hbm_copy(uint64_t dst, uint64_t src, uint64_t n16, unsigned *tiles,
                                                    uint32_t tiles_pre) {
  constexpr int kIt = 2;
  const uint32_t ntiles = static_cast<uint32_t>((n16 + kBlock * kIt - 1) / (kBlock * kIt));
  for_tiles(ntiles, tiles, tiles_pre, [&](uint64_t t) {
    const uint64_t i0 = t * kBlock * kIt + threadIdx.x;
    u32x4 v[kIt];
#pragma unroll
    for (int it = 0; it < kIt; ++it) {
      const uint64_t i = i0 + it * kBlock;
      if (i < n16) v[it] = __builtin_nontemporal_load(gptr<u32x4>(src + i * 16));
    }
#pragma unroll
    for (int it = 0; it < kIt; ++it) {
      const uint64_t i = i0 + it * kBlock;
      if (i < n16) __builtin_nontemporal_store(v[it], gptr_w<u32x4>(dst + i * 16));
    }
  });
}

// The encode's own traffic shape with no arithmetic (measurement probe): per stripe, the XOR of
// K input shards written to each of R output shards, in the RS encode kernel's tiles (2 x 16 B
// per lane, one 8 KiB column tile per block, XCD-contiguous tile order, non-temporal loads and
// stores) -- so K reads : R writes per column, as the encode.
__global__ __launch_bounds__(kBlock) void k_hbm_mix(ApplyArgs a) {
  constexpr int kIt = 2, kTile = kBlock * 16 * kIt;
  const int64_t C = a.size;
  const uint32_t tps = static_cast<uint32_t>((C + kTile - 1) / kTile);
  const uint32_t ntiles = tps * static_cast<uint32_t>(a.nstripes);
  for_tiles(ntiles, a.tiles, a.tiles_pre, [&](uint32_t t) {
    const uint32_t s = t / tps;
    const int64_t off0 = static_cast<int64_t>(t - s * tps) * kTile + threadIdx.x * 16;
    u32x4 acc[kIt] = {0u, 0u};
    for (int j = 0; j < a.K; ++j) {
      const uint64_t p = a.in[j].base + s * a.in[j].stride;
#pragma unroll
      for (int it = 0; it < kIt; ++it) {
        const int64_t o = off0 + it * kBlock * 16;
        if (o + 16 <= C) {
          acc[it] ^= __builtin_nontemporal_load(gptr<u32x4>(p + o));
        } else if (o < C) {
          const u32x2 h = *gptr<u32x2>(p + o);
          acc[it].x ^= h.x;
          acc[it].y ^= h.y;
        }
      }
    }
    for (int r = 0; r < a.R; ++r) {
      const uint64_t q = a.out[r].base + s * a.out[r].stride;
#pragma unroll
      for (int it = 0; it < kIt; ++it) {
        const int64_t o = off0 + it * kBlock * 16;
        if (o + 16 <= C) {
          __builtin_nontemporal_store(acc[it], gptr_w<u32x4>(q + o));
        } else if (o < C) {
          u32x2 h;
          h.x = acc[it].x;
          h.y = acc[it].y;
          *gptr_w<u32x2>(q + o) = h;
        }
      }
    }
  }, a.tile_phase);
}

// Decode-shape probe (measurement only; shares no code with the coding kernels or their tile
// helpers): per stripe, out = XOR of the K inputs -- the single-erasure decode's K reads : 1 write
// per column with the plainest streaming code.  A lane moves 16 B per step, IT steps kBlock*16 B
// apart (a tile is kBlock*16*IT bytes of every shard); block b takes G consecutive tiles (a grab)
// of a static partition, the grabs dealt XCD-contiguous (REMAP: XCD x = blocks b % 8 == x gets an
// eighth of the grabs in order) or round-robin; all K*IT loads of a tile are issued before the
// XOR.  bench.py times every (IT, G, REMAP) beside the decode as the decode's own ceiling.
struct ProbeXorArgs {
  int K;
  int nstripes;
  int64_t size;  // a multiple of kBlock * 16 * IT
  int grab;
  int remap;
  ShardRef in[kMaxK];
  ShardRef out;
};

template <int KC, int IT>
__global__ __launch_bounds__(kBlock) void k_probe_xor(ProbeXorArgs a) {
  constexpr int64_t kStep = kBlock * 16, kTile = kStep * IT;
  const int K = KC ? KC : a.K;
  const uint32_t tps = static_cast<uint32_t>(a.size / kTile);
  const uint32_t ntiles = tps * static_cast<uint32_t>(a.nstripes);
  const uint32_t G = static_cast<uint32_t>(a.grab), ngrabs = (ntiles + G - 1) / G;
  uint32_t g = blockIdx.x;
  if (a.remap) {
    const uint32_t nb = gridDim.x, per = nb >> 3, rem = nb & 7, x = blockIdx.x & 7;
    g = x * per + min(x, rem) + (blockIdx.x >> 3);
  }
  for (; g < ngrabs; g += gridDim.x) {
    const uint32_t t1 = min(ntiles, (g + 1) * G);
    for (uint32_t t = g * G; t < t1; ++t) {
      const uint32_t s = t / tps;
      const int64_t off = static_cast<int64_t>(t - s * tps) * kTile + threadIdx.x * 16;
      u32x4 acc[IT];
#pragma unroll
      for (int it = 0; it < IT; ++it) acc[it] = 0u;
      if constexpr (KC > 0) {
        u32x4 v[KC][IT];
#pragma unroll
        for (int j = 0; j < KC; ++j)
#pragma unroll
          for (int it = 0; it < IT; ++it)
            v[j][it] = __builtin_nontemporal_load(gptr<u32x4>(a.in[j].base + s * a.in[j].stride + off + it * kStep));
#pragma unroll
        for (int j = 0; j < KC; ++j)
#pragma unroll
          for (int it = 0; it < IT; ++it) acc[it] ^= v[j][it];
      } else {
        for (int j = 0; j < K; ++j)
#pragma unroll
          for (int it = 0; it < IT; ++it)
            acc[it] ^= __builtin_nontemporal_load(gptr<u32x4>(a.in[j].base + s * a.in[j].stride + off + it * kStep));
      }
#pragma unroll
      for (int it = 0; it < IT; ++it)
        __builtin_nontemporal_store(acc[it], gptr_w<u32x4>(a.out.base + s * a.out.stride + off + it * kStep));
    }
  }
}

// A small grid striding over the pieces, every lane holding its 4 x 16 B of a piece in flight
// before storing: enough bytes in flight for PCIe, while the H2D and D2H launches (on two
// streams) and the coding kernel between them all keep room on the CUs.  (One block per piece
// let each transfer fill the chip, so the two directions ran one after the other.)
constexpr int kCopyGrid = 256;
static_assert(kPieceBytes == kBlock * 16 * 4, "one piece = 4 x 16 B per lane");
__global__ __launch_bounds__(kBlock) void k_copy_pieces(const CopyPiece *list, int n) {
  for (int p = blockIdx.x; p < n; p += gridDim.x) {
    const CopyPiece g = list[p];
    const uint64_t n16 = g.bytes / 16;
    u32x4 v[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint64_t e = threadIdx.x + static_cast<uint64_t>(i) * kBlock;
      if (e < n16) v[i] = __builtin_nontemporal_load(gptr<u32x4>(g.src + e * 16));
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const uint64_t e = threadIdx.x + static_cast<uint64_t>(i) * kBlock;
      if (e < n16) __builtin_nontemporal_store(v[i], gptr_w<u32x4>(g.dst + e * 16));
    }
  }
}

// one block per XCD (blocks b, b+8, ... are dealt to one XCD), so the system-scope release
// fence of each block writes back every XCD's L2
constexpr int kSignalBlocks = 8;
__global__ __launch_bounds__(64) void k_signal(unsigned *counter, unsigned *flag, unsigned value) {
  __threadfence_system();
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == gridDim.x - 1) {
      __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(flag, value, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

}  // namespace

hipError_t launch_signal(unsigned *counter, unsigned *flag, unsigned value, hipStream_t st) {
  if (!counter || !flag) return hipErrorInvalidValue;
  return launch_kernel(&k_signal, dim3(kSignalBlocks), dim3(64), st, counter, flag, value);
}

hipError_t launch_copy_pieces(const CopyPiece *list, int n, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  // the grid does not matter from 64 to 4096 blocks (profiles/r01_v28_kcopy_grid.txt)
  return launch_kernel(&k_copy_pieces, dim3(std::min(n, kCopyGrid)), dim3(kBlock), st, list, n);
}

hipError_t launch_hbm_copy(void *dst, const void *src, uint64_t bytes, hipStream_t st) {
  if (!dst || !src || bytes % 16 != 0 || (reinterpret_cast<uint64_t>(dst) | reinterpret_cast<uint64_t>(src)) % 16)
    return hipErrorInvalidValue;
  const uint64_t n16 = bytes / 16, ntiles = (n16 + kBlock * 2 - 1) / (kBlock * 2);
  if (ntiles == 0) return hipSuccess;
  if (ntiles >= (1ull << 31)) return hipErrorInvalidValue;
  int grid = default_grid(ntiles);
  unsigned *const slot = tile_queue_slot(st, ntiles);
  unsigned *q = nullptr;
  uint32_t pre = 0;
  if (slot) {
    const int pg = persistent_grid(reinterpret_cast<const void *>(&k_hbm_copy), grid, st);
    if (pg > 0) {
      q = slot;
      pre = tiles_prefix(static_cast<uint32_t>(grid));
      grid = static_cast<int>(8 * pre) + pg;
    }
  }
  const hipError_t e = launch_kernel(&k_hbm_copy, dim3(grid), dim3(kBlock), st, reinterpret_cast<uint64_t>(dst),
                                     reinterpret_cast<uint64_t>(src), n16, q, pre);
  tile_queue_release(st, slot);
  return e;
}

hipError_t launch_hbm_mix(const ApplyArgs &a, hipStream_t st) {
  if (a.K < 1 || a.K > kMaxK || a.R < 1 || a.R > kMaxR || a.size % 8 != 0) return hipErrorInvalidValue;
  if (a.nstripes <= 0 || a.size == 0) return hipSuccess;
  const uint64_t tile = kBlock * 16 * 2;
  const uint64_t ntiles = ((a.size + tile - 1) / tile) * static_cast<uint64_t>(a.nstripes);
  if (ntiles >= (1ull << 31)) return hipErrorInvalidValue;
  return launch_tiled(&k_hbm_mix, default_grid(ntiles), st, a);
}

// variant = IT | G << 4 | REMAP << 8 (IT, G in {1, 2, 4})
hipError_t launch_probe_xor(const ShardRef *in, int K, ShardRef out, int nstripes, int64_t size, int variant,
                            hipStream_t st) {
  const int IT = variant & 15, G = (variant >> 4) & 15, remap = (variant >> 8) & 1;
  if (K < 1 || K > kMaxK || nstripes < 0 || (IT != 1 && IT != 2 && IT != 4) || (G != 1 && G != 2 && G != 4) ||
      size % (static_cast<int64_t>(kBlock) * 16 * IT) != 0)
    return hipErrorInvalidValue;
  if (nstripes == 0 || size == 0) return hipSuccess;
  ProbeXorArgs a;
  std::memset(&a, 0, sizeof(a));
  a.K = K;
  a.nstripes = nstripes;
  a.size = size;
  a.grab = G;
  a.remap = remap;
  for (int j = 0; j < K; ++j) a.in[j] = in[j];
  a.out = out;
  const uint64_t ntiles = static_cast<uint64_t>(size / (static_cast<int64_t>(kBlock) * 16 * IT)) * nstripes;
  const uint64_t grid = (ntiles + G - 1) / G;
  if (grid >= (1ull << 31)) return hipErrorInvalidValue;
  const auto go = [&](auto kern) { return launch_kernel(kern, dim3(static_cast<unsigned>(grid)), dim3(kBlock), st, a); };
  if (K == 6) return IT == 1 ? go(&k_probe_xor<6, 1>) : IT == 2 ? go(&k_probe_xor<6, 2>) : go(&k_probe_xor<6, 4>);
  if (K == 10) return IT == 1 ? go(&k_probe_xor<10, 1>) : IT == 2 ? go(&k_probe_xor<10, 2>) : go(&k_probe_xor<10, 4>);
  return IT == 1 ? go(&k_probe_xor<0, 1>) : IT == 2 ? go(&k_probe_xor<0, 2>) : go(&k_probe_xor<0, 4>);
}

hipError_t launch_gather(const GatherPiece *list, int n, char *dst, hipStream_t st) {
  if (n <= 0) return hipSuccess;
  return launch_kernel(&k_gather, dim3(n), dim3(kBlock), st, list, dst);
}

hipError_t launch_chunk_diff(const DiffArgs &a, hipStream_t st) {
  if (a.npairs < 1 || a.npairs > kMaxR || a.size % 8 != 0 || !a.flags) return hipErrorInvalidValue;
  if (a.nstripes <= 0 || a.size == 0) return hipSuccess;
  const uint64_t tile = kBlock * 16 * 2;
  const uint64_t ntiles = ((a.size + tile - 1) / tile) * static_cast<uint64_t>(a.nstripes);
  if (ntiles >= (1ull << 31)) return hipErrorInvalidValue;
  return launch_kernel(&k_chunk_diff, dim3(default_grid(ntiles)), dim3(kBlock), st, a);
}

hipError_t launch_stripe_magic(const MagicArgs &a, hipStream_t st) {
  if (a.nshards < 1 || a.nshards > kMaxMagicShards || a.size % 8 != 0) return hipErrorInvalidValue;
  if (a.nstripes <= 0) return hipSuccess;
  const uint64_t tile = kBlock * 16 * 2;
  const uint64_t ntiles = ((a.size + tile - 1) / tile) * static_cast<uint64_t>(a.nstripes);
  if (ntiles >= (1ull << 31) || a.size == 0) return a.size == 0 ? hipSuccess : hipErrorInvalidValue;
  return launch_kernel(&k_stripe_magic, dim3(default_grid(ntiles)), dim3(kBlock), st, a);
}

hipError_t launch_magic_finalize(const unsigned long long *acc, int nstripes, int64_t total_len, uint8_t *magic,
                                 hipStream_t st) {
  if (nstripes <= 0) return hipSuccess;
  return launch_kernel(&k_magic_finalize, dim3((nstripes + 255) / 256), dim3(256), st, acc, nstripes,
                     static_cast<uint64_t>(total_len), magic);
}

}  // namespace lsec
