// ec_route.cpp -- the routing of host-memory calls (route_host and its threshold table), the
// device set of the in-process static partition, the batched and per-stripe entry points of
// include/lstore_ec.h, and the per-stripe fn-pointers' direct retry.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdarg>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <cstdint>
#include <cstdio>

#include "ec_host.h"
#include "ec_jit.h"
#include "ec_numa.h"
#include "ec_engine.h"

namespace lsec {
namespace eng {

const RouteTable &routes() {
  static const RouteTable t = [] {
    const auto env = [](const char *name, long dflt) {
      const char *s = getenv(name);
      return s && *s ? atol(s) : dflt;
    };
    RouteTable r;
    r.cpus = usable_cpus();
    r.zerocopy_max = static_cast<size_t>(std::max(0L, env("LSEC_ZEROCOPY_KB", 4096))) << 10;
    r.coalesce_max = static_cast<size_t>(std::max(0L, env("LSEC_COALESCE_MB", 16))) << 20;
    r.own_pipeline_min = static_cast<size_t>(std::max(0L, env("LSEC_OWN_PIPELINE_MIN_KB", 4096))) << 10;
    r.own_pipeline_max = static_cast<int>(std::max(0L, env("LSEC_OWN_PIPELINE_MAX", std::max(2, r.cpus / 2))));
    r.own_pipeline_slot = env("LSEC_ZC_BIG", 1) != 0;
    r.own_dma_max = static_cast<int>(std::max(0L, env("LSEC_OWN_DMA_MAX", 2)));
    r.own_dma_min_bytes = 1u << 20;
    r.own_dma_min_run = static_cast<size_t>(std::max(0L, env("LSEC_OWN_DMA_MIN_RUN_KB", 1024))) << 10;
    r.defer_unpin_bytes = static_cast<size_t>(std::max(0L, env("LSEC_DEFER_UNPIN_MB", 0))) << 20;
    r.lone_blocks = static_cast<int>(std::min(16L, std::max(1L, env("LSEC_LONE_BLOCKS", 1))));
    r.server = env("LSEC_SERVER", 1) != 0;
    r.srv_nt_min = env("LSEC_SRV_NT_MIN_KB", -1) < 0 ? SIZE_MAX : static_cast<size_t>(env("LSEC_SRV_NT_MIN_KB", 0)) << 10;
    r.srv_early_out = env("LSEC_SRV_EARLY_OUT", 1) != 0;
    r.pin_in_place = getenv("LSEC_NO_HOST_REGISTER") == nullptr;
    r.pin_min_bytes = static_cast<size_t>(std::max(0L, env("LSEC_PIN_MIN_KB", 8192))) << 10;
    r.pin_min_run = static_cast<size_t>(std::max(0L, env("LSEC_PIN_MIN_RUN_KB", 6144))) << 10;
    r.kernel_copy = env("LSEC_KERNEL_COPY", 1) != 0;
    r.kernel_copy_max_run = 1u << 20;
    r.slot_pack_pool = static_cast<int>(env("LSEC_ZC_POOL", -1));
    r.slot_pack_inline = 2;
    r.staging_bytes = static_cast<size_t>(std::max(1L, env("LSEC_STAGING_MB", 128))) << 20;
    r.dev_staging_bytes = static_cast<size_t>(std::max(1L, env("LSEC_DEV_STAGING_MB", 512))) << 20;
    r.slot_budget = static_cast<size_t>(std::max(0L, env("LSEC_ZC_SLOTS_MB", 1024))) << 20;
    r.dispatch_batch = 96u << 20;
    const long hw = std::max(1u, std::thread::hardware_concurrency());
    r.copy_threads = static_cast<int>(std::max(1L, env("LSEC_COPY_THREADS", std::min(8L, hw))));
    r.spinners = std::max(1, r.cpus / 4);
    r.spin = std::chrono::microseconds(30);
    r.pollers = std::max(1, std::min(4, r.cpus / 8));
    return r;
  }();
  return t;
}

bool is_device_ptr(const void *ptr) {
  const PtrInfo i = query_ptr(ptr);
  return i.ok && (i.type == hipMemoryTypeDevice || i.type == hipMemoryTypeManaged);
}

// all k+m pointers of every stripe device memory?  then describe them as shard refs
// Returns 1 (device layout in sh), 0 (host memory), -1 (device and host pointers mixed, or an
// irregular device stride: refused rather than guessed).  A batch whose first chunk is device
// memory has every chunk of its first and last stripe checked; a multi-stripe batch whose first
// chunk is host memory has the last chunk of its first and last stripe checked, and a single
// stripe whose first chunk is host memory nothing more (each check is a query under a runtime
// lock that per-stripe calls contend on; a device pointer among host chunks faults the host
// copy, as it faults the reference's CPU code).
int device_layout(const lio_erasure_plan_t *p, char **ptrs, int nstripes, std::vector<lsec_shard_t> &sh) {
  const int km = p->data_strips + p->parity_strips;
  if (!is_device_ptr(ptrs[0])) {
    // A single-stripe call (LStore's per-stripe fn-pointer path) stops at its first chunk:
    // every extra query is a turn on a runtime lock that spins, and at 128 threads on 16 CPUs
    // one extra query per call cut 16 KiB decodes from 30.2 to 3.2-5.3 GiB/s with the CPU quota
    // spent spinning (profiles/r02_v32_zc_decode2.txt).
    if (nstripes == 1) return 0;
    for (int s : {0, nstripes - 1})
      for (int i : {0, km - 1})
        if (is_device_ptr(ptrs[static_cast<size_t>(s) * km + i])) return fail("stripe pointers mix device and host memory");
    return 0;
  }
  for (int s : {0, nstripes - 1})
    for (int i = 0; i < km; ++i)
      if (!is_device_ptr(ptrs[static_cast<size_t>(s) * km + i])) return fail("stripe pointers mix device and host memory");
  sh.resize(km);
  for (int i = 0; i < km; ++i) {
    sh[i].base = ptrs[i];
    sh[i].stride = nstripes > 1 ? static_cast<long long>(ptrs[km + i] - ptrs[i]) : 0;
  }
  for (int s = 2; s < nstripes; ++s)  // require a regular stride (one layout descriptor)
    for (int i = 0; i < km; ++i)
      if (ptrs[static_cast<size_t>(s) * km + i] != ptrs[i] + s * sh[i].stride)
        return fail("device stripe pointers are not regularly strided (stripe %d, shard %d)", s, i);
  return 1;
}

hipStream_t thread_stream() {
  // per-thread stream for the synchronous fn-pointer entry points, destroyed when the thread
  // exits (a caller that churns threads does not accumulate streams)
  struct Streams {
    std::map<int, hipStream_t> by_dev;
    ~Streams() {
      for (auto &kv : by_dev) (void)hipStreamDestroy(kv.second);
    }
  };
  static thread_local Streams streams;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  auto it = streams.by_dev.find(dev);
  if (it != streams.by_dev.end()) return it->second;
  hipStream_t s = nullptr;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return nullptr;
  streams.by_dev[dev] = s;
  return s;
}

// The one routing function of host-memory calls (RouteTable holds every threshold).  By the
// call's bytes B (inputs + outputs):
//   B <= zerocopy_max (4 MiB)        route 1, the stripe server (one stripe it can serve), else
//                                    route 2, this thread's own page-locked slot (zero-copy launch)
//   B <= coalesce_max (16 MiB)       from own_pipeline_min (4 MiB), while at most
//                                    own_pipeline_max such calls run, the call's own pipeline:
//                                    while at most own_dma_max run, route 4 pinned in place at the
//                                    lower own_dma_min_* thresholds (DMA, no packing), else route 2
//                                    (own slot); beyond own_pipeline_max, route 3, the device's
//                                    dispatcher (coalesced with concurrent calls)
//   larger                           route 4, the call's own staging pipeline (pinned in place
//                                    for DMA when pin_min_bytes / pin_min_run allow, else packed)
// Route 2 answers 1 when its slot would pass the device's page-locked budget; the call then
// falls to the next route.  Measured reasons: LStore's 1 MiB chunks make 9 MiB RS(6+3) stripes;
// their own pipeline skips the dispatcher's packing (RS(6+3) 1 MiB encode at one thread 15 -> 27
// GiB/s, Cauchy at 8 threads 19-23 -> 35-36) while few run, and with many the registrations
// contend on the runtime and the dispatcher's packed batches win (decode at 32 threads 38 vs 17
// GiB/s; profiles/r02_v36_route_1m.jsonl, gated vs dispatcher-only r02_v36_route_1m2.jsonl).
int route_host(PlanExt *e, char **ptrs, int nstripes, long long C, const std::vector<int> &in_ids,
               const std::vector<int> &out_ids, const void *image, int kind) {
  const RouteTable &rt = routes();
  const size_t bytes = static_cast<size_t>(nstripes) * (in_ids.size() + out_ids.size()) * C;
  static std::atomic<int> own_inflight{0};
  if (bytes <= rt.zerocopy_max) {
    const int rc = run_zerocopy(e, ptrs, nstripes, C, in_ids, out_ids, image, kind);
    if (rc != 1) return rc;
  }
  if (bytes > rt.coalesce_max) return run_host(e, ptrs, nstripes, C, in_ids, out_ids, image, kind);
  if (bytes >= rt.own_pipeline_min && rt.own_pipeline_max > 0) {
    const int running = own_inflight.fetch_add(1, std::memory_order_acq_rel) + 1;
    if (running <= rt.own_pipeline_max) {
      int rc;
      if (running <= rt.own_dma_max) {
        // few running: pinned in place and DMA'd, no packing (1 MiB Cauchy(6+3) decodes at one
        // thread 22.5 -> 31.5 GiB/s, the reference 29.4; level at two, 37.3 / 37.1;
        // profiles/r04_v3_fnptr_dma_ab.jsonl)
        rc = run_host(e, ptrs, nstripes, C, in_ids, out_ids, image, kind, nullptr, true);
      } else {
        rc = rt.own_pipeline_slot ? run_zerocopy(e, ptrs, nstripes, C, in_ids, out_ids, image, kind) : 1;
        if (rc == 1) rc = run_host(e, ptrs, nstripes, C, in_ids, out_ids, image, kind);
      }
      own_inflight.fetch_sub(1, std::memory_order_acq_rel);
      return rc;
    }
    own_inflight.fetch_sub(1, std::memory_order_acq_rel);
  }
  return run_coalesced(e, ptrs, nstripes, C, in_ids, out_ids, image, kind);
}

// Last resort of the per-stripe fn-pointers after a failed call (a pinned allocation or a
// registration refused, a dispatcher error): plain synchronous copies of the caller's chunks
// into per-thread device scratch, the kernel, and synchronous copies back -- no page-locked
// memory, no dispatcher, no kernel transport.  Still the GPU kernels: there is no CPU path.
int run_direct(PlanExt *e, char **ptrs, long long C, const std::vector<int> &in_ids, const std::vector<int> &out_ids,
               const void *image, int kind) {
  struct Scratch {
    int dev = -1;
    char *d = nullptr;
    size_t cap = 0;
    ~Scratch() {
      if (d) (void)hipFree(d);
    }
  };
  static thread_local Scratch sc;
  int dev = 0;
  HIP_OK(hipGetDevice(&dev));
  const size_t nin = in_ids.size(), nout = out_ids.size(), need = (nin + nout) * static_cast<size_t>(C);
  if (sc.dev != dev || sc.cap < need) {
    if (sc.d) {
      (void)hipSetDevice(sc.dev);
      (void)hipFree(sc.d);
      (void)hipSetDevice(dev);
    }
    sc.d = nullptr;
    sc.cap = 0;
    sc.dev = dev;
    HIP_OK(hipMalloc(&sc.d, need));
    sc.cap = need;
  }
  hipStream_t st = thread_stream();
  if (!st) return fail("no HIP stream");
  ShardRef in[kMaxDevs], out[kMaxDevs];
  for (size_t j = 0; j < nin; ++j) {
    HIP_OK(hipMemcpyAsync(sc.d + j * C, ptrs[in_ids[j]], C, hipMemcpyHostToDevice, st));
    in[j] = {reinterpret_cast<uint64_t>(sc.d) + j * C, 0};
  }
  for (size_t r = 0; r < nout; ++r) out[r] = {reinterpret_cast<uint64_t>(sc.d) + (nin + r) * C, 0};
  if (enqueue_apply(kind, image, static_cast<int>(nin), static_cast<int>(nout), in, out, 1, C, e->pub.packet_size, st, e->pub.w))
    return -1;
  for (size_t r = 0; r < nout; ++r) HIP_OK(hipMemcpyAsync(ptrs[out_ids[r]], sc.d + (nin + r) * C, C, hipMemcpyDeviceToHost, st));
  HIP_OK(hipStreamSynchronize(st));
  return 0;
}

// ---------------------------------------------------------------- host-path device set
// Host-memory calls run on the caller's current device unless lsec_set_host_devices() named a
// device set.  Then a batch above the coalescing limit is cut into contiguous stripe ranges,
// one per device, each driven by its own thread through that device's staging pipeline and
// PCIe link -- SURVEY §8e's static partition inside one LStore process -- and smaller calls go
// to the devices' dispatchers in turn.  Matrix images are per device (encode_cells /
// decode_entry are called on the device that runs the range).
std::mutex g_devs_mu;
std::vector<int> g_host_devs;  // empty: the caller's current device

std::atomic<unsigned> g_devs_version{0};  // bumped under g_devs_mu by every change

// the device set, as a per-thread copy refreshed only when lsec_set_host_devices changed it
// (no lock on the per-stripe path)
const std::vector<int> &host_devices() {
  thread_local std::vector<int> mine;
  thread_local unsigned seen = ~0u;
  const unsigned v = g_devs_version.load(std::memory_order_acquire);
  if (v != seen) {
    std::lock_guard<std::mutex> lk(g_devs_mu);
    mine = g_host_devs;
    seen = g_devs_version.load(std::memory_order_relaxed);
  }
  return mine;
}

struct DeviceGuard {
  int prev = -1;
  bool ok = true;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (dev != prev) ok = hipSetDevice(dev) == hipSuccess;
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

template <typename F>
int on_host_devices(int nstripes, size_t bytes, F &&fn) {
  const std::vector<int> devs = host_devices();
  if (devs.empty()) return fn(0, nstripes);
  if (devs.size() == 1 || nstripes < 2 || bytes <= routes().coalesce_max) {
    static std::atomic<unsigned> rr{0};
    const int dev = devs[rr.fetch_add(1) % devs.size()];
    DeviceGuard g(dev);
    if (!g.ok) return fail("cannot select device %d", dev);
    return fn(0, nstripes);
  }
  const int G = std::min(static_cast<int>(devs.size()), nstripes);
  std::vector<int> rc(G, 0);
  std::vector<std::string> err(G);
  auto work = [&](int g) {
    const int base = nstripes / G, extra = nstripes % G;
    const int s0 = g * base + std::min(g, extra), n = base + (g < extra ? 1 : 0);
    DeviceGuard dg(devs[g]);
    // each range packs with its device's node-local copy pool (ec_numa.h)
    const int node0 = tl_copy_node;
    tl_copy_node = lsec::numa::of_device(devs[g]).node;
    rc[g] = dg.ok ? fn(s0, n) : fail("cannot select device %d", devs[g]);
    tl_copy_node = node0;
    if (rc[g]) err[g] = tl_err;  // tl_err is per thread
  };
  std::vector<std::thread> th;
  for (int g = 1; g < G; ++g)
    th.emplace_back([&work, &devs, g] {
      lsec::numa::bind_this_thread(devs[g]);  // a range thread of its own: on its device's node
      work(g);
    });
  work(0);
  for (auto &t : th) t.join();
  for (int g = 0; g < G; ++g)
    if (rc[g]) return fail("device %d: %s", devs[g], err[g].c_str());
  return 0;
}


int encode_stripes_impl(PlanExt *e, char **ptrs, int nstripes, long long C) {
  PtrMemo memo;
  lio_erasure_plan_t *p = &e->pub;
  if (!ptrs) return fail("ptrs is NULL");
  if (check_geometry(p, C)) return -1;
  if (nstripes <= 0 || C == 0) return 0;
  std::vector<lsec_shard_t> sh;
  const int dl = device_layout(p, ptrs, nstripes, sh);
  if (dl < 0) return -1;
  if (dl) {
    hipStream_t st = thread_stream();
    if (!st) return fail("no HIP stream");
    if (encode_dev(e, sh.data(), nstripes, C, st)) return -1;
    HIP_OK(hipStreamSynchronize(st));
    return 0;
  }
  if (ensure_coding(e)) return -1;
  const int k = p->data_strips, km = k + p->parity_strips;
  const int R = encode_rows(e);
  std::vector<int> in_ids(k), out_ids(R);
  for (int j = 0; j < k; ++j) in_ids[j] = j;
  for (int r = 0; r < R; ++r) out_ids[r] = k + r;
  return on_host_devices(nstripes, static_cast<size_t>(nstripes) * (k + R) * C, [&](int s0, int n) {
    const void *cells = nullptr;
    if (encode_cells(e, &cells)) return -1;
    return route_host(e, ptrs + static_cast<size_t>(s0) * km, n, C, in_ids, out_ids, cells, kernel_kind(p->method, p->w));
  });
}

int decode_stripes_impl(PlanExt *e, char **ptrs, int nstripes, long long C, const int *erasures) {
  PtrMemo memo;
  lio_erasure_plan_t *p = &e->pub;
  if (!ptrs) return fail("ptrs is NULL");
  std::vector<int> ids;
  const int pr = parse_erasures(p, erasures, ids);
  if (pr < 0) return -1;
  if (pr == 1) return 0;
  if (check_geometry(p, C)) return -1;
  if (p->method == RAID4 && ids[0] >= p->data_strips) return 0;
  if (nstripes <= 0 || C == 0) return 0;
  std::vector<lsec_shard_t> sh;
  const int dl = device_layout(p, ptrs, nstripes, sh);
  if (dl < 0) return -1;
  if (dl) {
    hipStream_t st = thread_stream();
    if (!st) return fail("no HIP stream");
    if (decode_dev(e, sh.data(), nstripes, C, erasures, st)) return -1;
    HIP_OK(hipStreamSynchronize(st));
    return 0;
  }
  const int km = p->data_strips + p->parity_strips;
  return on_host_devices(nstripes, static_cast<size_t>(nstripes) * (p->data_strips + ids.size()) * C, [&](int s0, int n) {
    DecodeEntry *ent = nullptr;
    const void *cells = nullptr;
    if (decode_entry(e, ids, &ent, &cells)) return -1;
    return route_host(e, ptrs + static_cast<size_t>(s0) * km, n, C, ent->dp.survivors, ent->dp.erased, cells,
                         decode_kind(e, ent));
  });
}

int encode_stripes_magic_impl(PlanExt *e, char **ptrs, int nstripes, long long C, uint8_t *magic) {
  lio_erasure_plan_t *p = &e->pub;
  if (!ptrs || !magic) return fail("ptrs / magic is NULL");
  if (check_geometry(p, C)) return -1;
  if (nstripes <= 0 || C == 0) return 0;
  if (ensure_coding(e)) return -1;
  const int k = p->data_strips, km = k + p->parity_strips;
  const int R = encode_rows(e);
  if (R != p->parity_strips) return fail("stripe magic needs m parity rows");
  std::vector<int> in_ids(k), out_ids(R);
  for (int j = 0; j < k; ++j) in_ids[j] = j;
  for (int r = 0; r < R; ++r) out_ids[r] = k + r;
  return on_host_devices(nstripes, static_cast<size_t>(nstripes) * km * C, [&](int s0, int n) {
    const void *cells = nullptr;
    if (encode_cells(e, &cells)) return -1;
    return run_host(e, ptrs + static_cast<size_t>(s0) * km, n, C, in_ids, out_ids, cells, kernel_kind(p->method, p->w),
                    magic + 4 * static_cast<size_t>(s0));
  });
}

int stripes_magic_impl(PlanExt *e, char **ptrs, int nstripes, long long C, uint8_t *magic) {
  lio_erasure_plan_t *p = &e->pub;
  if (!ptrs || !magic) return fail("ptrs / magic is NULL");
  if (C < 0 || C % 8 != 0) return fail("block_size %lld is not a multiple of 8", C);
  if (nstripes <= 0 || C == 0) return 0;
  const int km = p->data_strips + p->parity_strips;
  std::vector<int> in_ids(km), none;
  for (int i = 0; i < km; ++i) in_ids[i] = i;
  return on_host_devices(nstripes, static_cast<size_t>(nstripes) * km * C, [&](int s0, int n) {
    return run_host(e, ptrs + static_cast<size_t>(s0) * km, n, C, in_ids, none, nullptr, KBYTEWISE,
                    magic + 4 * static_cast<size_t>(s0));
  });
}

int magic_dev_impl(PlanExt *e, const lsec_shard_t *sh, int nstripes, long long C, uint8_t *magic, hipStream_t st) {
  lio_erasure_plan_t *p = &e->pub;
  const int km = p->data_strips + p->parity_strips;
  if (km > kMaxDevs) return fail("stripe magic supports at most %d chunks", kMaxDevs);
  if (C < 0 || C % 8 != 0) return fail("block_size %lld is not a multiple of 8", C);
  if (nstripes <= 0 || C == 0) return 0;
  unsigned long long *acc = nullptr;
  HIP_OK(hipMallocAsync(reinterpret_cast<void **>(&acc), 16ull * nstripes, st));
  HIP_OK(hipMemsetAsync(acc, 0, 16ull * nstripes, st));
  lsec::MagicArgs ma;
  std::memset(&ma, 0, sizeof(ma));
  ma.size = C;
  ma.col0 = 0;
  ma.chunk = C;
  const int per = static_cast<int>(std::max(1LL, (1LL << 30) / std::max(1LL, C / 8192 + 1)));
  ShardRef msh[kMaxDevs];
  for (int s0 = 0; s0 < nstripes; s0 += per) {
    ma.nstripes = std::min(per, nstripes - s0);
    ma.acc = acc + 2ull * s0;
    for (int i = 0; i < km; ++i)
      msh[i] = {reinterpret_cast<uint64_t>(sh[i].base) + static_cast<uint64_t>(s0) * sh[i].stride, sh[i].stride};
    HIP_OK(launch_magic_groups(ma, msh, km, st));
  }
  HIP_OK(lsec::launch_magic_finalize(acc, nstripes, static_cast<int64_t>(km) * C, magic, st));
  HIP_OK(hipFreeAsync(acc, st));
  return 0;
}

// plan->encode_block / plan->decode_block
// Retry of a failed host-memory fn-pointer call through run_direct.  Geometry errors are not
// retried (they would fail again); a plan from et_generate_plan never has them.
int retry_direct(PlanExt *e, char **ptr, long long C, const std::vector<int> &ids) {
  const std::string first = tl_err;
  lio_erasure_plan_t *p = &e->pub;
  if (check_geometry(p, C) != 0) return -1;
  std::vector<lsec_shard_t> sh;
  if (device_layout(p, ptr, 1, sh) != 0) {
    tl_err = first;  // device pointers (or mixed): nothing to retry with another transport
    return -1;
  }
  int rc;
  if (ids.empty()) {  // encode
    const int k = p->data_strips;
    const void *cells = nullptr;
    rc = encode_cells(e, &cells);
    if (rc == 0) {
      const int R = encode_rows(e);
      std::vector<int> in_ids(k), out_ids(R);
      for (int j = 0; j < k; ++j) in_ids[j] = j;
      for (int r = 0; r < R; ++r) out_ids[r] = k + r;
      rc = run_direct(e, ptr, C, in_ids, out_ids, cells, kernel_kind(p->method, p->w));
    }
  } else {
    DecodeEntry *ent = nullptr;
    const void *cells = nullptr;
    rc = decode_entry(e, ids, &ent, &cells);
    if (rc == 0) rc = run_direct(e, ptr, C, ent->dp.survivors, ent->dp.erased, cells, decode_kind(e, ent));
  }
  if (rc == 0) {
    static std::atomic<bool> warned{false};
    if (!warned.exchange(true))
      fprintf(stderr, "lstore_ec: a stripe call failed (%s); retried with direct copies\n", first.c_str());
    return 0;
  }
  tl_err = first + "; direct retry: " + tl_err;
  return -1;
}

thread_local CallTrace tl_trace;

namespace {
bool call_trace_on() {
  static const bool on = getenv("LSEC_TRACE") != nullptr;
  return on;
}
// LSEC_TRACE=2: the lines are kept in memory and printed at exit, so that no write to stderr
// sits between one call and the next (the one-thread tail study, tools/gpu_fnptr_tail.sh)
bool call_trace_buffered() {
  static const bool b = [] {
    const char *e = getenv("LSEC_TRACE");
    return e && std::strcmp(e, "2") == 0;
  }();
  return b;
}
std::mutex g_trace_mu;
std::vector<std::string> *g_trace_lines = nullptr;  // leaked: printed by the exit handler
void print_trace_lines() {
  std::lock_guard<std::mutex> lk(g_trace_mu);
  if (g_trace_lines)
    for (const std::string &l : *g_trace_lines) fprintf(stderr, "%s\n", l.c_str());
}
void call_trace_begin() {
  tl_trace.active = true;
  tl_trace.line[0] = 0;
  tl_trace.t_call0 = std::chrono::steady_clock::now();
}
// the call's run_host phases (if it took route 4) with the time spent before run_host began
// (entry: pointer queries, decode image lookup, routing, staging acquisition) and after it ended
// (exit: staging release, return)
void call_trace_end() {
  const auto t = std::chrono::steady_clock::now();
  const auto ms = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
    return std::chrono::duration<double, std::milli>(b - a).count();
  };
  if (tl_trace.line[0]) {
    char buf[400];
    snprintf(buf, sizeof(buf), "%s, entry %.4f ms, exit %.4f ms, call %.4f ms", tl_trace.line, ms(tl_trace.t_call0, tl_trace.t_run0),
             ms(tl_trace.t_run1, t), ms(tl_trace.t_call0, t));
    if (call_trace_buffered()) {
      std::lock_guard<std::mutex> lk(g_trace_mu);
      if (!g_trace_lines) {
        g_trace_lines = new std::vector<std::string>();
        g_trace_lines->reserve(1 << 16);
        atexit(print_trace_lines);
      }
      if (g_trace_lines->size() < (1u << 21)) g_trace_lines->emplace_back(buf);  // (~0.5 GB at most)
    } else {
      fprintf(stderr, "%s\n", buf);
    }
  }
  tl_trace.active = false;
  tl_trace.line[0] = 0;
}
}  // namespace

void fp_encode_block(lio_erasure_plan_t *p, char **ptr, int block_size) {
  if (call_trace_on()) call_trace_begin();
  struct End {
    ~End() {
      if (tl_trace.active) call_trace_end();
    }
  } end_trace;
  if (ZcStats::on()) {
    tl_call_t0 = std::chrono::steady_clock::now();
    tl_call_cpu0 = thread_cpu_ns();
  }
  PlanExt *e = ext_of(p);
  if (!e) fatal("encode_block on a plan not created by this library");
  if (encode_stripes_impl(e, ptr, 1, block_size) == 0) return;
  // encode_block cannot report a status, and writing no (or stale) parity would be stamped with
  // a matching stripe magic by the caller (segment/jerasure.c:1850): retry once, then abort as
  // Jerasure exits on errors (jerasure.c:306-310).  tl_err then holds both attempts' reasons
  // ("<first>; direct retry: <second>", retry_direct).
  if (retry_direct(e, ptr, block_size, {}) == 0) return;
  fatal("encode_block (k=%d m=%d w=%d C=%d) failed: %s", p->data_strips, p->parity_strips, p->w, block_size,
        tl_err.c_str());
}

int fp_decode_block(lio_erasure_plan_t *p, char **ptr, int block_size, int *erasures) {
  if (call_trace_on()) call_trace_begin();
  struct End {
    ~End() {
      if (tl_trace.active) call_trace_end();
    }
  } end_trace;
  if (ZcStats::on()) {
    tl_call_t0 = std::chrono::steady_clock::now();
    tl_call_cpu0 = thread_cpu_ns();
  }
  PlanExt *e = ext_of(p);
  if (!e) return fail("not an lstore_ec plan");
  if (decode_stripes_impl(e, ptr, 1, block_size, erasures) == 0) return 0;
  std::vector<int> ids;
  if (parse_erasures(p, erasures, ids) != 0) return -1;
  if (p->method == RAID4 && ids[0] >= p->data_strips) return 0;
  return retry_direct(e, ptr, block_size, ids);
}

int fp_dummy(lio_erasure_plan_t *) { return 0; }

}  // namespace eng
}  // namespace lsec

using namespace lsec::eng;

extern "C" {

// ---- extensions
int et_encode_stripes(lio_erasure_plan_t *plan, char **ptrs, int nstripes, int block_size) {
  PlanExt *e = ext_of(plan);
  if (!e) return fail("not an lstore_ec plan");
  return encode_stripes_impl(e, ptrs, nstripes, block_size);
}

int et_decode_stripes(lio_erasure_plan_t *plan, char **ptrs, int nstripes, int block_size, int *erasures) {
  PlanExt *e = ext_of(plan);
  if (!e) return fail("not an lstore_ec plan");
  return decode_stripes_impl(e, ptrs, nstripes, block_size, erasures);
}

int lsec_encode_dev(lio_erasure_plan_t *plan, const lsec_shard_t *shards, int nstripes, long long block_size,
                    void *stream) {
  PlanExt *e = ext_of(plan);
  if (!e) return fail("not an lstore_ec plan");
  if (!shards) return fail("shards is NULL");
  return encode_dev(e, shards, nstripes, block_size, static_cast<hipStream_t>(stream));
}

int lsec_decode_dev(lio_erasure_plan_t *plan, const lsec_shard_t *shards, int nstripes, long long block_size,
                    const int *erasures, void *stream) {
  PlanExt *e = ext_of(plan);
  if (!e) return fail("not an lstore_ec plan");
  if (!shards) return fail("shards is NULL");
  return decode_dev(e, shards, nstripes, block_size, erasures, static_cast<hipStream_t>(stream));
}

int et_encode_stripes_magic(lio_erasure_plan_t *plan, char **ptrs, int nstripes, int block_size, char *magic) {
  PlanExt *e = ext_of(plan);
  if (!e) return fail("not an lstore_ec plan");
  return encode_stripes_magic_impl(e, ptrs, nstripes, block_size, reinterpret_cast<uint8_t *>(magic));
}

int et_stripes_magic(lio_erasure_plan_t *plan, char **ptrs, int nstripes, int block_size, char *magic) {
  PlanExt *e = ext_of(plan);
  if (!e) return fail("not an lstore_ec plan");
  return stripes_magic_impl(e, ptrs, nstripes, block_size, reinterpret_cast<uint8_t *>(magic));
}

int lsec_stripe_magic_dev(lio_erasure_plan_t *plan, const lsec_shard_t *shards, int nstripes, long long block_size,
                          void *magic, void *stream) {
  PlanExt *e = ext_of(plan);
  if (!e) return fail("not an lstore_ec plan");
  if (!shards || !magic) return fail("shards / magic is NULL");
  return magic_dev_impl(e, shards, nstripes, block_size, static_cast<uint8_t *>(magic), static_cast<hipStream_t>(stream));
}

int lsec_encode_magic_dev(lio_erasure_plan_t *plan, const lsec_shard_t *shards, int nstripes, long long block_size,
                          void *magic, void *stream) {
  PlanExt *e = ext_of(plan);
  if (!e) return fail("not an lstore_ec plan");
  if (!shards || !magic) return fail("shards / magic is NULL");
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int k = plan->data_strips, m = plan->parity_strips;
  // One pass: the encode kernel also accumulates the magic of the k inputs and m outputs.
  // Each lane keeps it in 32-bit dot-product chains (MagicLane, ec_kernels_impl.h), about
  // 3 VALU ops per data dword, so fusing wins at every k, m a single launch takes (m <= 8):
  // RS 12+4 5.9 ms fused vs 5.7 + 5.2 ms as two passes, Cauchy 6+3 5.9 vs 5.9 + 6.2 ms
  // (profiles/r01_v12_kbench_fused_magic.txt).
  const int kind = kernel_kind(plan->method, plan->w);
  const bool fuse = kind == KBYTEWISE || kind == KBITSLICED;
  if (fuse && m <= 8 && k <= lsec::kMaxK && !check_geometry(plan, block_size) && k + m <= lsec::kMaxMagicShards) {
    if (nstripes <= 0 || block_size == 0) return 0;
    const void *cells = nullptr;
    if (encode_cells(e, &cells)) return -1;
    if (encode_rows(e) != m) return fail("stripe magic needs m parity rows");
    unsigned long long *acc = nullptr;
    HIP_OK(hipMallocAsync(reinterpret_cast<void **>(&acc), 16ull * nstripes, st));
    HIP_OK(hipMemsetAsync(acc, 0, 16ull * nstripes, st));
    lsec::ApplyArgs a;
    std::memset(&a, 0, sizeof(a));
    a.cells = static_cast<const CoefCell *>(cells);
    a.K = k;
    a.R = m;
    a.size = block_size;
    a.packet = plan->packet_size;
    const int per = static_cast<int>(std::max(1LL, (1LL << 30) / std::max(1LL, block_size / 8192 + 1)));
    for (int s0 = 0; s0 < nstripes; s0 += per) {
      a.nstripes = std::min(per, nstripes - s0);
      a.magic_acc = acc + 2ull * s0;
      for (int j = 0; j < k; ++j)
        a.in[j] = {reinterpret_cast<uint64_t>(shards[j].base) + static_cast<uint64_t>(s0) * shards[j].stride, shards[j].stride};
      for (int r = 0; r < m; ++r)
        a.out[r] = {reinterpret_cast<uint64_t>(shards[k + r].base) + static_cast<uint64_t>(s0) * shards[k + r].stride,
                    shards[k + r].stride};
      HIP_OK(kind == KBITSLICED ? lsec::launch_bitsliced(a, st) : lsec::launch_bytewise_magic(a, st));
    }
    HIP_OK(lsec::launch_magic_finalize(acc, nstripes, static_cast<int64_t>(k + m) * block_size,
                                       static_cast<uint8_t *>(magic), st));
    HIP_OK(hipFreeAsync(acc, st));
    return 0;
  }
  if (encode_dev(e, shards, nstripes, block_size, st)) return -1;
  return magic_dev_impl(e, shards, nstripes, block_size, static_cast<uint8_t *>(magic), st);
}


int lsec_set_host_devices(const int *devices, int n) {
  std::vector<int> v;
  if (n > 0) {
    if (!devices) return fail("devices is NULL");
    int count = 0;
    if (lsec::quiet([&] { return hipGetDeviceCount(&count); }) != hipSuccess) {
      return fail("no HIP device");
    }
    for (int i = 0; i < n; ++i) {
      if (devices[i] < 0 || devices[i] >= count) return fail("device %d outside 0..%d", devices[i], count - 1);
      v.push_back(devices[i]);
    }
  }
  std::lock_guard<std::mutex> lk(g_devs_mu);
  g_host_devs.swap(v);
  g_devs_version.fetch_add(1, std::memory_order_release);
  return 0;
}

int lsec_abi_version(void) { return LSEC_ABI_VERSION; }

int lsec_device_count(void) {
  int n = 0;
  if (lsec::quiet([&] { return hipGetDeviceCount(&n); }) != hipSuccess) {
    return 0;
  }
  return n;
}

const char *lsec_last_error(void) { return tl_err.c_str(); }


int lsec_hbm_copy_dev(void *dst, const void *src, unsigned long long bytes, void *stream) {
  const hipError_t e = lsec::launch_hbm_copy(dst, src, bytes, static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return fail("lsec_hbm_copy_dev: %s", hipGetErrorString(e));
  return 0;
}

int lsec_hbm_mix_dev(const lsec_shard_t *shards, int k, int m, int nstripes, long long block_size, void *stream) {
  if (!shards || k < 1 || k > lsec::kMaxK || m < 1 || m > lsec::kMaxR || nstripes < 0 || block_size < 0 ||
      block_size % 8 != 0)
    return fail("lsec_hbm_mix_dev: bad arguments (k=%d m=%d nstripes=%d block_size=%lld)", k, m, nstripes, block_size);
  lsec::ApplyArgs a;
  std::memset(&a, 0, sizeof(a));
  a.K = k;
  a.R = m;
  a.nstripes = nstripes;
  a.size = block_size;
  for (int j = 0; j < k; ++j) a.in[j] = {reinterpret_cast<uint64_t>(shards[j].base), shards[j].stride};
  for (int r = 0; r < m; ++r) a.out[r] = {reinterpret_cast<uint64_t>(shards[k + r].base), shards[k + r].stride};
  const hipError_t e = lsec::launch_hbm_mix(a, static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return fail("lsec_hbm_mix_dev: %s", hipGetErrorString(e));
  return 0;
}


int lsec_hbm_decode_shape_dev(const lsec_shard_t *shards, int k, int nstripes, long long block_size, int variant,
                              void *stream) {
  if (!shards || k < 1 || k > lsec::kMaxK || nstripes < 0 || block_size < 0)
    return fail("lsec_hbm_decode_shape_dev: bad arguments (k=%d nstripes=%d block_size=%lld)", k, nstripes, block_size);
  lsec::ShardRef in[lsec::kMaxK];
  for (int j = 0; j < k; ++j) in[j] = {reinterpret_cast<uint64_t>(shards[j].base), shards[j].stride};
  const lsec::ShardRef out = {reinterpret_cast<uint64_t>(shards[k].base), shards[k].stride};
  const hipError_t e = lsec::launch_probe_xor(in, k, out, nstripes, block_size, variant, static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return fail("lsec_hbm_decode_shape_dev: %s", hipGetErrorString(e));
  return 0;
}

int lsec_device_numa(int dev, int *node, int *cpus, int max_cpus) {
  int n = 0;
  if (lsec::quiet([&] { return hipGetDeviceCount(&n); }) != hipSuccess) {
    n = 0;
  }
  if (dev < 0 || dev >= n) return fail("lsec_device_numa: no device %d", dev);
  const lsec::numa::Placement &pl = lsec::numa::of_device(dev);
  if (node) *node = pl.node;
  for (int i = 0; cpus && i < max_cpus && i < static_cast<int>(pl.cpus.size()); ++i) cpus[i] = pl.cpus[i];
  return static_cast<int>(pl.cpus.size());
}

// Test hook, not part of include/*.h: the placement of PCI function `bus` under the sysfs tree
// `root` (a fake tree in tests/test_numa.py), unfiltered by this process's affinity.
int lsec_test_numa_for_bus(const char *root, const char *bus, int *node, int *cpus, int max_cpus) {
  if (!root || !bus) return fail("lsec_test_numa_for_bus: NULL argument");
  const lsec::numa::Placement pl = lsec::numa::for_bus(root, bus, {});
  if (node) *node = pl.node;
  for (int i = 0; cpus && i < max_cpus && i < static_cast<int>(pl.cpus.size()); ++i) cpus[i] = pl.cpus[i];
  return static_cast<int>(pl.cpus.size());
}

}  // extern "C"
