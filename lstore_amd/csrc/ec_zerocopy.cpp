// ec_zerocopy.cpp -- routes 1 and 2 for small host calls: the stripe server when it takes the
// call (ec_stripe_server.cpp), else the calling thread's own page-locked slot, read and written
// by the coding kernel over PCIe (zero-copy), completed by a signal kernel's flag.  Also the
// per-device accounting of the page-locked memory both hold (PinnedBudget).
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

#include <immintrin.h>

#include "ec_server.h"
#include "ec_engine.h"

namespace lsec {
namespace eng {

// ---------------------------------------------------------------- zero-copy small calls
// LStore calls encode_block / decode_block once per stripe (16 KiB chunks by default,
// cjerase_16k.ex3:46) from many pool threads.  For such calls the DMA round trip (H2D, kernel,
// D2H, each a queue operation with its own fixed cost, plus the hops through a dispatcher
// thread) dominates: 78 us per 16 KiB Cauchy(6+3) call at one thread in round 1.  Here the
// calling thread copies its chunks into its own page-locked slot and the coding kernel reads
// and writes that slot over PCIe directly (zero-copy): one launch on the thread's stream and
// one synchronisation per call, no DMA and no other thread.  Chunks the caller already holds
// in page-locked memory are read and written in place, with no copies at all.
// Per-call bytes (inputs + outputs) served this way; LSEC_ZEROCOPY_KB.  4 MiB: calls of 1-4 MiB
// (RS(6+3) at 128 / 256 KiB chunks) ran 1.3-2.5x faster zero-copy than through the dispatcher
// at 1-128 threads (profiles/r02_v42_route_mid.jsonl).  Each thread keeps a page-locked slot as
// large as its largest such call.

// Completion signals of zero-copy calls (flag in coherent page-locked memory, arrival counter
// in device memory) are pooled per device and never freed: a poller (FlagWaits) may read a flag
// just as the thread that owned it exits.
struct SignalBlock {
  unsigned *flag, *dflag, *counter;
};
std::mutex g_signal_mu;
std::map<int, std::vector<SignalBlock>> &signal_pool() {
  static auto *p = new std::map<int, std::vector<SignalBlock>>();  // leaked with the blocks
  return *p;
}

struct ZcSlot {  // one calling thread's page-locked slot on one device
  char *h = nullptr;
  uint64_t d = 0;  // its device address
  size_t cap = 0;
  // completion: flag in coherent page-locked memory (the host spins on it), the signal
  // kernel's arrival counter in device memory, and the value the next call waits for
  unsigned *flag = nullptr, *dflag = nullptr, *counter = nullptr;
  unsigned seq = 0;
  int dev = -1;
  bool clean = true;  // every signal launched was seen: the block can serve another thread
  ZcSlot() = default;
  ZcSlot(const ZcSlot &) = delete;
  ZcSlot &operator=(const ZcSlot &) = delete;
  ~ZcSlot() {
    if (h) {
      (void)hipHostFree(h);
      PinnedBudget::global().release_slot(dev, cap);
    }
    if (flag && clean) {
      std::lock_guard<std::mutex> lk(g_signal_mu);
      signal_pool()[dev].push_back({flag, dflag, counter});
    }
  }
  int init_signal() {
    if (flag) return 0;
    HIP_OK(hipGetDevice(&dev));
    {
      std::lock_guard<std::mutex> lk(g_signal_mu);
      std::vector<SignalBlock> &pool = signal_pool()[dev];
      if (!pool.empty()) {
        flag = pool.back().flag;
        dflag = pool.back().dflag;
        counter = pool.back().counter;
        pool.pop_back();
        seq = __atomic_load_n(flag, __ATOMIC_ACQUIRE);  // continue the sequence the flag holds
        return 0;
      }
    }
    HIP_OK(hipHostMalloc(reinterpret_cast<void **>(&flag), 64, hipHostMallocCoherent));
    *flag = 0;
    void *dp = nullptr;
    HIP_OK(hipHostGetDevicePointer(&dp, flag, 0));
    dflag = static_cast<unsigned *>(dp);
    HIP_OK(hipMalloc(reinterpret_cast<void **>(&counter), 64));
    HIP_OK(hipMemset(counter, 0, 64));
    return 0;
  }
};

// Completes a zero-copy call: the signal kernel behind the coding kernel on `st`, then a spin
// on the flag (a flag seen ~8 us sooner than hipStreamSynchronize returns:
// tools/probes/zc_probe.hip, profiles/r02_v3_zc_probe.txt).  A call whose flag has not come
// after a second falls back to the stream's own status, so a failed launch is reported.
bool wait_flag(const unsigned *flag, unsigned v, hipStream_t st, int *rc);

int zc_complete(ZcSlot &sl, hipStream_t st) {
  const unsigned v = ++sl.seq == 0 ? ++sl.seq : sl.seq;
  const hipError_t e = lsec::launch_signal(sl.counter, sl.dflag, v, st);
  if (e != hipSuccess) return fail("signal launch: %s", hipGetErrorString(e));
  int rc = 0;
  if (!wait_flag(sl.flag, v, st, &rc)) sl.clean = false;
  return rc;
}

// regular stripe stride of device addresses a[s * per + i] (i < per): shard i of stripe s at
// a[i] + s * stride[i]; false if irregular
bool regular_refs(const std::vector<uint64_t> &a, int nstripes, size_t per, std::vector<int64_t> &stride) {
  stride.assign(per, 0);
  if (nstripes < 2) return true;
  for (size_t i = 0; i < per; ++i) stride[i] = static_cast<int64_t>(a[per + i] - a[i]);
  for (int s = 2; s < nstripes; ++s)
    for (size_t i = 0; i < per; ++i)
      if (a[s * per + i] != a[i] + static_cast<uint64_t>(s * stride[i])) return false;
  return true;
}

// LSEC_STATS phase clocks of the current call (ec_engine.h)
thread_local std::chrono::steady_clock::time_point tl_call_t0;
thread_local std::chrono::steady_clock::time_point tl_zc_t0;
thread_local long long tl_call_cpu0 = 0, tl_zc_cpu0 = 0;

long long thread_cpu_ns() {
  struct timespec ts;
  clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
  return static_cast<long long>(ts.tv_sec) * 1000000000LL + ts.tv_nsec;
}


ZcSlot &thread_zc_slot(int dev);

int run_zerocopy(PlanExt *e, char **ptrs, int nstripes, long long C, const std::vector<int> &in_ids,
                 const std::vector<int> &out_ids, const void *image, int kind) {
  if (ZcStats::on()) {
    tl_zc_t0 = std::chrono::steady_clock::now();
    tl_zc_cpu0 = thread_cpu_ns();
  }
  int dev = 0;
  HIP_OK(hipGetDevice(&dev));
  hipStream_t st = thread_stream();
  if (!st) return fail("no HIP stream");
  const lio_erasure_plan_t *p = &e->pub;
  const int km = p->data_strips + p->parity_strips;
  const size_t nin = in_ids.size(), nout = out_ids.size(), nio = nin + nout;
  ShardRef in[kMaxDevs], out[kMaxDevs];
  const bool aligned = kernel_transport_aligned(ptrs, nstripes, km, in_ids, out_ids, C, C);
  ZcSlot *slot = &thread_zc_slot(dev);
  if (slot->init_signal()) return -1;
  CallerPinned cp = caller_pinned(ptrs, nstripes, km, in_ids, out_ids, C, aligned);
  if (nstripes == 1 && routes().server) {
    const int rc = server_run(dev, e, ptrs, C, in_ids, out_ids, image, kind, &cp);
    if (rc != 1) {
      if (rc == 0) ZcStats::get().server.fetch_add(1, std::memory_order_relaxed);
      return rc;
    }
  }
  std::vector<int64_t> stride;
  if (cp.by_kernel && regular_refs(cp.dev, nstripes, nio, stride)) {
    // caller page-locked chunks: read and written in place over PCIe
    for (size_t j = 0; j < nin; ++j) in[j] = {cp.dev[j], stride[j]};
    for (size_t r = 0; r < nout; ++r) out[r] = {cp.dev[nin + r], stride[nin + r]};
    ZcStats::get().launch_direct.fetch_add(1, std::memory_order_relaxed);
    if (enqueue_apply(kind, image, static_cast<int>(nin), static_cast<int>(nout), in, out, nstripes, C, p->packet_size, st, p->w))
      return -1;
    return zc_complete(*slot, st);
  }
  const size_t need = static_cast<size_t>(nstripes) * nio * static_cast<size_t>(C);
  if (slot->cap < need) {
    const size_t cap = std::max<size_t>(need, 256u << 10);
    // all threads' slots on this device together stay within LSEC_ZC_SLOTS_MB (default 1 GiB of
    // page-locked memory per device, PinnedBudget); a call whose slot would pass it goes to the
    // dispatcher's shared staging instead
    if (!PinnedBudget::global().grow_slot(dev, slot->cap, cap)) return 1;
    if (slot->h) (void)hipHostFree(slot->h);
    slot->h = nullptr;
    slot->cap = 0;
    slot->d = 0;
    // coherent: the kernel's reads and writes of the slot go straight over PCIe, none stays in an L2
    char *h = nullptr;
    void *d = nullptr;
    if (quiet([&] { return hipHostMalloc(reinterpret_cast<void **>(&h), cap, hipHostMallocCoherent); }) != hipSuccess) {
      PinnedBudget::global().release_slot(dev, cap);
      return fail("zero-copy slot: cannot allocate %zu bytes of page-locked memory", cap);
    }
    if (quiet([&] { return hipHostGetDevicePointer(&d, h, 0); }) != hipSuccess || !d) {
      (void)hipHostFree(h);
      PinnedBudget::global().release_slot(dev, cap);
      return fail("zero-copy slot: no device address");
    }
    slot->h = h;
    slot->d = reinterpret_cast<uint64_t>(d);
    slot->cap = cap;
  }
  ZcStats::get().launch_slot.fetch_add(1, std::memory_order_relaxed);
  const bool stats = ZcStats::on();
  const auto tnow = [] { return std::chrono::steady_clock::now(); };
  const auto tns = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
    return static_cast<unsigned long long>(std::chrono::duration_cast<std::chrono::nanoseconds>(b - a).count());
  };
  auto t_last = stats ? tnow() : std::chrono::steady_clock::time_point{};
  // Packing: a call running alone (with at most one other) copies its own chunks -- one thread
  // packed a 1 MiB Cauchy(6+3) decode's 6 MiB in 164 us against 200 us on the 8-thread copy pool,
  // at a quarter of the CPU (profiles/r03_v20_slot_phases.txt; 1 MiB decodes at one thread
  // 19.1 -> 22.6 GiB/s, RS(6+3) 1 MiB encodes 12.9 -> 16.1).  Under concurrency the pool, whose
  // workers sit on the GPU's NUMA node, packs faster (8 threads: 46.0 pool vs 34.8 inline;
  // profiles/r03_v21_fnptr_fair.jsonl).  LSEC_ZC_POOL=1 / 0 forces either (A/B runs).
  const int pool_mode = routes().slot_pack_pool;
  static std::atomic<int> slot_calls{0};
  struct InFlight {
    std::atomic<int> &n;
    const int at;
    explicit InFlight(std::atomic<int> &c) : n(c), at(c.fetch_add(1, std::memory_order_acq_rel) + 1) {}
    ~InFlight() { n.fetch_sub(1, std::memory_order_acq_rel); }
  } inflight(slot_calls);
  const bool pool = pool_mode >= 0 ? pool_mode == 1 : inflight.at > routes().slot_pack_inline;
  const auto pack = [&](std::vector<CopyJob> &js) {
    if (pool) {
      copy_run(js, 64 << 10);
      return;
    }
    for (const CopyJob &j : js) host_copy(j.dst, j.src, j.bytes);
    _mm_sfence();  // the streamed bytes are visible before the launch (or the return) that follows
  };
  if (stats) ZcStats::get().s_alloc.fetch_add(tns(tl_zc_t0, t_last), std::memory_order_relaxed);
  const auto lap = [&](std::atomic<unsigned long long> &acc) {
    if (!stats) return;
    const auto t = tnow();
    acc.fetch_add(tns(t_last, t), std::memory_order_relaxed);
    t_last = t;
  };
  // slot layout: inputs [s][nin][C], then outputs [s][nout][C].  Calls of 1 MiB and more are
  // packed and computed in blocks of about 1 MiB (groups of stripes, or column blocks of a
  // single stripe): the copy pool packs block b+1 while the kernel of block b reads the slot over
  // PCIe, and a 7 MiB call no longer waits for all its packing before the GPU starts.
  const size_t in_bytes = static_cast<size_t>(nstripes) * nin * C;
  const int nblk = static_cast<int>(std::min<size_t>(16, std::max<size_t>(1, need >> 20)));
  const long long unit = packet_kind(kind) ? static_cast<long long>(p->w) * p->packet_size : 16;
  const bool by_cols = nstripes == 1 && nblk > 1 && C > unit;
  const int sg = by_cols ? 1 : (nstripes + nblk - 1) / nblk;                       // stripes per block
  const long long cl = by_cols ? ((C + nblk - 1) / nblk + unit - 1) / unit * unit : C;  // columns per block
  std::vector<CopyJob> jobs;
  for (int s0 = 0; s0 < nstripes; s0 += sg) {
    const int n = std::min(sg, nstripes - s0);
    for (long long c0 = 0; c0 < C; c0 += cl) {
      const long long len = std::min(cl, C - c0);
      jobs.clear();
      for (int s = s0; s < s0 + n; ++s)
        for (size_t j = 0; j < nin; ++j)
          jobs.push_back({slot->h + (s * nin + j) * C + c0, ptrs[static_cast<size_t>(s) * km + in_ids[j]] + c0,
                          static_cast<size_t>(len)});
      pack(jobs);
      lap(ZcStats::get().s_pack);
      for (size_t j = 0; j < nin; ++j) in[j] = {slot->d + (s0 * nin + j) * C + c0, static_cast<int64_t>(nin * C)};
      for (size_t r = 0; r < nout; ++r)
        out[r] = {slot->d + in_bytes + (s0 * nout + r) * C + c0, static_cast<int64_t>(nout * C)};
      if (enqueue_apply(kind, image, static_cast<int>(nin), static_cast<int>(nout), in, out, n, len, p->packet_size, st, p->w))
        return -1;
      lap(ZcStats::get().s_enq);
    }
  }
  if (zc_complete(*slot, st)) return -1;
  lap(ZcStats::get().s_wait);
  jobs.clear();
  for (int s = 0; s < nstripes; ++s)
    for (size_t r = 0; r < nout; ++r)
      jobs.push_back({ptrs[static_cast<size_t>(s) * km + out_ids[r]], slot->h + in_bytes + (s * nout + r) * C, static_cast<size_t>(C)});
  pack(jobs);
  lap(ZcStats::get().s_out);
  return 0;
}

ZcSlot &thread_zc_slot(int dev) {
  static thread_local std::map<int, std::unique_ptr<ZcSlot>> slots;
  std::unique_ptr<ZcSlot> &slot = slots[dev];
  if (!slot) slot.reset(new ZcSlot());
  return *slot;
}

}  // namespace eng
}  // namespace lsec

using namespace lsec::eng;

extern "C" {

// Test hook, not in include/ (no GPU): the zero-copy page-locked accounting (PinnedBudget) on a
// fresh instance with a slot budget of budget_mb per device: `ndev` devices each start their
// stripe server, every device but 0 fills its threads' slots with slot_mb slots, then device 0
// takes slot_mb slots until refused.  Returns how many it got; *server_mb = the servers' total.
long long lsec_test_pinned_budget(int ndev, long long budget_mb, long long slot_mb, long long *server_mb) {
  if (ndev < 1 || ndev > PinnedBudget::kDevs || budget_mb < 0 || slot_mb < 1) return fail("lsec_test_pinned_budget: bad arguments");
  PinnedBudget b(static_cast<size_t>(budget_mb) << 20);
  const size_t region = lsec::kSrvSlotBytes * lsec::kSrvSlots, slot = static_cast<size_t>(slot_mb) << 20;
  for (int d = 0; d < ndev; ++d) b.add_server(d, region);
  for (int d = 1; d < ndev; ++d)
    while (b.grow_slot(d, 0, slot)) {
    }
  long long n = 0;
  while (b.grow_slot(0, 0, slot)) ++n;
  size_t total = 0;
  for (int d = 0; d < ndev; ++d) total += b.server_bytes(d);
  if (server_mb) *server_mb = static_cast<long long>(total >> 20);
  return n;
}

}  // extern "C"
