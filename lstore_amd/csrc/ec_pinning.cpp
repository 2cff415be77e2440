// ec_pinning.cpp -- what kind of host memory a call hands over: runtime pointer queries (with a
// per-call memo), caller page-locked buffers (DMA in place; kernel transport for small runs of
// hipHostMalloc memory), and pageable batches pinned in place for DMA (InPlacePin).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdarg>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "ec_engine.h"

namespace lsec {

namespace {

// The engine thread that runs quiet()'s calls while a caller's error is pending: one persistent
// thread (a hand-off costs a few microseconds; a thread per call cost tens), started at first need
// and left running for the process's life.
class QuietThread {
 public:
  static QuietThread &get() {
    static QuietThread *t = new QuietThread();  // leaked: callers may still use it during exit
    return *t;
  }
  hipError_t run(const std::function<hipError_t()> &f) {
    // the caller's current device, so that device-relative calls (module loads, allocations) act
    // where they would have on the caller's thread (a successful call leaves the caller's error)
    int dev = -1;
    if (hipGetDevice(&dev) != hipSuccess) dev = -1;
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [this] { return job_ == nullptr; });  // one call at a time
    job_ = &f;
    dev_ = dev;
    ++seq_;
    const unsigned long long mine = seq_;
    cv_.notify_one();
    done_cv_.wait(lk, [&] { return finished_ == mine; });
    const hipError_t e = result_;
    job_ = nullptr;
    done_cv_.notify_all();
    return e;
  }

 private:
  QuietThread() { std::thread([this] { loop(); }).detach(); }
  void loop() {
    std::unique_lock<std::mutex> lk(mu_);
    for (;;) {
      cv_.wait(lk, [this] { return job_ != nullptr && finished_ != seq_; });
      const std::function<hipError_t()> *f = job_;
      const unsigned long long s = seq_;
      const int dev = dev_;
      lk.unlock();
      if (dev >= 0 && hipSetDevice(dev) != hipSuccess) (void)hipGetLastError();
      hipError_t e = (*f)();
      if (e != hipSuccess) (void)hipGetLastError();  // this thread's slot: the error is the engine's
      lk.lock();
      result_ = e;
      finished_ = s;
      done_cv_.notify_all();
    }
  }
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<hipError_t()> *job_ = nullptr;
  unsigned long long seq_ = 0, finished_ = 0;
  int dev_ = -1;
  hipError_t result_ = hipSuccess;
};

}  // namespace

hipError_t quiet(const std::function<hipError_t()> &f) {
  if (hipPeekAtLastError() == hipSuccess) {
    const hipError_t e = f();
    if (e != hipSuccess) (void)hipGetLastError();  // the slot was clear: this error is the engine's own
    return e;
  }
  // the caller's error is pending: run the call where its error cannot replace the caller's
  return QuietThread::get().run(f);
}

namespace eng {

std::atomic<unsigned long long> g_st_queries{0};  // runtime pointer queries (LSEC_STATS)

thread_local int tl_memo_depth = 0;
thread_local std::vector<std::pair<const void *, PtrInfo>> tl_memo;

PtrInfo query_ptr(const void *ptr) {
  if (tl_memo_depth > 0)
    for (const auto &kv : tl_memo)
      if (kv.first == ptr) return kv.second;
  PtrInfo r;
  hipPointerAttribute_t attr;
  g_st_queries.fetch_add(1, std::memory_order_relaxed);
  // (pageable host memory reports an error on some runtimes)
  if (quiet([&] { return hipPointerGetAttributes(&attr, ptr); }) == hipSuccess) {
    r.ok = true;
    r.type = attr.type;
    r.dev = attr.devicePointer;
  }
  if (tl_memo_depth > 0 && tl_memo.size() < 64) tl_memo.push_back({ptr, r});  // small: scanned linearly
  return r;
}

// Caller buffers that are already page-locked (hipHostMalloc'd, or hipHostRegister'ed by an
// allocator that pins its cache pages) need no packing: the DMA engines copy straight
// between them and the device slots, and the host copy pool stays idle.
bool is_pinned_host(const void *ptr) {
  const PtrInfo i = query_ptr(ptr);
  return i.ok && i.type == hipMemoryTypeHost;
}

// Ranges pinned in place by a running call (InPlacePin), page-rounded.  Another call that
// touches them must not take them for caller-pinned memory: the owner unregisters them when
// it returns, maybe while the other call's DMA is still queued.
std::mutex g_inplace_mu;
std::vector<std::pair<uintptr_t, uintptr_t>> g_inplace;
std::atomic<int> g_pins_held{0};  // calls holding in-place registrations right now (InPlacePin)

bool inplace_overlaps_locked(uintptr_t lo, uintptr_t hi) {
  for (const auto &r : g_inplace)
    if (lo < r.second && r.first < hi) return true;
  return false;
}

// Which caller page-locked memory a GPU kernel may touch in place.  Kernels read and write
// hipHostMalloc allocations in place (the stripe server's direct parts, the copy-piece kernel,
// a zero-copy launch over caller chunks); ranges the caller pinned with hipHostRegister move by
// DMA only.  Round 3 found that kernels over per-call registrations of pageable memory return
// stale bytes once the process recycles host memory (profiles/r03_v16_reg_repro.jsonl), while
// DMA over the same registrations stays exact (r03_v18_churn_default_routes.jsonl).  A caller's
// own registration of its arenas is the same mechanism, and what separates the two could not be
// named from the records, so registered memory gets the transport shown safe.
// hipHostMalloc memory answers hipHostGetFlags; a hipHostRegister'ed range does not
// (profiles/r04_alloc_kind_probe.jsonl).
bool kernel_visible_allocation(const char *p) {
  unsigned flags = 0;
  return quiet([&] { return hipHostGetFlags(&flags, const_cast<char *>(p)); }) == hipSuccess;
}

// p..p+len inside one page-locked allocation with a device alias?  (its device address in *dev;
// *kernel_ok: the allocation is one kernels may touch in place)
bool pinned_chunk(const char *p, size_t len, std::vector<PinnedAlloc> &seen, uint64_t *dev, bool *kernel_ok) {
  const uintptr_t u = reinterpret_cast<uintptr_t>(p);
  for (const PinnedAlloc &a : seen)
    if (u >= a.lo && u + len <= a.hi) {
      *dev = static_cast<uint64_t>(static_cast<intptr_t>(u) + a.delta);
      if (kernel_ok) *kernel_ok = a.kernel_ok;
      return true;
    }
  const PtrInfo i = query_ptr(p);
  if (!i.ok || i.type != hipMemoryTypeHost || !i.dev) return false;
  // The extent of the page-locked range around p, as host addresses: the pointer attributes give
  // it for both kinds; hipMemGetAddressRange gives the host range of hipHostMalloc memory only (for
  // a hipHostRegister'ed range its base is not a host address, tools/probes/unregister_probe.py),
  // so a caller-registered chunk never passed this check and was packed instead of DMA'd
  void *start = nullptr;
  size_t size = 0;
  if (quiet([&] {
        const hipError_t r = hipPointerGetAttribute(&start, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR,
                                                    reinterpret_cast<hipDeviceptr_t>(const_cast<char *>(p)));
        return r != hipSuccess ? r
                               : hipPointerGetAttribute(&size, HIP_POINTER_ATTRIBUTE_RANGE_SIZE,
                                                        reinterpret_cast<hipDeviceptr_t>(const_cast<char *>(p)));
      }) != hipSuccess)
    return false;
  const uintptr_t lo = reinterpret_cast<uintptr_t>(start), hi = lo + size;
  if (u < lo || u + len > hi) return false;
  const intptr_t delta = reinterpret_cast<intptr_t>(i.dev) - static_cast<intptr_t>(u);
  const bool kok = kernel_visible_allocation(p);
  seen.push_back({lo, hi, delta, kok});
  *dev = reinterpret_cast<uint64_t>(i.dev);
  if (kernel_ok) *kernel_ok = kok;
  return true;
}

bool caller_pinned_aliases(char **ptrs, int nstripes, int km, const std::vector<int> &in_ids,
                           const std::vector<int> &out_ids, long long C, std::vector<PinnedAlloc> &seen,
                           std::vector<uint64_t> &dev);

CallerPinned caller_pinned(char **ptrs, int nstripes, int km, const std::vector<int> &in_ids, const std::vector<int> &out_ids,
                           long long C, bool kernel_ok) {
  CallerPinned r;
  if (nstripes < 1) return r;
  // A first chunk that is not page-locked settles it, with no lock: every path below returns
  // "not pinned" for it too, and taking memory for pageable is always safe.  (Per-stripe calls
  // from hundreds of threads queued on this mutex.)
  if (tl_memo_depth > 0)
    for (const auto &kv : tl_memo)  // a chunk of this call already known not to be page-locked
      if (!kv.second.ok || kv.second.type != hipMemoryTypeHost)
        for (const std::vector<int> *ids : {&in_ids, &out_ids})
          for (int id : *ids)
            if (ptrs[id] == kv.first) return r;
  if (!in_ids.empty() && !is_pinned_host(ptrs[in_ids[0]])) return r;
  std::lock_guard<std::mutex> lk(g_inplace_mu);
  if (!g_inplace.empty()) {
    for (int s = 0; s < nstripes; ++s)
      for (const std::vector<int> *ids : {&in_ids, &out_ids})
        for (int id : *ids) {
          const uintptr_t a = reinterpret_cast<uintptr_t>(ptrs[static_cast<size_t>(s) * km + id]);
          if (inplace_overlaps_locked(a & ~(kPage - 1), (a + static_cast<uintptr_t>(C) + kPage - 1) & ~(kPage - 1))) return r;
        }
  }
  // every staged shard of the first and last stripe page-locked?  (a stray pageable pointer in
  // between stays correct for DMA -- hipMemcpyAsync accepts pageable memory too, only slower;
  // the kernel transport checks every chunk, caller_pinned_aliases)
  std::vector<PinnedAlloc> seen;
  uint64_t d = 0;
  for (int s : {0, nstripes - 1}) {
    for (int id : in_ids)
      if (!pinned_chunk(ptrs[static_cast<size_t>(s) * km + id], static_cast<size_t>(C), seen, &d, nullptr)) return r;
    for (int id : out_ids)
      if (!pinned_chunk(ptrs[static_cast<size_t>(s) * km + id], static_cast<size_t>(C), seen, &d, nullptr)) return r;
  }
  r.pinned = true;
  r.by_kernel = kernel_ok && caller_pinned_aliases(ptrs, nstripes, km, in_ids, out_ids, C, seen, r.dev);
  return r;
}

namespace {
std::atomic<int> g_guard_calls{0}, g_guard_stalls{0}, g_guard_level{0};
std::atomic<long long> g_guard_until_ns{0};
std::mutex g_guard_mu;

long long steady_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

bool guard_on() {
  static const bool on = [] {
    const char *e = getenv("LSEC_INPLACE_GUARD");
    return !(e && *e == '0');
  }();
  return on;
}
}  // namespace

bool inplace_suspended() {
  if (!guard_on()) return false;
  const long long until = g_guard_until_ns.load(std::memory_order_relaxed);
  return until != 0 && steady_ns() < until;
}

void note_inplace_drain(size_t bytes, double drain_ms) {
  if (!guard_on()) return;
  const bool stall = drain_ms > 5.0 && static_cast<double>(bytes) / (drain_ms * 1e-3) < 1e9;
  const int calls = g_guard_calls.fetch_add(1, std::memory_order_relaxed) + 1;
  const int stalls = stall ? g_guard_stalls.fetch_add(1, std::memory_order_relaxed) + 1 : g_guard_stalls.load(std::memory_order_relaxed);
  if (stalls >= 3) {
    std::lock_guard<std::mutex> lk(g_guard_mu);
    if (g_guard_stalls.load(std::memory_order_relaxed) < 3) return;  // another thread suspended just now
    const int level = std::min(g_guard_level.fetch_add(1, std::memory_order_relaxed), 4);
    const long long secs = 30LL << level;  // 30 s, 60, 120, 240, 480 (10 min cap below)
    const long long s2 = std::min(secs, 600LL);
    g_guard_until_ns.store(steady_ns() + s2 * 1000000000LL, std::memory_order_relaxed);
    g_guard_calls.store(0, std::memory_order_relaxed);
    g_guard_stalls.store(0, std::memory_order_relaxed);
    fprintf(stderr, "liblstore_ec: DMA from host pages pinned in place stalled (%.1f ms for %zu B); pinning in place "
                    "suspended for %lld s, calls pack into page-locked staging (LSEC_INPLACE_GUARD=0 turns this off)\n",
            drain_ms, bytes, s2);
  } else if (calls >= 64) {  // a fresh window
    g_guard_calls.store(0, std::memory_order_relaxed);
    g_guard_stalls.store(0, std::memory_order_relaxed);
  }
}

bool InPlacePin::pin(char **ptrs, int nstripes, int km, const std::vector<int> &in_ids, const std::vector<int> &out_ids,
                     long long C, size_t min_bytes, size_t min_run) {
  if (!routes().pin_in_place || inplace_suspended()) return false;
  std::vector<std::pair<char *, char *>> pieces;
  pieces.reserve(static_cast<size_t>(nstripes) * (in_ids.size() + out_ids.size()));
  for (int s = 0; s < nstripes; ++s) {
    for (int id : in_ids) pieces.push_back({ptrs[static_cast<size_t>(s) * km + id], ptrs[static_cast<size_t>(s) * km + id] + C});
    for (int id : out_ids) pieces.push_back({ptrs[static_cast<size_t>(s) * km + id], ptrs[static_cast<size_t>(s) * km + id] + C});
  }
  std::sort(pieces.begin(), pieces.end());
  std::vector<std::pair<char *, char *>> regions;
  for (const auto &pc : pieces) {
    if (!regions.empty() && pc.first < regions.back().second) return false;  // overlapping chunks
    if (!regions.empty() && pc.first == regions.back().second)
      regions.back().second = pc.second;
    else
      regions.push_back(pc);
    if (regions.size() > kMaxRegions) return false;
  }
  size_t total = 0;
  for (const auto &r : regions) total += static_cast<size_t>(r.second - r.first);
  if (total < min_bytes) return false;  // packing a small batch is cheaper than the syscalls
  // Each DMA from registered pageable memory has a fixed cost on top of the bytes, so pin
  // only when the copies the pinned path will issue (one per run of host-contiguous chunks,
  // stripe by stripe) average >= pin_min_run; smaller runs pack faster.  History: round 1's
  // 4 MiB; 2.5 MiB from round 2 (profiles/r02_v38_sweep_c5.jsonl vs r02_v25: 800 KiB lost half
  // the rate at 1.5-2.25 MiB runs); 6 MiB from round 5, once one-region batches moved to strided
  // copies: the remaining per-run decodes at 2.5-4.5 MiB runs reached 0.76-0.87 of the link
  // pinned against 0.91-0.93 packed (RS(4+2) 1 MiB 0.769 -> 0.906, RS(6+3) 1 MiB 0.837 -> 0.913;
  // profiles/r05_v10_dma2d_ab.jsonl).
  size_t runs = 0;
  for (const std::vector<int> *ids : {&in_ids, &out_ids}) {
    const char *end = nullptr;
    for (int s = 0; s < nstripes; ++s)
      for (int id : *ids) {
        const char *b = ptrs[static_cast<size_t>(s) * km + id];
        if (b != end) ++runs;
        end = b + C;
      }
  }
  if (runs == 0) return false;
  // One region (an encode over [stripe][k+m][C] batches: every chunk moves) is one registration,
  // and its runs repeat at one stride, so they go as strided copies (issue_runs) whatever their
  // length: the per-copy cost the threshold prices is gone.  Several regions (a decode's
  // survivors with the unused parity between stripes) keep one copy per run.
  // (A lone stripe or two have no stride to share: they keep the threshold.)
  if ((regions.size() > 1 || nstripes < 4) && total / runs < min_run) return false;
  // (after the cheap checks: a query per region end)
  // Never register pages someone has already page-locked: HIP keeps one registration per range,
  // so registering a caller's registered arena again succeeds and our unregister at the end of
  // the call then drops the CALLER's registration (its own hipHostUnregister later fails with
  // hipErrorHostMemoryNotRegistered, and its kernels lose the mapping; round 5,
  // tools/probes/unregister_probe.py).  Such memory is page-locked already: it packs (or DMAs in
  // place when caller_pinned recognised it) instead.
  for (const auto &r : regions)
    for (const char *q : {static_cast<const char *>(r.first), static_cast<const char *>(r.second - 1)}) {
      const PtrInfo i = query_ptr(q);
      if (i.ok && i.type != hipMemoryTypeUnregistered) return false;
    }
  {
    // claim the page-rounded regions, so a concurrent call over the same pages packs
    std::lock_guard<std::mutex> lk(g_inplace_mu);
    for (const auto &r : regions) {
      const uintptr_t lo = reinterpret_cast<uintptr_t>(r.first) & ~(kPage - 1);
      const uintptr_t hi = (reinterpret_cast<uintptr_t>(r.second) + kPage - 1) & ~(kPage - 1);
      if (inplace_overlaps_locked(lo, hi)) {
        claimed_.clear();
        return false;
      }
      claimed_.push_back({lo, hi});
    }
    for (size_t i = 1; i < claimed_.size(); ++i)
      if (claimed_[i].first < claimed_[i - 1].second) {  // two (sorted) regions share a page
        claimed_.clear();
        return false;
      }
    g_inplace.insert(g_inplace.end(), claimed_.begin(), claimed_.end());
  }
  // whole pages (the claims above are page-rounded and disjoint)
  for (const auto &r : regions) {
    char *lo = reinterpret_cast<char *>(reinterpret_cast<uintptr_t>(r.first) & ~(kPage - 1));
    char *hi = reinterpret_cast<char *>((reinterpret_cast<uintptr_t>(r.second) + kPage - 1) & ~(kPage - 1));
    if (quiet([&] { return hipHostRegister(lo, static_cast<size_t>(hi - lo), hipHostRegisterPortable | hipHostRegisterMapped); }) !=
        hipSuccess) {
      g_pins_held.fetch_add(1, std::memory_order_acq_rel);  // (release() counts this call out)
      release();
      return false;
    }
    held_.push_back(lo);
  }
  g_pins_held.fetch_add(1, std::memory_order_acq_rel);
  return true;
}

namespace {
void unregister_all(const std::vector<char *> &held) {
  if (held.empty()) return;
  // hipHostUnregister waits for an idle device: running stripe servers step aside meanwhile
  servers_yield_begin();
  for (char *b : held)
    if (quiet([&] { return hipHostUnregister(b); }) != hipSuccess) {
      static std::atomic<bool> told{false};
      if (!told.exchange(true)) fprintf(stderr, "liblstore_ec: hipHostUnregister(%p) failed\n", static_cast<void *>(b));
    }
  servers_yield_end();
}

void unclaim(const std::vector<std::pair<uintptr_t, uintptr_t>> &claimed) {
  if (claimed.empty()) return;
  std::lock_guard<std::mutex> lk(g_inplace_mu);
  for (const auto &c : claimed) {
    auto it = std::find(g_inplace.begin(), g_inplace.end(), c);
    if (it != g_inplace.end()) g_inplace.erase(it);
  }
}

// hipHostUnregister waits until every queue of the device is idle (tools/probes/
// unregister_wait_probe.cpp: 4.5 ms behind another thread's 256 MiB copy, and no progress at all
// while that thread re-submits after each hipStreamSynchronize), so two callers' registrations
// released at the ends of their calls march in lockstep.  With LSEC_DEFER_UNPIN_MB the release
// goes to this thread instead: the ranges stay claimed (no other call takes or re-registers them)
// until they are unregistered, and a caller whose release would put more than the cap in flight
// waits for the backlog.  Leaked singleton: registrations still pending at exit go with the process.
class Unpinner {
 public:
  static Unpinner &get() {
    static Unpinner *u = new Unpinner();
    return *u;
  }
  // until nothing is pending (lsec_host_unpin_drain)
  void drain() {
    std::unique_lock<std::mutex> lk(mu_);
    done_.wait(lk, [&] { return exiting_ || (pending_ == 0 && q_.empty()); });
  }
  // at exit, before the runtime's own teardown (registered after it, so run before it): a bounded
  // wait, since an unregister waits for work other threads may still have on the device
  // After the wait, whatever is still queued is dropped with no runtime call: the thread starts no
  // unregister once the runtime's teardown may be under way (the registrations go
  // with the process).
  static void drain_at_exit() {
    Unpinner &u = get();
    std::unique_lock<std::mutex> lk(u.mu_);
    u.done_.wait_for(lk, std::chrono::seconds(2), [&] { return u.pending_ == 0 && u.q_.empty(); });
    u.exiting_ = true;
    u.q_.clear();
    u.work_.notify_all();
    u.done_.notify_all();
  }
  void put(std::vector<char *> held, std::vector<std::pair<uintptr_t, uintptr_t>> claimed, size_t bytes, size_t cap) {
    std::unique_lock<std::mutex> lk(mu_);
    done_.wait(lk, [&] { return exiting_ || pending_ == 0 || pending_ + bytes <= cap; });
    if (exiting_) return;  // (the process is exiting: the registrations go with it)
    q_.push_back({std::move(held), std::move(claimed), bytes});
    pending_ += bytes;
    work_.notify_one();
  }

 private:
  struct Item {
    std::vector<char *> held;
    std::vector<std::pair<uintptr_t, uintptr_t>> claimed;
    size_t bytes;
  };
  Unpinner() {
    std::thread([this] { loop(); }).detach();
    std::atexit(drain_at_exit);
  }
  void loop() {
    for (;;) {
      Item it;
      {
        std::unique_lock<std::mutex> lk(mu_);
        work_.wait(lk, [&] { return !q_.empty() || exiting_; });
        if (exiting_) return;
        it = std::move(q_.front());
        q_.pop_front();
      }
      unregister_all(it.held);
      unclaim(it.claimed);
      std::lock_guard<std::mutex> lk(mu_);
      pending_ -= it.bytes;
      done_.notify_all();
    }
  }
  std::mutex mu_;
  std::condition_variable work_, done_;
  std::deque<Item> q_;
  size_t pending_ = 0;
  bool exiting_ = false;  // set by drain_at_exit: no unregister starts after it
};
}  // namespace

std::atomic<Unpinner *> g_unpinner{nullptr};  // set once the first deferred release made it

int in_place_calls() { return g_pins_held.load(std::memory_order_acquire); }

void InPlacePin::release() {
  if (held_.empty() && claimed_.empty()) return;
  const bool others = g_pins_held.fetch_sub(1, std::memory_order_acq_rel) > 1;
  const size_t cap = routes().defer_unpin_bytes;
  // deferred only while another call is in flight: alone, the unregister is immediate (the runtime
  // re-registers recently registered pages in microseconds, and nothing else of ours is running)
  if (cap > 0 && others && !held_.empty()) {
    g_unpinner.store(&Unpinner::get(), std::memory_order_release);
    size_t bytes = 0;
    for (const auto &c : claimed_) bytes += c.second - c.first;
    Unpinner::get().put(std::move(held_), std::move(claimed_), bytes, cap);
    held_.clear();
    claimed_.clear();
    return;
  }
  unregister_all(held_);
  held_.clear();
  unclaim(claimed_);
  claimed_.clear();
}

void add_run(std::vector<DmaRun> &v, char *dst, const char *src, size_t n) {
  if (!v.empty() && v.back().dst + v.back().bytes == dst && v.back().src + v.back().bytes == src)
    v.back().bytes += n;
  else
    v.push_back({dst, src, n});
}

// kernel transport pieces of one chunk (addresses already device-visible)
// (returns 0 when either address is 0 -- a host byte outside the pinned regions -- so the
// caller stops before launching)
size_t add_pieces(lsec::CopyPiece *pl, size_t n, uint64_t src, uint64_t dst, size_t len) {
  if (src == 0 || dst == 0) return 0;
  for (size_t o = 0; o < len; o += lsec::kPieceBytes) pl[n++] = {src + o, dst + o, std::min<uint64_t>(lsec::kPieceBytes, len - o)};
  return n;
}

KernelCopy kernel_copy_policy() { return routes().kernel_copy ? KernelCopy::kCallerPinned : KernelCopy::kNever; }

// every transferred chunk (and column block) 16-byte aligned, as the copy-piece kernel needs
bool kernel_transport_aligned(char **ptrs, int nstripes, int km, const std::vector<int> &in_ids,
                              const std::vector<int> &out_ids, long long C, long long cb) {
  if (C % 16 != 0 || cb % 16 != 0) return false;
  for (int s = 0; s < nstripes; ++s)
    for (const std::vector<int> *ids : {&in_ids, &out_ids})
      for (int id : *ids)
        if (reinterpret_cast<uintptr_t>(ptrs[static_cast<size_t>(s) * km + id]) % 16 != 0) return false;
  return true;
}

// Caller page-locked buffers with small runs (average < 1 MiB: DMA of 384 KiB runs from
// hipHostMalloc memory moves ~20 GiB/s, profiles/r01_v27_kernel_copy_ab.txt) move by kernel,
// once EVERY chunk is checked: page-locked, inside one allocation, with a device address
// (a pageable chunk between pinned ones is harmless to a DMA but would fault a kernel).  The
// check costs ~0.06 us per chunk (tools/probes/pinned_attr_probe.cpp).  dev[i] gets the device
// address of chunk i, in the order stripe, then in_ids, then out_ids.
// (called by caller_pinned with g_inplace_mu held)
bool caller_pinned_aliases(char **ptrs, int nstripes, int km, const std::vector<int> &in_ids,
                           const std::vector<int> &out_ids, long long C, std::vector<PinnedAlloc> &seen,
                           std::vector<uint64_t> &dev) {
  size_t runs = 0, total = 0;
  for (const std::vector<int> *ids : {&in_ids, &out_ids}) {
    const char *end = nullptr;
    for (int s = 0; s < nstripes; ++s)
      for (int id : *ids) {
        const char *b = ptrs[static_cast<size_t>(s) * km + id];
        if (b != end) ++runs;
        end = b + C;
        total += static_cast<size_t>(C);
      }
  }
  if (runs == 0 || total / runs >= routes().kernel_copy_max_run) return false;
  dev.clear();
  dev.reserve(static_cast<size_t>(nstripes) * (in_ids.size() + out_ids.size()));
  for (int s = 0; s < nstripes; ++s)
    for (const std::vector<int> *ids : {&in_ids, &out_ids})
      for (int id : *ids) {
        uint64_t d = 0;
        bool kok = false;
        if (!pinned_chunk(ptrs[static_cast<size_t>(s) * km + id], static_cast<size_t>(C), seen, &d, &kok) || !kok) return false;
        dev.push_back(d);
      }
  return true;
}

void split_pieces(std::vector<lsec::CopyPiece> &v, uint64_t src, uint64_t dst, size_t len) {
  for (size_t o = 0; o < len; o += lsec::kPieceBytes) v.push_back({src + o, dst + o, std::min<uint64_t>(lsec::kPieceBytes, len - o)});
}

// Runs that repeat with one stripe stride on both sides (the p chunks a stripe moves, stripe after
// stripe: p = 1 for encode's k data chunks, 2 for a decode whose erasure splits the survivors) go
// as p strided copies (hipMemcpy2DAsync, one row per stripe) instead of one copy per run: per-copy
// gaps hold one copy per 4 MiB run to 49.5 GB/s of the link's 57.6 H2D, and 1-2 MiB D2H runs to
// 10-45 GB/s, where the strided copy runs at 57.6 / 57.0 (profiles/r05_v10_rect_probe.jsonl).
// LSEC_DMA_2D=0 issues one copy per run.
// Rows this wide already move at 0.97+ of the link one copy at a time, and strided copies of them
// lost to plain copies when two processes shared the device's DMA engines (c4, Cauchy-good(10+4)
// 4 MiB, 40 MiB rows, two ranks on one GPU: 14.9 against 23.2 GiB/s per rank pageable encode;
// one process alone 51.3 against 48.7; profiles/r05_v18_c4_dma2d_ab.jsonl).
constexpr size_t kMaxLatticeRow = 16u << 20;

struct Lattice {
  size_t period = 0, rows = 0;
  ptrdiff_t sp = 0, dp = 0;
};

// the longest lattice starting at v[i]: `period` runs repeated `rows` times at strides sp / dp
Lattice lattice_at(const std::vector<DmaRun> &v, size_t i) {
  Lattice best;
  const size_t n = v.size();
  for (size_t p = 1; p <= 8 && i + p < n; ++p) {
    const ptrdiff_t sp = v[i + p].src - v[i].src, dp = v[i + p].dst - v[i].dst;
    if (sp <= 0 || dp <= 0) continue;
    bool fits = true;  // every lane's row fits its pitch, and is narrower than kMaxLatticeRow
    for (size_t l = 0; l < p && fits; ++l)
      fits = static_cast<size_t>(sp) >= v[i + l].bytes && static_cast<size_t>(dp) >= v[i + l].bytes && v[i + l].bytes < kMaxLatticeRow;
    if (!fits) continue;
    size_t rows = 1;
    for (;; ++rows) {
      const size_t b = i + rows * p;
      if (b + p > n) break;
      bool same = true;
      for (size_t l = 0; l < p && same; ++l)
        same = v[b + l].bytes == v[i + l].bytes && v[b + l].src - v[b + l - p].src == sp && v[b + l].dst - v[b + l - p].dst == dp;
      if (!same) break;
    }
    if (rows >= 2 && rows * p > best.rows * best.period) best = {p, rows, sp, dp};
  }
  return best;
}

namespace {
// [p, p + span) inside one allocation or registered range: a strided copy is validated against
// the allocation holding its first byte, and in-place pinning registers only the chunks a call
// moves, so a lattice over a decode's survivors can step over unregistered chunks
// (hipMemcpy2DAsync: invalid argument)
bool one_range(const char *p, size_t span) {
  void *start = nullptr;
  size_t size = 0;
  const hipDeviceptr_t d = reinterpret_cast<hipDeviceptr_t>(const_cast<char *>(p));
  if (quiet([&] {
        const hipError_t r = hipPointerGetAttribute(&start, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR, d);
        return r != hipSuccess ? r : hipPointerGetAttribute(&size, HIP_POINTER_ATTRIBUTE_RANGE_SIZE, d);
      }) != hipSuccess)
    return false;
  const uintptr_t lo = reinterpret_cast<uintptr_t>(start), u = reinterpret_cast<uintptr_t>(p);
  return u >= lo && u + span <= lo + size;
}

bool lattice_in_ranges(const std::vector<DmaRun> &v, size_t i, const Lattice &g) {
  size_t lo_s = SIZE_MAX, hi_s = 0, lo_d = SIZE_MAX, hi_d = 0;
  for (size_t l = 0; l < g.period; ++l) {
    const DmaRun &a = v[i + l], &b = v[i + (g.rows - 1) * g.period + l];
    lo_s = std::min(lo_s, reinterpret_cast<size_t>(a.src));
    hi_s = std::max(hi_s, reinterpret_cast<size_t>(b.src) + b.bytes);
    lo_d = std::min(lo_d, reinterpret_cast<size_t>(a.dst));
    hi_d = std::max(hi_d, reinterpret_cast<size_t>(b.dst) + b.bytes);
  }
  return one_range(reinterpret_cast<const char *>(lo_s), hi_s - lo_s) &&
         one_range(reinterpret_cast<const char *>(lo_d), hi_d - lo_d);
}
}  // namespace

hipError_t issue_runs(const std::vector<DmaRun> &v, hipMemcpyKind kind, hipStream_t st) {
  static const bool strided = [] {
    const char *e = getenv("LSEC_DMA_2D");
    return !(e && *e == '0');
  }();
  for (size_t i = 0; i < v.size();) {
    const Lattice g = strided ? lattice_at(v, i) : Lattice{};
    const size_t end = g.rows >= 2 ? i + g.period * g.rows : i + 1;
    if (g.rows >= 2 && lattice_in_ranges(v, i, g)) {
      for (size_t l = 0; l < g.period; ++l) {
        const DmaRun &r = v[i + l];
        const hipError_t e = hipMemcpy2DAsync(r.dst, static_cast<size_t>(g.dp), r.src, static_cast<size_t>(g.sp), r.bytes, g.rows, kind, st);
        if (e != hipSuccess) return e;
      }
    } else {  // (a lattice over more than one range: its runs one by one)
      for (size_t j = i; j < end; ++j) {
        const hipError_t e = hipMemcpyAsync(v[j].dst, v[j].src, v[j].bytes, kind, st);
        if (e != hipSuccess) return e;
      }
    }
    i = end;
  }
  return hipSuccess;
}

}  // namespace eng
}  // namespace lsec

// Test hook, not part of include/*.h: how issue_runs would group n DMA runs (dst[i], src[i],
// bytes[i], in issue order) into strided lattices, before the registered-range check (which needs
// the runtime).  Writes (first run, period, rows, src pitch, dst pitch) per group to out; a lone
// run is period 1, rows 1.  Returns the number of groups, or -1 when out_cap is too small.
// include/lstore_ec.h: wait until every in-place registration a call left to the background
// unpinner is dropped (before the caller registers host memory with HIP itself)
// Test hook, not part of include/*.h: the in-place stall guard without a GPU.  op 0: reset (no
// suspension, empty window); op 1: report one pinned call's drain (bytes, drain_ms); op 2: 1 while
// pinning in place is suspended, else 0.
extern "C" int lsec_test_inplace_guard(int op, unsigned long long bytes, double drain_ms) {
  using namespace lsec::eng;
  if (op == 0) {
    g_guard_calls.store(0);
    g_guard_stalls.store(0);
    g_guard_level.store(0);
    g_guard_until_ns.store(0);
    return 0;
  }
  if (op == 1) {
    note_inplace_drain(static_cast<size_t>(bytes), drain_ms);
    return 0;
  }
  return inplace_suspended() ? 1 : 0;
}

extern "C" int lsec_host_unpin_drain(void) {
  if (lsec::eng::Unpinner *u = lsec::eng::g_unpinner.load(std::memory_order_acquire)) u->drain();
  return 0;
}

extern "C" int lsec_test_lattices(const uint64_t *dst, const uint64_t *src, const uint64_t *bytes, int n, int64_t *out,
                                  int out_cap) {
  std::vector<lsec::eng::DmaRun> v;
  for (int i = 0; i < n; ++i)
    v.push_back({reinterpret_cast<char *>(dst[i]), reinterpret_cast<const char *>(src[i]), static_cast<size_t>(bytes[i])});
  int groups = 0;
  for (size_t i = 0; i < v.size();) {
    const lsec::eng::Lattice g = lsec::eng::lattice_at(v, i);
    const bool lat = g.rows >= 2;
    if (groups >= out_cap) return -1;
    int64_t *o = out + 5 * groups++;
    o[0] = static_cast<int64_t>(i);
    o[1] = lat ? static_cast<int64_t>(g.period) : 1;
    o[2] = lat ? static_cast<int64_t>(g.rows) : 1;
    o[3] = lat ? g.sp : 0;
    o[4] = lat ? g.dp : 0;
    i += lat ? g.period * g.rows : 1;
  }
  return groups;
}
