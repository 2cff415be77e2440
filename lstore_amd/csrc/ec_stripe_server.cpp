// ec_stripe_server.cpp -- route 1: the host side of the persistent stripe server (ec_server.hip):
// slot claims, posts, waits, the idle retirement and relaunch, and the stop / settle protocol.
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

// ---------------------------------------------------------------- stripe server (host side)
// Per-stripe calls up to kSlotBytes per part are served by the persistent stripe server
// (ec_server.hip): the calling thread claims slots, copies its chunks' column blocks into them
// (or, for page-locked caller chunks, just names their device addresses), posts one descriptor
// per part and spins on the parts' done flags.  No launch, no DMA and no other host thread per
// call; the server's workgroups serve the parts of many callers in parallel.  The server exits
// after 2 ms without work and is relaunched by the next caller (or by a waiting one that finds
// it gone).  LSEC_SERVER=0 turns it off.
// the stripe server's answer time limit (LSEC test hook lsec_test_server_hold) and its hold
std::atomic<int> g_srv_timeout_ms{5000};
std::atomic<int> g_srv_hold{0};
std::atomic<unsigned long long> g_st_srv_timeouts{0};
// In-place releases running (servers_yield_begin / _end): no server launches meanwhile
std::atomic<int> g_srv_yield{0};
std::atomic<unsigned long long> g_st_srv_yields{0};
std::mutex g_registry_mu;  // the registry of servers (creation, and the walks of stop_all / yield)

class StripeServer {
 public:
  static StripeServer *for_device(int dev) {
    // every per-stripe call asks: a lock-free read once the device's server exists
    static std::atomic<StripeServer *> fast[64] = {};
    if (dev >= 0 && dev < 64)
      if (StripeServer *f = fast[dev].load(std::memory_order_acquire)) return f;
    static std::map<int, StripeServer *> all;  // intentionally leaked: lives until exit
    std::lock_guard<std::mutex> lk(g_registry_mu);
    StripeServer *&r = all[dev];
    if (!r) {
      r = new StripeServer(dev);
      registry().push_back(r);
      static std::once_flag once;
      std::call_once(once, [] { atexit(stop_all); });
    }
    if (dev >= 0 && dev < 64) fast[dev].store(r, std::memory_order_release);
    return r;
  }

  // 0 served, -1 error, 1 not servable here (the caller takes another path)
  int run(PlanExt *e, char **ptrs, long long C, const std::vector<int> &in_ids, const std::vector<int> &out_ids,
          const void *image, int kind, const CallerPinned *cp) {
    const auto t_enter = std::chrono::steady_clock::now();
    const bool stats = ZcStats::on();
    const long long c_enter = stats ? thread_cpu_ns() : 0;
    long long c_post = 0, c_waited = 0;
    const size_t nin = in_ids.size(), nout = out_ids.size(), nio = nin + nout;
    const auto refuse = [] {
      ZcStats::get().not_servable.fetch_add(1, std::memory_order_relaxed);
      return 1;
    };
    if (nin < 1 || nout < 1 || nin > lsec::kSrvMaxK || nout > lsec::kSrvMaxR) return refuse();
    if (kind != KBYTEWISE && kind != KBITSLICED) return refuse();
    // a server that cannot be set up or launched is never posted to: the call takes its own
    // zero-copy launch or the dispatcher (a post nobody will serve would strand its slots)
    if (broken_.load(std::memory_order_acquire)) return refuse();
    if (init_once()) {
      broken_ = true;
      return refuse();
    }
    const lio_erasure_plan_t *p = &e->pub;
    const bool direct = cp && cp->by_kernel;
    // calls whose parts the server reads and writes in the caller's own buffers: a server that
    // cannot be stopped while any is in flight ends the process (stop_and_settle)
    struct DirectCall {
      std::atomic<int> *n;
      explicit DirectCall(std::atomic<int> *c) : n(c) {
        if (n) n->fetch_add(1, std::memory_order_acq_rel);
      }
      ~DirectCall() {
        if (n) n->fetch_sub(1, std::memory_order_acq_rel);
      }
    } direct_call(direct ? &direct_inflight_ : nullptr);
    // parts: column blocks of about 4 KiB per shard (one 256-lane x 16 B pass), whole
    // super-packets for the bit-sliced layout, at most kMaxParts of them
    const long long unit = kind == KBITSLICED ? 8LL * p->packet_size : 16;
    const long long max_len = direct ? C : static_cast<long long>(kSlotBytes / nio) / unit * unit;
    if (max_len < std::min<long long>(unit, C)) return refuse();
    // column bytes per part: 4 KiB (4-16 KiB parts measured level, profiles/r02_v22_server_part_ab.jsonl)
    constexpr long long target = 4096;
    long long len = std::min(std::max<long long>(unit, target / unit * unit), max_len);
    if ((C + len - 1) / len > kMaxParts) {
      len = ((C + kMaxParts - 1) / kMaxParts + unit - 1) / unit * unit;
      if (len > max_len) return refuse();
    }
    if (len > C) len = C;
    int nparts = static_cast<int>((C + len - 1) / len);
    int slot[kMaxParts];
    if (!claim(nparts, slot)) {
      // under load: fewer, larger parts (as many columns as a slot holds), then a short wait for
      // slots to come free -- the other route, a launch of this call's own, costs the host far
      // more CPU per call than a wait (profiles/r02_v28_zc_routes.txt)
      bool got = false;
      g_st_claim_misses.fetch_add(1, std::memory_order_relaxed);
      if (len < std::min(max_len, C)) {
        len = std::min(max_len, C);
        nparts = static_cast<int>((C + len - 1) / len);
        got = claim(nparts, slot);
      }
      const auto t0 = std::chrono::steady_clock::now();
      while (!got && std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(50)) {
        std::this_thread::yield();
        g_st_claim_spins.fetch_add(1, std::memory_order_relaxed);
        got = claim(nparts, slot);
      }
      if (!got) {
        ZcStats::get().no_slots.fetch_add(1, std::memory_order_relaxed);
        return 1;
      }
    }
    uint32_t want[kMaxParts];
    const bool nt = static_cast<size_t>(C) * nin >= routes().srv_nt_min;
    for (int q = 0; q < nparts; ++q) {
      const int sl = slot[q];
      const long long c0 = static_cast<long long>(q) * len, n = std::min(len, C - c0);
      lsec::SrvDesc &d = sh_->desc[sl];
      d.kind = kind == KBITSLICED ? lsec::kSrvBitsliced : lsec::kSrvBytewise;
      d.K = static_cast<uint32_t>(nin);
      d.R = static_cast<uint32_t>(nout);
      d.packet = static_cast<uint32_t>(p->packet_size);
      d.size = static_cast<uint64_t>(n);
      d.cells = reinterpret_cast<uint64_t>(image);
      d.cstride = static_cast<uint32_t>(nin);
      if (direct) {
        for (size_t j = 0; j < nin; ++j) d.in[j] = cp->dev[j] + static_cast<uint64_t>(c0);
        for (size_t r = 0; r < nout; ++r) d.out[r] = cp->dev[nin + r] + static_cast<uint64_t>(c0);
      } else {
        char *region = data_ + static_cast<size_t>(sl) * kSlotBytes;
        const uint64_t dregion = data_dev_ + static_cast<uint64_t>(sl) * kSlotBytes;
        for (size_t j = 0; j < nin; ++j) {
          // plain stores: for these 4 KiB pieces streaming ones cost 15 -> 18 us p50 at one
          // thread (the server reads them back from DRAM instead of the host's caches;
          // profiles/r03_v27_fnptr_fair.jsonl); calls of srv_nt_min bytes and more stream
          if (nt) host_copy(region + j * n, ptrs[in_ids[j]] + c0, static_cast<size_t>(n));
          else std::memcpy(region + j * n, ptrs[in_ids[j]] + c0, static_cast<size_t>(n));
          d.in[j] = dregion + j * n;
        }
        if (nt) _mm_sfence();
        for (size_t r = 0; r < nout; ++r) d.out[r] = dregion + (nin + r) * n;
      }
      want[q] = ++seq_[sl] == 0 ? ++seq_[sl] : seq_[sl];
      __atomic_store_n(&sh_->post[lsec::srv_wg(sl)][lsec::srv_word(sl)], want[q], __ATOMIC_RELEASE);
    }
    const auto t_post = std::chrono::steady_clock::now();
    if (stats) c_post = thread_cpu_ns();
    int rc = ensure_running(false);
    const auto t0 = std::chrono::steady_clock::now();
    auto last_check = t0;
    const unsigned *flags[kMaxParts];
    for (int q = 0; q < nparts; ++q) flags[q] = &sh_->done[slot[q]][0];
    const auto timeout = std::chrono::milliseconds(g_srv_timeout_ms.load(std::memory_order_relaxed));
    bool late = false;
    // outputs of parts [0, copied) are in the caller's buffers: a spinning wait copies each part out
    // as soon as it and the parts before it are done, while the server serves the later ones (a
    // 64 KiB decode's 16 parts finish over ~9 us; profiles/r04_v4_phases_64k.txt)
    int copied = 0;
    const auto copy_out = [&](int upto) {
      for (; copied < upto; ++copied) {
        const long long c0 = static_cast<long long>(copied) * len, n = std::min(len, C - c0);
        const char *region = data_ + static_cast<size_t>(slot[copied]) * kSlotBytes;
        for (size_t r = 0; r < nout; ++r) std::memcpy(ptrs[out_ids[r]] + c0, region + (nin + r) * n, static_cast<size_t>(n));
      }
    };
    using CopyOut = decltype(copy_out);
    const WaitProgress early{[](void *ctx, int upto) { (*static_cast<const CopyOut *>(ctx))(upto); },
                             const_cast<void *>(static_cast<const void *>(&copy_out))};
    const WaitProgress *progress = !direct && routes().srv_early_out ? &early : nullptr;
    // spin or park (FlagWaits) until every part is done, checking every 500 us that the server
    // has not retired meanwhile (it retires only after 2 ms without work; at 100 us slices a
    // loaded box woke 1.5 parked waiters per call just to check, profiles/r02_v30_zc_phases3.txt)
    while (rc == 0 && !flag_wait(flags, want, nparts, std::chrono::microseconds(500), progress)) {
      const auto now = std::chrono::steady_clock::now();
      if (now - last_check > std::chrono::microseconds(500)) {
        last_check = now;
        if ((rc = ensure_running(true))) break;
      }
      if (now - t0 > timeout) {
        late = true;
        break;
      }
    }
    if (rc != 0 || late) {
      // No answer in time (a throttled box, a stuck server) or no server: stop it and wait until
      // it has left, so no post of this call can be served after the call returns -- for
      // page-locked callers the server writes the caller's own buffers.  Parts served meanwhile
      // count; the others are cancelled and the call takes another route (return 1).
      g_st_srv_timeouts.fetch_add(1, std::memory_order_relaxed);
      std::lock_guard<std::mutex> lk(mu_);
      const int served = stop_and_settle(nparts, slot, want);
      if (served < 0) return 1;  // a server that would not stop: its slots stay claimed for good
      if (served != nparts) {
        release(nparts, slot);
        return 1;
      }
      rc = 0;
    }
    const auto t_waited = std::chrono::steady_clock::now();
    if (stats) c_waited = thread_cpu_ns();
    static const bool trace = getenv("LSEC_TRACE") != nullptr;
    if (trace) {  // calls slower than 1 ms: where the time went
      const auto t_end = std::chrono::steady_clock::now();
      const auto us = [](std::chrono::steady_clock::duration d) { return std::chrono::duration<double, std::micro>(d).count(); };
      if (t_end - t_post > std::chrono::milliseconds(1))
        fprintf(stderr, "[lsec trace] server call %d parts (slots %d..): ensure %.1f us, wait %.1f us, rc %d\n", nparts, slot[0],
                us(t0 - t_post), us(t_end - t0), rc);
    }
    if (rc == 0)
      last_seen_us_.store(std::chrono::duration_cast<std::chrono::microseconds>(
                              std::chrono::steady_clock::now().time_since_epoch()).count(),
                          std::memory_order_relaxed);
    if (rc == 0 && !direct) copy_out(nparts);
    release(nparts, slot);
    if (rc == 0 && stats) {
      ZcStats &z = ZcStats::get();
      const auto ns = [](std::chrono::steady_clock::duration d) {
        return static_cast<unsigned long long>(std::chrono::duration_cast<std::chrono::nanoseconds>(d).count());
      };
      const auto t_done = std::chrono::steady_clock::now();
      if (tl_call_t0.time_since_epoch().count() && t_enter > tl_call_t0) z.t_setup.fetch_add(ns(t_enter - tl_call_t0), std::memory_order_relaxed);
      if (tl_zc_t0.time_since_epoch().count() && t_enter > tl_zc_t0) z.t_zc.fetch_add(ns(t_enter - tl_zc_t0), std::memory_order_relaxed);
      z.t_post.fetch_add(ns(t_post - t_enter), std::memory_order_relaxed);
      z.t_wait.fetch_add(ns(t_waited - t_post), std::memory_order_relaxed);
      z.t_out.fetch_add(ns(t_done - t_waited), std::memory_order_relaxed);
      const long long c_done = thread_cpu_ns();
      if (tl_call_cpu0 && c_enter > tl_call_cpu0) z.c_setup.fetch_add(c_enter - tl_call_cpu0, std::memory_order_relaxed);
      if (tl_zc_cpu0 && c_enter > tl_zc_cpu0) z.c_zc.fetch_add(c_enter - tl_zc_cpu0, std::memory_order_relaxed);
      z.c_post.fetch_add(c_post - c_enter, std::memory_order_relaxed);
      z.c_wait.fetch_add(c_waited - c_post, std::memory_order_relaxed);
      z.c_out.fetch_add(c_done - c_waited, std::memory_order_relaxed);
    }
    return rc;
  }

 private:
  static constexpr size_t kSlotBytes = lsec::kSrvSlotBytes;  // chunk bytes of one part (inputs + outputs)
  static constexpr int kMaxParts = 16;

  explicit StripeServer(int dev) : dev_(dev) {
    for (auto &b : busy_) b.store(0);
    for (auto &q : seq_) q = 0;
  }

  static std::vector<StripeServer *> &registry() {
    // leaked: stop_all runs from atexit and must find it intact (a function-local static
    // constructed after the atexit registration would be destroyed before stop_all runs)
    static std::vector<StripeServer *> *r = new std::vector<StripeServer *>();
    return *r;
  }
  // at exit: stop every running server and let it drain (its stop word is read on every idle poll)
  static void stop_all() {
    std::lock_guard<std::mutex> rk(g_registry_mu);
    for (StripeServer *s : registry()) {
      std::lock_guard<std::mutex> lk(s->mu_);
      if (s->sh_) s->stop_and_settle(0, nullptr, nullptr);
    }
  }

 public:
  // test hook (lsec_test_server_hold): stop every server, so the next launch takes the new hold
  static void restart_all() { stop_all(); }
  // servers_yield_begin: stop the running launches.  No part is cancelled: what was posted and
  // not yet served stays posted, and the next launch serves it (as after an idle retirement).
  static void stop_running() {
    std::lock_guard<std::mutex> rk(g_registry_mu);
    for (StripeServer *s : registry()) {
      if (!s->running_.load(std::memory_order_acquire)) continue;
      std::lock_guard<std::mutex> lk(s->mu_);
      if (s->sh_ && s->running_) {
        s->stop_and_settle(0, nullptr, nullptr);
        s->yield_stopped_.store(true, std::memory_order_release);
        g_st_srv_yields.fetch_add(1, std::memory_order_relaxed);
      }
    }
  }
  // servers_yield_end, the last release done: relaunch the servers a release stopped, so calls
  // posted meanwhile are served now rather than at their wait loop's next check
  static void relaunch_yielded() {
    std::lock_guard<std::mutex> rk(g_registry_mu);
    for (StripeServer *s : registry())
      if (s->yield_stopped_.exchange(false, std::memory_order_acq_rel)) (void)s->ensure_running(false);
  }

 private:
  // Stop the running server and wait (bounded) until it has left.  The stop word is final (the
  // kernel picks nothing after it sees it, ec_server.hip), so the launch leaves after the parts
  // its workgroups are serving; afterwards nothing can serve a post until the next launch, which
  // takes served[] from done[].  Of this call's parts, those served count; the rest are
  // cancelled by setting done to the posted value, so no later launch serves them.  Returns
  // the number served.  mu_ held.
  // A server still there after 30 s (a hung device) may yet write whatever it was serving.  If
  // any call in flight has the server write the caller's own page-locked buffers in place
  // (direct_inflight_), the process ends: those buffers may not be handed back while a kernel can
  // write them.  Otherwise it writes only its own slot region: the server is marked broken (no
  // call posts to it again), the caller abandons its slots, and -1 is returned.
  int stop_and_settle(int nparts, const int *slot, const uint32_t *want) {
    if (zombie_) return -1;
    if (running_) {
      for (int g = 0; g < lsec::kSrvWG; ++g) __atomic_store_n(&sh_->post[g][lsec::kSrvSlotsPerWG], 1u, __ATOMIC_RELEASE);
      const auto t0 = std::chrono::steady_clock::now();
      for (;;) {
        const hipError_t q = hipEventQuery(ev_);
        if (q == hipSuccess) break;
        if (q != hipErrorNotReady) {  // the device failed: nothing runs there any more
          (void)hipGetLastError();
          broken_ = true;
          break;
        }
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(kStopWaitS)) {
          if (direct_inflight_.load(std::memory_order_acquire) > 0)
            fatal("the stripe server on device %d did not stop within %d s while it serves page-locked caller "
                  "buffers in place", dev_, kStopWaitS);
          broken_ = true;
          zombie_ = true;
          fprintf(stderr, "liblstore_ec: the stripe server on device %d did not stop within %d s; its slots are "
                  "abandoned and this device's per-stripe calls take other routes\n", dev_, kStopWaitS);
          return -1;
        }
        std::this_thread::sleep_for(std::chrono::microseconds(100));
      }
      running_ = false;
    }
    int served = 0;
    for (int q = 0; q < nparts; ++q) {
      unsigned *d = &sh_->done[slot[q]][0];
      if (__atomic_load_n(d, __ATOMIC_ACQUIRE) == want[q]) ++served;
      else __atomic_store_n(d, want[q], __ATOMIC_RELEASE);
    }
    return served;
  }

  bool claim(int n, int *slot) {
    static std::atomic<unsigned> next{0};
    thread_local unsigned base = next.fetch_add(7919) % lsec::kSrvSlots;
    int got = 0;
    for (int k = 0; k < lsec::kSrvSlots && got < n; ++k) {
      const int s = static_cast<int>((base + k) % lsec::kSrvSlots);
      uint8_t z = 0;
      // look before the locked exchange: under load most slots are busy, and a failed
      // exchange on every one of them from every thread kept the flag lines bouncing
      if (busy_[s].load(std::memory_order_relaxed) == 0 && busy_[s].compare_exchange_strong(z, 1)) slot[got++] = s;
    }
    if (got < n) {
      release(got, slot);
      return false;
    }
    return true;
  }
  void release(int n, const int *slot) {
    for (int q = 0; q < n; ++q) busy_[slot[q]].store(0, std::memory_order_release);
  }

  int init_once() {
    if (ready_.load(std::memory_order_acquire)) return 0;
    std::lock_guard<std::mutex> lk(mu_);
    if (ready_.load()) return 0;
    DeviceGuardLite g(dev_);
    int lo = 0, hi = 0;
    HIP_OK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    HIP_OK(hipStreamCreateWithPriority(&st_, hipStreamNonBlocking, hi));  // a hardware queue of its own
    HIP_OK(hipEventCreateWithFlags(&ev_, hipEventDisableTiming));
    HIP_OK(hipMalloc(reinterpret_cast<void **>(&votes_), 64));
    HIP_OK(hipMemset(votes_, 0, 64));
    HIP_OK(hipHostMalloc(reinterpret_cast<void **>(&sh_), sizeof(lsec::SrvShared), hipHostMallocCoherent));
    std::memset(static_cast<void *>(sh_), 0, sizeof(lsec::SrvShared));
    void *p = nullptr;
    HIP_OK(hipHostGetDevicePointer(&p, sh_, 0));
    sh_dev_ = reinterpret_cast<uint64_t>(p);
    // the slot region: about 93 MiB per device, accounted as the device's server memory, apart
    // from the threads' slot budget (PinnedBudget)
    const size_t region = kSlotBytes * lsec::kSrvSlots;
    if (quiet([&] { return hipHostMalloc(reinterpret_cast<void **>(&data_), region, hipHostMallocCoherent); }) != hipSuccess) {
      return fail("stripe server: cannot allocate its slots");
    }
    PinnedBudget::global().add_server(dev_, region);
    HIP_OK(hipHostGetDevicePointer(&p, data_, 0));
    data_dev_ = reinterpret_cast<uint64_t>(p);
    ready_.store(true, std::memory_order_release);
    return 0;
  }

  int ensure_running(bool check) {
    // the server retires after 2 ms without work: past 1.5 ms since a part was last seen done,
    // ask the runtime whether it is still there before relying on it
    const int64_t now = std::chrono::duration_cast<std::chrono::microseconds>(
                            std::chrono::steady_clock::now().time_since_epoch()).count();
    if (!check && now - last_seen_us_.load(std::memory_order_relaxed) > 1500) check = true;
    if (!check && running_.load(std::memory_order_acquire)) return 0;
    if (running_.load(std::memory_order_acquire)) {
      // one liveness query per 200 us for all threads: after the cgroup throttles the process
      // every waiter's slice expires at once, and each asking the runtime (under mu_) kept a
      // 128-thread process throttled (profiles/r02_v32_zc_decode2.txt)
      int64_t prev = last_check_us_.load(std::memory_order_relaxed);
      if (now - prev < 200 || !last_check_us_.compare_exchange_strong(prev, now)) return 0;
    }
    std::lock_guard<std::mutex> lk(mu_);
    if (broken_) return fail("stripe server: unusable after an earlier failure");
    if (running_ && check) {
      const hipError_t q = hipEventQuery(ev_);
      if (q == hipSuccess) running_ = false;
      else if (q != hipErrorNotReady) {
        broken_ = true;
        return fail("stripe server: %s", hipGetErrorString(q));
      }
    }
    if (running_) return 0;
    // an in-place release is waiting for the device to go idle (servers_yield_begin): no launch
    // until it is done; the posting caller's wait loop asks again within 500 us.  Checked under
    // mu_, which the release's stop also takes, so a launch that got in first is stopped by it.
    if (g_srv_yield.load(std::memory_order_acquire) > 0) return 0;
    for (int g = 0; g < lsec::kSrvWG; ++g) sh_->post[g][lsec::kSrvSlotsPerWG] = 0;  // stop word
    lsec::SrvArgs a;
    a.shared = reinterpret_cast<lsec::SrvShared *>(sh_dev_);
    a.votes = votes_;
    a.idle_ticks = 200000;  // 2 ms at the 100 MHz wall clock
    a.hold = g_srv_hold.load(std::memory_order_relaxed) ? 1u : 0u;
    a.pad = 0;
    DeviceGuardLite g(dev_);
    hipError_t err = hipMemsetAsync(votes_, 0, sizeof(int), st_);
    if (err == hipSuccess) err = lsec::launch_stripe_server(a, st_);
    if (err == hipSuccess) err = hipEventRecord(ev_, st_);
    if (err != hipSuccess) {
      broken_ = true;
      return fail("stripe server launch: %s", hipGetErrorString(err));
    }
    running_ = true;
    return 0;
  }

  struct DeviceGuardLite {  // (DeviceGuard is defined further down)
    int prev = -1;
    explicit DeviceGuardLite(int dev) {
      if (hipGetDevice(&prev) != hipSuccess) prev = -1;
      if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuardLite() {
      if (prev >= 0) (void)hipSetDevice(prev);
    }
  };

  int dev_;
  lsec::SrvShared *sh_ = nullptr;
  uint64_t sh_dev_ = 0;
  char *data_ = nullptr;
  uint64_t data_dev_ = 0;
  std::atomic<uint8_t> busy_[lsec::kSrvSlots];
  uint32_t seq_[lsec::kSrvSlots];
  std::atomic<bool> ready_{false};
  std::mutex mu_;
  hipStream_t st_ = nullptr;
  hipEvent_t ev_ = nullptr;
  int *votes_ = nullptr;
  std::atomic<bool> running_{false};
  std::atomic<bool> broken_{false};
  bool zombie_ = false;                 // a launch that would not stop (mu_)
  std::atomic<int> direct_inflight_{0};  // calls whose parts the server serves in the caller's buffers
  static constexpr int kStopWaitS = 30;  // how long stop_and_settle waits for a launch to leave
  std::atomic<int64_t> last_seen_us_{0};
  std::atomic<int64_t> last_check_us_{0};
  std::atomic<bool> yield_stopped_{false};  // stopped by a release (stop_running), to relaunch after it
};

int server_run(int dev, PlanExt *e, char **ptrs, long long C, const std::vector<int> &in_ids,
               const std::vector<int> &out_ids, const void *image, int kind, const CallerPinned *cp) {
  return StripeServer::for_device(dev)->run(e, ptrs, C, in_ids, out_ids, image, kind, cp);
}

void servers_restart() { StripeServer::restart_all(); }

// hipHostUnregister waits until the device is idle, and a running stripe server never is while
// per-stripe calls keep coming: beside one thread of back-to-back 16 KiB calls a 1 MiB call pinned
// in place made no progress for 4 s (tools/probes/mixed_sizes_probe.c).  So a release stops the
// running servers first and holds off launches until it is done; calls posted meanwhile are
// served by the launch their wait loop makes after it (within 500 us).
void servers_yield_begin() {
  g_srv_yield.fetch_add(1, std::memory_order_acq_rel);
  StripeServer::stop_running();
}
void servers_yield_end() {
  if (g_srv_yield.fetch_sub(1, std::memory_order_acq_rel) == 1) StripeServer::relaunch_yielded();
}

}  // namespace eng
}  // namespace lsec

using namespace lsec::eng;

extern "C" {

// Test hook, not part of include/*.h: hold = 1 makes stripe servers launched from now on poll
// but serve nothing (a server that never answers); timeout_ms sets how long a call waits for
// its parts (default 5000).  Running servers are stopped so the next launch takes the setting.
// Returns the number of server calls that have timed out (or lost their server) so far.
long long lsec_test_server_hold(int hold, int timeout_ms) {
  if (hold >= 0) g_srv_hold.store(hold ? 1 : 0);
  if (timeout_ms > 0) g_srv_timeout_ms.store(timeout_ms);
  if (hold >= 0) servers_restart();
  return static_cast<long long>(g_st_srv_timeouts.load());
}

}  // extern "C"
