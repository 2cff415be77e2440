// ec_waits.cpp -- completion waits of the zero-copy routes: a few spinners, futex parking with
// lock-free records, and poller threads that watch GPU-written flags and wake the parked.
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

#include <linux/futex.h>
#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <climits>
#include <cstring>
#include "ec_engine.h"

namespace lsec {
namespace eng {

// ---------------------------------------------------------------- waiting for completion flags
// CPUs this process may keep busy: the affinity mask, capped by the cgroup CPU quota (a GPU box
// may show the whole machine's CPUs and grant a share of them).
int usable_cpus() {
  static const int n = [] {
    int c = 1;
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof(set), &set) == 0) c = std::max(1, CPU_COUNT(&set));
    if (FILE *f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
      char q[32] = {0};
      long long period = 0;
      if (fscanf(f, "%31s %lld", q, &period) == 2 && strcmp(q, "max") != 0 && period > 0)
        c = std::min<long long>(c, std::max(1LL, (atoll(q) + period - 1) / period));
      fclose(f);
    }
    return c;
  }();
  return n;
}

// Completion waits.  LStore calls encode_block from up to 300 pool threads; a waiter that spins
// (or yields) holds a CPU, and with more waiters than CPUs the spinning starves the threads whose
// calls are done -- on a cgroup quota it also burns the quota and gets the whole process
// throttled.  So at most a quarter of the usable CPUs spin; every other waiter parks on a futex
// word of its own, and poller threads watch the parked waiters' flags (written by the GPU, which
// cannot wake a thread) and wake them.
//
// Parking is lock-free: each thread owns a record in a static table (its flags and wanted values
// copied in, published under a sequence lock), and the pollers scan the table.  An earlier form
// (one poller holding one mutex over a list of condition variables while it scanned and
// notified) capped per-stripe calls at ~150k/s: at 32 and 128 threads an RS(6+3) 16 KiB encode
// ran 12.5-13.7 GiB/s against 20.9 at 8 threads, with CPUs to spare
// (profiles/r02_v28_zc_routes.txt).  Every flag a record can name stays mapped for the life of
// the process (server done lines; zero-copy flags come from a pool that is never freed), so a
// poller that reads a record just as its waiter leaves reads valid memory.
// LSEC_STATS counters of the waiting machinery (printed with ZcStats at exit)
std::atomic<unsigned long long> g_st_parks{0}, g_st_spin_hits{0}, g_st_claim_misses{0}, g_st_claim_spins{0},
    g_st_wakes{0}, g_st_slices{0};

class FlagWaits {
 public:
  static constexpr int kMaxFlags = 16;  // flags one wait covers (StripeServer::kMaxParts)

  static FlagWaits &get() {
    static FlagWaits *w = new FlagWaits();  // leaked: the poller threads outlive static destruction
    return *w;
  }

  // Waits until every flags[i] reaches wants[i] (wrapping u32 sequences: wants[i] - *flags[i] <= 0),
  // or up to `slice`; true when all are reached.  Callers loop, doing their own checks between
  // slices.  One wait covers all the parts of a call: the parts land on different server
  // workgroups and finish in any order (a wait per part could park and wake its thread once
  // per part under load).
  bool wait(const unsigned *const *flags, const unsigned *wants, int n, std::chrono::microseconds slice,
            const WaitProgress *pr = nullptr) {
    int from = 0, told = 0;
    // reached_all, telling the caller (pr) each time the reached prefix grows
    const auto check = [&] {
      const bool all = reached_all(flags, wants, n, from);
      if (pr && from > told) pr->fn(pr->ctx, told = from);
      return all;
    };
    if (check()) return true;
    Record *rec = n <= kMaxFlags ? my_record() : nullptr;
    if (!rec) {  // no record: spin, then yield, then nap
      const auto t0 = std::chrono::steady_clock::now();
      for (unsigned i = 0;; ++i) {
        if (check()) return true;
        if (i < 500) {
          __builtin_ia32_pause();
          continue;
        }
        const auto dt = std::chrono::steady_clock::now() - t0;
        if (dt > slice) return false;
        if (dt < std::chrono::microseconds(200)) std::this_thread::yield();
        else std::this_thread::sleep_for(std::chrono::microseconds(20));
      }
    }
    const auto t0 = std::chrono::steady_clock::now();
    // spin only while waits are short: under load (waits of 100s of us) a spinner holds a CPU
    // for nothing that the callers' copies need
    const bool short_waits = recent_us_.load(std::memory_order_relaxed) < 2 * spin_.count();
    const int active = spinners_.fetch_add(1, std::memory_order_relaxed) + 1;
    if (short_waits && active <= spin_limit_) {
      for (unsigned i = 1;; ++i) {
        if (check()) {
          spinners_.fetch_sub(1, std::memory_order_relaxed);
          note(t0);
          g_st_spin_hits.fetch_add(1, std::memory_order_relaxed);
          return true;
        }
        __builtin_ia32_pause();
        if ((i & 63) == 0 && std::chrono::steady_clock::now() - t0 > spin_) break;
      }
    }
    spinners_.fetch_sub(1, std::memory_order_relaxed);
    // park: publish the flags still outstanding, then sleep on the record's futex word
    const int m = n - from;
    rec->seq.fetch_add(1, std::memory_order_relaxed);  // odd: fields changing
    std::atomic_thread_fence(std::memory_order_release);
    for (int i = 0; i < m; ++i) {
      rec->flags[i].store(flags[from + i], std::memory_order_relaxed);
      rec->wants[i].store(wants[from + i], std::memory_order_relaxed);
    }
    rec->n.store(m, std::memory_order_relaxed);
    rec->word.store(0, std::memory_order_relaxed);
    rec->seq.fetch_add(1, std::memory_order_release);  // even: published
    rec->active.store(1, std::memory_order_seq_cst);
    g_st_parks.fetch_add(1, std::memory_order_relaxed);
    if (sleeping_.load(std::memory_order_seq_cst) > 0) {  // a poller sleeps: new work for it
      epoch_.fetch_add(1, std::memory_order_seq_cst);
      futex_wake(&epoch_, INT32_MAX);
    }
    const auto deadline = t0 + slice;
    while (rec->word.load(std::memory_order_acquire) == 0 && !reached_all(flags, wants, n, from)) {
      const auto now = std::chrono::steady_clock::now();
      if (now >= deadline) break;
      futex_wait(&rec->word, 0, std::chrono::duration_cast<std::chrono::nanoseconds>(deadline - now));
    }
    rec->active.store(0, std::memory_order_release);
    if (!check()) {
      g_st_slices.fetch_add(1, std::memory_order_relaxed);
      return false;
    }
    note(t0);
    return true;
  }
  bool wait(const unsigned *flag, unsigned want, std::chrono::microseconds slice) {
    return wait(&flag, &want, 1, slice);
  }

 private:
  static constexpr int kMaxRecords = 4096;  // threads that have parked at least once

  struct alignas(64) Record {
    std::atomic<uint32_t> seq{0};   // sequence lock over n / flags / wants (odd while writing)
    std::atomic<uint32_t> word{0};  // futex word: set to 1 by the poller that wakes the waiter
    std::atomic<int> active{0};     // 1 while the waiter is parked
    std::atomic<int> n{0};
    std::atomic<const unsigned *> flags[kMaxFlags];
    std::atomic<unsigned> wants[kMaxFlags];
  };

  // this thread's record; a thread that exits returns it for reuse
  Record *my_record() {
    struct Owner {
      int idx = -1;
      ~Owner() {
        if (idx >= 0) FlagWaits::get().free_record(idx);
      }
    };
    static thread_local Owner own;
    if (own.idx < 0) own.idx = alloc_record();
    return own.idx < 0 ? nullptr : &records_[own.idx];
  }
  int alloc_record() {
    std::lock_guard<std::mutex> lk(free_mu_);
    if (!free_.empty()) {
      const int i = free_.back();
      free_.pop_back();
      return i;
    }
    const int i = used_.load(std::memory_order_relaxed);
    if (i >= kMaxRecords) return -1;
    used_.store(i + 1, std::memory_order_release);
    return i;
  }
  void free_record(int i) {
    records_[i].active.store(0, std::memory_order_release);
    std::lock_guard<std::mutex> lk(free_mu_);
    free_.push_back(i);
  }

  static void futex_wait(std::atomic<uint32_t> *w, uint32_t v, std::chrono::nanoseconds t) {
    struct timespec ts;
    ts.tv_sec = static_cast<time_t>(t.count() / 1000000000);
    ts.tv_nsec = static_cast<long>(t.count() % 1000000000);
    syscall(SYS_futex, reinterpret_cast<uint32_t *>(w), FUTEX_WAIT_PRIVATE, v, &ts, nullptr, 0);
  }
  static void futex_wake(std::atomic<uint32_t> *w, int n) {
    syscall(SYS_futex, reinterpret_cast<uint32_t *>(w), FUTEX_WAKE_PRIVATE, n, nullptr, nullptr, 0);
  }

  // moving average of completed waits (us), 1/8 weight per sample
  void note(std::chrono::steady_clock::time_point t0) {
    const long us = static_cast<long>(
        std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0).count());
    const long old = recent_us_.load(std::memory_order_relaxed);
    recent_us_.store(old + (us - old) / 8, std::memory_order_relaxed);
  }

  static bool reached(const unsigned *flag, unsigned want) {
    return static_cast<int>(__atomic_load_n(flag, __ATOMIC_ACQUIRE) - want) >= 0;
  }
  // all of flags[from, n) reached; advances `from` past the ones that are
  static bool reached_all(const unsigned *const *flags, const unsigned *wants, int n, int &from) {
    while (from < n && reached(flags[from], wants[from])) ++from;
    return from == n;
  }

  FlagWaits() {
    // from a sweep of both (profiles/r02_v22_wait_sweep.jsonl): a quarter of the usable CPUs
    // spin, for up to 30 us (an unloaded call completes in 14-20 us)
    spin_limit_ = routes().spinners;
    spin_ = routes().spin;
    // pollers: one per 8 usable CPUs, at most 4
    npollers_ = routes().pollers;
    for (int p = 0; p < npollers_; ++p) std::thread([this, p] { poll(p); }).detach();
  }

  // poller p scans records p, p + npollers, ...: wakes every parked waiter whose flags have all
  // come; sleeps on epoch_ while none of its records is parked
  void poll(int p) {
    const unsigned *f[kMaxFlags];
    unsigned wv[kMaxFlags];
    for (;;) {
      bool any = false;
      const int hi = used_.load(std::memory_order_acquire);
      for (int i = p; i < hi; i += npollers_) {
        Record &r = records_[i];
        if (!r.active.load(std::memory_order_acquire)) continue;
        any = true;
        const uint32_t s1 = r.seq.load(std::memory_order_acquire);
        if (s1 & 1u) continue;
        const int m = r.n.load(std::memory_order_relaxed);
        if (m < 1 || m > kMaxFlags) continue;
        for (int j = 0; j < m; ++j) {
          f[j] = r.flags[j].load(std::memory_order_relaxed);
          wv[j] = r.wants[j].load(std::memory_order_relaxed);
        }
        std::atomic_thread_fence(std::memory_order_acquire);
        if (r.seq.load(std::memory_order_relaxed) != s1) continue;  // rewritten meanwhile
        int from = 0;
        if (!reached_all(f, wv, m, from)) continue;
        if (r.word.exchange(1, std::memory_order_acq_rel) == 0) {
          futex_wake(&r.word, 1);
          g_st_wakes.fetch_add(1, std::memory_order_relaxed);
        }
      }
      if (any) {  // flags are written by the GPU: poll, a few us apart
        for (int i = 0; i < 32; ++i) __builtin_ia32_pause();
        std::this_thread::yield();
        continue;
      }
      // nothing parked here: sleep until a waiter parks (it bumps epoch_ when it sees a sleeper)
      const uint32_t e = epoch_.load(std::memory_order_seq_cst);
      sleeping_.fetch_add(1, std::memory_order_seq_cst);
      bool now_any = false;
      const int hi2 = used_.load(std::memory_order_acquire);
      for (int i = p; i < hi2 && !now_any; i += npollers_) now_any = records_[i].active.load(std::memory_order_seq_cst) != 0;
      if (!now_any) futex_wait(&epoch_, e, std::chrono::milliseconds(10));
      sleeping_.fetch_sub(1, std::memory_order_seq_cst);
    }
  }

  int spin_limit_ = 1;                   // waiters allowed to spin at once (LSEC_WAIT_SPINNERS)
  std::chrono::microseconds spin_{100};  // how long one spins before parking (LSEC_WAIT_SPIN_US)
  int npollers_ = 1;
  std::atomic<int> spinners_{0};
  std::atomic<long> recent_us_{0};
  std::atomic<uint32_t> epoch_{0};
  std::atomic<int> sleeping_{0};
  std::atomic<int> used_{0};
  Record records_[kMaxRecords];
  std::mutex free_mu_;
  std::vector<int> free_;
};

// Waits until flag reaches v (wrapping u32 sequence) through FlagWaits.  Bounded: after 2 s
// the caller checks its stream for an error.
bool wait_flag(const unsigned *flag, unsigned v, hipStream_t st, int *rc) {
  const auto t0 = std::chrono::steady_clock::now();
  while (!FlagWaits::get().wait(flag, v, std::chrono::milliseconds(1))) {
    if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
      const hipError_t e = hipStreamSynchronize(st);
      if (static_cast<int>(__atomic_load_n(flag, __ATOMIC_ACQUIRE) - v) >= 0) return true;
      *rc = fail("zero-copy call: completion flag never came (%s)", hipGetErrorString(e));
      return false;
    }
  }
  return true;
}

bool flag_wait(const unsigned *const *flags, const unsigned *wants, int n, std::chrono::microseconds slice,
               const WaitProgress *progress) {
  return FlagWaits::get().wait(flags, wants, n, slice, progress);
}

}  // namespace eng
}  // namespace lsec

using namespace lsec::eng;

extern "C" {

// Self-test of the completion waits (FlagWaits: spinners, lock-free parking, pollers) with the
// flags written by host threads instead of the GPU: `threads` waiters, each with a producer that
// sets its 1..16 flags in random order after a random delay of 0-300 us, `iters` rounds.  Every
// wait must end with all its flags set and within 2 s.  Test hook, not part of include/*.h;
// needs no GPU.  Returns 0, or -1 with a message.
int lsec_selftest_waits(int threads, int iters) {
  if (threads < 1 || threads > 512 || iters < 1) return fail("lsec_selftest_waits: bad arguments");
  struct alignas(64) Pair {
    unsigned flags[16][16];  // one 64-byte line per flag, as the server's done lines
    std::atomic<int> ready{-1};
    int n = 1;
  };
  std::vector<std::unique_ptr<Pair>> pairs;
  for (int t = 0; t < threads; ++t) {
    pairs.emplace_back(new Pair());
    std::memset(pairs.back()->flags, 0, sizeof(pairs.back()->flags));
    pairs.back()->n = 1 + (t * 7) % 16;
  }
  std::atomic<int> bad{0};
  std::atomic<unsigned long long> progress_calls{0};
  const unsigned long long parks0 = g_st_parks.load(), wakes0 = g_st_wakes.load();
  std::vector<std::thread> th;
  for (int t = 0; t < threads; ++t) {
    th.emplace_back([&, t] {  // producer
      Pair &p = *pairs[t];
      uint64_t x = 0x9E3779B97F4A7C15ull * (t + 1);
      for (int it = 0; it < iters && !bad.load(); ++it) {
        while (p.ready.load(std::memory_order_acquire) < it && !bad.load()) std::this_thread::yield();
        x ^= x << 13, x ^= x >> 7, x ^= x << 17;
        std::this_thread::sleep_for(std::chrono::microseconds(x % 300));
        int order[16];
        for (int i = 0; i < p.n; ++i) order[i] = i;
        for (int i = p.n - 1; i > 0; --i) std::swap(order[i], order[(x >> (i % 48)) % (i + 1)]);
        for (int i = 0; i < p.n; ++i) __atomic_store_n(&p.flags[order[i]][0], static_cast<unsigned>(it + 1), __ATOMIC_RELEASE);
      }
    });
    th.emplace_back([&, t] {  // waiter
      Pair &p = *pairs[t];
      const unsigned *f[16];
      unsigned want[16];
      for (int i = 0; i < p.n; ++i) f[i] = &p.flags[i][0];
      // the progress hook (WaitProgress): every prefix it reports must be reached, and grow
      struct Seen {
        const unsigned *const *f;
        const unsigned *want;
        int n, last;
        std::atomic<int> *bad;
        std::atomic<unsigned long long> *calls;
      } seen{f, want, p.n, 0, &bad, &progress_calls};
      const WaitProgress pr{[](void *ctx, int upto) {
                              Seen &z = *static_cast<Seen *>(ctx);
                              z.calls->fetch_add(1, std::memory_order_relaxed);
                              bool ok = upto > z.last && upto <= z.n;
                              for (int i = 0; ok && i < upto; ++i)
                                ok = static_cast<int>(__atomic_load_n(z.f[i], __ATOMIC_ACQUIRE) - z.want[i]) >= 0;
                              if (!ok) z.bad->store(3);
                              z.last = upto;
                            },
                            &seen};
      for (int it = 0; it < iters && !bad.load(); ++it) {
        for (int i = 0; i < p.n; ++i) want[i] = static_cast<unsigned>(it + 1);
        p.ready.store(it, std::memory_order_release);
        const auto t0 = std::chrono::steady_clock::now();
        for (;;) {
          seen.last = 0;  // each wait reports prefixes from the start
          if (FlagWaits::get().wait(f, want, p.n, std::chrono::microseconds(500), (it & 1) ? &pr : nullptr)) break;
          if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
            bad.store(1);
            return;
          }
        }
        for (int i = 0; i < p.n; ++i)
          if (static_cast<int>(__atomic_load_n(f[i], __ATOMIC_ACQUIRE) - want[i]) < 0) {
            bad.store(2);
            return;
          }
      }
    });
  }
  for (auto &x : th) x.join();
  {  // the flags stay mapped for the life of the process, as the engine's own do: a poller may
     // still read the record of a waiter that has just left (found by ThreadSanitizer)
    static std::mutex mu;
    static auto *kept = new std::vector<std::unique_ptr<Pair>>();  // leaked on purpose
    std::lock_guard<std::mutex> lk(mu);
    for (auto &p : pairs) kept->push_back(std::move(p));
  }
  if (bad.load() == 1) return fail("lsec_selftest_waits: a wait did not end within 2 s of its flags");
  if (bad.load() == 2) return fail("lsec_selftest_waits: a wait returned before all its flags were set");
  if (bad.load() == 3) return fail("lsec_selftest_waits: a progress report named a flag not yet set, or shrank");
  // delays up to 300 us against a 30 us spin: long runs must have parked and been woken
  if (static_cast<long long>(threads) * iters >= 200 && (g_st_parks.load() == parks0 || g_st_wakes.load() == wakes0))
    return fail("lsec_selftest_waits: no waiter parked or was woken by a poller");
  if (static_cast<long long>(threads) * iters >= 200 && progress_calls.load() == 0)
    return fail("lsec_selftest_waits: no spinning wait reported progress");
  return 0;
}

}  // extern "C"
