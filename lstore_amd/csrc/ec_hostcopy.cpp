// ec_hostcopy.cpp -- host copies of the engine: streaming (non-temporal) copies, the NUMA-local
// copy pool that packs and unpacks staging, and the pinned ring behind h2d_pieces / d2h_pieces
// (the verification path's scattered transfers).
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

#include <pthread.h>
#include <sched.h>

#include <immintrin.h>

#include <condition_variable>
#include <random>

#include "ec_host.h"
#include "ec_numa.h"
#include "ec_engine.h"

namespace lsec {
namespace eng {

// ---------------------------------------------------------------- host copy pool
// Host-memory callers hand over pageable buffers (cache pages, parity on the stack,
// segment/jerasure.c:1315), so bytes must be packed into pinned staging before DMA.  One
// CPU thread copies ~10 GB/s, well below PCIe Gen5, so packing/unpacking is spread over a
// small process-wide worker pool (LSEC_COPY_THREADS, default min(8, cores)); the calling
// thread works too.
// NUMA node whose copy pool packs this thread's staging: set by threads that work for one
// device (its dispatcher, the threads of a split host batch), -1 elsewhere
thread_local int tl_copy_node = -1;

// Copy with non-temporal (streaming) stores: the destination is a page-locked slot the GPU
// reads next, or a caller buffer well outside the caches, so neither is worth the
// read-for-ownership of ordinary stores, and the GPU's reads of the slot find no dirty CPU lines
// to snoop.  Own-slot calls at one thread: 1 MiB Cauchy(6+3) decodes 18.6-20.6 -> 21.9-22.5 GiB/s,
// RS(6+3) 1 MiB encodes 13.7 -> 15.5, 256 KiB 11.1 -> 12.7 (profiles/r03_v25_slot_phases_nt.txt).
// The caller issues _mm_sfence() before anything that publishes the bytes.
void stream_copy(char *dst, const char *src, size_t n) {
  while (n && (reinterpret_cast<uintptr_t>(dst) & 15)) {
    *dst++ = *src++;
    --n;
  }
  for (; n >= 64; n -= 64, dst += 64, src += 64) {
    const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i *>(src));
    const __m128i b = _mm_loadu_si128(reinterpret_cast<const __m128i *>(src + 16));
    const __m128i c = _mm_loadu_si128(reinterpret_cast<const __m128i *>(src + 32));
    const __m128i d = _mm_loadu_si128(reinterpret_cast<const __m128i *>(src + 48));
    _mm_stream_si128(reinterpret_cast<__m128i *>(dst), a);
    _mm_stream_si128(reinterpret_cast<__m128i *>(dst + 16), b);
    _mm_stream_si128(reinterpret_cast<__m128i *>(dst + 32), c);
    _mm_stream_si128(reinterpret_cast<__m128i *>(dst + 48), d);
  }
  if (n) std::memcpy(dst, src, n);
}

// LSEC_NT_COPY=0: plain memcpy instead of streaming stores for the host copies (A/B runs).  Read
// once when the library loads, before any copy thread exists.
const bool g_nt_copies = [] {
  const char *v = getenv("LSEC_NT_COPY");
  return !v || *v != '0';
}();
bool nt_copies() { return g_nt_copies; }

void host_copy(char *dst, const char *src, size_t n) {
  if (nt_copies()) stream_copy(dst, src, n);
  else std::memcpy(dst, src, n);
}

class CopyPool {
 public:
  // one pool per NUMA node (workers pinned to the node's CPUs, ec_numa.h), plus an unpinned one
  static CopyPool &get() {
    static std::mutex mu;
    static auto *pools = new std::map<int, CopyPool *>();  // intentionally leaked: workers live until exit
    std::lock_guard<std::mutex> lk(mu);
    CopyPool *&p = (*pools)[tl_copy_node];
    if (!p) p = new CopyPool(tl_copy_node);
    return *p;
  }

  // piece: bytes per work item (every worker gets a share of large chunks)
  void run(std::vector<CopyJob> &jobs, size_t kPiece = 512 << 10) {
    std::vector<CopyJob> pieces;
    pieces.reserve(jobs.size());
    for (const CopyJob &j : jobs)
      for (size_t o = 0; o < j.bytes; o += kPiece)
        pieces.push_back({j.dst + o, j.src + o, std::min(kPiece, j.bytes - o)});
    if (pieces.empty()) return;
    if (workers_.empty() || pieces.size() == 1) {
      for (const CopyJob &j : pieces) host_copy(j.dst, j.src, j.bytes);
      _mm_sfence();
      return;
    }
    Batch b;
    b.jobs = pieces.data();
    b.n = pieces.size();
    {
      std::lock_guard<std::mutex> lk(mu_);
      queue_.push_back(&b);
    }
    cv_.notify_all();
    work(b, false);
    std::unique_lock<std::mutex> lk(mu_);
    auto it = std::find(queue_.begin(), queue_.end(), &b);
    if (it != queue_.end()) queue_.erase(it);  // no new worker can pick it up now
    done_cv_.wait(lk, [&] { return b.finished == b.n && b.users == 0; });
  }

 private:
  struct Batch {
    const CopyJob *jobs = nullptr;
    size_t n = 0;
    std::atomic<size_t> next{0};
    size_t finished = 0;  // guarded by mu_
    int users = 0;        // workers inside work() for this batch, guarded by mu_
  };

  explicit CopyPool(int node) {
    const int n = routes().copy_threads;
    std::vector<int> cpus;
    if (node >= 0) cpus = node_cpus(node);
    for (int i = 1; i < n; ++i)
      workers_.emplace_back([this, cpus] {
        if (!cpus.empty()) {
          cpu_set_t set;
          CPU_ZERO(&set);
          for (int c : cpus) CPU_SET(c, &set);
          (void)pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
        }
        loop();
      });
    for (auto &t : workers_) t.detach();
  }

  // the CPUs of a node, from any device placed on it
  static std::vector<int> node_cpus(int node) {
    int n = 0;
    (void)quiet([&] { return hipGetDeviceCount(&n); });
    for (int d = 0; d < n; ++d)
      if (lsec::numa::of_device(d).node == node) return lsec::numa::of_device(d).cpus;
    return {};
  }

  // copies pieces until none are left; the caller of work() must hold a `users` reference
  void work(Batch &b, bool worker) {
    size_t mine = 0;
    for (size_t i; (i = b.next.fetch_add(1)) < b.n; ++mine) host_copy(b.jobs[i].dst, b.jobs[i].src, b.jobs[i].bytes);
    _mm_sfence();  // this thread's streamed bytes are visible before the batch is reported done
    std::lock_guard<std::mutex> lk(mu_);
    b.finished += mine;
    if (worker) --b.users;
    if (b.finished == b.n && b.users == 0) done_cv_.notify_all();
  }

  void loop() {
    for (;;) {
      Batch *b = nullptr;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] {
          for (Batch *q : queue_)
            if (q->next.load() < q->n) return true;
          return false;
        });
        for (Batch *q : queue_)
          if (q->next.load() < q->n) { b = q; ++b->users; break; }
      }
      if (b) work(*b, true);
    }
  }

  std::vector<std::thread> workers_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  std::vector<Batch *> queue_;
};

void copy_run(std::vector<CopyJob> &jobs, size_t piece) { CopyPool::get().run(jobs, piece); }

}  // namespace eng

using namespace eng;

void parallel_copy(std::vector<HostCopy> &jobs) {
  std::vector<CopyJob> j;
  j.reserve(jobs.size());
  for (const HostCopy &h : jobs) j.push_back({h.dst, h.src, h.bytes});
  CopyPool::get().run(j);
}

namespace {

// Two pinned buffers per device for h2d_pieces / d2h_pieces.  The mutex serialises users;
// `pending` survives a call, so the next user waits for the last DMA out of a buffer before
// it refills it.
struct PinnedRing {
  static constexpr size_t kBytes = 32u << 20;
  std::mutex mu;
  char *buf[2] = {nullptr, nullptr};
  hipEvent_t ev[2] = {nullptr, nullptr};
  bool pending[2] = {false, false};

  static PinnedRing *for_device(int dev) {
    static std::mutex m;
    static std::map<int, PinnedRing *> all;  // intentionally leaked: lives until exit
    std::lock_guard<std::mutex> lk(m);
    PinnedRing *&r = all[dev];
    if (!r) r = new PinnedRing();
    return r;
  }
  int ready() {
    for (int b = 0; b < 2; ++b) {
      if (!buf[b]) HIP_OK(hipHostMalloc(reinterpret_cast<void **>(&buf[b]), kBytes, hipHostMallocDefault));
      if (!ev[b]) HIP_OK(hipEventCreateWithFlags(&ev[b], hipEventDisableTiming));
    }
    return 0;
  }
  int wait(int b) {
    if (!pending[b]) return 0;
    pending[b] = false;
    HIP_OK(hipEventSynchronize(ev[b]));
    return 0;
  }
};

PinnedRing *ring_here() {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  return PinnedRing::for_device(dev);
}

}  // namespace

int h2d_pieces(const std::vector<DevPiece> &pieces, void *stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  PinnedRing *R = ring_here();
  if (!R) return fail("h2d_pieces: no HIP device");
  std::lock_guard<std::mutex> lk(R->mu);
  if (R->ready()) return -1;
  int b = 0;
  size_t fill = 0;
  char *span = nullptr;  // device address of buf[b][0]
  std::vector<CopyJob> jobs;
  auto flush = [&]() -> int {
    if (fill == 0) return 0;
    CopyPool::get().run(jobs);
    jobs.clear();
    HIP_OK(hipMemcpyAsync(span, R->buf[b], fill, hipMemcpyHostToDevice, st));
    HIP_OK(hipEventRecord(R->ev[b], st));
    R->pending[b] = true;
    b ^= 1;
    fill = 0;
    return 0;
  };
  for (const DevPiece &p : pieces) {
    for (size_t done = 0; done < p.bytes;) {
      if (fill > 0 && p.dev + done != span + fill && flush()) return -1;  // not contiguous on the device
      if (fill == 0) {
        if (R->wait(b)) return -1;
        span = p.dev + done;
      }
      const size_t take = std::min(p.bytes - done, PinnedRing::kBytes - fill);
      if (p.host)
        jobs.push_back({R->buf[b] + fill, p.host + done, take});
      else
        std::memset(R->buf[b] + fill, 0, take);
      fill += take;
      done += take;
      if (fill == PinnedRing::kBytes && flush()) return -1;
    }
  }
  return flush();
}

static int d2h_pieces_direct(const std::vector<DevPiece> &pieces, hipStream_t st);

namespace {

// Scattered pieces (many small ones far apart, e.g. one rebuilt chunk per stripe of a stage)
// are first gathered on the device into one contiguous buffer by one kernel launch; the D2H
// then moves only useful bytes in a few large DMAs instead of one small DMA per piece.
int d2h_gathered(const std::vector<DevPiece> &pieces, hipStream_t st) {
  std::vector<lsec::GatherPiece> list(pieces.size());
  size_t total = 0;
  for (size_t i = 0; i < pieces.size(); ++i) {
    if (pieces[i].bytes % 8 || reinterpret_cast<uintptr_t>(pieces[i].dev) % 8) return 1;  // not gatherable
    list[i] = {reinterpret_cast<uint64_t>(pieces[i].dev), total, pieces[i].bytes};
    total += pieces[i].bytes;
  }
  char *buf = nullptr;
  HIP_OK(hipMallocAsync(reinterpret_cast<void **>(&buf), total + sizeof(lsec::GatherPiece) * list.size(), st));
  lsec::GatherPiece *dlist = reinterpret_cast<lsec::GatherPiece *>(buf + total);  // total is a multiple of 8
  hipError_t e = hipMemcpyAsync(dlist, list.data(), sizeof(lsec::GatherPiece) * list.size(), hipMemcpyHostToDevice, st);
  if (e == hipSuccess) e = lsec::launch_gather(dlist, static_cast<int>(list.size()), buf, st);
  std::vector<DevPiece> packed(pieces.size());
  for (size_t i = 0; i < pieces.size(); ++i) packed[i] = {buf + list[i].dst_off, pieces[i].host, pieces[i].bytes};
  int rc = e == hipSuccess ? d2h_pieces_direct(packed, st) : fail("gather: %s", hipGetErrorString(e));
  (void)hipFreeAsync(buf, st);
  return rc;
}

}  // namespace

int d2h_pieces(const std::vector<DevPiece> &pieces, void *stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  // far-apart small pieces: gather on the device first (a DMA per piece costs ~40 us)
  size_t small = 0;
  for (size_t i = 1; i < pieces.size(); ++i)
    small += pieces[i].dev != pieces[i - 1].dev + pieces[i - 1].bytes && pieces[i].bytes < (4u << 20);
  if (small >= 4) {
    const int rc = d2h_gathered(pieces, st);
    if (rc <= 0) return rc;  // 1: not gatherable, fall through to per-window DMAs
  }
  return d2h_pieces_direct(pieces, st);
}

static int d2h_pieces_direct(const std::vector<DevPiece> &pieces, hipStream_t st) {
  PinnedRing *R = ring_here();
  if (!R) return fail("d2h_pieces: no HIP device");
  // windows: device ranges of at most one ring buffer, covering runs of pieces whose gaps are
  // small (a gap is transferred and discarded: cheaper than another DMA below ~1 MiB)
  struct Window {
    char *dev;
    size_t len;
    char *alloc_end;           // a window never crosses the end of the allocation it starts in
    std::vector<CopyJob> out;  // src = offset into the window (fixed up at unpack time)
  };
  constexpr size_t kGap = 1u << 20;
  std::vector<Window> win;
  char *abase = nullptr, *aend = nullptr;  // allocation of the last piece looked up
  for (const DevPiece &p : pieces)
    for (size_t done = 0; done < p.bytes;) {
      char *d = p.dev + done;
      const size_t take = std::min(p.bytes - done, PinnedRing::kBytes);
      if (!(d >= abase && d < aend)) {
        hipDeviceptr_t b = nullptr;
        size_t sz = 0;
        if (quiet([&] { return hipMemGetAddressRange(&b, &sz, d); }) != hipSuccess) {
          b = d;  // unknown extent: no gap merging past this piece
          sz = p.bytes - done;
        }
        abase = static_cast<char *>(b);
        aend = abase + sz;
      }
      const bool fits = !win.empty() && d >= win.back().dev + win.back().len && d <= win.back().dev + win.back().len + kGap &&
                        d + take <= win.back().alloc_end && d >= abase && win.back().dev >= abase &&
                        static_cast<size_t>(d + take - win.back().dev) <= PinnedRing::kBytes;
      if (!fits) win.push_back({d, 0, aend, {}});
      Window &w = win.back();
      w.out.push_back({p.host + done, reinterpret_cast<const char *>(d - w.dev), take});
      w.len = static_cast<size_t>(d + take - w.dev);
      done += take;
    }
  std::lock_guard<std::mutex> lk(R->mu);
  if (R->ready()) return -1;
  auto unpack = [&](size_t i) -> int {
    const int b = static_cast<int>(i & 1);
    if (R->wait(b)) return -1;
    for (CopyJob &j : win[i].out) j.src = R->buf[b] + reinterpret_cast<uintptr_t>(j.src);
    CopyPool::get().run(win[i].out);
    return 0;
  };
  for (size_t i = 0; i < win.size(); ++i) {
    const int b = static_cast<int>(i & 1);
    if (i >= 2 && unpack(i - 2)) return -1;  // frees buffer b
    if (R->wait(b)) return -1;
    HIP_OK(hipMemcpyAsync(R->buf[b], win[i].dev, win[i].len, hipMemcpyDeviceToHost, st));
    HIP_OK(hipEventRecord(R->ev[b], st));
    R->pending[b] = true;
  }
  for (size_t i = win.size() >= 2 ? win.size() - 2 : 0; i < win.size(); ++i)
    if (unpack(i)) return -1;
  return 0;
}
}  // namespace lsec

using namespace lsec::eng;

extern "C" {

// Self-test of the host copies (test hook, not in include/): stream_copy and the copy pool
// over `cases` random (source offset, destination offset, length) triples, lengths 0..300 KiB,
// against memcpy; bytes around each destination must stay untouched.  0 / -1.
int lsec_selftest_copies(int cases, unsigned seed) {
  if (cases < 1) return fail("lsec_selftest_copies: bad arguments");
  std::mt19937 rng(seed);
  const size_t cap = (300u << 10) + 256;
  std::vector<char> src(cap + 64), dst(cap + 64), want(cap + 64);
  for (auto &c : src) c = static_cast<char>(rng());
  for (int i = 0; i < cases; ++i) {
    const size_t so = rng() % 64, doff = rng() % 64;
    size_t n = rng() % 4 == 0 ? rng() % 256 : rng() % (300u << 10);
    for (auto &c : dst) c = static_cast<char>(0xA5);
    want = dst;
    std::memcpy(&want[doff], &src[so], n);
    if (i % 2) {
      stream_copy(&dst[doff], &src[so], n);
      _mm_sfence();
    } else {
      std::vector<CopyJob> jobs{{&dst[doff], &src[so], n}};
      CopyPool::get().run(jobs, 1 + rng() % (64u << 10));
    }
    if (std::memcmp(dst.data(), want.data(), dst.size()) != 0)
      return fail("lsec_selftest_copies: case %d (src +%zu, dst +%zu, %zu B, %s) differs", i, so, doff, n,
                  i % 2 ? "stream_copy" : "copy pool");
  }
  return 0;
}

}  // extern "C"
