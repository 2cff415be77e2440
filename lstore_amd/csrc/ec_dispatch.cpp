// ec_dispatch.cpp -- route 3: the per-device dispatcher thread, which coalesces concurrent
// host calls into one H2D + one kernel per group + one D2H (group commit).
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

#include <condition_variable>
#include <deque>

#include "ec_numa.h"
#include "ec_engine.h"

namespace lsec {
namespace eng {

// ---------------------------------------------------------------- request coalescing
// The unmodified segment driver calls encode_block / decode_block once per stripe, from up
// to 300 gop pool threads at once (segment/jerasure.c:1847, :245, :1937; lio_config.c:87).
// One H2D + kernel + D2H round trip per 16 KiB stripe would leave the GPU idle between tiny
// transfers, so small host-memory calls are handed to a per-device dispatcher thread that
// coalesces everything queued at that moment: requests with the same matrix image and
// geometry share ONE staging region, ONE H2D, ONE kernel launch and ONE D2H (group commit).
// Two staging slots alternate so packing batch n+1 overlaps the GPU work of batch n.
struct HostReq {
  char **ptrs = nullptr;
  int nstripes = 0, km = 0, kind = 0, packet = 0, w = 8;
  bool pinned = false;  // caller buffers page-locked: DMA in place, no packing
  // pinned with small runs, every chunk checked: moved by the copy-piece kernel; dev = the
  // chunks' device addresses (stripe, then in_ids, then out_ids -- caller_pinned_aliases)
  bool by_kernel = false;
  std::vector<uint64_t> dev;
  long long C = 0;
  std::vector<int> in_ids, out_ids;
  const void *image = nullptr;
  int rc = 0;
  std::string err;
  bool done = false;
  std::mutex mu;
  std::condition_variable cv;
  size_t bytes() const { return static_cast<size_t>(nstripes) * (in_ids.size() + out_ids.size()) * C; }
  bool same_group(const HostReq &o) const {
    return image == o.image && kind == o.kind && C == o.C && packet == o.packet && w == o.w && in_ids.size() == o.in_ids.size() &&
           out_ids.size() == o.out_ids.size();
  }
};


class Dispatcher {
 public:
  static Dispatcher *for_device(int dev) {
    static std::mutex mu;
    static std::map<int, Dispatcher *> all;  // intentionally leaked: lives until exit
    std::lock_guard<std::mutex> lk(mu);
    auto it = all.find(dev);
    if (it != all.end()) return it->second;
    Dispatcher *d = new Dispatcher(dev);
    all[dev] = d;
    return d;
  }

  int run(HostReq &r) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      q_.push_back(&r);
    }
    cv_.notify_one();
    std::unique_lock<std::mutex> lk(r.mu);
    r.cv.wait(lk, [&] { return r.done; });
    if (r.rc) tl_err = r.err;
    return r.rc;
  }

 private:
  struct Group {
    std::vector<HostReq *> reqs;
    std::vector<int> first;  // stripe offset of each request inside the group
    int nstripes = 0;
    size_t off = 0;          // byte offset of the group inside the slot
  };
  struct Slot {
    char *d = nullptr, *h = nullptr;
    size_t cap = 0;
    lsec::CopyPiece *pl = nullptr;  // copy pieces of by_kernel requests (page-locked)
    size_t pl_cap = 0;
    hipEvent_t done = nullptr;
    std::vector<Group> groups;
    std::string err;
  };


  explicit Dispatcher(int dev) : dev_(dev) { std::thread([this] { loop(); }).detach(); }

  static size_t group_bytes(const Group &g) {
    const HostReq &r = *g.reqs[0];
    return static_cast<size_t>(g.nstripes) * (r.in_ids.size() + r.out_ids.size()) * r.C;
  }

  void finish(Slot &sl) {
    if (sl.groups.empty()) return;
    std::string err = sl.err;
    if (err.empty() && hipEventSynchronize(sl.done) != hipSuccess) err = "dispatcher: event sync failed";
    if (!err.empty()) {  // whatever was enqueued must not outlive the callers' buffers or the slot
      (void)hipStreamSynchronize(s_in_);
      (void)hipStreamSynchronize(s_out_);
    }
    std::vector<CopyJob> jobs;
    if (err.empty()) {
      for (const Group &g : sl.groups) {
        const HostReq &r0 = *g.reqs[0];
        const size_t C = static_cast<size_t>(r0.C), nin = r0.in_ids.size(), nout = r0.out_ids.size();
        const char *outb = sl.h + g.off + static_cast<size_t>(g.nstripes) * nin * C;
        for (size_t q = 0; q < g.reqs.size(); ++q) {
          const HostReq &r = *g.reqs[q];
          if (r.pinned) continue;  // its D2H went straight into its buffers
          for (int s = 0; s < r.nstripes; ++s)
            for (size_t o = 0; o < nout; ++o)
              jobs.push_back({r.ptrs[static_cast<size_t>(s) * r.km + r.out_ids[o]],
                              outb + ((static_cast<size_t>(g.first[q]) + s) * nout + o) * C, C});
        }
      }
      copy_run(jobs);
    }
    for (const Group &g : sl.groups)
      for (HostReq *r : g.reqs) {
        std::lock_guard<std::mutex> lk(r->mu);
        r->rc = err.empty() ? 0 : -1;
        r->err = err;
        r->done = true;
        r->cv.notify_all();
      }
    sl.groups.clear();
    sl.err.clear();
  }

  // pack + enqueue one batch into `sl`; errors are recorded in sl.err (reported at finish)
  void launch(Slot &sl, std::vector<HostReq *> &batch) {
    for (HostReq *r : batch) {  // group compatible requests
      Group *g = nullptr;
      for (Group &x : sl.groups)
        if (x.reqs[0]->same_group(*r)) { g = &x; break; }
      if (!g) {
        sl.groups.emplace_back();
        g = &sl.groups.back();
      }
      g->reqs.push_back(r);
      g->first.push_back(g->nstripes);
      g->nstripes += r->nstripes;
    }
    size_t total = 0;
    for (Group &g : sl.groups) {
      g.off = total;
      total += (group_bytes(g) + 255) & ~static_cast<size_t>(255);
    }
    auto hip_err = [&](hipError_t e, const char *what) {
      if (e != hipSuccess && sl.err.empty()) sl.err = std::string("dispatcher: ") + what + ": " + hipGetErrorString(e);
      return e == hipSuccess;
    };
    if (sl.cap < total) {
      if (sl.d) (void)hipFree(sl.d);
      if (sl.h) (void)hipHostFree(sl.h);
      sl.d = sl.h = nullptr;
      // grow geometrically up to the batch budget: pinning a fresh region costs milliseconds
      // per call, so creeping batch sizes must not re-pin on every growth step
      const size_t cap = std::max({total, std::min(2 * sl.cap, routes().dispatch_batch + (1u << 20)), size_t(32u << 20)});
      sl.cap = 0;
      if (!hip_err(hipMalloc(&sl.d, cap), "hipMalloc") ||
          !hip_err(hipHostMalloc(reinterpret_cast<void **>(&sl.h), cap, hipHostMallocDefault), "hipHostMalloc"))
        return;
      sl.cap = cap;
    }
    // Inputs: pageable requests are packed into the pinned slot and leave in one DMA per run
    // of neighbouring requests; pinned requests are DMA'd from their own buffers.  Outputs
    // mirror that (finish() unpacks only the pageable ones).
    std::vector<CopyJob> jobs;
    std::vector<DmaRun> h2d, d2h;
    std::vector<lsec::CopyPiece> kin, kout;  // by_kernel requests
    for (const Group &g : sl.groups) {
      const HostReq &r0 = *g.reqs[0];
      const size_t C = static_cast<size_t>(r0.C), nin = r0.in_ids.size(), nout = r0.out_ids.size();
      const size_t out0 = g.off + static_cast<size_t>(g.nstripes) * nin * C;
      for (size_t q = 0; q < g.reqs.size(); ++q) {
        const HostReq &r = *g.reqs[q];
        const size_t ib = g.off + static_cast<size_t>(g.first[q]) * nin * C;
        const size_t ob = out0 + static_cast<size_t>(g.first[q]) * nout * C;
        if (r.by_kernel) {
          const size_t nio = nin + nout;
          for (int s = 0; s < r.nstripes; ++s) {
            for (size_t j = 0; j < nin; ++j)
              split_pieces(kin, r.dev[s * nio + j], reinterpret_cast<uint64_t>(sl.d) + ib + (static_cast<size_t>(s) * nin + j) * C, C);
            for (size_t o = 0; o < nout; ++o)
              split_pieces(kout, reinterpret_cast<uint64_t>(sl.d) + ob + (static_cast<size_t>(s) * nout + o) * C,
                           r.dev[s * nio + nin + o], C);
          }
        } else if (r.pinned) {
          for (int s = 0; s < r.nstripes; ++s) {
            for (size_t j = 0; j < nin; ++j)
              add_run(h2d, sl.d + ib + (static_cast<size_t>(s) * nin + j) * C, r.ptrs[static_cast<size_t>(s) * r.km + r.in_ids[j]], C);
            for (size_t o = 0; o < nout; ++o)
              add_run(d2h, r.ptrs[static_cast<size_t>(s) * r.km + r.out_ids[o]], sl.d + ob + (static_cast<size_t>(s) * nout + o) * C, C);
          }
        } else {
          for (int s = 0; s < r.nstripes; ++s)
            for (size_t j = 0; j < nin; ++j)
              jobs.push_back({sl.h + ib + (static_cast<size_t>(s) * nin + j) * C, r.ptrs[static_cast<size_t>(s) * r.km + r.in_ids[j]], C});
          add_run(h2d, sl.d + ib, sl.h + ib, static_cast<size_t>(r.nstripes) * nin * C);
          add_run(d2h, sl.h + ob, sl.d + ob, static_cast<size_t>(r.nstripes) * nout * C);
        }
      }
    }
    copy_run(jobs);
    if (!kin.empty() || !kout.empty()) {
      const size_t need = kin.size() + kout.size();
      if (sl.pl_cap < need) {
        const size_t cap = std::max(need, 2 * sl.pl_cap + 4096);
        if (sl.pl) (void)hipHostFree(sl.pl);
        sl.pl = nullptr;
        sl.pl_cap = 0;
        if (!hip_err(hipHostMalloc(reinterpret_cast<void **>(&sl.pl), cap * sizeof(lsec::CopyPiece), hipHostMallocDefault),
                     "hipHostMalloc")) {
          sl.pl = nullptr;
          return;
        }
        sl.pl_cap = cap;
      }
      std::copy(kin.begin(), kin.end(), sl.pl);
      std::copy(kout.begin(), kout.end(), sl.pl + kin.size());
    }
    if (!hip_err(issue_runs(h2d, hipMemcpyHostToDevice, s_in_), "H2D")) return;
    if (!kin.empty() && !hip_err(lsec::launch_copy_pieces(sl.pl, static_cast<int>(kin.size()), s_in_), "H2D pieces")) return;
    if (!hip_err(hipEventRecord(in_done_, s_in_), "event") || !hip_err(hipStreamWaitEvent(s_out_, in_done_, 0), "wait"))
      return;
    for (const Group &g : sl.groups) {
      const HostReq &r0 = *g.reqs[0];
      const size_t C = static_cast<size_t>(r0.C);
      const int nin = static_cast<int>(r0.in_ids.size()), nout = static_cast<int>(r0.out_ids.size());
      const size_t in_bytes = static_cast<size_t>(g.nstripes) * nin * C;
      char *dbase = sl.d + g.off;
      ShardRef in[kMaxDevs], out[kMaxDevs];
      for (int j = 0; j < nin; ++j)
        in[j] = {reinterpret_cast<uint64_t>(dbase) + static_cast<uint64_t>(j) * C, static_cast<int64_t>(nin * C)};
      for (int o = 0; o < nout; ++o)
        out[o] = {reinterpret_cast<uint64_t>(dbase) + in_bytes + static_cast<uint64_t>(o) * C, static_cast<int64_t>(nout * C)};
      if (enqueue_apply(r0.kind, r0.image, nin, nout, in, out, g.nstripes, r0.C, r0.packet, s_out_, r0.w) != 0) {
        if (sl.err.empty()) sl.err = tl_err;
        return;
      }
    }
    if (!hip_err(issue_runs(d2h, hipMemcpyDeviceToHost, s_out_), "D2H")) return;
    if (!kout.empty() &&
        !hip_err(lsec::launch_copy_pieces(sl.pl + kin.size(), static_cast<int>(kout.size()), s_out_), "D2H pieces"))
      return;
    hip_err(hipEventRecord(sl.done, s_out_), "event");
  }

  void loop() {
    // this device's host thread: on its NUMA node, packing with that node's copy pool, and
    // allocating its page-locked staging from there
    lsec::numa::bind_this_thread(dev_);
    tl_copy_node = lsec::numa::of_device(dev_).node;
    if (hipSetDevice(dev_) != hipSuccess || hipStreamCreateWithFlags(&s_in_, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&s_out_, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreateWithFlags(&in_done_, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&slot_[0].done, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&slot_[1].done, hipEventDisableTiming) != hipSuccess) {
      broken_ = "dispatcher: cannot create HIP streams/events";
    }
    int cur = 0;
    for (;;) {
      std::vector<HostReq *> batch;
      {
        std::unique_lock<std::mutex> lk(mu_);
        const bool pending = !slot_[cur ^ 1].groups.empty();
        if (!pending) cv_.wait(lk, [&] { return !q_.empty(); });
        size_t bytes = 0;
        while (!q_.empty() && (batch.empty() || bytes + q_.front()->bytes() <= routes().dispatch_batch)) {
          bytes += q_.front()->bytes();
          batch.push_back(q_.front());
          q_.pop_front();
        }
      }
      if (!batch.empty()) {
        if (!broken_.empty()) slot_[cur].err = broken_;
        else launch(slot_[cur], batch);
        if (slot_[cur].groups.empty()) {  // launch failed before grouping
          for (HostReq *r : batch) {
            std::lock_guard<std::mutex> lk(r->mu);
            r->rc = -1;
            r->err = slot_[cur].err.empty() ? broken_ : slot_[cur].err;
            r->done = true;
            r->cv.notify_all();
          }
          slot_[cur].err.clear();
        }
      }
      finish(slot_[cur ^ 1]);  // complete the previous batch while this one runs
      cur ^= 1;
    }
  }

  int dev_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<HostReq *> q_;
  Slot slot_[2];
  hipStream_t s_in_ = nullptr, s_out_ = nullptr;
  hipEvent_t in_done_ = nullptr;
  std::string broken_;
};

int run_coalesced(PlanExt *e, char **ptrs, int nstripes, long long C, const std::vector<int> &in_ids,
                  const std::vector<int> &out_ids, const void *image, int kind) {
  int dev = 0;
  HIP_OK(hipGetDevice(&dev));
  HostReq r;
  r.ptrs = ptrs;
  r.nstripes = nstripes;
  r.km = e->pub.data_strips + e->pub.parity_strips;
  r.C = C;
  r.in_ids = in_ids;
  r.out_ids = out_ids;
  r.image = image;
  r.kind = kind;
  r.packet = e->pub.packet_size;
  r.w = e->pub.w;
  CallerPinned cp = caller_pinned(ptrs, nstripes, r.km, in_ids, out_ids, C,
                                  kernel_copy_policy() != KernelCopy::kNever &&
                                      kernel_transport_aligned(ptrs, nstripes, r.km, in_ids, out_ids, C, C));
  r.pinned = cp.pinned;
  r.by_kernel = cp.by_kernel;
  r.dev.swap(cp.dev);
  return Dispatcher::for_device(dev)->run(r);
}

}  // namespace eng
}  // namespace lsec
