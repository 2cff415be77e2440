// ec_staging.cpp -- route 4: a host call's own staging pipeline (pack or pin in place -> H2D ->
// kernel -> D2H -> unpack, three slots on two streams), used for host batches above the
// dispatcher's limit and for the magic-fused encode of the segment adapter.
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

#include "ec_engine.h"

namespace lsec {
namespace eng {

// ---------------------------------------------------------------- host staging pool
// Each staging object owns a copy-in stream, a compute/copy-out stream and kSlots slots of
// pinned + device memory, so that for consecutive batches  H2D(b+1) || kernel(b) -> D2H(b)
// and the host packs b+2 / unpacks b-1 meanwhile (PCIe is full duplex).
constexpr int kSlots = 3;

struct Staging {
  int dev = -1;
  hipStream_t s_in = nullptr, s_out = nullptr;
  struct Slot {
    char *d = nullptr;   // device: [nb][nin][C] then [nb][nout][C]
    char *h = nullptr;   // pinned host, same layout
    size_t cap = 0;      // bytes at d
    size_t hcap = 0;     // bytes at h (grown on its own: see ensure_slot)
    hipEvent_t in_done = nullptr, done = nullptr;
    bool pending = false;
    // what to unpack when `done` fires
    char **ptrs = nullptr;
    int s0 = 0, nb = 0;
    long long c0 = 0, clen = 0;  // column block of each shard this slot carries
    // kernel transport (small host runs pinned in place): the slot's copy pieces, page-locked
    lsec::CopyPiece *pl = nullptr;
    size_t pl_cap = 0;
  } slot[kSlots];
  ~Staging() {
    for (auto &s : slot) {
      if (s.pl) (void)hipHostFree(s.pl);
      if (s.d) (void)hipFree(s.d);
      if (s.h) (void)hipHostFree(s.h);
      if (s.done) (void)hipEventDestroy(s.done);
      if (s.in_done) (void)hipEventDestroy(s.in_done);
    }
    if (s_in) (void)hipStreamDestroy(s_in);
    if (s_out) (void)hipStreamDestroy(s_out);
  }
};

std::mutex g_pool_mu;
std::map<int, std::vector<Staging *>> g_pool;

Staging *acquire_staging(int dev) {
  {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    auto &v = g_pool[dev];
    if (!v.empty()) {
      Staging *s = v.back();
      v.pop_back();
      return s;
    }
  }
  Staging *s = new Staging();
  s->dev = dev;
  if (hipStreamCreateWithFlags(&s->s_in, hipStreamNonBlocking) != hipSuccess ||
      hipStreamCreateWithFlags(&s->s_out, hipStreamNonBlocking) != hipSuccess) {
    delete s;
    return nullptr;
  }
  for (auto &sl : s->slot)
    if (hipEventCreateWithFlags(&sl.done, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&sl.in_done, hipEventDisableTiming) != hipSuccess) {
      delete s;
      return nullptr;
    }
  return s;
}

// Device halves larger than the packed geometry's (the in-place DMA geometry, dev_staging_bytes:
// up to ~256 MiB a slot) are kept by at most kKeepLarge pooled stagings per device; a staging that
// comes back with them beyond that gives them up (the next large call regrows them).  Otherwise the
// HBM the pool holds for the life of the process grew with the peak count of concurrent large
// pinned calls: 16 threads of RS(6+3) 1 MiB batches kept ~12 GiB.
constexpr int kKeepLarge = 2;

bool large_device_half(const Staging *s) {
  for (const auto &sl : s->slot)
    if (sl.cap > routes().staging_bytes / 2) return true;
  return false;
}

void release_staging(Staging *s) {
  bool shrink = false;
  {
    std::lock_guard<std::mutex> lk(g_pool_mu);
    if (large_device_half(s)) {
      int large = 0;
      for (const Staging *o : g_pool[s->dev]) large += large_device_half(o);
      shrink = large >= kKeepLarge;
    }
  }
  if (shrink)
    for (auto &sl : s->slot)
      if (sl.cap > routes().staging_bytes / 2) {
        (void)quiet([&] { return hipFree(sl.d); });  // (every slot was drained before the release)
        sl.d = nullptr;
        sl.cap = 0;
      }
  std::lock_guard<std::mutex> lk(g_pool_mu);
  g_pool[s->dev].push_back(s);
}


// Slots are sized for a full batch (half the staging budget) the first time, so that a
// small first call does not leave them too small for the next one: re-pinning 64 MiB of
// host memory costs more than moving it over PCIe.  need_host = false (pinned callers, see
// below) needs only the device half.  The two halves grow independently: a pinned caller's
// larger device geometry (dev_staging_bytes) must not free the host half a packed caller
// will want again, or alternating pinned encodes and packed decodes re-pin the host half on
// every call (a 2x host-path loss the round-5 c5 sweep showed).
int ensure_slot(Staging::Slot &sl, size_t bytes, bool need_host = true) {
  const size_t cap = std::max(bytes, routes().staging_bytes / 2);
  if (sl.cap < bytes) {
    if (sl.d) (void)hipFree(sl.d);
    sl.d = nullptr;
    sl.cap = 0;
    HIP_OK(hipMalloc(&sl.d, cap));
    sl.cap = cap;
  }
  if (need_host && sl.hcap < bytes) {
    if (sl.h) (void)hipHostFree(sl.h);
    sl.h = nullptr;
    sl.hcap = 0;
    HIP_OK(hipHostMalloc(reinterpret_cast<void **>(&sl.h), cap, hipHostMallocDefault));
    sl.hcap = cap;
  }
  return 0;
}

// Stripe magic partial sums over `km` shards in checksum order (sh[i] = shard i), in launches
// of at most kMaxMagicShards shards; `ma` carries everything else.
hipError_t launch_magic_groups(lsec::MagicArgs ma, const ShardRef *sh, int km, hipStream_t st) {
  ma.total_shards = km;
  for (int i0 = 0; i0 < km; i0 += lsec::kMaxMagicShards) {
    ma.shard0 = i0;
    ma.nshards = std::min(lsec::kMaxMagicShards, km - i0);
    for (int i = 0; i < ma.nshards; ++i) ma.sh[i] = sh[i0 + i];
    const hipError_t err = lsec::launch_stripe_magic(ma, st);
    if (err != hipSuccess) return err;
  }
  return hipSuccess;
}

// Shared driver of the host-memory paths.  For each stripe, `in_ids` name the shards that
// go to the GPU and `out_ids` the shards that come back (encode: data -> parity; decode:
// survivors -> erased).  The kernel runs on the packed staging layout.
//
// Work is cut into batches of about half the staging budget: whole stripes when a stripe
// fits, otherwise column blocks of every shard of one stripe (the codes act column-wise --
// bytewise on any 8-byte boundary, bitsliced on super-packet boundaries -- so a block is a
// valid independent sub-stripe).
int run_host(PlanExt *e, char **ptrs, int nstripes, long long C, const std::vector<int> &in_ids,
             const std::vector<int> &out_ids, const void *cells, int kind, uint8_t *magic_host, bool eager_pin) {
  lio_erasure_plan_t *p = &e->pub;
  const int km = p->data_strips + p->parity_strips;
  // staged position of every device id (for the stripe magic, which covers all k+m chunks)
  std::vector<int> where(km, -1);  // >= 0: input slot j; <= -2: output slot (-2 - r)
  for (size_t j = 0; j < in_ids.size(); ++j) where[in_ids[j]] = static_cast<int>(j);
  for (size_t r = 0; r < out_ids.size(); ++r) where[out_ids[r]] = -2 - static_cast<int>(r);
  if (magic_host) {
    for (int i = 0; i < km; ++i)
      if (where[i] == -1) return fail("stripe magic needs all %d chunks staged", km);
  }
  const int nin = static_cast<int>(in_ids.size()), nout = static_cast<int>(out_ids.size());
  int dev = 0;
  HIP_OK(hipGetDevice(&dev));
  const size_t per_col = static_cast<size_t>(nin + nout);  // staging bytes per column byte
  // Batch geometry for a staging budget: whole stripes per slot when a stripe fits half the
  // budget, else column blocks of one stripe (packet codes cut at super-packet boundaries)
  long long cb = C;
  int nb_max = 1;
  const auto geometry = [&](size_t budget) {
    cb = C;
    if (per_col * C > budget / 2) {
      const long long align = packet_kind(kind) ? static_cast<long long>(p->w) * p->packet_size : 8192;
      cb = static_cast<long long>(budget / 2 / per_col) / align * align;
      if (cb < align) cb = align;
      if (cb >= C) cb = C;
    }
    nb_max = cb < C ? 1 : static_cast<int>(std::max<size_t>(1, std::min<size_t>(nstripes, budget / 2 / (per_col * C))));
  };
  geometry(routes().staging_bytes);
  Staging *stg = acquire_staging(dev);
  if (!stg) return fail("cannot create staging streams");
  int rc = 0;
  std::vector<CopyJob> jobs;
  unsigned long long *dacc = nullptr;
  uint8_t *dmagic = nullptr;
  if (magic_host) {
    hipError_t err = hipMallocAsync(reinterpret_cast<void **>(&dacc), 16ull * nstripes + 4ull * nstripes, stg->s_out);
    if (err == hipSuccess) err = hipMemsetAsync(dacc, 0, 16ull * nstripes, stg->s_out);
    if (err != hipSuccess) {
      delete stg;
      return fail("magic workspace: %s", hipGetErrorString(err));
    }
    dmagic = reinterpret_cast<uint8_t *>(dacc + 2ull * nstripes);
  }

  // LSEC_TRACE=1: wall time of the phases of this call on stderr
  static const bool trace = getenv("LSEC_TRACE") != nullptr;
  const auto now = [] { return std::chrono::steady_clock::now(); };
  const auto ms = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
    return std::chrono::duration<double, std::milli>(b - a).count();
  };
  const auto t_pin0 = now();
  // pinned callers (or pageable ones pinned in place for this call): DMA straight between
  // their buffers and the device slots.  `inplace` is declared before the staging users, so
  // its registrations outlive every DMA (all are drained before run_host returns).
  InPlacePin inplace;
  const KernelCopy kpol = kernel_copy_policy();
  const bool aligned = kpol != KernelCopy::kNever && kernel_transport_aligned(ptrs, nstripes, km, in_ids, out_ids, C, cb);
  CallerPinned cp = caller_pinned(ptrs, nstripes, km, in_ids, out_ids, C, aligned);
  const bool caller_pinned = cp.pinned;
  const auto t_reg0 = now();
  const RouteTable &rt = routes();
  const bool pinned = caller_pinned || inplace.pin(ptrs, nstripes, km, in_ids, out_ids, C,
                                                   eager_pin ? rt.own_dma_min_bytes : rt.pin_min_bytes,
                                                   eager_pin ? rt.own_dma_min_run : rt.pin_min_run);
  const std::vector<uint64_t> &calias = cp.dev;  // caller-pinned chunks moved by kernel: their device addresses
  const bool caller_by_kernel = cp.by_kernel;
  const size_t nio = in_ids.size() + out_ids.size();
  // device address of byte c0 of chunk (stripe s, list position i: inputs, then outputs)
  const auto dev_at = [&](int s, size_t i, int, long long c0) -> uint64_t {
    return calias[static_cast<size_t>(s) * nio + i] + static_cast<uint64_t>(c0);
  };
  // small caller page-locked runs move by kernel over their device addresses: one launch per
  // direction instead of a DMA per run (256 KiB runs move at 18 GB/s by DMA, 54 GB/s by one
  // kernel: profiles/r01_v27_zerocopy_probe.txt)
  const bool by_kernel = caller_by_kernel;
  // Outputs go back by kernel too.  GPU-initiated reads and writes of host memory share ~52 GB/s
  // (profiles/r01_v28_host_trace.txt), but DMA of the same small registered runs is slower still:
  // kernel in + DMA out gave 17-30 GiB/s encode against 28-32 (profiles/r01_v28_kcopy_modes.txt).
  const bool out_by_kernel = by_kernel;
  // DMA in place stages nothing on the host: the slots are device memory only, so they take the
  // device budget, and wide stripes move whole (RS(20+6) at 4 MiB: 80 MiB runs instead of twenty
  // 2.5 MiB column-block runs per stripe)
  if (pinned && !by_kernel) geometry(std::max(rt.dev_staging_bytes, rt.staging_bytes));
  // A lone stripe DMA'd in place (LStore's per-stripe calls on route 4) in column blocks: each
  // block's chunks repeat at the chunk stride, so a block moves as one strided copy each way
  // (issue_runs), and block b+1's H2D runs under block b's kernel and D2H
  if (pinned && !by_kernel && nstripes == 1 && rt.lone_blocks > 1 && cb == C) {
    const long long align = packet_kind(kind) ? static_cast<long long>(p->w) * p->packet_size : 8192;
    const long long b = (C / rt.lone_blocks + align - 1) / align * align;
    if (b < C) cb = b;
  }
  const size_t slot_bytes = per_col * static_cast<size_t>(cb) * nb_max;
  // One batch (a lone stripe's call, LStore's per-stripe pattern) has nothing to overlap.  Pinned
  // in place and alone, its H2D, kernel and D2H go in order on one stream: no cross-stream event
  // between the H2D and the kernel (~20 us in the two-thread timeline, r05_v15); 1 MiB decodes at
  // one thread 30.6 -> 32.4 / 33.1 GiB/s.  With other calls in flight, two streams let the copies
  // of different calls interleave on the link: 43.6 / 44.6 against 40.5 / 40.5 at two threads
  // (profiles/r05_v17_fnptr_one_stream_auto.jsonl).  LSEC_ONE_STREAM=1 / 0 forces either.
  static const int one_stream_env = [] {
    const char *e = getenv("LSEC_ONE_STREAM");
    return e && *e ? (*e == '1' ? 1 : 0) : -1;
  }();
  const bool one_batch = nb_max >= nstripes && cb >= C;
  const bool one_stream = one_batch && (one_stream_env == 1 || (one_stream_env < 0 && inplace.held() && in_place_calls() == 1));
  const hipStream_t s_h2d = one_stream ? stg->s_out : stg->s_in;
  const auto t_loop0 = now();
  std::vector<DmaRun> runs;

  auto unpack = [&](Staging::Slot &sl) -> int {
    if (!sl.pending) return 0;
    sl.pending = false;
    if (hipEventSynchronize(sl.done) != hipSuccess) return fail("staging event sync failed");
    if (pinned) return 0;  // the D2H already landed in the caller's buffers
    const size_t len = static_cast<size_t>(sl.clen);
    const char *outb = sl.h + static_cast<size_t>(sl.nb) * nin * len;
    jobs.clear();
    for (int s = 0; s < sl.nb; ++s)
      for (int r = 0; r < nout; ++r)
        jobs.push_back({sl.ptrs[static_cast<size_t>(sl.s0 + s) * km + out_ids[r]] + sl.c0,
                        outb + (static_cast<size_t>(s) * nout + r) * len, len});
    copy_run(jobs);
    return 0;
  };

  int which = 0;
  for (int s0 = 0; s0 < nstripes && rc == 0; s0 += nb_max) {
    const int nb = std::min(nb_max, nstripes - s0);
    for (long long c0 = 0; c0 < C && rc == 0; c0 += cb, which = (which + 1) % kSlots) {
      const long long clen = std::min(cb, C - c0);
      const size_t len = static_cast<size_t>(clen);
      Staging::Slot &sl = stg->slot[which];
      if ((rc = unpack(sl))) break;
      if ((rc = ensure_slot(sl, slot_bytes, !pinned))) break;
      const size_t in_bytes = static_cast<size_t>(nb) * nin * len;
      const size_t out_off = in_bytes;
      hipError_t err;
      size_t npin = 0;  // kernel transport: input pieces at sl.pl[0, npin), output pieces after
      if (by_kernel) {
        const size_t per = (len + lsec::kPieceBytes - 1) / lsec::kPieceBytes;
        const size_t need = per * static_cast<size_t>(nb) * (nin + nout);
        if (sl.pl_cap < need) {
          if (sl.pl) (void)hipHostFree(sl.pl);
          sl.pl = nullptr;
          sl.pl_cap = 0;
          const size_t cap = std::max(need, per * static_cast<size_t>(nb_max) * (nin + nout));
          if (quiet([&] { return hipHostMalloc(reinterpret_cast<void **>(&sl.pl), cap * sizeof(lsec::CopyPiece), hipHostMallocDefault); }) !=
              hipSuccess) {
            sl.pl = nullptr;
            rc = fail("cannot allocate the copy-piece list");
            break;
          }
          sl.pl_cap = cap;
        }
        for (int s = 0; s < nb; ++s)
          for (int j = 0; j < nin; ++j)
            if (rc == 0 && !(npin = add_pieces(sl.pl, npin, dev_at(s0 + s, static_cast<size_t>(j), in_ids[j], c0),
                                              reinterpret_cast<uint64_t>(sl.d) + (static_cast<size_t>(s) * nin + j) * len, len)))
              rc = fail("kernel transport: host chunk outside the pinned regions");
        if (rc) break;
        err = lsec::launch_copy_pieces(sl.pl, static_cast<int>(npin), s_h2d);
      } else if (pinned) {
        runs.clear();
        for (int s = 0; s < nb; ++s)
          for (int j = 0; j < nin; ++j)
            add_run(runs, sl.d + (static_cast<size_t>(s) * nin + j) * len, ptrs[static_cast<size_t>(s0 + s) * km + in_ids[j]] + c0,
                    len);
        err = issue_runs(runs, hipMemcpyHostToDevice, s_h2d);
      } else {
        jobs.clear();
        for (int s = 0; s < nb; ++s)
          for (int j = 0; j < nin; ++j)
            jobs.push_back({sl.h + (static_cast<size_t>(s) * nin + j) * len,
                            ptrs[static_cast<size_t>(s0 + s) * km + in_ids[j]] + c0, len});
        copy_run(jobs);
        err = hipMemcpyAsync(sl.d, sl.h, in_bytes, hipMemcpyHostToDevice, s_h2d);
      }
      if (s_h2d != stg->s_out) {
        if (err == hipSuccess) err = hipEventRecord(sl.in_done, s_h2d);
        if (err == hipSuccess) err = hipStreamWaitEvent(stg->s_out, sl.in_done, 0);
      }
      if (err != hipSuccess) { rc = fail("H2D: %s", hipGetErrorString(err)); break; }
      ShardRef in[kMaxDevs], out[kMaxDevs];
      for (int j = 0; j < nin; ++j)
        in[j] = {reinterpret_cast<uint64_t>(sl.d) + static_cast<uint64_t>(j) * len, static_cast<int64_t>(nin * len)};
      for (int r = 0; r < nout; ++r)
        out[r] = {reinterpret_cast<uint64_t>(sl.d) + out_off + static_cast<uint64_t>(r) * len, static_cast<int64_t>(nout * len)};
      if (nout > 0 && (rc = enqueue_apply(kind, cells, nin, nout, in, out, nb, clen, p->packet_size, stg->s_out, p->w))) break;
      if (magic_host) {
        lsec::MagicArgs ma;
        std::memset(&ma, 0, sizeof(ma));
        ma.nstripes = nb;
        ma.size = clen;
        ma.col0 = c0;
        ma.chunk = C;
        ma.acc = dacc + 2ull * s0;
        ShardRef msh[kMaxDevs];
        for (int i = 0; i < km; ++i) msh[i] = where[i] >= 0 ? in[where[i]] : out[-2 - where[i]];
        err = launch_magic_groups(ma, msh, km, stg->s_out);
        if (err != hipSuccess) { rc = fail("magic launch: %s", hipGetErrorString(err)); break; }
      }
      if (nout > 0 && out_by_kernel) {
        size_t n = npin;
        for (int s = 0; s < nb; ++s)
          for (int r = 0; r < nout; ++r)
            if (rc == 0 && !(n = add_pieces(sl.pl, n, reinterpret_cast<uint64_t>(sl.d) + out_off + (static_cast<size_t>(s) * nout + r) * len,
                                            dev_at(s0 + s, static_cast<size_t>(nin + r), out_ids[r], c0), len)))
              rc = fail("kernel transport: host chunk outside the pinned regions");
        if (rc) break;
        err = lsec::launch_copy_pieces(sl.pl + npin, static_cast<int>(n - npin), stg->s_out);
      } else if (nout > 0 && pinned) {
        runs.clear();
        for (int s = 0; s < nb; ++s)
          for (int r = 0; r < nout; ++r)
            add_run(runs, ptrs[static_cast<size_t>(s0 + s) * km + out_ids[r]] + c0,
                    sl.d + out_off + (static_cast<size_t>(s) * nout + r) * len, len);
        err = issue_runs(runs, hipMemcpyDeviceToHost, stg->s_out);
      } else if (nout > 0) {
        err = hipMemcpyAsync(sl.h + out_off, sl.d + out_off, static_cast<size_t>(nb) * nout * len, hipMemcpyDeviceToHost,
                             stg->s_out);
      }
      if (err == hipSuccess) err = hipEventRecord(sl.done, stg->s_out);
      if (err != hipSuccess) { rc = fail("D2H: %s", hipGetErrorString(err)); break; }
      sl.pending = true;
      sl.ptrs = ptrs;
      sl.s0 = s0;
      sl.nb = nb;
      sl.c0 = c0;
      sl.clen = clen;
    }
  }
  if (magic_host && rc == 0) {
    hipError_t err = lsec::launch_magic_finalize(dacc, nstripes, static_cast<int64_t>(km) * C, dmagic, stg->s_out);
    if (err == hipSuccess) err = hipMemcpyAsync(magic_host, dmagic, 4ull * nstripes, hipMemcpyDeviceToHost, stg->s_out);
    if (err != hipSuccess) rc = fail("magic finalize: %s", hipGetErrorString(err));
  }
  const auto t_drain0 = now();
  // drain in submission order
  for (int i = 0; i < kSlots; ++i) {
    const int r2 = unpack(stg->slot[(which + i) % kSlots]);
    if (!rc) rc = r2;
  }
  if (rc == 0 && inplace.held()) {  // the in-place stall guard (ec_engine.h)
    const size_t moved = static_cast<size_t>(nstripes) * (in_ids.size() + out_ids.size()) * static_cast<size_t>(C);
    note_inplace_drain(moved, ms(t_loop0, now()));
  }
  if (trace && rc == 0) {  // every slot drained: no transfer still reads or writes the pins
    const auto t_rel0 = now();
    inplace.release();  // (the destructor would, after this print)
    const auto t_end = now();
    char line[320];
    snprintf(line, sizeof(line), "[lsec trace] host call %d stripes, %d in / %d out x %lld B (%s): pin %.4f ms (query %.4f, register %.4f), "
                    "submit %.4f ms, drain %.4f ms, unpin %.4f ms",
            nstripes, nin, nout, C, by_kernel ? "kernel transport" : pinned ? "pinned DMA" : "packed", ms(t_pin0, t_loop0),
            ms(t_pin0, t_reg0), ms(t_reg0, t_loop0),
            ms(t_loop0, t_drain0), ms(t_drain0, t_rel0), ms(t_rel0, t_end));
    if (tl_trace.active) {  // a fn-pointer call: it prints the line with its entry and exit times
      memcpy(tl_trace.line, line, sizeof(line));
      tl_trace.t_run0 = t_pin0;
      tl_trace.t_run1 = t_end;
    } else {
      fprintf(stderr, "%s\n", line);
    }
  }
  if (dacc) {
    if (hipStreamSynchronize(stg->s_out) != hipSuccess && !rc) rc = fail("magic sync failed");
    (void)hipFreeAsync(dacc, stg->s_out);
  }
  if (rc) {
    (void)hipStreamSynchronize(stg->s_in);
    (void)hipStreamSynchronize(stg->s_out);
    delete stg;  // do not recycle streams in an unknown state
  } else {
    release_staging(stg);
  }
  return rc;
}

}  // namespace eng
}  // namespace lsec

// Test hook, not part of include/*.h: the staging pool of device dev -- out[0] = pooled stagings,
// out[1] = those holding device halves larger than the packed geometry's, out[2] = device bytes
// their slots hold.  0.
extern "C" int lsec_test_staging_pool(int dev, long long *out) {
  using namespace lsec::eng;
  std::lock_guard<std::mutex> lk(g_pool_mu);
  long long n = 0, large = 0, bytes = 0;
  for (const Staging *s : g_pool[dev]) {
    ++n;
    large += large_device_half(s);
    for (const auto &sl : s->slot) bytes += static_cast<long long>(sl.cap);
  }
  out[0] = n;
  out[1] = large;
  out[2] = bytes;
  return 0;
}
