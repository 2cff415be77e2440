// ec_engine.h -- internal interface between the engine's host-side files (not part of the C ABI;
// include/lstore_ec.h is).  The engine is split by route:
//
//   ec_plan.cpp           plan service: et_* plan entry points, matrices, device images, decode
//                         entries, check_geometry, enqueue_apply (every kernel launch of a coding
//                         job goes through it), the device-resident core
//   ec_route.cpp          the routing function (route_host) and its threshold table (RouteTable),
//                         the batched / per-stripe entry points, the device set, the direct retry
//   ec_stripe_server.cpp  route 1: the persistent stripe server (host side of ec_server.hip)
//   ec_zerocopy.cpp       route 2: a thread's own page-locked slot (zero-copy launch)
//   ec_dispatch.cpp       route 3: the per-device dispatcher (coalesced DMA batches)
//   ec_staging.cpp        route 4: the call's own staging pipeline (packed or pinned-in-place DMA)
//   ec_pinning.cpp        pointer queries, caller page-locked memory, in-place pinning
//   ec_hostcopy.cpp       streaming host copies and the NUMA-local copy pool
//   ec_waits.cpp          completion waits (spinners, futex parking, pollers)
//
// There is no CPU compute path: every byte of parity or recovered data is produced by the HIP
// kernels (ec_kernels*.hip, ec_server.hip, ec_jit.cpp's compiled networks).
#pragma once

#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "../../include/lstore_ec.h"
#include "ec_hiperr.h"
#include "ec_kernels.h"
#include "gf8.h"

namespace lsec {
namespace eng {

using lsec::CoefCell;
using lsec::ShardRef;

// ---------------------------------------------------------------- errors
extern thread_local std::string tl_err;  // lsec_last_error()
int fail(const char *fmt, ...) __attribute__((format(printf, 1, 2)));         // tl_err = message; -1
[[noreturn]] void fatal(const char *fmt, ...) __attribute__((format(printf, 1, 2)));

#define HIP_OK(expr)                                                                             \
  do {                                                                                           \
    hipError_t e_ = (expr);                                                                      \
    if (e_ != hipSuccess) return fail("%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, __LINE__); \
  } while (0)


// ---------------------------------------------------------------- plans (ec_plan.cpp)
enum KernelKind { KNONE = 0, KBYTEWISE = 1, KBITSLICED = 2, KBITMATRIX = 3, KWORDWISE = 4, KBITSLICEDW = 5 };

// devices per stripe: Jerasure takes k + m <= 2^w (reed_sol.c:247-248, cauchy.c:139), 256 at w = 8.
// The engine takes that at w = 8 and for the bitmatrix codes (LSEC_MAX_DEVS), and up to
// kMaxDevs = 1024 for the GF(2^16) / GF(2^32) matrix codes (RS, r6, Cauchy); the segment adapters
// keep LSEC_MAX_DEVS, which sizes their ABI structs.  Inputs beyond lsec::kMaxK per launch run as
// several launches over the grouped image layout (ec_kernels.h).
constexpr int kMaxDevs = LSEC_MAX_DEVS_WIDE;
int max_devs(int method, int w);

struct DecodeEntry {
  lsec::gf8::DecodePlan dp;
  bool xor_only = false;  // GF(2^8) rows of 0 / 1 only (XOR of survivors)
  std::map<int, CoefCell *> dev_cells;  // device -> e x k cells
  std::vector<uint32_t> masks;          // bitmatrix codes: (e*w) x k row masks; wordwise: e x k x w products
  std::map<int, uint32_t *> dev_masks;
  std::vector<uint32_t> wrows;          // wordwise: the e x k GF(2^w) decode rows (XOR networks)
};

constexpr int kFastDevs = 16;  // devices whose encode image pointer is cached lock-free

struct PlanImpl {
  std::mutex mu;
  // Lock-free fast path of the per-stripe calls (up to 300 pool threads share one plan): set
  // once under mu, after what they publish is complete, and never cleared before the plan is
  // destroyed (the caller may not use a plan it destroys).
  std::atomic<bool> coding_fast{false};
  std::atomic<const void *> enc_fast[kFastDevs] = {};
  // process-unique id: per-thread caches key on it, not on the address (a destroyed plan's
  // address can come back for a new plan)
  const unsigned long long serial = next_serial();
  static unsigned long long next_serial() {
    static std::atomic<unsigned long long> n{0};
    return ++n;
  }
  lsec::gf8::Mat coding;   // GF(2^8) matrix the kernels apply (m x k)
  lsec::gfw::Mat coding_w; // GF(2^16) / GF(2^32) matrix codes (m x k)
  bool coding_ready = false;
  std::map<int, CoefCell *> enc_cells;                   // device -> m x k cells
  std::vector<uint32_t> enc_masks;                       // bitmatrix codes: (m*w) x k row masks;
                                                         // wordwise: m x k x w products
  std::map<int, uint32_t *> enc_dev_masks;
  std::map<std::vector<int>, DecodeEntry> decode_cache;  // sorted erased ids -> entry
};

// The public struct must stay first: callers only ever see &PlanExt::pub, and
// et_destroy_plan / the fn-pointers recover the extension from it.
struct PlanExt {
  lio_erasure_plan_t pub;
  uint64_t magic;
  PlanImpl *impl;
};
constexpr uint64_t kPlanMagic = 0x4C53454350414E31ull;  // "LSECPAN1"

PlanExt *ext_of(lio_erasure_plan_t *p);
bool liberation_family(int method);
int kernel_kind(int method, int w);
bool uses_u32_image(int kind);
bool packet_kind(int kind);
int form_matrices(lio_erasure_plan_t *p, bool with_schedule);
int fp_form_encoding(lio_erasure_plan_t *p);
int fp_form_decoding(lio_erasure_plan_t *p);
int ensure_coding(PlanExt *e);
int encode_rows(const PlanExt *e);
int encode_cells(PlanExt *e, const void **out);
int parse_erasures(const lio_erasure_plan_t *p, const int *erasures, std::vector<int> &ids);
int decode_entry(PlanExt *e, const std::vector<int> &ids, DecodeEntry **out, const void **cells);
int decode_kind(const PlanExt *e, const DecodeEntry *ent);
int check_geometry(const lio_erasure_plan_t *p, long long block_size);
int enqueue_apply(int kind, const void *image, int K, int R, const ShardRef *in, const ShardRef *out, int nstripes,
                  long long size, int packet, hipStream_t st, int w = 8);
int encode_dev(PlanExt *e, const lsec_shard_t *sh, int nstripes, long long C, hipStream_t st);
int decode_dev(PlanExt *e, const lsec_shard_t *sh, int nstripes, long long C, const int *erasures, hipStream_t st);
void fp_encode_block(lio_erasure_plan_t *p, char **ptr, int block_size);         // ec_route.cpp
int fp_dummy(lio_erasure_plan_t *);                                            // ec_route.cpp
int encode_stripes_impl(PlanExt *e, char **ptrs, int nstripes, long long C);  // ec_route.cpp
int decode_stripes_impl(PlanExt *e, char **ptrs, int nstripes, long long C, const int *erasures);
int fp_decode_block(lio_erasure_plan_t *p, char **ptr, int block_size, int *erasures);  // ec_route.cpp

// ---------------------------------------------------------------- the routing table (ec_route.cpp)
// Every threshold of the host-memory routes, read once: the defaults are the measured ones
// (DESIGN.md §2 gives each one's record), environment variables override them for A/B runs, and
// the concurrency limits derive from the CPUs this process may use (usable_cpus: the affinity
// mask capped by the cgroup quota).  route_host (ec_route.cpp) is the one routing function.
struct RouteTable {
  int cpus;                    // usable_cpus()
  // route choice by a call's bytes (inputs + outputs)
  size_t zerocopy_max;         // LSEC_ZEROCOPY_KB = 4096: up to here, routes 1-2 (server, own slot)
  size_t coalesce_max;         // LSEC_COALESCE_MB = 16: up to here, route 3 (dispatcher)
  size_t own_pipeline_min;     // LSEC_OWN_PIPELINE_MIN_KB = 4096: from here to coalesce_max, a call's own pipeline ...
  int own_pipeline_max;        // LSEC_OWN_PIPELINE_MAX = max(2, cpus / 2): ... while this few run
  bool own_pipeline_slot;      // LSEC_ZC_BIG = 1: that pipeline is the own slot (route 2), else route 4
  int own_dma_max;             // LSEC_OWN_DMA_MAX = 2: while at most this many own pipelines run, each
                               // takes route 4 pinned in place (DMA, no packing) ...
  size_t own_dma_min_bytes;    // 1 MiB: ... when the call has this many bytes ...
  size_t own_dma_min_run;      // LSEC_OWN_DMA_MIN_RUN_KB = 1024: ... and its DMA runs average this
  size_t defer_unpin_bytes;    // LSEC_DEFER_UNPIN_MB = 0 (off): > 0 lets a background thread drop a
                               // call's in-place registrations after it returns while another call
                               // holds registrations, at most this many bytes pending
                               // (hipHostUnregister waits for the whole device to idle).  Off by
                               // default: a registration that outlives its call maps pages the caller
                               // may free and reuse, and another HIP user in the process would take
                               // them for page-locked memory
  int lone_blocks;             // LSEC_LONE_BLOCKS = 1: a lone stripe DMA'd in place moves in this many
                               // column blocks (block b+1's H2D under block b's kernel and D2H)
  bool server;                 // LSEC_SERVER = 1: route 1 on
  size_t srv_nt_min;           // LSEC_SRV_NT_MIN_KB (off): server calls copying this much in use streaming stores
  bool srv_early_out;          // LSEC_SRV_EARLY_OUT = 1: a spinning server caller copies each part's
                               // outputs out as soon as that part is done, while later parts are served
  // transports
  bool pin_in_place;           // LSEC_NO_HOST_REGISTER unset: pageable batches may be pinned in place for DMA
  size_t pin_min_bytes;        // LSEC_PIN_MIN_KB = 8192: ... when the batch has at least this many bytes
  size_t pin_min_run;          // LSEC_PIN_MIN_RUN_KB = 6144: ... and its DMA copies average this run
                               //   (waived for one-region batches of >= 4 stripes: strided copies)
  bool kernel_copy;            // LSEC_KERNEL_COPY != 0: hipHostMalloc'd caller runs may move by kernel
  size_t kernel_copy_max_run;  // 1 MiB: ... when their runs average less
  int slot_pack_pool;          // LSEC_ZC_POOL: -1 (default) own-slot calls pack on the pool when
                               // more than slot_pack_inline run, else on the calling thread; 0 / 1 force
  int slot_pack_inline;        // 2
  // sizes
  size_t staging_bytes;        // LSEC_STAGING_MB = 128: route 4's page-locked budget per pipeline
  size_t dev_staging_bytes;    // LSEC_DEV_STAGING_MB = 512: route 4's device slots when it DMAs in place
                               // (no page-locked staging: only HBM, so whole stripes of wide codes fit)
  size_t slot_budget;          // LSEC_ZC_SLOTS_MB = 1024: route 2's slots per device (PinnedBudget)
  size_t dispatch_batch;       // 96 MiB packed per dispatcher batch
  int copy_threads;            // LSEC_COPY_THREADS = min(8, hardware threads): copy pool per NUMA node
  // waits
  int spinners;                // max(1, cpus / 4) waiters spin at once, ...
  std::chrono::microseconds spin;  // ... for up to 30 us; the rest park
  int pollers;                 // max(1, min(4, cpus / 8)) poller threads wake the parked
};
const RouteTable &routes();

// ---------------------------------------------------------------- host copies (ec_hostcopy.cpp)
struct CopyJob {
  char *dst;
  const char *src;
  size_t bytes;
};

// NUMA node whose copy pool packs this thread's staging: set by threads that work for one device
// (its dispatcher, the threads of a split host batch), -1 elsewhere
extern thread_local int tl_copy_node;
void stream_copy(char *dst, const char *src, size_t n);  // non-temporal stores; _mm_sfence() before publishing
void host_copy(char *dst, const char *src, size_t n);    // stream_copy, or memcpy under LSEC_NT_COPY=0
// every job copied, spread over the copy pool of this thread's node (the caller works too), in
// pieces of at most `piece` bytes; the bytes are visible when it returns
void copy_run(std::vector<CopyJob> &jobs, size_t piece = 512 << 10);

// ---------------------------------------------------------------- host memory kinds (ec_pinning.cpp)
extern std::atomic<unsigned long long> g_st_queries;  // runtime pointer queries (LSEC_STATS)
// Pointer attributes.  Every hipPointerGetAttributes takes a lock of the HIP runtime; per-stripe
// calls from tens of threads made 10-20 queries each and spent most of their time queued on it
// (an RS(6+3) 16 KiB call: 3 us of set-up at one thread, 140-360 us at 32 before this memo, 12 us
// after; LSEC_STATS phase means, profiles/r02_v30_zc_phases.txt for the after-state).  Within
// one public call the caller's buffers cannot change kind, so a
// call answers repeated queries from a per-call memo (PtrMemo: the entry points of the batched
// and per-stripe calls open one; with none open every query goes to the runtime).
struct PtrInfo {
  bool ok = false;  // the query succeeded (ROCm 7 also answers for pageable memory: type Unregistered)
  hipMemoryType type = hipMemoryTypeHost;
  void *dev = nullptr;  // its device address
};
extern thread_local int tl_memo_depth;
extern thread_local std::vector<std::pair<const void *, PtrInfo>> tl_memo;
struct PtrMemo {
  PtrMemo() {
    if (tl_memo_depth++ == 0) tl_memo.clear();
  }
  ~PtrMemo() {
    if (--tl_memo_depth == 0) tl_memo.clear();
  }
  PtrMemo(const PtrMemo &) = delete;
  PtrMemo &operator=(const PtrMemo &) = delete;
};

PtrInfo query_ptr(const void *ptr);
bool is_pinned_host(const void *ptr);
bool is_device_ptr(const void *ptr);

// Ranges pinned in place by a running call (InPlacePin), page-rounded.  Another call that
// touches them must not take them for caller-pinned memory: the owner unregisters them when
// it returns, maybe while the other call's DMA is still queued.
extern std::mutex g_inplace_mu;
extern std::vector<std::pair<uintptr_t, uintptr_t>> g_inplace;
constexpr uintptr_t kPage = 4096;
bool inplace_overlaps_locked(uintptr_t lo, uintptr_t hi);

// A page-locked allocation a call has verified: [lo, hi) host bytes, device alias = host + delta.
// A chunk inside one needs no further runtime query (each takes a runtime lock; a page-locked
// per-stripe call made ~11 of them under g_inplace_mu: RS(6+3) 16 KiB at 128 threads spent
// 430 us of its 450 us in this set-up, profiles/r02_v45_zc_phases.txt).
struct PinnedAlloc {
  uintptr_t lo, hi;
  intptr_t delta;
  bool kernel_ok;  // a hipHostMalloc allocation: GPU kernels may read and write it in place
};

struct CallerPinned {
  bool pinned = false, by_kernel = false;
  std::vector<uint64_t> dev;  // by_kernel: device address of every chunk (caller_pinned_aliases order)
};

// Caller page-locked buffers.  pinned: every staged chunk of the first and last stripe is
// page-locked (a stray pageable chunk in between stays correct -- hipMemcpyAsync accepts
// pageable memory too, only slower).  by_kernel (asked with kernel_ok): small runs, and EVERY
// chunk checked to have a device address -- see caller_pinned_aliases.  The whole decision is
// one pass under g_inplace_mu, with every chunk's page range checked against the in-flight
// in-place registrations first: a range a concurrent InPlacePin has claimed (it claims before
// it registers and releases after it unregisters) is never taken for caller-pinned memory,
// since its owner may unregister it while this call's DMA or copy kernel still reads it.
CallerPinned caller_pinned(char **ptrs, int nstripes, int km, const std::vector<int> &in_ids, const std::vector<int> &out_ids,
                           long long C, bool kernel_ok);

// Pageable caller buffers of a large batch are pinned in place for the duration of the call
// when they form a few dense regions: hipHostRegister pins at 190-450 GB/s on the box
// (tools/hostreg_probe.py) while packing copies at ~20 GB/s per thread, so the DMA engines
// then read and write the caller's pages directly and the host cores stay idle.  Regions are
// exactly the caller's chunks merged where they touch (LStore: a cache page of k data chunks,
// a parity buffer), so no other buffer shares a registration.  Any failure (already
// registered by another call, too many regions) keeps the packing path.
class InPlacePin {
 public:
  ~InPlacePin() { release(); }
  // DMA only: a GPU kernel never reads or writes registered pageable pages.  (Kernels reading
  // and writing them in place -- a registered zero-copy route and a copy-piece transport for
  // pageable batches, both opt-in in rounds 1-3 -- returned stale bytes and wrote into pages the
  // caller had since reused, once host arrays were freed and reallocated between calls;
  // tools/reg_stress.py --churn, profiles/r03_v16_reg_repro.jsonl.  DMA over the same
  // registrations stayed exact: r03_v18_churn_default_routes.jsonl.)
  // min_bytes / min_run: the batch's smallest total and average DMA run worth pinning
  // (RouteTable pin_min_* for batches, own_dma_min_* for a lone call's own pipeline)
  bool pin(char **ptrs, int nstripes, int km, const std::vector<int> &in_ids, const std::vector<int> &out_ids,
           long long C, size_t min_bytes, size_t min_run);
  void release();
  bool held() const { return !held_.empty(); }

 private:
  static constexpr size_t kMaxRegions = 1024;
  std::vector<char *> held_;
  std::vector<std::pair<uintptr_t, uintptr_t>> claimed_;
};

// calls holding in-place registrations at this moment (this one included when it holds some)
int in_place_calls();

// The in-place stall guard.  DMA from pages pinned in place can stall for tens of milliseconds when
// the process keeps unmapping and remapping host memory while calls run (round 6: per-stripe
// calls on buffers that are each a fresh mmap, munmapped after the call, at two threads: ~25 ms per
// call in the drain against ~0.3 ms packed; profiles/r06_v2_free_after_churn.jsonl).  run_host
// reports every pinned call's drain; three stalls (under 1 GB/s and over 5 ms) within 64 calls
// suspend in-place pinning -- calls pack into the engine's page-locked staging instead -- for 30 s,
// doubling on every recurrence up to 10 min.  LSEC_INPLACE_GUARD=0 turns the guard off.
void note_inplace_drain(size_t bytes, double drain_ms);
bool inplace_suspended();

// DMA runs: pieces whose source and destination both continue the previous piece merge
// into one copy (LStore's k data chunks of a stripe sit back to back in one cache page, so
// a stripe's inputs usually become a single k*C transfer)
struct DmaRun {
  char *dst;
  const char *src;
  size_t bytes;
};

void add_run(std::vector<DmaRun> &v, char *dst, const char *src, size_t n);
hipError_t issue_runs(const std::vector<DmaRun> &v, hipMemcpyKind kind, hipStream_t st);
size_t add_pieces(lsec::CopyPiece *pl, size_t n, uint64_t src, uint64_t dst, size_t len);
void split_pieces(std::vector<lsec::CopyPiece> &v, uint64_t src, uint64_t dst, size_t len);

// Kernel transport policy, LSEC_KERNEL_COPY read per call:
//   unset  caller page-locked buffers with small runs move by kernel (DMA of their 384 KiB runs
//          moves 17-20 GiB/s at C = 64 KiB, the kernel 30 / 38: profiles/r01_v28_kcopy_pinned.txt);
//          pageable batches with small runs are packed
//   0      never
// (Until round 3, `1` also pinned pageable batches in place for the copy kernel; kernels over
// per-call registrations of pageable pages are gone, see InPlacePin.)
enum class KernelCopy { kNever, kCallerPinned };
KernelCopy kernel_copy_policy();
bool kernel_transport_aligned(char **ptrs, int nstripes, int km, const std::vector<int> &in_ids,
                              const std::vector<int> &out_ids, long long C, long long cb);

// ---------------------------------------------------------------- routes
// route 4, the call's own staging pipeline (ec_staging.cpp); magic_host: stripe magics too
// eager_pin: pin pageable chunks in place at the lower own_dma_min_* thresholds (a lone call's own
// pipeline, route_host), else at pin_min_*
int run_host(PlanExt *e, char **ptrs, int nstripes, long long C, const std::vector<int> &in_ids,
             const std::vector<int> &out_ids, const void *cells, int kind, uint8_t *magic_host = nullptr,
             bool eager_pin = false);
hipError_t launch_magic_groups(lsec::MagicArgs ma, const ShardRef *sh, int km, hipStream_t st);
// route 3, the device's dispatcher (ec_dispatch.cpp)
int run_coalesced(PlanExt *e, char **ptrs, int nstripes, long long C, const std::vector<int> &in_ids,
                  const std::vector<int> &out_ids, const void *image, int kind);
// routes 1 and 2 (ec_zerocopy.cpp): the stripe server, else this thread's own slot; 1 = the
// slot would pass its page-locked budget (the caller takes another route)
int run_zerocopy(PlanExt *e, char **ptrs, int nstripes, long long C, const std::vector<int> &in_ids,
                 const std::vector<int> &out_ids, const void *image, int kind);
hipStream_t thread_stream();  // this thread's stream on the current device (ec_route.cpp)

// ---------------------------------------------------------------- waits (ec_waits.cpp)
int usable_cpus();  // affinity mask, capped by the cgroup CPU quota
// until every flags[i] reaches wants[i] (wrapping u32 sequences) or `slice` passes; true when
// all have.  n <= kMaxWaitFlags parks on a futex when spinning does not pay.
constexpr int kMaxWaitFlags = 16;
// Called by a spinning wait each time flags[0, upto) have all been reached (in order), so the caller
// can consume finished parts while the rest are served.  A parked waiter reports on waking.
struct WaitProgress {
  void (*fn)(void *ctx, int upto);
  void *ctx;
};
bool flag_wait(const unsigned *const *flags, const unsigned *wants, int n, std::chrono::microseconds slice,
               const WaitProgress *progress = nullptr);
// flag reaches v, bounded: after 2 s the stream's status decides (false, *rc = -1 with a message)
bool wait_flag(const unsigned *flag, unsigned v, hipStream_t st, int *rc);
extern std::atomic<unsigned long long> g_st_parks, g_st_spin_hits, g_st_claim_misses, g_st_claim_spins, g_st_wakes,
    g_st_slices;

// ---------------------------------------------------------------- stripe server (ec_stripe_server.cpp)
// 0 served, -1 error, 1 not servable here (the caller takes another route)
int server_run(int dev, PlanExt *e, char **ptrs, long long C, const std::vector<int> &in_ids,
               const std::vector<int> &out_ids, const void *image, int kind, const CallerPinned *cp);
void servers_restart();  // stop every server (the next launch takes new test settings)
// Around a hipHostUnregister (ec_pinning.cpp), which waits until the device is idle: running
// stripe servers are stopped and none is launched until the matching end (ec_stripe_server.cpp)
void servers_yield_begin();
void servers_yield_end();
extern std::atomic<int> g_srv_timeout_ms, g_srv_hold;
extern std::atomic<unsigned long long> g_st_srv_timeouts;

// ---------------------------------------------------------------- LSEC_STATS
// Routes taken by zero-copy calls, printed at exit with LSEC_STATS=1: served by the stripe
// server, refused by it (no free slots: claim failed, or not servable), then run as their own
// launch (kernel over the caller's page-locked chunks, or over this thread's slot)
extern thread_local std::chrono::steady_clock::time_point tl_call_t0;  // fn-pointer entry (LSEC_STATS)
// LSEC_TRACE of a fn-pointer call: run_host leaves its phase line here (line[0] != 0) instead of
// printing it, and the fn-pointer prints it with the time before run_host (entry) and after it (exit)
struct CallTrace {
  bool active = false;
  std::chrono::steady_clock::time_point t_call0, t_run0, t_run1;
  char line[320] = {0};
};
extern thread_local CallTrace tl_trace;
extern thread_local std::chrono::steady_clock::time_point tl_zc_t0;    // run_zerocopy entry (LSEC_STATS)
extern thread_local long long tl_call_cpu0, tl_zc_cpu0;           // this thread's CPU ns at both

long long thread_cpu_ns();

struct ZcStats {
  std::atomic<unsigned long long> server{0}, no_slots{0}, not_servable{0}, launch_direct{0}, launch_slot{0};
  // server-served calls, wall time per phase (ns): fn-pointer entry -> server (plan checks,
  // layout and pinned-memory lookups), claim + copies in + posts, wait, copies out
  std::atomic<unsigned long long> t_setup{0}, t_zc{0}, t_post{0}, t_wait{0}, t_out{0};
  std::atomic<unsigned long long> c_setup{0}, c_zc{0}, c_post{0}, c_wait{0}, c_out{0};  // thread CPU ns
  // own-slot calls, wall time (ns): slot allocation, packing the inputs, enqueueing the block
  // kernels, waiting for the last one, copying the outputs back
  std::atomic<unsigned long long> s_alloc{0}, s_pack{0}, s_enq{0}, s_wait{0}, s_out{0};
  static bool on() {
    static const bool v = getenv("LSEC_STATS") != nullptr;
    return v;
  }
  static ZcStats &get() {
    static ZcStats *s = [] {
      ZcStats *p = new ZcStats();  // leaked: read by the atexit printer
      if (getenv("LSEC_STATS")) atexit([] {
        ZcStats &z = get();
        fprintf(stderr, "[lsec stats] zero-copy calls: server %llu, server out of slots %llu, not servable %llu, "
                "own launch (caller page-locked) %llu, own launch (slot) %llu\n", z.server.load(), z.no_slots.load(),
                z.not_servable.load(), z.launch_direct.load(), z.launch_slot.load());
        fprintf(stderr, "[lsec stats] waits: spin hits %llu, parks %llu, poller wakes %llu, timed-out slices %llu; "
                "claims missed %llu, claim retries %llu; runtime pointer queries %llu\n", g_st_spin_hits.load(),
                g_st_parks.load(), g_st_wakes.load(), g_st_slices.load(), g_st_claim_misses.load(), g_st_claim_spins.load(),
                g_st_queries.load());
        const double n = static_cast<double>(std::max(1ULL, z.server.load())) * 1e3;
        fprintf(stderr, "[lsec stats] server calls, mean wall us: setup %.2f (of it in run_zerocopy %.2f), claim+copy-in+post %.2f, "
                "wait %.2f, copy-out %.2f\n", z.t_setup.load() / n, z.t_zc.load() / n, z.t_post.load() / n, z.t_wait.load() / n,
                z.t_out.load() / n);
        fprintf(stderr, "[lsec stats] server calls, mean thread CPU us: setup %.2f (of it in run_zerocopy %.2f), claim+copy-in+post "
                "%.2f, wait %.2f, copy-out %.2f\n", z.c_setup.load() / n, z.c_zc.load() / n, z.c_post.load() / n,
                z.c_wait.load() / n, z.c_out.load() / n);
        const double ns = static_cast<double>(std::max(1ULL, z.launch_slot.load())) * 1e3;
        fprintf(stderr, "[lsec stats] own-slot calls, mean wall us: slot %.2f, pack %.2f, enqueue %.2f, wait %.2f, copy-out %.2f\n",
                z.s_alloc.load() / ns, z.s_pack.load() / ns, z.s_enq.load() / ns, z.s_wait.load() / ns, z.s_out.load() / ns);
      });
      return p;
    }();
    return *s;
  }
};

// Page-locked memory of the zero-copy routes, accounted per device (per GPU its own
// host thread, streams, buffers and pinned staging).  Two kinds:
//   server   each device's stripe server holds a fixed region of kSrvSlots x 96 KiB (93 MiB),
//            allocated at its first call and never charged against the slot budget, so a
//            device's server can neither be refused nor shrink the threads' slots
//   slots    the per-thread zero-copy slots on a device together stay within LSEC_ZC_SLOTS_MB
//            (default 1024) on that device; a call whose slot would pass it goes to the dispatcher
// So with the in-process device set over 8 GPUs (lsec_set_host_devices) every device's threads
// get the same slot budget one device's do (round 3 charged both kinds to one process-wide
// 1 GiB: eight servers took 744 MiB of it).  The worst-case page-locked total is in
// INTEGRATION.md; tests/test_budget.py checks this arithmetic for 1 and 8 devices.
class PinnedBudget {
 public:
  static constexpr int kDevs = 64;  // device ids beyond share the last entry
  explicit PinnedBudget(size_t slot_budget) : budget_(slot_budget) {
    for (int d = 0; d < kDevs; ++d) {
      slots_[d].store(0);
      server_[d].store(0);
    }
  }
  static PinnedBudget &global() {
    static PinnedBudget *b = new PinnedBudget(routes().slot_budget);  // leaked: slots outlive statics
    return *b;
  }
  // a thread's slot on `dev` grows from old_cap to new_cap bytes: false if the device's slots
  // would pass the budget (nothing is charged then)
  bool grow_slot(int dev, size_t old_cap, size_t new_cap) {
    std::atomic<size_t> &u = slots_[idx(dev)];
    size_t cur = u.load(std::memory_order_relaxed);
    do {
      if (cur - old_cap + new_cap > budget_) return false;
    } while (!u.compare_exchange_weak(cur, cur - old_cap + new_cap, std::memory_order_relaxed));
    return true;
  }
  void release_slot(int dev, size_t cap) { slots_[idx(dev)].fetch_sub(cap, std::memory_order_relaxed); }
  void add_server(int dev, size_t bytes) { server_[idx(dev)].fetch_add(bytes, std::memory_order_relaxed); }
  size_t slot_bytes(int dev) const { return slots_[idx(dev)].load(std::memory_order_relaxed); }
  size_t server_bytes(int dev) const { return server_[idx(dev)].load(std::memory_order_relaxed); }
  size_t budget() const { return budget_; }

 private:
  static int idx(int dev) { return dev < 0 ? 0 : std::min(dev, kDevs - 1); }
  const size_t budget_;
  std::atomic<size_t> slots_[kDevs];
  std::atomic<size_t> server_[kDevs];
};

}  // namespace eng
}  // namespace lsec
