// ec_verify.cpp -- GPU-batched stripe verification and repair for LStore's erasure segment
// (SURVEY.md §8f row 3): the read path (segjerase_read_func, src/lio/segment/jerasure.c:
// 1255-1631) and the full byte-level inspection / repair (segjerase_inspect_full_func,
// :347-732).
//
// Both run the reference's per-stripe decision procedure:
//   1. majority vote over the k+m stored 4-byte magics (first group with the largest count
//      wins ties; :1383-1438, :474-502)
//   2. jerase_control_check (:202-269) with the devices outside the quorum marked bad:
//        cksum magic (segment magic_cksum = 1): rebuild the bad devices, adler32 over the
//          k+m chunks must equal the quorum magic (je_cksum_compare, :188-194)
//        legacy magic (magic_cksum = 0): slide a window of "control" chunks over the good
//          devices, rebuild bad + controls and require every rebuilt control to equal the
//          stored one
//      decode_block writes the rebuilt bad devices IN PLACE, so a failed check leaves its
//      (wrong) rebuild in the stripe for the steps that follow
//   3. on failure, jerase_brute_recovery (:321-339): first the last successful brute-force
//      bad set of this pass (bm_brute_used, :587-589, :1485), checked in place, then every
//      erasure combination of 1..m devices (1..m-1 in legacy mode) in lexicographic order,
//      each checked on swapped-in work buffers (not in place); first pass wins.
//
// Here every step is a batch over many stripes: chunks are staged once in HBM in logical
// order [W][n][C]; one check = one decode launch (rebuilt chunks go to per-stripe rebuild
// slots) plus one adler32 or chunk-compare launch over a contiguous range of staged stripes
// sharing the bad set; in-place effects are mirrored by copying rebuild slots back into the
// staged chunks of the stripes that failed.  Failures are gathered into a second stage and
// resolved in stripe order, batching the brute-force search across stripes.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <chrono>
#include <cstdio>
#include <string>
#include <cstdlib>
#include <cstring>
#include <map>
#include <vector>

#include "../../include/lstore_ec.h"
#include "ec_hiperr.h"
#include "ec_host.h"
#include "ec_kernels.h"

namespace {

constexpr uint8_t kZeroMagic[4] = {0, 0, 0, 0};
using Magic = std::array<uint8_t, 4>;

// stripes staged per batch: LSEC_VERIFY_MB of HBM for chunks + rebuild slots (default 4 GiB)
size_t verify_budget() {
  static const size_t b = [] {
    const char *s = getenv("LSEC_VERIFY_MB");
    return static_cast<size_t>(std::max(16L, s ? atol(s) : 4096L)) << 20;
  }();
  return b;
}

// LSEC_TRACE=1: per-phase wall times of a read / inspection on stderr (synchronises the
// stage stream at each mark, so the times add up).
struct Trace {
  const char *what;
  hipStream_t st = nullptr;
  bool on = getenv("LSEC_TRACE") != nullptr;
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  std::string line;
  explicit Trace(const char *w) : what(w) {}
  void mark(const char *phase) {
    if (!on) return;
    if (st) (void)hipStreamSynchronize(st);
    const auto now = std::chrono::steady_clock::now();
    char buf[96];
    snprintf(buf, sizeof(buf), " %s %.2f ms", phase, std::chrono::duration<double, std::milli>(now - t).count());
    line += buf;
    t = now;
  }
  ~Trace() {
    if (on) fprintf(stderr, "lsec trace %s:%s\n", what, line.c_str());
  }
};

// W stripes of n logical chunks in HBM ([W][n][C]) plus m rebuild slots per stripe
struct Stage {
  int W = 0, n = 0, m = 0;
  size_t C = 0;
  char *d = nullptr, *slots = nullptr;
  uint8_t *dmag = nullptr;
  int *dflag = nullptr;
  hipStream_t st = nullptr;
  std::vector<uint8_t> hmag;
  std::vector<int> hflag;

  Stage() = default;
  Stage(const Stage &) = delete;
  Stage &operator=(const Stage &) = delete;
  ~Stage() { release(); }
  // Stream-ordered allocations from the device's memory pool: a verification pass allocates
  // and frees a stage per bad-set group, and hipMalloc / hipFree (a device-wide sync) per
  // group cost more than the group's work.  See keep_pool().
  void release() {
    if (d) (void)hipFreeAsync(d, st);
    if (slots) (void)hipFreeAsync(slots, st);
    if (dmag) (void)hipFreeAsync(dmag, st);
    if (dflag) (void)hipFreeAsync(dflag, st);
    d = slots = nullptr;
    dmag = nullptr;
    dflag = nullptr;
  }
  int alloc(int W_, int n_, int m_, size_t C_, hipStream_t s) {
    release();
    W = W_, n = n_, m = m_, C = C_, st = s;
    if (W == 0) return 0;
    if (hipMallocAsync(reinterpret_cast<void **>(&d), static_cast<size_t>(W) * n * C, st) != hipSuccess ||
        hipMallocAsync(reinterpret_cast<void **>(&slots), static_cast<size_t>(W) * m * C, st) != hipSuccess ||
        hipMallocAsync(reinterpret_cast<void **>(&dmag), static_cast<size_t>(W) * 4, st) != hipSuccess ||
        hipMallocAsync(reinterpret_cast<void **>(&dflag), sizeof(int) * W, st) != hipSuccess)
      return -1;
    hmag.assign(static_cast<size_t>(W) * 4, 0);
    hflag.assign(W, 0);
    return 0;
  }
  char *chunk(int w, int j) const { return d + (static_cast<size_t>(w) * n + j) * C; }
  char *slot(int w, int r) const { return slots + (static_cast<size_t>(w) * m + r) * C; }
};

// copy whole staged stripes src[idx[i]] -> dst[i]
int gather(const Stage &src, const std::vector<int> &idx, Stage &dst) {
  for (size_t i = 0; i < idx.size(); ++i)
    if (hipMemcpyAsync(dst.chunk(static_cast<int>(i), 0), src.chunk(idx[i], 0), static_cast<size_t>(src.n) * src.C,
                       hipMemcpyDeviceToDevice, dst.st) != hipSuccess)
      return -1;
  return 0;
}

int gather_new(const Stage &src, const std::vector<int> &idx, Stage &dst) {
  if (dst.alloc(static_cast<int>(idx.size()), src.n, src.m, src.C, src.st) != 0) return -1;
  return gather(src, idx, dst);
}

// shard refs for stripes w0.. of a stage: device j reads/writes its rebuild slot when
// slot_of[j] >= 0, else its staged chunk
std::vector<lsec_shard_t> refs(const Stage &S, int w0, const std::vector<int> &slot_of) {
  std::vector<lsec_shard_t> r(S.n);
  for (int j = 0; j < S.n; ++j)
    r[j] = slot_of[j] >= 0 ? lsec_shard_t{S.slot(w0, slot_of[j]), static_cast<long long>(S.m * S.C)}
                           : lsec_shard_t{S.chunk(w0, j), static_cast<long long>(S.n * S.C)};
  return r;
}

int stage_magic(lio_erasure_plan_t *plan, Stage &S, int w0, int cnt, const std::vector<int> &slot_of) {
  std::vector<lsec_shard_t> sh = refs(S, w0, slot_of);
  if (lsec_stripe_magic_dev(plan, sh.data(), cnt, static_cast<int>(S.C), S.dmag + static_cast<size_t>(w0) * 4, S.st) != 0)
    return -1;
  if (hipMemcpyAsync(&S.hmag[static_cast<size_t>(w0) * 4], S.dmag + static_cast<size_t>(w0) * 4, static_cast<size_t>(cnt) * 4,
                     hipMemcpyDeviceToHost, S.st) != hipSuccess)
    return -1;
  return hipStreamSynchronize(S.st) == hipSuccess ? 0 : -1;
}

// Result of jerase_control_check over a contiguous range of staged stripes sharing one bad
// set.  After a pass, device j as the reference's eptr[j] sees it is rebuild slot
// slot_of[j] (>= 0) or the staged chunk.
struct Check {
  std::vector<char> pass;
  std::vector<int> slot_of;
};

// Where a check mirrors decode_block's in-place writes for the stripes that fail it:
// stripe t of the checked range maps to stripe at[t] of *dst (-1: not mirrored).
struct InPlace {
  Stage *dst = nullptr;
  std::vector<int> at;
};

int mirror(const Stage &S, int w0, int t, const std::vector<int> &bad, const std::vector<int> &slot_of, const InPlace *ip) {
  if (!ip || ip->at[t] < 0) return 0;
  for (int b : bad)
    if (hipMemcpyAsync(ip->dst->chunk(ip->at[t], b), S.slot(w0 + t, slot_of[b]), S.C, hipMemcpyDeviceToDevice, S.st) != hipSuccess)
      return -1;
  return 0;
}

// magic: quorum magics of the range ([cnt][4]) in cksum mode, nullptr in legacy mode.
// want_magic (legacy): also leave adler32 over eptr in S.hmag (the magic a repair writes).
int control_check(lio_erasure_plan_t *plan, Stage &S, int w0, int cnt, const std::vector<int> &bad, const uint8_t *magic,
                  bool want_magic, Check &out, const InPlace *ip = nullptr) {
  const int n = S.n, m = S.m, C = static_cast<int>(S.C);
  out.pass.assign(cnt, 1);
  out.slot_of.assign(n, -1);
  if (cnt == 0) return 0;
  std::vector<char> badmap(n, 0);
  for (int b : bad) badmap[b] = 1;
  auto decode = [&](const std::vector<int> &er) -> int {
    std::fill(out.slot_of.begin(), out.slot_of.end(), -1);
    for (size_t r = 0; r < er.size(); ++r) out.slot_of[er[r]] = static_cast<int>(r);
    if (er.empty()) return 0;
    // raid4 leaves a lost parity alone (raid4.c:48).  In a check in place (the first check, the
    // carried guess: eptr[b] = ptr[b], jerasure.c:226) the reference's buffer then still holds
    // the staged chunk, so its rebuild slot starts as that chunk; in the combination search the
    // buffer is a pwork leftover (:284), which the slot's own leftover stands for.
    if (ip && plan->method == RAID4)
      for (int b : bad)
        if (b >= n - m &&
            hipMemcpy2DAsync(S.slot(w0, out.slot_of[b]), S.m * S.C, S.chunk(w0, b), S.n * S.C, S.C, cnt,
                             hipMemcpyDeviceToDevice, S.st) != hipSuccess)
          return lsec::set_error("control check: cannot stage a raid4 parity chunk");
    std::vector<int> e(er);
    e.push_back(-1);
    std::vector<lsec_shard_t> sh = refs(S, w0, out.slot_of);
    return lsec_decode_dev(plan, sh.data(), cnt, C, e.data(), S.st);
  };
  if (magic) {  // cksum magic: rebuild the bad devices (if any), then adler32 must match
    if (decode(bad) != 0 || stage_magic(plan, S, w0, cnt, out.slot_of) != 0) return -1;
    for (int t = 0; t < cnt; ++t) {
      out.pass[t] = std::memcmp(&S.hmag[static_cast<size_t>(w0 + t) * 4], magic + 4 * t, 4) == 0;
      if (!out.pass[t] && mirror(S, w0, t, bad, out.slot_of, ip) != 0) return -1;
    }
    return hipStreamSynchronize(S.st) == hipSuccess ? 0 : -1;
  }
  // legacy magic: windows of control chunks (jerasure.c:218-266); a stripe stops at its
  // first failing window, whose rebuild of the bad devices is what stays in place
  const int n_ctl_max = m - static_cast<int>(bad.size());
  int control_index = -1;
  do {
    std::vector<int> er, ctl;
    for (int i = 0; i < n; ++i)
      if ((!badmap[i] && static_cast<int>(ctl.size()) < n_ctl_max && i > control_index) || badmap[i]) {
        er.push_back(i);
        if (!badmap[i]) {
          ctl.push_back(i);
          control_index = i;
        }
      }
    if (decode(er) != 0) return -1;
    if (ctl.empty()) {
      if (n_ctl_max > 0) control_index = n - 1;  // nothing left to control: done
      else break;                               // m devices bad: nothing can be checked
      continue;
    }
    // up to m - |bad| control chunks: compared in launches of at most kMaxR pairs (the kernel
    // only sets flags, so the launches OR into one flag per stripe)
    if (hipMemsetAsync(S.dflag + w0, 0, sizeof(int) * cnt, S.st) != hipSuccess)
      return lsec::set_error("control check: hipMemsetAsync failed");
    for (size_t p0 = 0; p0 < ctl.size(); p0 += lsec::kMaxR) {
      lsec::DiffArgs da;
      std::memset(&da, 0, sizeof(da));
      da.npairs = static_cast<int>(std::min<size_t>(lsec::kMaxR, ctl.size() - p0));
      da.nstripes = cnt;
      da.size = S.C;
      da.flags = S.dflag + w0;
      for (int p = 0; p < da.npairs; ++p) {
        const int c = ctl[p0 + p];
        da.a[p] = {reinterpret_cast<uint64_t>(S.slot(w0, out.slot_of[c])), static_cast<int64_t>(m * S.C)};
        da.b[p] = {reinterpret_cast<uint64_t>(S.chunk(w0, c)), static_cast<int64_t>(n * S.C)};
      }
      if (lsec::launch_chunk_diff(da, S.st) != hipSuccess) return lsec::set_error("control check: chunk compare launch failed");
    }
    if (hipMemcpyAsync(&S.hflag[w0], S.dflag + w0, sizeof(int) * cnt, hipMemcpyDeviceToHost, S.st) != hipSuccess ||
        hipStreamSynchronize(S.st) != hipSuccess)
      return lsec::set_error("control check: flag copy failed");
    for (int t = 0; t < cnt; ++t)
      if (S.hflag[w0 + t] && out.pass[t]) {
        out.pass[t] = 0;
        if (mirror(S, w0, t, bad, out.slot_of, ip) != 0) return -1;
      }
  } while (control_index < n - 1);
  if (want_magic && stage_magic(plan, S, w0, cnt, out.slot_of) != 0) return -1;
  return hipStreamSynchronize(S.st) == hipSuccess ? 0 : -1;  // rebuild slots are read next
}

bool next_combo(std::vector<int> &c, int n) {  // lexicographic next e-subset of 0..n-1
  const int e = static_cast<int>(c.size());
  int i = e - 1;
  while (i >= 0 && c[i] == n - e + i) --i;
  if (i < 0) return false;
  ++c[i];
  for (int j = i + 1; j < e; ++j) c[j] = c[j - 1] + 1;
  return true;
}

// A passed check: the bad set it rebuilt, the rebuilt bytes of those devices, and (legacy
// mode) adler32 over the repaired stripe.  Stripes that failed their first check also keep
// `full`: every chunk as the reference's stripe buffer holds it at the end (eptr of the
// passing check, or the buffer with the in-place rebuilds of the failed checks).
struct Repair {
  bool ok = false;
  std::vector<int> bad;       // ascending
  std::vector<char> rebuilt;  // bad.size() x C, in `bad` order
  std::vector<char> full;     // n x C, or empty
  uint8_t magic[4] = {0, 0, 0, 0};
};

// Queue the device->host copies that capture a passed check for stripe w of S into rp (the
// rebuilt devices, and with `full` every chunk as eptr holds it); one d2h_pieces call then
// moves a whole batch of stripes.  rp's buffers must stay put until that call.
void capture_q(const Stage &S, int w, const Check &ck, const std::vector<int> &bad, Repair &rp, bool full,
               std::vector<lsec::DevPiece> &q) {
  rp.ok = true;
  rp.bad = bad;
  rp.rebuilt.resize(bad.size() * S.C);
  for (size_t i = 0; i < bad.size(); ++i) q.push_back({S.slot(w, ck.slot_of[bad[i]]), &rp.rebuilt[i * S.C], S.C});
  std::memcpy(rp.magic, &S.hmag[static_cast<size_t>(w) * 4], 4);
  if (full) {
    rp.full.resize(static_cast<size_t>(S.n) * S.C);
    for (int j = 0; j < S.n; ++j)
      q.push_back({ck.slot_of[j] >= 0 ? S.slot(w, ck.slot_of[j]) : S.chunk(w, j), &rp.full[static_cast<size_t>(j) * S.C], S.C});
  }
}

int capture(const Stage &S, int w, const Check &ck, const std::vector<int> &bad, Repair &rp, bool full = false) {
  std::vector<lsec::DevPiece> q;
  capture_q(S, w, ck, bad, rp, full, q);
  return lsec::d2h_pieces(q, S.st);
}

// the stripe buffer of an unresolved stripe (with the in-place rebuilds of its failed checks)
int capture_lost(const Stage &S, int w, Repair &rp) {
  rp.ok = false;
  rp.full.resize(static_cast<size_t>(S.n) * S.C);
  return hipMemcpy(rp.full.data(), S.chunk(w, 0), rp.full.size(), hipMemcpyDeviceToHost) == hipSuccess ? 0 : -1;
}

std::vector<uint8_t> flat(const std::vector<Magic> &mg, const std::vector<int> &ids) {
  std::vector<uint8_t> f(ids.size() * 4);
  for (size_t i = 0; i < ids.size(); ++i) std::memcpy(&f[i * 4], mg[ids[i]].data(), 4);
  return f;
}

// The combination search of jerase_brute_recovery (jerase_brute_recurse, :271-314) for every
// stripe of F at once: out[t] = the first passing combination in the reference's order.
int brute_enumerate(lio_erasure_plan_t *plan, Stage &F, const std::vector<Magic> &magic, bool cksum, bool want_magic,
                    std::vector<Repair> &out) {
  const int n = F.n, m = F.m, W = F.W;
  out.assign(W, Repair());
  std::vector<int> rem(W);
  for (int t = 0; t < W; ++t) rem[t] = t;
  Stage G;  // the still-unresolved stripes, once they are at most half of F
  Stage *cur = &F;
  std::vector<int> cur_ids = rem;  // F index of each stripe of *cur
  const int emax = cksum ? m : m - 1;
  for (int e = 1; e <= emax && !rem.empty(); ++e) {
    std::vector<int> combo(e);
    for (int i = 0; i < e; ++i) combo[i] = i;
    do {
      const std::vector<uint8_t> mg = flat(magic, cur_ids);
      Check ck;
      if (control_check(plan, *cur, 0, cur->W, combo, cksum ? mg.data() : nullptr, want_magic, ck) != 0) return -1;
      std::vector<int> still;
      std::vector<lsec::DevPiece> q;
      for (int i = 0; i < cur->W; ++i) {
        const int t = cur_ids[i];
        if (!std::binary_search(rem.begin(), rem.end(), t)) continue;
        if (ck.pass[i])
          capture_q(*cur, i, ck, combo, out[t], true, q);
        else
          still.push_back(t);
      }
      if (lsec::d2h_pieces(q, cur->st) != 0) return -1;
      rem.swap(still);
      if (cur == &F && !rem.empty() && rem.size() * 2 <= static_cast<size_t>(F.W)) {
        if (gather_new(F, rem, G) != 0) return -1;
        cur = &G;
        cur_ids = rem;
      }
    } while (!rem.empty() && next_combo(combo, n));
  }
  return 0;
}

struct BruteState {  // bm_brute_used / badmap_brute of one read or inspection pass
  bool used = false;
  std::vector<int> guess;
};

// jerase_brute_recovery for the stripes staged in F0 (in stripe order, already carrying the
// in-place effects of their failed first check), resolved in order with the carried guess.
int resolve_failing(lio_erasure_plan_t *plan, Stage &F0, const std::vector<Magic> &mg, bool cksum, bool want_magic,
                    BruteState &bs, std::vector<Repair> &out) {
  const int nf = F0.W;
  out.assign(nf, Repair());
  int pos = 0;
  while (pos < nf) {
    std::vector<int> rem;
    for (int t = pos; t < nf; ++t) rem.push_back(t);
    Stage T;
    if (gather_new(F0, rem, T) != 0) return -1;
    if (!bs.used) {  // no guess yet: the combination search decides, up to the first success
      std::vector<Repair> r;
      if (brute_enumerate(plan, T, std::vector<Magic>(mg.begin() + pos, mg.end()), cksum, want_magic, r) != 0) return -1;
      int s0 = 0;
      for (; s0 < T.W && !r[s0].ok; ++s0)
        if (capture_lost(T, s0, out[pos + s0]) != 0) return -1;
      if (s0 == T.W) return 0;  // every remaining stripe is unrecoverable
      out[pos + s0] = std::move(r[s0]);
      bs.used = true;
      bs.guess = out[pos + s0].bad;
      pos += s0 + 1;
      continue;
    }
    // the guess first, in place
    InPlace ip{&T, rem};
    for (int t = 0; t < T.W; ++t) ip.at[t] = t;
    const std::vector<uint8_t> tm = flat(mg, rem);
    Check ck;
    if (control_check(plan, T, 0, T.W, bs.guess, cksum ? tm.data() : nullptr, want_magic, ck, &ip) != 0) return -1;
    const std::vector<int> g = bs.guess;
    int t = 0;
    for (; t < T.W; ++t) {
      if (ck.pass[t]) {
        if (capture(T, t, ck, g, out[pos + t], true) != 0) return -1;
        continue;
      }
      // the guess failed: search this stripe (its staged chunks now hold the guess's rebuild)
      Stage one;
      std::vector<Repair> r;
      if (gather_new(T, {t}, one) != 0 || brute_enumerate(plan, one, {mg[pos + t]}, cksum, want_magic, r) != 0) return -1;
      out[pos + t] = std::move(r[0]);
      if (!out[pos + t].ok && capture_lost(T, t, out[pos + t]) != 0) return -1;
      if (out[pos + t].ok && out[pos + t].bad != g) {  // new guess: later stripes start over
        bs.guess = out[pos + t].bad;
        break;
      }
    }
    pos += std::min(t + 1, T.W);
  }
  return 0;
}

// The reference's procedure over W stripes staged in S (stripe order): first check with each
// stripe's quorum bad set, then brute force for the failures.  res[w] = 0 passed the first
// check, 1 repaired by the search, -1 unrecoverable; rp[w] holds the rebuilt devices
// (captured when the bad set is non-empty, or always when want_magic).
int verify_batch(lio_erasure_plan_t *plan, Stage &S, const std::vector<std::vector<int>> &bad, const std::vector<Magic> &mg,
                 bool cksum, bool want_magic, BruteState &bs, std::vector<int> &res, std::vector<Repair> &rp) {
  const int W = S.W;
  res.assign(W, 0);
  rp.assign(W, Repair());
  std::map<std::vector<int>, std::vector<int>> groups;
  for (int w = 0; w < W; ++w) groups[bad[w]].push_back(w);
  // A group runs over the whole stage (the other stripes' results are ignored) when that is
  // cheaper than gathering it: it is the most common bad set, it holds at least a quarter of
  // the stage, or the stage is small (<= 1 GiB: a full decode + magic pass is ~0.3 ms of HBM
  // time, less than the launches of a per-stripe gather).  Smaller groups are gathered.
  auto big = std::max_element(groups.begin(), groups.end(),
                              [](const auto &a, const auto &b) { return a.second.size() < b.second.size(); });
  const bool small_stage = static_cast<size_t>(W) * (S.n + S.m) * S.C <= (1ull << 30);
  Trace tr("verify_batch");
  tr.st = S.st;
  std::vector<char> fail(W, 0);
  for (auto it = groups.begin(); it != groups.end(); ++it) {
    Stage G;
    Stage *T = &S;
    std::vector<int> ids;  // S index of each stripe of *T
    InPlace ip{&S, {}};
    if (it == big || small_stage || it->second.size() * 4 >= static_cast<size_t>(W)) {
      for (int w = 0; w < W; ++w) {
        ids.push_back(w);
        ip.at.push_back(bad[w] == it->first ? w : -1);
      }
    } else {
      ids = it->second;
      ip.at = ids;
      if (gather_new(S, ids, G) != 0) return -1;
      T = &G;
    }
    const std::vector<uint8_t> tm = flat(mg, ids);
    Check ck;
    tr.mark("group");
    if (control_check(plan, *T, 0, static_cast<int>(ids.size()), it->first, cksum ? tm.data() : nullptr, want_magic, ck, &ip) != 0)
      return -1;
    tr.mark("check");
    std::vector<lsec::DevPiece> q;
    for (size_t i = 0; i < ids.size(); ++i) {
      const int w = ids[i];
      if (bad[w] != it->first) continue;
      if (!ck.pass[i]) fail[w] = 1;
      else if (!it->first.empty() || want_magic) capture_q(*T, static_cast<int>(i), ck, it->first, rp[w], false, q);
    }
    if (lsec::d2h_pieces(q, T->st) != 0) return -1;
    tr.mark("capture");
  }
  std::vector<int> failing;
  for (int w = 0; w < W; ++w)
    if (fail[w]) failing.push_back(w);
  if (failing.empty()) return 0;
  Stage F0;
  std::vector<Repair> r;
  std::vector<Magic> fm;
  for (int w : failing) fm.push_back(mg[w]);
  if (gather_new(S, failing, F0) != 0 || resolve_failing(plan, F0, fm, cksum, want_magic, bs, r) != 0) return -1;
  for (size_t i = 0; i < failing.size(); ++i) {
    res[failing[i]] = r[i].ok ? 1 : -1;
    rp[failing[i]] = std::move(r[i]);
  }
  return 0;
}

// majority vote over the magics of one stripe; keys[j] == nullptr = unreadable device
struct Quorum {
  Magic magic{};
  int count = 0;
  bool none = false;  // every device unreadable
  std::vector<int> members, bad;
};

Quorum vote(int n, const std::vector<const uint8_t *> &keys) {
  Quorum q;
  std::vector<const uint8_t *> gk;
  std::vector<std::vector<int>> gm;
  for (int j = 0; j < n; ++j) {
    if (!keys[j]) {  // unreadable: a group of its own that can never be the quorum's magic
      gk.push_back(nullptr);
      gm.push_back({j});
      continue;
    }
    size_t g = 0;
    for (; g < gk.size(); ++g)
      if (gk[g] && std::memcmp(gk[g], keys[j], 4) == 0) break;
    if (g == gk.size()) {
      gk.push_back(keys[j]);
      gm.push_back({});
    }
    gm[g].push_back(j);
  }
  size_t best = 0;  // first group with the largest count
  for (size_t g = 1; g < gk.size(); ++g)
    if (gm[g].size() > gm[best].size()) best = g;
  if (!gk[best]) {
    q.none = true;
    for (int j = 0; j < n; ++j) q.bad.push_back(j);
    return q;
  }
  std::memcpy(q.magic.data(), gk[best], 4);
  q.count = static_cast<int>(gm[best].size());
  q.members = gm[best];
  for (size_t g = 0; g < gk.size(); ++g)
    if (g != best) q.bad.insert(q.bad.end(), gm[g].begin(), gm[g].end());
  std::sort(q.bad.begin(), q.bad.end());
  return q;
}

bool all_zero(const char *p, size_t C) {
  for (size_t b = 0; b < C; ++b)
    if (p[b]) return false;
  return true;
}

// Keep up to two verification budgets of freed stage memory in the current device's default
// pool between calls (the default release threshold of 0 hands it back at every sync).
void keep_pool() {
  int dev = 0;
  hipMemPool_t pool = nullptr;
  if (lsec::quiet([&] {
        const hipError_t r = hipGetDevice(&dev);
        return r != hipSuccess ? r : hipDeviceGetDefaultMemPool(&pool, dev);
      }) != hipSuccess)
    return;
  uint64_t keep = 2 * verify_budget();
  (void)lsec::quiet([&] { return hipMemPoolSetAttribute(pool, hipMemPoolAttrReleaseThreshold, &keep); });
}

int stripes_per_batch(int n, int m, size_t C) {
  return static_cast<int>(std::max<size_t>(1, verify_budget() / ((static_cast<size_t>(n) + m) * C)));
}

}  // namespace

extern "C" {

// ============================================================================ read
int lsec_segment_read(lio_erasure_plan_t *plan, char **dev, int nstripes, int chunk, int n_shift, long long first_stripe,
                      int flags, char *data_out, int *status) {
  if (!plan || !dev || !data_out) return lsec::set_error("lsec_segment_read: plan, dev or data_out is NULL");
  if (nstripes < 0 || chunk <= 0 || chunk % 8 != 0 || n_shift < 0 || first_stripe < 0)
    return lsec::set_error("lsec_segment_read: bad geometry (nstripes=%d chunk=%d n_shift=%d first_stripe=%lld)", nstripes,
                           chunk, n_shift, first_stripe);
  const int k = plan->data_strips, m = plan->parity_strips, n = k + m;
  if (k < 1 || m < 1 || n > LSEC_MAX_DEVS) return lsec::set_error("lsec_segment_read: k+m=%d outside 2..%d", n, LSEC_MAX_DEVS);
  const size_t C = static_cast<size_t>(chunk), lchunk = C + 4;
  const bool paranoid = flags & LSEC_READ_PARANOID, cksum = !(flags & LSEC_MAGIC_LEGACY);
  if (nstripes == 0) return 0;
  Trace tr("read");
  // logical chunk j of stripe s lives on device (j - ss*n_shift) mod n  (lun.c:1178-1223)
  auto phys = [&](long long ss, int j) { return static_cast<int>(((j - ss * n_shift) % n + n) % n); };
  auto rec = [&](int s, int j) -> const char * {  // [magic | chunk] record, nullptr if unreadable
    const int d = phys(first_stripe + s, j);
    return dev[d] ? dev[d] + static_cast<size_t>(s) * lchunk : nullptr;
  };

  // ---- 1. quorum and the reference's data_ok classification, per stripe (host)
  enum { kOk = 0, kRecovered = 1, kBlank = 2, kLost = -1 };
  std::vector<int> st(nstripes, kOk);
  std::vector<Quorum> q(nstripes);
  std::vector<int> work;
  for (int s = 0; s < nstripes; ++s) {
    std::vector<const uint8_t *> keys(n);
    for (int j = 0; j < n; ++j) keys[j] = reinterpret_cast<const uint8_t *>(rec(s, j));
    q[s] = vote(n, keys);
    if (q[s].none) {
      st[s] = kLost;
      continue;
    }
    int data_ok = 1;
    if (q[s].count != n) {
      int nd = 0;
      for (int j : q[s].members) nd += j < k;
      if (nd != k) data_ok = 0;
    } else if (std::memcmp(kZeroMagic, q[s].magic.data(), 4) == 0) {
      bool nonzero = false;
      for (int j = 0; j < n && !nonzero; ++j) nonzero = !all_zero(rec(s, j) + 4, C);
      data_ok = nonzero ? 1 : 2;
    }
    if (data_ok == 1) {  // every data device in the quorum: verified in paranoid mode only (:1440-1442),
                         // also when a parity device is unreadable
      if (paranoid) work.push_back(s);
    } else if (data_ok == 2) {
      st[s] = kBlank;
    } else if (q[s].count < k) {
      st[s] = kLost;
    } else {
      work.push_back(s);
    }
  }

  // ---- 2. verification / repair on the GPU, in stripe order, budget-sized batches
  tr.mark("classify");
  std::vector<Repair> repair(nstripes);
  hipStream_t stream = nullptr;
  if (!work.empty()) keep_pool();
  if (!work.empty() && hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess)
    return lsec::set_error("lsec_segment_read: cannot create a HIP stream");
  tr.st = stream;
  BruteState bs;
  int rc = 0;
  const int wmax = stripes_per_batch(n, m, C);
  for (size_t b0 = 0; b0 < work.size() && rc == 0; b0 += wmax) {
    const int W = static_cast<int>(std::min<size_t>(wmax, work.size() - b0));
    Stage S;
    if (S.alloc(W, n, m, C, stream) != 0) {
      rc = lsec::set_error("lsec_segment_read: cannot allocate a %d-stripe stage in HBM", W);
      break;
    }
    std::vector<std::vector<int>> bad(W);
    std::vector<Magic> mg(W);
    std::vector<lsec::DevPiece> pieces;  // chunks in staging order; unreadable devices stage zeros
    pieces.reserve(static_cast<size_t>(W) * n);
    for (int w = 0; w < W; ++w) {
      const int s = work[b0 + w];
      bad[w] = q[s].bad;
      mg[w] = q[s].magic;
      for (int j = 0; j < n; ++j) {
        const char *p = rec(s, j);
        pieces.push_back({S.chunk(w, j), p ? const_cast<char *>(p) + 4 : nullptr, C});
      }
    }
    if (lsec::h2d_pieces(pieces, stream) != 0) rc = -1;
    tr.mark("stage");
    std::vector<int> res;
    std::vector<Repair> rp;
    if (rc || verify_batch(plan, S, bad, mg, cksum, false, bs, res, rp) != 0) { rc = -1; break; }
    tr.mark("verify");
    for (int w = 0; w < W; ++w) {
      const int s = work[b0 + w];
      if (res[w] < 0) st[s] = kLost;
      else if (!rp[w].bad.empty() && rp[w].bad.front() < k) st[s] = kRecovered;  // user data was rebuilt
      repair[s] = std::move(rp[w]);
    }
  }
  tr.st = nullptr;
  if (stream) (void)hipStreamDestroy(stream);
  if (rc) return -1;

  // ---- 3. user data out: originals, with rebuilt data devices swapped in
  int unrecoverable = 0;
  std::vector<lsec::HostCopy> jobs;
  for (int s = 0; s < nstripes; ++s) {
    if (status) status[s] = st[s];
    char *out = data_out + static_cast<size_t>(s) * k * C;
    if (st[s] == kBlank) {
      std::memset(out, 0, static_cast<size_t>(k) * C);
      continue;
    }
    if (st[s] == kLost) {
      ++unrecoverable;
      continue;
    }
    const Repair &rp = repair[s];
    for (int j = 0; j < k; ++j) {
      const auto it = std::find(rp.bad.begin(), rp.bad.end(), j);
      const char *src = !rp.full.empty()    ? &rp.full[static_cast<size_t>(j) * C]
                        : it != rp.bad.end() ? &rp.rebuilt[static_cast<size_t>(it - rp.bad.begin()) * C]
                                             : rec(s, j) + 4;
      jobs.push_back({out + static_cast<size_t>(j) * C, src, C});
    }
  }
  lsec::parallel_copy(jobs);
  tr.mark("copyout");
  return unrecoverable;
}

// ============================================================================ inspect
int lsec_segment_inspect(lio_erasure_plan_t *plan, char *buf, int nstripes, int chunk, int flags, int *stripe_status,
                         unsigned char *badmap, unsigned char *rewrite, lsec_inspect_state_t *state) {
  if (!plan || !buf || !state) return lsec::set_error("lsec_segment_inspect: plan, buf or state is NULL");
  if (nstripes < 0 || chunk <= 0 || chunk % 8 != 0)
    return lsec::set_error("lsec_segment_inspect: bad geometry (nstripes=%d chunk=%d)", nstripes, chunk);
  const int k = plan->data_strips, m = plan->parity_strips, n = k + m;
  if (k < 1 || m < 1 || n > LSEC_MAX_DEVS) return lsec::set_error("lsec_segment_inspect: k+m=%d outside 2..%d", n, LSEC_MAX_DEVS);
  const size_t C = static_cast<size_t>(chunk), lchunk = C + 4;
  const bool do_fix = flags & LSEC_INSPECT_FIX, cksum = !(flags & LSEC_MAGIC_LEGACY);
  if (nstripes == 0) return 0;
  auto rec = [&](int s, int j) { return buf + (static_cast<size_t>(s) * n + j) * lchunk; };

  // ---- 1. host classification (segment/jerasure.c:474-560)
  std::vector<int> st(nstripes, LSEC_STRIPE_OK);
  std::vector<Quorum> q(nstripes);
  std::vector<int> work;  // stripes that go through jerase_control_check
  for (int s = 0; s < nstripes; ++s) {
    std::vector<const uint8_t *> keys(n);
    for (int j = 0; j < n; ++j) keys[j] = reinterpret_cast<const uint8_t *>(rec(s, j));
    q[s] = vote(n, keys);
    bool good_magic = std::memcmp(kZeroMagic, q[s].magic.data(), 4) != 0;
    if (!good_magic) {
      bool nonzero = false;
      for (int j = 0; j < n && !nonzero; ++j) nonzero = !all_zero(rec(s, j) + 4, C);
      if (nonzero) {
        good_magic = true;
      } else if (q[s].count == n) {  // completely empty stripe: skipped
        st[s] = LSEC_STRIPE_EMPTY;
        continue;
      }
    }
    if ((!good_magic && q[s].count != n) || q[s].count < k) {
      st[s] = LSEC_STRIPE_LOST_MAGIC;
      continue;
    }
    work.push_back(s);
  }

  // ---- 2. GPU: control check of every remaining stripe, brute force for the failures
  BruteState bs;
  bs.used = state->brute_used != 0;
  for (int j = 0; j < n; ++j)
    if (state->brute_badmap[j]) bs.guess.push_back(j);
  std::vector<Repair> fix(nstripes);
  std::vector<std::vector<int>> final_bad(nstripes);
  for (int s = 0; s < nstripes; ++s) final_bad[s] = q[s].bad;
  hipStream_t stream = nullptr;
  if (!work.empty()) keep_pool();
  if (!work.empty() && hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess)
    return lsec::set_error("lsec_segment_inspect: cannot create a HIP stream");
  const int wmax = stripes_per_batch(n, m, C);
  int rc = 0;
  for (size_t b0 = 0; b0 < work.size() && rc == 0; b0 += wmax) {
    const int W = static_cast<int>(std::min<size_t>(wmax, work.size() - b0));
    Stage S;
    if (S.alloc(W, n, m, C, stream) != 0) {
      rc = lsec::set_error("lsec_segment_inspect: cannot allocate a %d-stripe stage in HBM", W);
      break;
    }
    // stage the chunks ([magic | chunk] records -> chunks), packed into large DMAs
    std::vector<lsec::DevPiece> pieces;
    pieces.reserve(static_cast<size_t>(W) * n);
    for (int w = 0; w < W; ++w)
      for (int j = 0; j < n; ++j) pieces.push_back({S.chunk(w, j), rec(work[b0 + w], j) + 4, C});
    if (lsec::h2d_pieces(pieces, stream) != 0) rc = -1;
    std::vector<std::vector<int>> bad(W);
    std::vector<Magic> mg(W);
    for (int w = 0; w < W; ++w) {
      bad[w] = q[work[b0 + w]].bad;
      mg[w] = q[work[b0 + w]].magic;
    }
    std::vector<int> res;
    std::vector<Repair> rp;
    if (rc || verify_batch(plan, S, bad, mg, cksum, !cksum, bs, res, rp) != 0) { rc = -1; break; }
    for (int w = 0; w < W; ++w) {
      const int s = work[b0 + w];
      if (res[w] == 0) {
        st[s] = q[s].count != n ? LSEC_STRIPE_BAD_MAGIC : LSEC_STRIPE_OK;
      } else if (res[w] > 0) {
        st[s] = LSEC_STRIPE_REPAIRED;
        final_bad[s] = rp[w].bad;
      } else {
        st[s] = LSEC_STRIPE_LOST_MISMATCH;
        // the search leaves the last combination it tried in badmap (jerase_brute_recurse, :283-289)
        const int emax = cksum ? m : m - 1;
        final_bad[s].clear();
        for (int j = n - emax; j < n && emax > 0; ++j) final_bad[s].push_back(j);
      }
      fix[s] = std::move(rp[w]);
    }
  }
  if (stream) (void)hipStreamDestroy(stream);
  if (rc) return -1;
  state->brute_used = bs.used;
  std::memset(state->brute_badmap, 0, sizeof(state->brute_badmap));
  for (int j : bs.guess) state->brute_badmap[j] = 1;

  // ---- 3. report and, with do_fix, repair the buffer in place (:614-640)
  for (int s = 0; s < nstripes; ++s) {
    const int x = st[s];
    if (stripe_status) stripe_status[s] = x;
    if (badmap) {
      std::memset(badmap + static_cast<size_t>(s) * n, 0, n);
      for (int j : final_bad[s]) badmap[static_cast<size_t>(s) * n + j] = 1;
    }
    if (rewrite) std::memset(rewrite + static_cast<size_t>(s) * n, (do_fix && !cksum) ? 1 : 0, n);
    if (x == LSEC_STRIPE_EMPTY) ++state->empty_stripes;
    if (x == LSEC_STRIPE_REPAIRED || x == LSEC_STRIPE_LOST_MISMATCH) ++state->silent_errors;
    if (x == LSEC_STRIPE_LOST_MAGIC || x == LSEC_STRIPE_LOST_MISMATCH) ++state->unrecoverable;
    if (x != LSEC_STRIPE_OK && x != LSEC_STRIPE_EMPTY) ++state->bad_stripes;
    const bool skip = x == LSEC_STRIPE_EMPTY || x == LSEC_STRIPE_LOST_MAGIC || x == LSEC_STRIPE_LOST_MISMATCH ||
                      (x == LSEC_STRIPE_OK && cksum);
    const Repair &rp = fix[s];
    if (do_fix && !cksum && x == LSEC_STRIPE_LOST_MISMATCH) {
      // the whole range is written back (:464-470), including the failed checks' in-place rebuilds
      for (int j = 0; j < n; ++j) std::memcpy(rec(s, j) + 4, &rp.full[static_cast<size_t>(j) * C], C);
    }
    if (!do_fix || skip) continue;
    const uint8_t *magic = cksum ? q[s].magic.data() : rp.magic;  // legacy: adler32 of the repaired stripe
    std::vector<char> isbad(n, 0);
    for (int j : final_bad[s]) isbad[j] = 1;
    for (int j = 0; j < n; ++j) {
      if (!isbad[j] && cksum) continue;
      char *r = rec(s, j);
      std::memcpy(r, magic, 4);
      const auto it = std::find(rp.bad.begin(), rp.bad.end(), j);
      if (!rp.full.empty()) std::memcpy(r + 4, &rp.full[static_cast<size_t>(j) * C], C);
      else if (it != rp.bad.end()) std::memcpy(r + 4, &rp.rebuilt[static_cast<size_t>(it - rp.bad.begin()) * C], C);
      if (rewrite) rewrite[static_cast<size_t>(s) * n + j] = 1;
    }
  }
  return 0;
}

}  // extern "C"
