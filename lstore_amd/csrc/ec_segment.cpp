// ec_segment.cpp -- batched adapter for LStore's erasure segment write path.
//
// segjerase_write_func (src/lio/segment/jerasure.c:1640-1895) does, per stripe of a
// whole-stripe-aligned write: point ptr[0..k) into the user page, ptr[k..k+m) into the parity
// buffer, encode_block (:1847), je_cksum_calc over the k+m chunks (:1850), and hand the LUN
// child 2(k+m) iovecs [magic | chunk] (:1826-1844).  The LUN child places logical chunk j of
// stripe s on physical device i = the one with (i + s*n_shift) % (k+m) == j, at device offset
// s*(C+4) (lun_row_decompose, lun.c:1140-1246).
//
// lsec_segment_write does the same for N stripes in one call: parity and magics are
// computed on the GPU (one staging pipeline for the whole batch, parity DMA'd straight into
// the device images), then the data chunks and magics are laid into the images on the host
// copy pool.  The images are byte-identical to what the reference path writes
// (tests/test_segment.py).
#include <cstring>
#include <vector>

#include "../../include/lstore_ec.h"
#include "ec_host.h"

extern "C" {

int lsec_segment_write(lio_erasure_plan_t *plan, const char *data, int nstripes, int chunk, int n_shift,
                       long long first_stripe, char **dev) {
  if (!plan || !data || !dev || nstripes < 0 || chunk <= 0 || n_shift < 0 || first_stripe < 0) return -1;
  const int k = plan->data_strips, m = plan->parity_strips, n = k + m;
  const size_t C = static_cast<size_t>(chunk), lchunk = C + 4;
  if (nstripes == 0) return 0;
  // ptr[] as segjerase_write_func builds it; parity slots point straight into the images
  std::vector<char *> ptrs(static_cast<size_t>(nstripes) * n);
  std::vector<int> phys_of(static_cast<size_t>(n));
  for (int s = 0; s < nstripes; ++s) {
    const long long ss = first_stripe + s;
    for (int i = 0; i < n; ++i) phys_of[(i + ss * n_shift) % n] = i;  // logical chunk -> device
    for (int j = 0; j < k; ++j)
      ptrs[static_cast<size_t>(s) * n + j] = const_cast<char *>(data) + (static_cast<size_t>(s) * k + j) * C;
    for (int r = 0; r < m; ++r)
      ptrs[static_cast<size_t>(s) * n + k + r] = dev[phys_of[k + r]] + static_cast<size_t>(s) * lchunk + 4;
  }
  std::vector<char> magic(static_cast<size_t>(nstripes) * 4);
  if (et_encode_stripes_magic(plan, ptrs.data(), nstripes, chunk, magic.data()) != 0) return -1;
  // data chunks and every chunk's magic into the images
  std::vector<lsec::HostCopy> jobs;
  jobs.reserve(static_cast<size_t>(nstripes) * k);
  for (int s = 0; s < nstripes; ++s) {
    const long long ss = first_stripe + s;
    for (int i = 0; i < n; ++i) {
      char *slot = dev[i] + static_cast<size_t>(s) * lchunk;
      std::memcpy(slot, &magic[static_cast<size_t>(s) * 4], 4);
      const int j = static_cast<int>((i + ss * n_shift) % n);
      if (j < k) jobs.push_back({slot + 4, ptrs[static_cast<size_t>(s) * n + j], C});
    }
  }
  lsec::parallel_copy(jobs);
  return 0;
}

}  // extern "C"

// ============================================================================ read side
// lsec_segment_read: segjerase_read_func (segment/jerasure.c:1255-1631) for whole stripes,
// with the verification / repair of SURVEY.md §8f row 3 done in GPU batches:
//   1. majority vote over the k+m stored magics per stripe (:1383-1438), host side
//   2. paranoid stripes (and every stripe that must be repaired) are checked against the
//      quorum magic with the GPU adler32 kernel (je_cksum_compare, :188-194)
//   3. stripes with bad / missing chunks are rebuilt with one decode launch per distinct
//      bad-device pattern (jerase_control_check, :202-269) and re-checked
//   4. stripes that still fail go to the brute-force search (jerase_brute_recovery,
//      :321-339): every erasure combination of 1..m devices in the reference's order, each
//      combination one decode + one magic launch over all still-failing stripes; a stripe is
//      resolved by the first combination whose rebuild matches its magic.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <map>

namespace {

struct StripeInfo {
  uint8_t magic[4];      // quorum magic
  std::vector<int> bad;  // devices outside the quorum (or unreadable)
  int status = 0;        // 0 ok, 1 recovered, 2 blank, -1 unrecoverable
  bool check = false;    // needs a checksum verification on the GPU
  bool repair = false;   // needs a rebuild
};

bool next_combo(std::vector<int> &c, int n) {  // lexicographic next e-subset of 0..n-1
  const int e = static_cast<int>(c.size());
  int i = e - 1;
  while (i >= 0 && c[i] == n - e + i) --i;
  if (i < 0) return false;
  ++c[i];
  for (int j = i + 1; j < e; ++j) c[j] = c[j - 1] + 1;
  return true;
}

}  // namespace

extern "C" int lsec_segment_read(lio_erasure_plan_t *plan, char **dev, int nstripes, int chunk, int n_shift,
                                 long long first_stripe, int paranoid, char *data_out, int *status) {
  if (!plan || !dev || !data_out || nstripes < 0 || chunk <= 0 || n_shift < 0 || first_stripe < 0) return -1;
  const int k = plan->data_strips, m = plan->parity_strips, n = k + m;
  const size_t C = static_cast<size_t>(chunk), lchunk = C + 4;
  if (nstripes == 0) return 0;
  static const uint8_t kEmpty[4] = {0, 0, 0, 0};
  // logical chunk j of stripe s lives on device (j - ss*n_shift) mod n  (lun.c:1178-1223)
  auto phys = [&](long long ss, int j) { return static_cast<int>(((j - ss * n_shift) % n + n) % n); };
  auto chunk_ptr = [&](int s, int j) -> const char * {
    const int d = phys(first_stripe + s, j);
    return dev[d] ? dev[d] + static_cast<size_t>(s) * lchunk : nullptr;
  };

  // ---- 1. quorum, per stripe (host)
  std::vector<StripeInfo> st(nstripes);
  for (int s = 0; s < nstripes; ++s) {
    StripeInfo &si = st[s];
    std::vector<const uint8_t *> keys;
    std::vector<std::vector<int>> members;
    bool read_error = false;
    for (int j = 0; j < n; ++j) {
      const char *p = chunk_ptr(s, j);
      if (!p) {  // unreadable device: never part of a quorum, forces paranoid handling
        read_error = true;
        keys.push_back(nullptr);
        members.push_back({j});
        continue;
      }
      bool found = false;
      for (size_t g = 0; g < keys.size(); ++g)
        if (keys[g] && std::memcmp(keys[g], p, 4) == 0) {
          members[g].push_back(j);
          found = true;
          break;
        }
      if (!found) {
        keys.push_back(reinterpret_cast<const uint8_t *>(p));
        members.push_back({j});
      }
    }
    size_t best = 0;  // first group with the largest count (ties keep the earlier group)
    for (size_t g = 1; g < keys.size(); ++g)
      if (members[g].size() > members[best].size()) best = g;
    if (!keys[best]) {  // only unreadable devices
      si.status = -1;
      continue;
    }
    std::memcpy(si.magic, keys[best], 4);
    const int count = static_cast<int>(members[best].size());
    for (size_t g = 0; g < keys.size(); ++g)
      if (g != best) si.bad.insert(si.bad.end(), members[g].begin(), members[g].end());
    std::sort(si.bad.begin(), si.bad.end());
    int data_ok = 1;
    if (count != n) {
      int nd = 0;
      for (int j : members[best]) nd += j < k;
      if (nd != k) data_ok = 0;
    } else if (std::memcmp(kEmpty, si.magic, 4) == 0) {
      bool nonzero = false;
      for (int j = 0; j < n && !nonzero; ++j) {
        const char *p = chunk_ptr(s, j) + 4;
        for (size_t b = 0; b < C; ++b)
          if (p[b]) { nonzero = true; break; }
      }
      data_ok = nonzero ? 1 : 2;
    }
    const bool para = paranoid || read_error;
    if (data_ok == 1) {
      si.check = para;
    } else if (data_ok == 2) {
      si.status = 2;
    } else if (count < k) {
      si.status = -1;
    } else {
      si.repair = true;
    }
  }

  // ---- device work, in batches of stripes that need it
  std::vector<int> work;
  for (int s = 0; s < nstripes; ++s)
    if (st[s].check || st[s].repair) work.push_back(s);
  hipStream_t stream = nullptr;
  char *dbuf = nullptr, *dwork = nullptr;
  uint8_t *dmag = nullptr;
  std::vector<uint8_t> hmag;
  int rc = 0;
  std::vector<char> rebuilt;  // host copy of rebuilt data chunks: [work][k][C]
  std::map<int, size_t> rebuilt_at;
  if (!work.empty()) {
    const size_t W = work.size();
    if (hipStreamCreateWithFlags(&stream, hipStreamNonBlocking) != hipSuccess) return -1;
    if (hipMalloc(&dbuf, W * n * C) != hipSuccess || hipMalloc(&dwork, W * n * C) != hipSuccess ||
        hipMalloc(&dmag, W * 4) != hipSuccess) {
      rc = -1;
    }
    hmag.resize(W * 4);
    // stage every chunk of the work stripes, logical order [w][n][C]
    for (size_t w = 0; w < W && rc == 0; ++w)
      for (int j = 0; j < n; ++j) {
        const char *p = chunk_ptr(work[w], j);
        char *dst = dbuf + (w * n + j) * C;
        if (p) {
          if (hipMemcpyAsync(dst, p + 4, C, hipMemcpyHostToDevice, stream) != hipSuccess) rc = -1;
        } else if (hipMemsetAsync(dst, 0, C, stream) != hipSuccess) {
          rc = -1;
        }
      }
    auto refs = [&](char *base, std::vector<lsec_shard_t> &sh) {
      sh.resize(n);
      for (int j = 0; j < n; ++j) sh[j] = {base + static_cast<size_t>(j) * C, static_cast<long long>(n * C)};
    };
    // run `erasures` over the listed work stripes (indices into work), copy of the originals in
    // dwork, then magic -> returns the subset whose rebuild matches the stripe's quorum magic
    auto try_pattern = [&](const std::vector<size_t> &idx, const std::vector<int> &erasures,
                           std::vector<size_t> &ok) -> int {
      ok.clear();
      if (idx.empty()) return 0;
      for (size_t t = 0; t < idx.size(); ++t)
        if (hipMemcpyAsync(dwork + t * n * C, dbuf + idx[t] * n * C, n * C, hipMemcpyDeviceToDevice, stream) != hipSuccess)
          return -1;
      std::vector<lsec_shard_t> sh;
      refs(dwork, sh);
      if (!erasures.empty()) {
        std::vector<int> er(erasures);
        er.push_back(-1);
        if (lsec_decode_dev(plan, sh.data(), static_cast<int>(idx.size()), chunk, er.data(), stream) != 0) return -1;
      }
      if (lsec_stripe_magic_dev(plan, sh.data(), static_cast<int>(idx.size()), chunk, dmag, stream) != 0) return -1;
      if (hipMemcpyAsync(hmag.data(), dmag, idx.size() * 4, hipMemcpyDeviceToHost, stream) != hipSuccess) return -1;
      if (hipStreamSynchronize(stream) != hipSuccess) return -1;
      for (size_t t = 0; t < idx.size(); ++t) {
        if (std::memcmp(&hmag[t * 4], st[work[idx[t]]].magic, 4) != 0) continue;
        ok.push_back(idx[t]);
        if (!erasures.empty()) {  // keep the rebuilt data chunks
          const size_t at = rebuilt.size();
          rebuilt.resize(at + static_cast<size_t>(k) * C);
          if (hipMemcpy(&rebuilt[at], dwork + t * n * C, static_cast<size_t>(k) * C, hipMemcpyDeviceToHost) != hipSuccess)
            return -1;
          rebuilt_at[work[idx[t]]] = at;
        }
      }
      return 0;
    };
    // 2 + 3: plain checks, and rebuilds grouped by bad-device pattern (jerase_control_check)
    std::map<std::vector<int>, std::vector<size_t>> groups;
    for (size_t w = 0; w < W; ++w) groups[st[work[w]].repair ? st[work[w]].bad : std::vector<int>()].push_back(w);
    std::vector<size_t> failing;
    for (auto &g : groups) {
      if (rc) break;
      std::vector<size_t> ok;
      if (try_pattern(g.second, g.first, ok) != 0) { rc = -1; break; }
      std::vector<char> good(W, 0);
      for (size_t w : ok) {
        good[w] = 1;
        st[work[w]].status = g.first.empty() ? 0 : 1;
      }
      for (size_t w : g.second)
        if (!good[w]) failing.push_back(w);
    }
    // 4: brute force over erasure combinations of 1..m devices (jerase_brute_recovery)
    std::sort(failing.begin(), failing.end());
    for (int e = 1; e <= m && !failing.empty() && rc == 0; ++e) {
      std::vector<int> combo(e);
      for (int i = 0; i < e; ++i) combo[i] = i;
      do {
        std::vector<size_t> ok;
        if (try_pattern(failing, combo, ok) != 0) { rc = -1; break; }
        for (size_t w : ok) st[work[w]].status = 1;
        std::vector<size_t> rest;
        std::set_difference(failing.begin(), failing.end(), ok.begin(), ok.end(), std::back_inserter(rest));
        failing.swap(rest);
      } while (!failing.empty() && next_combo(combo, n));
    }
    for (size_t w : failing) st[work[w]].status = -1;
  }
  if (dbuf) (void)hipFree(dbuf);
  if (dwork) (void)hipFree(dwork);
  if (dmag) (void)hipFree(dmag);
  if (stream) (void)hipStreamDestroy(stream);
  if (rc) return -1;

  // ---- user data out
  int unrecoverable = 0;
  std::vector<lsec::HostCopy> jobs;
  for (int s = 0; s < nstripes; ++s) {
    if (status) status[s] = st[s].status;
    char *out = data_out + static_cast<size_t>(s) * k * C;
    if (st[s].status == 2) {
      std::memset(out, 0, static_cast<size_t>(k) * C);
      continue;
    }
    if (st[s].status < 0) {
      ++unrecoverable;
      continue;
    }
    auto it = rebuilt_at.find(s);
    for (int j = 0; j < k; ++j) {
      const char *src = it != rebuilt_at.end() ? &rebuilt[it->second + static_cast<size_t>(j) * C] : chunk_ptr(s, j) + 4;
      jobs.push_back({out + static_cast<size_t>(j) * C, src, C});
    }
  }
  lsec::parallel_copy(jobs);
  return unrecoverable;
}
