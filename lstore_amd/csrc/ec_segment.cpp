// ec_segment.cpp -- batched adapter for LStore's erasure segment write path.
//
// segjerase_write_func (src/lio/segment/jerasure.c:1640-1895) does, per stripe of a
// whole-stripe-aligned write: point ptr[0..k) into the user page, ptr[k..k+m) into the parity
// buffer, encode_block (:1847), je_cksum_calc over the k+m chunks (:1850), and hand the LUN
// child 2(k+m) iovecs [magic | chunk] (:1826-1844).  The LUN child places logical chunk j of
// stripe s on physical device i = the one with (i + s*n_shift) % (k+m) == j, at device offset
// s*(C+4) (lun_row_decompose, lun.c:1140-1246).
//
// lsec_segment_write does the same for N stripes in one call (lsec_segment_write_iov from a
// scatter list with straddling stripes and error pages, as the cache hands pages over): parity and magics are
// computed on the GPU (one staging pipeline for the whole batch, parity DMA'd straight into
// the device images), then the data chunks and magics are laid into the images on the host
// copy pool.  The images are byte-identical to what the reference path writes
// (tests/test_segment.py).
#include <sys/uio.h>

#include <algorithm>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/lstore_ec.h"
#include "ec_host.h"

namespace {

// Engine-owned parity buffers of the image form, reused across calls: a fresh 100+ MiB
// allocation per call would pay the kernel's zeroing of every page it faults in.  At most
// kKeep are kept; a call that finds none large enough allocates (and may keep) its own.
class ParityPool {
 public:
  struct Buf {
    char *p = nullptr;
    size_t cap = 0;
  };
  static ParityPool &get() {
    static ParityPool *pool = new ParityPool();  // leaked: lives until exit
    return *pool;
  }
  // the smallest kept buffer that fits (a small call must not take a big one from the next big call)
  Buf acquire(size_t bytes) {
    std::lock_guard<std::mutex> lk(mu_);
    size_t best = free_.size();
    for (size_t i = 0; i < free_.size(); ++i)
      if (free_[i].cap >= bytes && (best == free_.size() || free_[i].cap < free_[best].cap)) best = i;
    if (best < free_.size()) {
      Buf b = free_[best];
      kept_ -= b.cap;
      free_.erase(free_.begin() + static_cast<long>(best));
      return b;
    }
    Buf b;
    b.p = static_cast<char *>(malloc(bytes));
    b.cap = b.p ? bytes : 0;
    return b;
  }
  // keep at most kKeep buffers and kKeepBytes in total, the smallest first (one large segment
  // write does not pin its parity heap for the life of the process)
  void release(Buf b) {
    std::lock_guard<std::mutex> lk(mu_);
    if (b.cap > kKeepBytes) {
      free(b.p);
      return;
    }
    free_.push_back(b);
    kept_ += b.cap;
    std::sort(free_.begin(), free_.end(), [](const Buf &x, const Buf &y) { return x.cap < y.cap; });
    while (free_.size() > kKeep || kept_ > kKeepBytes) {
      kept_ -= free_.back().cap;
      free(free_.back().p);
      free_.pop_back();
    }
  }

 private:
  static constexpr size_t kKeep = 4;
  static constexpr size_t kKeepBytes = 256u << 20;
  std::mutex mu_;
  size_t kept_ = 0;
  std::vector<Buf> free_;
};

// A chunk of zeros for stripes that start in an error page (segjerase_write_func points them at
// a zeroed `empty` chunk, segment/jerasure.c:1816-1822).  One per chunk size, never freed: the
// iovec form hands out pointers to it.
const char *zero_chunk(size_t C) {
  static std::mutex mu;
  static auto *chunks = new std::map<size_t, char *>();  // leaked with the chunks
  std::lock_guard<std::mutex> lk(mu);
  char *&z = (*chunks)[C];
  if (!z) z = static_cast<char *>(calloc(C, 1));
  return z;
}

// Data chunk pointers of a scatter list (segjerase_write_func, segment/jerasure.c:1786-1831):
// stripe s covers bytes [s*k*C, (s+1)*k*C) of the concatenated pieces.  A stripe inside one
// piece is used in place; a stripe straddling pieces is gathered into `straddle` (k*C bytes
// per straddling stripe, in stripe order; error pages inside it read as zeros); a stripe whose
// first piece is an error page (iov_base NULL) gets zero chunks.  straddle == nullptr only
// counts: *straddles = the number of straddling stripes.  0 / -1.
int resolve_data(const char *fn, int k, const struct iovec *iov, int n_iov, int nstripes, size_t C, char *straddle,
                 size_t straddle_bytes, std::vector<char *> *dp, size_t *straddles) {
  const size_t dsize = static_cast<size_t>(k) * C;
  if (n_iov < 0) return lsec::set_error("%s: n_iov=%d", fn, n_iov);
  std::vector<size_t> piece_start(static_cast<size_t>(n_iov) + 1, 0);
  for (int i = 0; i < n_iov; ++i) piece_start[i + 1] = piece_start[i] + iov[i].iov_len;
  if (piece_start[n_iov] < dsize * static_cast<size_t>(nstripes))
    return lsec::set_error("%s: %zu bytes in the scatter list for %d stripes of %zu", fn, piece_start[n_iov], nstripes,
                           dsize);
  std::vector<int> first_piece(static_cast<size_t>(nstripes));
  size_t nstraddle = 0;
  int pi = 0;
  for (int s = 0; s < nstripes; ++s) {
    const size_t off = static_cast<size_t>(s) * dsize;
    while (piece_start[pi + 1] <= off) ++pi;
    first_piece[s] = pi;
    if (iov[pi].iov_base && piece_start[pi + 1] < off + dsize) ++nstraddle;
  }
  if (straddles) *straddles = nstraddle;
  if (!dp) return 0;
  if (nstraddle * dsize > straddle_bytes)
    return lsec::set_error("%s: %zu straddling stripes need %zu bytes of straddle buffer, %zu given", fn, nstraddle,
                           nstraddle * dsize, straddle_bytes);
  dp->assign(static_cast<size_t>(nstripes) * k, nullptr);
  const char *zero = zero_chunk(C);
  if (!zero) return lsec::set_error("%s: cannot allocate a zero chunk", fn);
  size_t used = 0;
  for (int s = 0; s < nstripes; ++s) {
    const size_t off = static_cast<size_t>(s) * dsize;
    const int p0 = first_piece[s];
    char *base;
    if (!iov[p0].iov_base) {
      for (int j = 0; j < k; ++j) (*dp)[static_cast<size_t>(s) * k + j] = const_cast<char *>(zero);
      continue;
    }
    if (piece_start[p0 + 1] >= off + dsize) {
      base = static_cast<char *>(iov[p0].iov_base) + (off - piece_start[p0]);
    } else {
      base = straddle + used;
      used += dsize;
      size_t got = 0;
      for (int q = p0; got < dsize; ++q) {
        const size_t from = off + got - piece_start[q];
        const size_t take = std::min(iov[q].iov_len - from, dsize - got);
        if (iov[q].iov_base) std::memcpy(base + got, static_cast<const char *>(iov[q].iov_base) + from, take);
        else std::memset(base + got, 0, take);  // an error page inside a straddling stripe: zeros
        got += take;
      }
    }
    for (int j = 0; j < k; ++j) (*dp)[static_cast<size_t>(s) * k + j] = base + static_cast<size_t>(j) * C;
  }
  return 0;
}

// ptr[] as segjerase_write_func builds it (:1812-1836): data chunk j of stripe s at
// data_ptrs[s*k + j], parity chunk r at parity + (s*m + r)*C (the per-op parity buffer,
// parity_used advancing by C per parity chunk, :1836-1843)
std::vector<char *> stripe_ptrs(int k, int m, char *const *data_ptrs, int nstripes, char *parity, size_t C) {
  const int n = k + m;
  std::vector<char *> ptrs(static_cast<size_t>(nstripes) * n);
  for (int s = 0; s < nstripes; ++s) {
    for (int j = 0; j < k; ++j) ptrs[static_cast<size_t>(s) * n + j] = data_ptrs[static_cast<size_t>(s) * k + j];
    for (int r = 0; r < m; ++r) ptrs[static_cast<size_t>(s) * n + k + r] = parity + (static_cast<size_t>(s) * m + r) * C;
  }
  return ptrs;
}

// The image form's shared body: data chunk j of stripe s at data_ptrs[s*k + j] (any host memory;
// chunks may alias, e.g. the zero chunk of an error page).
//   1. parity and magics on the GPU, the parity into one contiguous engine buffer: with LStore's
//      contiguous cache page of data that makes the whole call two long host runs, which the
//      host path pins in place and DMAs (no packing; parity written straight into the images
//      was one 64 KiB run per chunk, so every byte was packed and unpacked)
//   2. meanwhile, on another thread, the data chunks into the images: they do not depend on
//      the encode (only the 4-byte magics do)
//   3. parity chunks and magics into the images
// The images are the LUN child's placement of the iovec stream lsec_segment_encode_iov returns.
int write_stripes(lio_erasure_plan_t *plan, char *const *data_ptrs, int nstripes, int chunk, int n_shift,
                  long long first_stripe, char **dev) {
  const int k = plan->data_strips, m = plan->parity_strips, n = k + m;
  const size_t C = static_cast<size_t>(chunk), lchunk = C + 4;
  if (nstripes == 0) return 0;
  ParityPool::Buf pb = ParityPool::get().acquire(static_cast<size_t>(nstripes) * m * C);
  if (!pb.p) return lsec::set_error("lsec_segment_write: cannot allocate %zu bytes of parity", static_cast<size_t>(nstripes) * m * C);
  std::vector<char *> ptrs = stripe_ptrs(k, m, data_ptrs, nstripes, pb.p, C);
  // logical chunk j of stripe s lives on device (j - s*n_shift) mod n (lun_row_decompose)
  const auto device_of = [&](int s, int j) {
    const long long ss = first_stripe + s;
    return static_cast<int>(((j - ss * n_shift) % n + n) % n);
  };
  std::vector<lsec::HostCopy> data_jobs, par_jobs;
  data_jobs.reserve(static_cast<size_t>(nstripes) * k);
  par_jobs.reserve(static_cast<size_t>(nstripes) * m);
  for (int s = 0; s < nstripes; ++s)
    for (int j = 0; j < n; ++j) {
      char *slot = dev[device_of(s, j)] + static_cast<size_t>(s) * lchunk + 4;
      (j < k ? data_jobs : par_jobs).push_back({slot, ptrs[static_cast<size_t>(s) * n + j], C});
    }
  std::thread data_copies([&data_jobs] { lsec::parallel_copy(data_jobs); });
  std::vector<char> magic(static_cast<size_t>(nstripes) * 4);
  const int rc = et_encode_stripes_magic(plan, ptrs.data(), nstripes, chunk, magic.data());
  data_copies.join();
  if (rc == 0) {
    lsec::parallel_copy(par_jobs);
    for (int s = 0; s < nstripes; ++s)
      for (int i = 0; i < n; ++i) std::memcpy(dev[i] + static_cast<size_t>(s) * lchunk, &magic[static_cast<size_t>(s) * 4], 4);
  }
  ParityPool::get().release(pb);
  return rc;
}

int check_args(const char *fn, lio_erasure_plan_t *plan, const void *data, int nstripes, int chunk, int n_shift,
               long long first_stripe, char **dev) {
  if (!plan || !data || !dev) return lsec::set_error("%s: plan, data or dev is NULL", fn);
  if (nstripes < 0 || chunk <= 0 || n_shift < 0 || first_stripe < 0)
    return lsec::set_error("%s: bad geometry (nstripes=%d chunk=%d n_shift=%d first_stripe=%lld)", fn, nstripes, chunk,
                           n_shift, first_stripe);
  const int k = plan->data_strips, m = plan->parity_strips, n = k + m;
  if (k < 1 || m < 1 || n > LSEC_MAX_DEVS) return lsec::set_error("%s: k+m=%d outside 2..%d", fn, n, LSEC_MAX_DEVS);
  for (int i = 0; i < n; ++i)
    if (!dev[i]) return lsec::set_error("%s: dev[%d] is NULL", fn, i);
  return 0;
}

}  // namespace

extern "C" {

int lsec_segment_write(lio_erasure_plan_t *plan, const char *data, int nstripes, int chunk, int n_shift,
                       long long first_stripe, char **dev) {
  if (check_args("lsec_segment_write", plan, data, nstripes, chunk, n_shift, first_stripe, dev)) return -1;
  const int k = plan->data_strips;
  std::vector<char *> dp(static_cast<size_t>(nstripes) * k);
  for (size_t i = 0; i < dp.size(); ++i) dp[i] = const_cast<char *>(data) + i * static_cast<size_t>(chunk);
  return write_stripes(plan, dp.data(), nstripes, chunk, n_shift, first_stripe, dev);
}

// The user data as the cache hands it over (segjerase_write_func, segment/jerasure.c:1786-1825):
// a scatter list; a stripe inside one piece is used in place, a stripe straddling pieces is
// gathered into a contiguous copy first (:1795-1811), and a stripe that starts in an error page
// (iov_base NULL) is written as zero data chunks (:1816, :1823-1831).
int lsec_segment_write_iov(lio_erasure_plan_t *plan, const struct iovec *iov, int n_iov, int nstripes, int chunk,
                           int n_shift, long long first_stripe, char **dev) {
  static const char *fn = "lsec_segment_write_iov";
  if (check_args(fn, plan, iov, nstripes, chunk, n_shift, first_stripe, dev)) return -1;
  const int k = plan->data_strips;
  const size_t C = static_cast<size_t>(chunk);
  size_t nstraddle = 0;
  if (resolve_data(fn, k, iov, n_iov, nstripes, C, nullptr, 0, nullptr, &nstraddle)) return -1;
  std::vector<char> arena(nstraddle * k * C);
  std::vector<char *> dp;
  if (resolve_data(fn, k, iov, n_iov, nstripes, C, arena.data(), arena.size(), &dp, nullptr)) return -1;
  return write_stripes(plan, dp.data(), nstripes, chunk, n_shift, first_stripe, dev);
}

long long lsec_segment_straddle_bytes(lio_erasure_plan_t *plan, const struct iovec *iov, int n_iov, int nstripes,
                                      int chunk) {
  static const char *fn = "lsec_segment_straddle_bytes";
  if (!plan || !iov || nstripes < 0 || chunk <= 0) return lsec::set_error("%s: bad arguments", fn);
  size_t nstraddle = 0;
  if (resolve_data(fn, plan->data_strips, iov, n_iov, nstripes, static_cast<size_t>(chunk), nullptr, 0, nullptr,
                   &nstraddle))
    return -1;
  return static_cast<long long>(nstraddle * plan->data_strips * static_cast<size_t>(chunk));
}

// The reference's own hand-off, with no data copy (segjerase_write_func, segment/jerasure.c:
// 1780-1858): per stripe, ptr[] into the user's pages and the parity buffer, one encode + magic
// (on the GPU, for all stripes at once), and 2(k+m) iovecs [magic | chunk] in logical chunk
// order -- the tbuf segment_write hands the LUN child (:1852-1853).
int lsec_segment_encode_iov(lio_erasure_plan_t *plan, const struct iovec *iov, int n_iov, int nstripes, int chunk,
                            char *parity, char *magic, char *straddle, long long straddle_bytes, struct iovec *out,
                            int out_cap) {
  static const char *fn = "lsec_segment_encode_iov";
  if (!plan || !iov || !parity || !magic || !out || nstripes < 0 || chunk <= 0 || straddle_bytes < 0)
    return lsec::set_error("%s: bad arguments", fn);
  const int k = plan->data_strips, m = plan->parity_strips, n = k + m;
  if (k < 1 || m < 1 || n > LSEC_MAX_DEVS) return lsec::set_error("%s: k+m=%d outside 2..%d", fn, n, LSEC_MAX_DEVS);
  if (static_cast<long long>(nstripes) * 2 * n > out_cap)
    return lsec::set_error("%s: %d stripes need %lld iovecs, out_cap=%d", fn, nstripes, static_cast<long long>(nstripes) * 2 * n,
                           out_cap);
  if (nstripes == 0) return 0;
  const size_t C = static_cast<size_t>(chunk);
  std::vector<char *> dp;
  if (resolve_data(fn, k, iov, n_iov, nstripes, C, straddle, static_cast<size_t>(straddle_bytes), &dp, nullptr)) return -1;
  std::vector<char *> ptrs = stripe_ptrs(k, m, dp.data(), nstripes, parity, C);
  if (et_encode_stripes_magic(plan, ptrs.data(), nstripes, chunk, magic) != 0) return -1;
  for (int s = 0; s < nstripes; ++s)
    for (int i = 0; i < n; ++i) {
      struct iovec *o = out + (static_cast<size_t>(s) * n + i) * 2;
      o[0].iov_base = magic + static_cast<size_t>(s) * 4;
      o[0].iov_len = 4;
      o[1].iov_base = ptrs[static_cast<size_t>(s) * n + i];
      o[1].iov_len = C;
    }
  return nstripes * 2 * n;
}

}  // extern "C"
