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

#include <cstring>
#include <vector>

#include "../../include/lstore_ec.h"
#include "ec_host.h"

namespace {

// The shared body: data chunk j of stripe s at data_ptrs[s*k + j] (any host memory; chunks may
// alias, e.g. the zero chunk of an error page).  Parity is encoded straight into the images.
int write_stripes(lio_erasure_plan_t *plan, char *const *data_ptrs, int nstripes, int chunk, int n_shift,
                  long long first_stripe, char **dev) {
  const int k = plan->data_strips, m = plan->parity_strips, n = k + m;
  const size_t C = static_cast<size_t>(chunk), lchunk = C + 4;
  if (nstripes == 0) return 0;
  // ptr[] as segjerase_write_func builds it; parity slots point straight into the images
  std::vector<char *> ptrs(static_cast<size_t>(nstripes) * n);
  std::vector<int> phys_of(static_cast<size_t>(n));
  for (int s = 0; s < nstripes; ++s) {
    const long long ss = first_stripe + s;
    for (int i = 0; i < n; ++i) phys_of[(i + ss * n_shift) % n] = i;  // logical chunk -> device
    for (int j = 0; j < k; ++j) ptrs[static_cast<size_t>(s) * n + j] = data_ptrs[static_cast<size_t>(s) * k + j];
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
  if (check_args("lsec_segment_write_iov", plan, iov, nstripes, chunk, n_shift, first_stripe, dev)) return -1;
  if (n_iov < 0) return lsec::set_error("lsec_segment_write_iov: n_iov=%d", n_iov);
  const int k = plan->data_strips;
  const size_t C = static_cast<size_t>(chunk), dsize = static_cast<size_t>(k) * C;
  size_t total = 0;
  for (int i = 0; i < n_iov; ++i) total += iov[i].iov_len;
  if (total < dsize * static_cast<size_t>(nstripes))
    return lsec::set_error("lsec_segment_write_iov: %zu bytes in the scatter list for %d stripes of %zu", total, nstripes,
                           dsize);
  // pass 1: the piece each stripe starts in, and which stripes straddle pieces
  std::vector<int> first_piece(static_cast<size_t>(nstripes));
  std::vector<size_t> piece_start(static_cast<size_t>(n_iov) + 1, 0);
  for (int i = 0; i < n_iov; ++i) piece_start[i + 1] = piece_start[i] + iov[i].iov_len;
  size_t nstraddle = 0;
  int pi = 0;
  for (int s = 0; s < nstripes; ++s) {
    const size_t off = static_cast<size_t>(s) * dsize;
    while (piece_start[pi + 1] <= off) ++pi;
    first_piece[s] = pi;
    if (iov[pi].iov_base && piece_start[pi + 1] < off + dsize) ++nstraddle;
  }
  // pass 2: chunk pointers; straddling stripes gathered into one arena
  std::vector<char> arena(nstraddle * dsize);
  std::vector<char> empty(C, 0);
  std::vector<char *> dp(static_cast<size_t>(nstripes) * k);
  size_t used = 0;
  for (int s = 0; s < nstripes; ++s) {
    const size_t off = static_cast<size_t>(s) * dsize;
    const int p0 = first_piece[s];
    char *base;
    if (!iov[p0].iov_base) {
      for (int j = 0; j < k; ++j) dp[static_cast<size_t>(s) * k + j] = empty.data();
      continue;
    }
    if (piece_start[p0 + 1] >= off + dsize) {
      base = static_cast<char *>(iov[p0].iov_base) + (off - piece_start[p0]);
    } else {
      base = arena.data() + used;
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
    for (int j = 0; j < k; ++j) dp[static_cast<size_t>(s) * k + j] = base + static_cast<size_t>(j) * C;
  }
  return write_stripes(plan, dp.data(), nstripes, chunk, n_shift, first_stripe, dev);
}

}  // extern "C"
