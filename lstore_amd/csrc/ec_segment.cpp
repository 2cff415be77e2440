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
  if (!plan || !data || !dev) return lsec::set_error("lsec_segment_write: plan, data or dev is NULL");
  if (nstripes < 0 || chunk <= 0 || n_shift < 0 || first_stripe < 0)
    return lsec::set_error("lsec_segment_write: bad geometry (nstripes=%d chunk=%d n_shift=%d first_stripe=%lld)", nstripes,
                           chunk, n_shift, first_stripe);
  const int k = plan->data_strips, m = plan->parity_strips, n = k + m;
  if (k < 1 || m < 1 || n > LSEC_MAX_DEVS) return lsec::set_error("lsec_segment_write: k+m=%d outside 2..%d", n, LSEC_MAX_DEVS);
  for (int i = 0; i < n; ++i)
    if (!dev[i]) return lsec::set_error("lsec_segment_write: dev[%d] is NULL", i);
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
