// ec_plan.cpp -- the plan service of liblstore_ec.so: et_new_plan / et_generate_plan /
// et_destroy_plan and the plan's fn-pointers (form_*), with the same arguments, return codes and
// struct contents as src/lio/erasure_tools.c; the coding matrices and their per-device images
// (encode image per plan, decode image per erasure pattern, built once and cached); and the
// device-resident core (enqueue_apply: every coding launch, for every route).
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

#include <strings.h>

#include <array>
#include <cstdio>

#include "ec_jit.h"
#include "ec_engine.h"

#include <unistd.h>

extern "C" const char *JE_method[N_JE_METHODS] = {"reed_sol_van", "reed_sol_r6_op", "cauchy_orig", "cauchy_good",
                                                  "blaum_roth",   "liberation",     "liber8tion",  "raid4"};

namespace lsec {
namespace eng {

thread_local std::string tl_err;

int fail(const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  tl_err = buf;
  return -1;
}

// Ends the process with a reason that survives it: written to fd 2 with write(2) (no stdio
// buffer to lose) and appended to the file LSEC_FATAL_LOG names, if set -- a test runner that
// captures fd 2 into a temporary file loses that file when the process aborts (VERDICT r03:
// an abort in a GPU suite run whose reason never reached the log).
[[noreturn]] void fatal(const char *fmt, ...) {
  char buf[1024];
  int n = snprintf(buf, sizeof(buf), "liblstore_ec: fatal: ");
  va_list ap;
  va_start(ap, fmt);
  n += vsnprintf(buf + n, sizeof(buf) - n - 2, fmt, ap);
  va_end(ap);
  n = std::min<int>(n, sizeof(buf) - 2);
  buf[n++] = '\n';
  if (write(2, buf, n) < 0) {
  }
  if (const char *path = getenv("LSEC_FATAL_LOG"))
    if (FILE *f = fopen(path, "a")) {
      fwrite(buf, 1, n, f);
      fclose(f);
    }
  abort();
}

int max_devs(int method, int w) {
  const bool matrix = method == REED_SOL_VAN || method == REED_SOL_R6_OP || method == CAUCHY_ORIG || method == CAUCHY_GOOD;
  return matrix && (w == 16 || w == 32) ? kMaxDevs : LSEC_MAX_DEVS;
}

PlanExt *ext_of(lio_erasure_plan_t *p) {
  if (!p) return nullptr;
  PlanExt *e = reinterpret_cast<PlanExt *>(p);
  return e->magic == kPlanMagic ? e : nullptr;
}

bool liberation_family(int method) { return method == BLAUM_ROTH || method == LIBERATION || method == LIBER8TION; }

// Which kernel applies a plan:
//   RS / r6 at w = 8 -> bytewise GF(2^8); at w = 16 / 32 -> wordwise GF(2^w)
//   Cauchy at w = 8 -> bit-sliced GF(2^8); at w = 16 / 32 -> bit-sliced GF(2^w)
//   liberation family -> generic GF(2) bitmatrix; raid4 -> bytewise XOR (w unused, raid4.c)
int kernel_kind(int method, int w) {
  if (liberation_family(method)) return w >= 2 && w <= lsec::kMaxW ? KBITMATRIX : KNONE;
  if (method == RAID4) return KBYTEWISE;
  const bool wide = (w == 16 || w == 32);
  if (w != 8 && !wide) return KNONE;
  switch (method) {
    case REED_SOL_VAN:
    case REED_SOL_R6_OP:
      return wide ? KWORDWISE : KBYTEWISE;
    case CAUCHY_ORIG:
    case CAUCHY_GOOD:
      return wide ? KBITSLICEDW : KBITSLICED;
    default:
      return KNONE;
  }
}

bool uses_u32_image(int kind) { return kind == KBITMATRIX || kind == KWORDWISE || kind == KBITSLICEDW; }
bool packet_kind(int kind) { return kind == KBITSLICED || kind == KBITMATRIX || kind == KBITSLICEDW; }

int *to_int_array(const lsec::gfw::Mat &m) {
  int *a = static_cast<int *>(malloc(sizeof(int) * m.size()));
  for (size_t i = 0; i < m.size(); ++i) a[i] = static_cast<int>(m[i]);
  return a;
}

// word image of an R x K GF(2^w) matrix for k_gfw_wordwise: [(r*K + j)*w + b] = M[r][j] * x^b
std::vector<uint32_t> word_image(const lsec::gfw::Mat &mat, int rows, int cols, int w) {
  std::vector<uint32_t> img(static_cast<size_t>(rows) * cols * w);
  for (int i = 0; i < rows * cols; ++i) lsec::make_word_cell(mat[i], w, &img[static_cast<size_t>(i) * w]);
  return img;
}

// bitmatrix row masks for the generic bitmatrix kernels: NW = mask_words(w) words per (row, input),
// bit x of word [((r*w+l)*k + j)*NW + q] = B[r*w+l][j*w + 32q + x]
std::vector<uint32_t> bitmatrix_masks(const int *bm, int k, int m, int w) {
  const int nw = lsec::mask_words(w);
  std::vector<uint32_t> mk(static_cast<size_t>(m) * w * k * nw, 0u);
  for (int row = 0; row < m * w; ++row)
    for (int j = 0; j < k; ++j)
      for (int x = 0; x < w; ++x)
        if (bm[static_cast<size_t>(row) * k * w + j * w + x])
          mk[(static_cast<size_t>(row) * k + j) * nw + x / 32] |= 1u << (x % 32);
  return mk;
}

// Image rows per output row and elements per (row, input) of a kernel kind's image.
int image_rows_per_output(int kind, int w) { return kind == KBITMATRIX ? w : 1; }
int image_unit(int kind, int w) {
  return kind == KBITMATRIX ? lsec::mask_words(w) : (kind == KWORDWISE || kind == KBITSLICEDW) ? w : 1;
}

// The grouped layout of ec_kernels.h for images of more than lsec::kMaxK inputs: `rows` image
// rows of K inputs x `unit` elements, row-major -> groups of kMaxK inputs, each row-major.
template <typename T>
void group_image(std::vector<T> &img, int rows, int K, int unit) {
  if (K <= lsec::kMaxK) return;
  std::vector<T> out(img.size());
  size_t o = 0;
  for (int k0 = 0; k0 < K; k0 += lsec::kMaxK) {
    const int kg = std::min(lsec::kMaxK, K - k0);
    for (int r = 0; r < rows; ++r) {
      const T *src = &img[(static_cast<size_t>(r) * K + k0) * unit];
      std::copy(src, src + static_cast<size_t>(kg) * unit, &out[o]);
      o += static_cast<size_t>(kg) * unit;
    }
  }
  img.swap(out);
}

int *to_int_array(const lsec::gf8::Mat &m) {
  int *a = static_cast<int *>(malloc(sizeof(int) * m.size()));
  for (size_t i = 0; i < m.size(); ++i) a[i] = m[i];
  return a;
}

int *to_int_array(const std::vector<int> &v) {
  int *a = static_cast<int *>(malloc(sizeof(int) * v.size()));
  std::memcpy(a, v.data(), sizeof(int) * v.size());
  return a;
}

int **schedule_array(const std::vector<std::array<int, 5>> &ops) {
  int **s = static_cast<int **>(malloc(sizeof(int *) * (ops.size() + 1)));
  for (size_t i = 0; i < ops.size(); ++i) {
    s[i] = static_cast<int *>(malloc(sizeof(int) * 5));
    std::memcpy(s[i], ops[i].data(), sizeof(int) * 5);
  }
  s[ops.size()] = static_cast<int *>(malloc(sizeof(int) * 5));
  s[ops.size()][0] = -1;
  return s;
}

// Builds the plan's public matrix objects (what erasure_tools.c's form_* routines build,
// erasure_tools.c:101-292) and the kernel's GF matrix.  `with_schedule` distinguishes
// form_encoding_matrix (matrix + bitmatrix + schedule) from form_decoding_matrix.
int form_matrices(lio_erasure_plan_t *p, bool with_schedule) {
  PlanExt *e = ext_of(p);
  if (!e) return -1;
  std::lock_guard<std::mutex> lk(e->impl->mu);
  const int k = p->data_strips, m = p->parity_strips, w = p->w;
  lsec::gf8::Mat mat;
  switch (p->method) {
    case RAID4:
      e->impl->coding.assign(k, 1);
      e->impl->coding_ready = true;
      e->impl->coding_fast.store(true, std::memory_order_release);
      return 0;
    case REED_SOL_VAN:
    case REED_SOL_R6_OP: {
      if (!p->encode_matrix) {
        const bool r6 = p->method == REED_SOL_R6_OP;
        if (w == 8) {
          if (!(r6 ? lsec::gf8::reed_sol_r6(k, mat) : lsec::gf8::reed_sol_vandermonde(k, m, mat)))
            return fail("cannot form %s matrix for k=%d m=%d w=%d", JE_method[p->method], k, m, w);
          p->encode_matrix = to_int_array(mat);
        } else {
          lsec::gfw::Mat wm;
          const bool ok = (w == 16 || w == 32) &&
                          (r6 ? lsec::gfw::reed_sol_r6(k, w, wm) : lsec::gfw::reed_sol_vandermonde(k, m, w, wm));
          if (!ok) return fail("cannot form %s matrix for k=%d m=%d w=%d", JE_method[p->method], k, m, w);
          p->encode_matrix = to_int_array(wm);
        }
      }
      break;
    }
    case CAUCHY_ORIG:
    case CAUCHY_GOOD: {
      if (!p->encode_matrix) {
        const bool orig = p->method == CAUCHY_ORIG;
        if (w == 8) {
          if (!(orig ? lsec::gf8::cauchy_original(k, m, mat) : lsec::gf8::cauchy_good(k, m, mat)))
            return fail("cannot form %s matrix for k=%d m=%d w=%d", JE_method[p->method], k, m, w);
          p->encode_matrix = to_int_array(mat);
          p->encode_bitmatrix = to_int_array(lsec::gf8::to_bitmatrix(k, m, mat));
        } else {
          lsec::gfw::Mat wm;
          const bool ok = (w == 16 || w == 32) &&
                          (orig ? lsec::gfw::cauchy_original(k, m, w, wm) : lsec::gfw::cauchy_good(k, m, w, wm));
          if (!ok) return fail("cannot form %s matrix for k=%d m=%d w=%d", JE_method[p->method], k, m, w);
          p->encode_matrix = to_int_array(wm);
          p->encode_bitmatrix = to_int_array(lsec::gfw::to_bitmatrix(k, m, w, wm));
        }
      }
      if (with_schedule && !p->encode_schedule) {
        std::vector<int> bm(p->encode_bitmatrix, p->encode_bitmatrix + static_cast<size_t>(k) * m * w * w);
        p->encode_schedule = schedule_array(lsec::gf8::smart_schedule(k, m, w, bm));
      }
      break;
    }
    case BLAUM_ROTH:
    case LIBERATION:
    case LIBER8TION: {
      if (!p->encode_bitmatrix) {
        std::vector<int> bm = p->method == LIBERATION   ? lsec::gf8::liberation_bitmatrix(k, w)
                              : p->method == BLAUM_ROTH ? lsec::gf8::blaum_roth_bitmatrix(k, w)
                                                        : lsec::gf8::liber8tion_bitmatrix(k);
        if (bm.empty()) return fail("cannot form %s bitmatrix for k=%d w=%d", JE_method[p->method], k, w);
        p->encode_bitmatrix = to_int_array(bm);
      }
      if (with_schedule && !p->encode_schedule) {
        std::vector<int> bm(p->encode_bitmatrix, p->encode_bitmatrix + static_cast<size_t>(k) * m * w * w);
        p->encode_schedule = schedule_array(lsec::gf8::smart_schedule(k, m, w, bm));
      }
      break;
    }
    default:
      return fail("invalid method %d", p->method);
  }
  if (e->impl->coding_ready) return 0;
  const int kind = kernel_kind(p->method, w);
  if (kind == KBITMATRIX) {
    if (!p->encode_bitmatrix) return 0;
    e->impl->enc_masks = bitmatrix_masks(p->encode_bitmatrix, k, m, w);
    group_image(e->impl->enc_masks, m * w, k, lsec::mask_words(w));
    e->impl->coding_ready = true;
    e->impl->coding_fast.store(true, std::memory_order_release);
  } else if (p->encode_matrix) {
    const int rows = (p->method == REED_SOL_R6_OP) ? 2 : m;
    if (kind == KWORDWISE || kind == KBITSLICEDW) {
      e->impl->coding_w.resize(static_cast<size_t>(rows) * k);
      for (size_t i = 0; i < e->impl->coding_w.size(); ++i) e->impl->coding_w[i] = static_cast<uint32_t>(p->encode_matrix[i]);
      e->impl->enc_masks = word_image(e->impl->coding_w, rows, k, w);
      group_image(e->impl->enc_masks, rows, k, w);
    } else {
      e->impl->coding.resize(static_cast<size_t>(rows) * k);
      for (size_t i = 0; i < e->impl->coding.size(); ++i) e->impl->coding[i] = static_cast<uint8_t>(p->encode_matrix[i]);
    }
    e->impl->coding_ready = true;
    e->impl->coding_fast.store(true, std::memory_order_release);
  }
  return 0;
}

// fn-pointer versions, with the reference's return-code behaviour
int fp_form_encoding(lio_erasure_plan_t *p) {
  if (!p) return -1;
  return form_matrices(p, true);
}

int fp_form_decoding(lio_erasure_plan_t *p) {
  if (!p) return -1;
  // "Already formed so skip step": every *_form_coding_matrix returns 0 at once when its
  // matrix (Cauchy) or bitmatrix (liberation family) exists (erasure_tools.c:137, :152, :169,
  // :184, :198), whatever the schedule
  const bool cauchy = p->method == CAUCHY_ORIG || p->method == CAUCHY_GOOD;
  const bool formed = cauchy ? p->encode_matrix != nullptr : liberation_family(p->method) && p->encode_bitmatrix != nullptr;
  const int rc = form_matrices(p, false);
  if (rc || formed) return rc;
  // ... and -1 when it has just formed it while the schedule is still unset (:142, :159,
  // :176, :190, :204)
  if ((cauchy || liberation_family(p->method)) && !p->encode_schedule) return -1;
  return 0;
}

int ensure_coding(PlanExt *e) {
  if (e->impl->coding_fast.load(std::memory_order_acquire)) return 0;
  {
    std::lock_guard<std::mutex> lk(e->impl->mu);
    if (e->impl->coding_ready) return 0;
  }
  return form_matrices(&e->pub, true);
}

void host_cells(const lsec::gf8::Mat &mat, int rows, int cols, std::vector<CoefCell> &cells) {
  cells.resize(static_cast<size_t>(rows) * cols);
  for (int i = 0; i < rows * cols; ++i) lsec::make_cell(mat[i], cells[i]);
  // flag plain-XOR rows (any launch whose first row is one takes the XOR-row kernel path)
  for (int r = 0; r < rows; ++r) {
    bool ones = true;
    for (int j = 0; j < cols && ones; ++j) ones = mat[static_cast<size_t>(r) * cols + j] == 1;
    if (ones) cells[static_cast<size_t>(r) * cols].pad |= lsec::kCellXorRow;
  }
}

int upload_cells(const std::vector<CoefCell> &h, CoefCell **out) {
  CoefCell *d = nullptr;
  HIP_OK(hipMalloc(&d, sizeof(CoefCell) * h.size()));
  hipError_t err = hipMemcpy(d, h.data(), sizeof(CoefCell) * h.size(), hipMemcpyHostToDevice);
  if (err != hipSuccess) {
    (void)hipFree(d);
    return fail("hipMemcpy(cells): %s", hipGetErrorString(err));
  }
  *out = d;
  return 0;
}

// output rows of the encode image (m; 2 for r6, 1 for raid4)
int encode_rows(const PlanExt *e) {
  const int kind = kernel_kind(e->pub.method, e->pub.w);
  if (kind == KBITMATRIX) return e->pub.parity_strips;
  if (kind == KWORDWISE || kind == KBITSLICEDW) return static_cast<int>(e->impl->coding_w.size()) / e->pub.data_strips;
  return static_cast<int>(e->impl->coding.size()) / e->pub.data_strips;
}

int upload_masks(const std::vector<uint32_t> &h, uint32_t **out) {
  uint32_t *d = nullptr;
  HIP_OK(hipMalloc(&d, sizeof(uint32_t) * h.size()));
  hipError_t err = hipMemcpy(d, h.data(), sizeof(uint32_t) * h.size(), hipMemcpyHostToDevice);
  if (err != hipSuccess) {
    (void)hipFree(d);
    return fail("hipMemcpy(masks): %s", hipGetErrorString(err));
  }
  *out = d;
  return 0;
}

int encode_cells_locked(PlanExt *e, int dev, const void **out);

// encode image on the current device: CoefCell[m][k] (matrix codes) or row masks (bitmatrix)
int encode_cells(PlanExt *e, const void **out) {
  if (ensure_coding(e)) return -1;
  int dev = 0;
  HIP_OK(hipGetDevice(&dev));
  if (dev >= 0 && dev < kFastDevs)
    if (const void *f = e->impl->enc_fast[dev].load(std::memory_order_acquire)) {
      *out = f;
      return 0;
    }
  std::lock_guard<std::mutex> lk(e->impl->mu);
  const int rc = encode_cells_locked(e, dev, out);
  if (rc == 0 && dev >= 0 && dev < kFastDevs) e->impl->enc_fast[dev].store(*out, std::memory_order_release);
  return rc;
}

int encode_cells_locked(PlanExt *e, int dev, const void **out) {
  if (uses_u32_image(kernel_kind(e->pub.method, e->pub.w))) {
    auto it = e->impl->enc_dev_masks.find(dev);
    if (it == e->impl->enc_dev_masks.end()) {
      uint32_t *d = nullptr;
      if (upload_masks(e->impl->enc_masks, &d)) return -1;
      it = e->impl->enc_dev_masks.emplace(dev, d).first;
      if (kernel_kind(e->pub.method, e->pub.w) == KWORDWISE)  // RS / r6 at w = 16 / 32: a bit-sliced network
        lsec::jit::bind_w(d, e->impl->coding_w.data(), encode_rows(e), e->pub.data_strips, e->pub.w);
      else if (kernel_kind(e->pub.method, e->pub.w) == KBITMATRIX)  // liberation family: a packet network
        lsec::jit::bind_pkt(d, e->impl->enc_masks.data(), encode_rows(e), e->pub.data_strips, e->pub.w, e->pub.packet_size);
      else if (kernel_kind(e->pub.method, e->pub.w) == KBITSLICEDW)  // Cauchy at w = 16 / 32: the same
        lsec::jit::bind_pkt_field(d, e->impl->coding_w.data(), encode_rows(e), e->pub.data_strips, e->pub.w,
                                  e->pub.packet_size);
    }
    *out = it->second;
    return 0;
  }
  auto it = e->impl->enc_cells.find(dev);
  if (it != e->impl->enc_cells.end()) {
    *out = it->second;
    return 0;
  }
  const int k = e->pub.data_strips;
  const int rows = static_cast<int>(e->impl->coding.size()) / k;
  std::vector<CoefCell> h;
  host_cells(e->impl->coding, rows, k, h);
  group_image(h, rows, k, 1);
  CoefCell *d = nullptr;
  if (upload_cells(h, &d)) return -1;
  e->impl->enc_cells[dev] = d;
  if (kernel_kind(e->pub.method, e->pub.w) == KBYTEWISE) {  // wide codes: an XOR network, compiled in the background
    lsec::jit::bind(d, e->impl->coding.data(), rows, k);
  } else if (kernel_kind(e->pub.method, e->pub.w) == KBITSLICED) {  // Cauchy w = 8: a packet network (A/B knob)
    std::vector<uint32_t> c32(e->impl->coding.begin(), e->impl->coding.end());
    lsec::jit::bind_pkt_field(d, c32.data(), rows, k, 8, e->pub.packet_size);
  }
  *out = d;
  return 0;
}

// Parses a -1 terminated erasure list.  Returns 0 with the sorted distinct ids, 1 if the
// list is empty (nothing to do), -1 if unrecoverable / invalid.
int parse_erasures(const lio_erasure_plan_t *p, const int *erasures, std::vector<int> &ids) {
  const int k = p->data_strips, m = p->parity_strips;
  ids.clear();
  if (!erasures) return fail("erasures is NULL");
  int listed = 0;
  for (int i = 0; erasures[i] != -1; ++i) {
    const int x = erasures[i];
    if (x < 0 || x >= k + m) return fail("erasure id %d out of range 0..%d", x, k + m - 1);
    ++listed;
    if (std::find(ids.begin(), ids.end(), x) == ids.end()) ids.push_back(x);
    if (listed > 4 * (k + m)) return fail("erasure list not terminated");
  }
  std::sort(ids.begin(), ids.end());
  if (p->method == RAID4 && listed > 1) return fail("raid4 recovers one device (raid4.c:47)");
  if (static_cast<int>(ids.size()) > m) return fail("%zu erasures exceed m=%d", ids.size(), m);
  if (ids.empty()) return 1;
  return 0;
}

int decode_entry_locked(PlanExt *e, const std::vector<int> &ids, int dev, DecodeEntry **out, const void **cells);

// decode entry (host plan + device cells on the current device).  Entries are never moved or
// freed before the plan is destroyed, so each thread keeps its last lookup and repeats of it
// (a degraded read decodes the same pattern stripe after stripe) skip the plan mutex.
int decode_entry(PlanExt *e, const std::vector<int> &ids, DecodeEntry **out, const void **cells) {
  if (ensure_coding(e)) return -1;
  int dev = 0;
  HIP_OK(hipGetDevice(&dev));
  struct Last {
    unsigned long long serial = 0;
    int dev = -1;
    std::vector<int> ids;
    DecodeEntry *ent = nullptr;
    const void *cells = nullptr;
  };
  thread_local Last last;
  if (last.serial == e->impl->serial && last.dev == dev && last.ids == ids) {
    *out = last.ent;
    *cells = last.cells;
    return 0;
  }
  int rc;
  {
    std::lock_guard<std::mutex> lk(e->impl->mu);
    rc = decode_entry_locked(e, ids, dev, out, cells);
  }
  if (rc == 0) {
    last.serial = e->impl->serial;
    last.dev = dev;
    last.ids = ids;
    last.ent = *out;
    last.cells = *cells;
  }
  return rc;
}

int decode_entry_locked(PlanExt *e, const std::vector<int> &ids, int dev, DecodeEntry **out, const void **cells) {
  const int kind = kernel_kind(e->pub.method, e->pub.w);
  const bool bitm = uses_u32_image(kind);
  auto it = e->impl->decode_cache.find(ids);
  if (it == e->impl->decode_cache.end()) {
    DecodeEntry ent;
    const int k = e->pub.data_strips;
    if (kind == KWORDWISE || kind == KBITSLICEDW) {
      const int w = e->pub.w;
      const int m = static_cast<int>(e->impl->coding_w.size()) / k;
      lsec::gfw::DecodePlan wp;
      if (!lsec::gfw::make_decode(k, m, w, e->impl->coding_w, ids, wp)) return fail("decoding matrix is singular");
      ent.dp.survivors = wp.survivors;
      ent.dp.erased = wp.erased;
      ent.masks = word_image(wp.rows, static_cast<int>(wp.erased.size()), k, w);
      group_image(ent.masks, static_cast<int>(wp.erased.size()), k, w);
      ent.xor_only = std::all_of(wp.rows.begin(), wp.rows.end(), [](uint32_t c) { return c <= 1u; });
      if (ent.xor_only) ent.dp.rows.assign(wp.rows.begin(), wp.rows.end());  // 0 / 1 as GF(2^8) cells
      ent.wrows.assign(wp.rows.begin(), wp.rows.end());
    } else if (kind == KBITMATRIX) {
      const lio_erasure_plan_t *p = &e->pub;
      // solves for the lost data bits only (gf8.cpp make_bit_decode): milliseconds even for the
      // widest liberation plans (k = 254, w = 257), where inverting the whole survivor bitmatrix
      // as jerasure_invert_bitmatrix does (jerasure.c:1049-1104) would take hours
      std::vector<int> bm(p->encode_bitmatrix, p->encode_bitmatrix + static_cast<size_t>(k) * p->parity_strips * p->w * p->w);
      if (!lsec::gf8::make_bit_decode(k, p->parity_strips, p->w, bm, ids, ent.dp, ent.masks))
        return fail("decoding bitmatrix is singular");
      group_image(ent.masks, static_cast<int>(ent.dp.erased.size()) * p->w, k, lsec::mask_words(p->w));
    } else {
      const int m = static_cast<int>(e->impl->coding.size()) / k;
      if (!lsec::gf8::make_decode(k, m, e->impl->coding, ids, ent.dp)) return fail("decoding matrix is singular");
      ent.xor_only = std::all_of(ent.dp.rows.begin(), ent.dp.rows.end(), [](int c) { return c == 0 || c == 1; });
    }
    it = e->impl->decode_cache.emplace(ids, std::move(ent)).first;
  }
  DecodeEntry &ent = it->second;
  if (bitm && !ent.xor_only) {
    auto dm = ent.dev_masks.find(dev);
    if (dm == ent.dev_masks.end()) {
      uint32_t *d = nullptr;
      if (upload_masks(ent.masks, &d)) return -1;
      dm = ent.dev_masks.emplace(dev, d).first;
      if (kind == KWORDWISE)
        lsec::jit::bind_w(d, ent.wrows.data(), static_cast<int>(ent.dp.erased.size()), e->pub.data_strips, e->pub.w);
      else if (kind == KBITMATRIX)
        lsec::jit::bind_pkt(d, ent.masks.data(), static_cast<int>(ent.dp.erased.size()), e->pub.data_strips, e->pub.w,
                            e->pub.packet_size);
      else if (kind == KBITSLICEDW)
        lsec::jit::bind_pkt_field(d, ent.wrows.data(), static_cast<int>(ent.dp.erased.size()), e->pub.data_strips,
                                  e->pub.w, e->pub.packet_size);
    }
    *out = &ent;
    *cells = dm->second;
    return 0;
  }
  auto dc = ent.dev_cells.find(dev);
  if (dc == ent.dev_cells.end()) {
    std::vector<CoefCell> h;
    host_cells(ent.dp.rows, static_cast<int>(ent.dp.erased.size()), e->pub.data_strips, h);
    group_image(h, static_cast<int>(ent.dp.erased.size()), e->pub.data_strips, 1);
    CoefCell *d = nullptr;
    if (upload_cells(h, &d)) return -1;
    dc = ent.dev_cells.emplace(dev, d).first;
    if (!ent.xor_only && kernel_kind(e->pub.method, e->pub.w) == KBYTEWISE) {
      lsec::jit::bind(d, ent.dp.rows.data(), static_cast<int>(ent.dp.erased.size()), e->pub.data_strips);
    } else if (!ent.xor_only && kernel_kind(e->pub.method, e->pub.w) == KBITSLICED) {
      std::vector<uint32_t> c32(ent.dp.rows.begin(), ent.dp.rows.end());
      lsec::jit::bind_pkt_field(d, c32.data(), static_cast<int>(ent.dp.erased.size()), e->pub.data_strips, 8,
                                e->pub.packet_size);
    }
  }
  *out = &ent;
  *cells = dc->second;
  return 0;
}

// A decode that only XORs survivors (a lost data shard rebuilt from P0, whose Cauchy-good /
// RS row is all ones) is layout- and field-agnostic, so Cauchy packets and GF(2^16) / GF(2^32)
// words go through the bytewise kernel's plain-XOR path (0 / 1 cells) instead.
int decode_kind(const PlanExt *e, const DecodeEntry *ent) {
  const int kind = kernel_kind(e->pub.method, e->pub.w);
  const bool field = kind == KBITSLICED || kind == KWORDWISE || kind == KBITSLICEDW;
  return field && ent->xor_only ? KBYTEWISE : kind;
}

int check_geometry(const lio_erasure_plan_t *p, long long block_size) {
  const int k = p->data_strips, m = p->parity_strips;
  const int lim = max_devs(p->method, p->w);
  if (k < 1 || m < 1 || k + m > lim) return fail("k=%d m=%d: k+m outside 2..%d (w=%d)", k, m, lim, p->w);
  if (block_size < 0 || block_size % 8 != 0) return fail("block_size %lld is not a multiple of 8", block_size);
  const int kind = kernel_kind(p->method, p->w);
  if (kind == KNONE)
    return fail("method %s (w=%d) has no GPU kernel in this build", JE_method[p->method], p->w);
  if (packet_kind(kind)) {
    const long long sp = static_cast<long long>(p->w) * p->packet_size;
    if (p->packet_size <= 0 || p->packet_size % 4 != 0 || block_size % sp != 0)
      return fail("block_size %lld is not a multiple of w*packet_size = %lld", block_size, sp);
  }
  if (liberation_family(p->method) && m != 2) return fail("%s needs m == 2", JE_method[p->method]);
  return 0;
}

// Cauchy at w = 8 (KBITSLICED): the generic bit-sliced kernel or the compiled packet network, by
// shape.  Round 6 (profiles/r06_v13_cauchy8_kernels_ab.txt: every c5 shape at C = 1, 4, 8 MiB, one
// allocation each, interleaved): since the bit-sliced kernel took the work-sharing tail (round 5)
// and the XCD tile phase (round 6), neither of which the networks have, it beats the network on
// every shape with R <= 4 by 0.3-2.5 % -- at 4 dwords per lane from K = 16, and from K = 10 at
// chunks of 4 MiB and up; 1 dword otherwise -- while the network keeps (20+6) (R = 6; up to 3.8 %
// ahead at 4 MiB).  0: the network (where one is compiled), else the bit-sliced kernel's dwords per
// lane.  lsec_test_set_cauchy8_policy(1) gives the network every shape it has one for (tests).
std::atomic<int> g_c8_policy{0};

int cauchy8_bitsliced_dw(int K, int R, long long size) {
  if (g_c8_policy.load(std::memory_order_relaxed) == 1 || R > 4) return 0;
  if (K >= 16 || (K >= 10 && size >= (4LL << 20))) return 4;
  return 1;
}

// Enqueue out[r] = rows[r] . in  for every stripe, splitting R into launches of <= 8 rows
// (<= 2 for the bitmatrix kernel) and K into groups of <= lsec::kMaxK inputs.  `image` is the
// CoefCell[R][K] matrix image, the uint32 row masks [((r*w+l)*K + j)*NW + q] (KBITMATRIX) or the
// word products [(r*K + j)*w + b] (KWORDWISE / KBITSLICEDW), grouped when K > kMaxK.
int enqueue_apply(int kind, const void *image, int K, int R, const ShardRef *in, const ShardRef *out,
                  int nstripes, long long size, int packet, hipStream_t st, int w) {
  const bool net = kind == KBYTEWISE   ? lsec::bytewise_variant() == 0 && lsec::jit::wants_xornet(R, K)
                   : kind == KWORDWISE ? lsec::bitsliced_variant() == 0 && lsec::jit::wants_gfw_net(R, K, w)
                                       : false;
  ShardRef tin[lsec::kMaxK], tout[lsec::kMaxR];  // a w = 16 / 32 network's ragged tail, below
  if (net) {
    if (hipFunction_t fn = lsec::jit::ready(image, R, K)) {  // the matrix's compiled XOR network
      // w = 16 / 32 networks take whole tiles only: the tail columns go to the generic kernel
      const long long whole = kind == KWORDWISE ? size / lsec::jit::gfw_tile(w, R) * lsec::jit::gfw_tile(w, R) : size;
      // batches split so tile indices stay 32-bit, as below
      const long long per = std::max(1LL, (1LL << 30) / std::max(1LL, size / 4096 + 1));
      ShardRef bi[lsec::jit::kMaxCols], bo[lsec::jit::kMaxRows];
      for (int s0 = 0; whole > 0 && s0 < nstripes; s0 += static_cast<int>(std::min<long long>(per, nstripes))) {
        const int n = static_cast<int>(std::min<long long>(per, nstripes - s0));
        for (int j = 0; j < K; ++j) bi[j] = {in[j].base + static_cast<uint64_t>(s0) * in[j].stride, in[j].stride};
        for (int r = 0; r < R; ++r) bo[r] = {out[r].base + static_cast<uint64_t>(s0) * out[r].stride, out[r].stride};
        const hipError_t err = lsec::jit::launch(fn, R, K, bi, bo, n, whole, st, kind == KWORDWISE ? w : 8);
        if (err != hipSuccess) return fail("xor network launch failed: %s", hipGetErrorString(err));
      }
      if (whole == size) return 0;
      for (int j = 0; j < K; ++j) tin[j] = {in[j].base + static_cast<uint64_t>(whole), in[j].stride};
      for (int r = 0; r < R; ++r) tout[r] = {out[r].base + static_cast<uint64_t>(whole), out[r].stride};
      in = tin;
      out = tout;
      size -= whole;
    }
  }
  // Cauchy w = 8: the shape's kernel (cauchy8_bitsliced_dw; 0 = the network)
  const int c8_dw = kind == KBITSLICED && w == 8 && lsec::bitsliced_variant() == 0 ? cauchy8_bitsliced_dw(K, R, size) : 0;
  if ((kind == KBITMATRIX || kind == KBITSLICEDW || kind == KBITSLICED) && lsec::bitsliced_variant() == 0 && c8_dw == 0 &&
      lsec::jit::wants_pktnet(R, K, w) &&
      lsec::jit::pkt_aligned(in, K, out, R, w, packet))
    if (hipFunction_t fn = lsec::jit::ready(image, R, K)) {  // the bitmatrix's compiled packet network
      const hipError_t err = lsec::jit::launch_pkt(fn, R, K, in, out, nstripes, size, packet, w, st);
      if (err != hipSuccess) return fail("packet network launch failed: %s", hipGetErrorString(err));
      return 0;
    }
  const int rmax = kind == KBITMATRIX ? 2 : ((kind == KBITSLICEDW || kind == KWORDWISE) && w == 32) ? 4 : 8;
  const int rpr = image_rows_per_output(kind, w), unit = image_unit(kind, w);
  // input groups of at most kMaxK (grouped image layout); groups after the first accumulate
  for (int k0 = 0; k0 < K; k0 += lsec::kMaxK) {
    const int kg = std::min(lsec::kMaxK, K - k0);
    const size_t group_base = static_cast<size_t>(k0) * R * rpr * unit;  // earlier groups: kMaxK inputs each
    for (int r0 = 0; r0 < R; r0 += rmax) {
      lsec::ApplyArgs a;
      std::memset(&a, 0, sizeof(a));
      a.K = kg;
      a.R = std::min(rmax, R - r0);
      a.accumulate = k0 > 0;
      const size_t at = group_base + static_cast<size_t>(r0) * rpr * kg * unit;
      if (uses_u32_image(kind)) {  // w words per (row, input), or mask words per (bit-row, input)
        a.masks = static_cast<const uint32_t *>(image) + at;
        a.w = w;
      } else {
        a.cells = static_cast<const CoefCell *>(image) + at;
      }
      a.nstripes = nstripes;
      a.size = size;
      a.packet = packet;
      for (int j = 0; j < kg; ++j) a.in[j] = in[k0 + j];
      for (int r = 0; r < a.R; ++r) a.out[r] = out[r0 + r];
      // split very large batches so tile indices stay 32-bit
      const long long per = std::max(1LL, (1LL << 30) / std::max(1LL, size / 4096 + 1));
      for (int s0 = 0; s0 < nstripes; s0 += static_cast<int>(std::min<long long>(per, nstripes))) {
        lsec::ApplyArgs b = a;
        b.nstripes = static_cast<int>(std::min<long long>(per, nstripes - s0));
        for (int j = 0; j < kg; ++j) b.in[j].base = in[k0 + j].base + static_cast<uint64_t>(s0) * in[k0 + j].stride;
        for (int r = 0; r < b.R; ++r) b.out[r].base = out[r0 + r].base + static_cast<uint64_t>(s0) * out[r0 + r].stride;
        const hipError_t err = kind == KBYTEWISE    ? lsec::launch_bytewise(b, st)
                               : kind == KBITMATRIX ? lsec::launch_bitmatrix(b, st)
                               : kind == KWORDWISE  ? lsec::launch_wordwise(b, st)
                               : kind == KBITSLICEDW ? lsec::launch_gfw_bitsliced(b, st)
                                                    : lsec::launch_bitsliced(b, st, 0, c8_dw);
        if (err != hipSuccess) return fail("kernel launch failed: %s", hipGetErrorString(err));
      }
    }
  }
  return 0;
}

// ---------------------------------------------------------------- device-resident core
int encode_dev(PlanExt *e, const lsec_shard_t *sh, int nstripes, long long C, hipStream_t st) {
  lio_erasure_plan_t *p = &e->pub;
  if (check_geometry(p, C)) return -1;
  if (nstripes <= 0 || C == 0) return 0;
  const void *cells = nullptr;
  if (encode_cells(e, &cells)) return -1;
  const int k = p->data_strips;
  const int R = encode_rows(e);  // m (2 for r6, 1 for raid4)
  ShardRef in[kMaxDevs], out[kMaxDevs];
  for (int j = 0; j < k; ++j) in[j] = {reinterpret_cast<uint64_t>(sh[j].base), sh[j].stride};
  for (int r = 0; r < R; ++r) out[r] = {reinterpret_cast<uint64_t>(sh[k + r].base), sh[k + r].stride};
  return enqueue_apply(kernel_kind(p->method, p->w), cells, k, R, in, out, nstripes, C, p->packet_size, st, p->w);
}

// returns 0 (done or nothing to do) / -1
int decode_dev(PlanExt *e, const lsec_shard_t *sh, int nstripes, long long C, const int *erasures,
               hipStream_t st) {
  lio_erasure_plan_t *p = &e->pub;
  std::vector<int> ids;
  const int pr = parse_erasures(p, erasures, ids);
  if (pr < 0) return -1;
  if (pr == 1) return 0;
  if (check_geometry(p, C)) return -1;
  if (p->method == RAID4 && ids[0] >= p->data_strips) return 0;  // raid4.c:48 leaves lost parity alone
  if (nstripes <= 0 || C == 0) return 0;
  DecodeEntry *ent = nullptr;
  const void *cells = nullptr;
  if (decode_entry(e, ids, &ent, &cells)) return -1;
  const int k = p->data_strips;
  ShardRef in[kMaxDevs], out[kMaxDevs];
  for (int j = 0; j < k; ++j) {
    const lsec_shard_t &s = sh[ent->dp.survivors[j]];
    in[j] = {reinterpret_cast<uint64_t>(s.base), s.stride};
  }
  const int R = static_cast<int>(ent->dp.erased.size());
  for (int r = 0; r < R; ++r) {
    const lsec_shard_t &s = sh[ent->dp.erased[r]];
    out[r] = {reinterpret_cast<uint64_t>(s.base), s.stride};
  }
  return enqueue_apply(decode_kind(e, ent), cells, k, R, in, out, nstripes, C, p->packet_size, st, p->w);
}

}  // namespace eng

using namespace eng;

int set_error(const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  tl_err = buf;
  return -1;
}


void make_word_cell(uint32_t c, int w, uint32_t *out) {
  for (int b = 0; b < w; ++b, c = gfw::times_x(c, w)) out[b] = (w == 16) ? (c | (c << 16)) : c;
}

void make_cell(uint8_t c, CoefCell &cell) {
  uint8_t ta[8], tb[8], tc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int n = 0; n < 8; ++n) {
    ta[n] = gf8::mul(c, static_cast<uint8_t>(n));
    tb[n] = gf8::mul(c, static_cast<uint8_t>(n << 3));
    if (n < 4) tc[n] = gf8::mul(c, static_cast<uint8_t>(n << 6));
  }
  auto pack = [](const uint8_t *b) {
    return static_cast<uint32_t>(b[0]) | (static_cast<uint32_t>(b[1]) << 8) | (static_cast<uint32_t>(b[2]) << 16) |
           (static_cast<uint32_t>(b[3]) << 24);
  };
  cell.coef = c;
  cell.pad = 0;
  cell.ta_lo = pack(ta);
  cell.ta_hi = pack(ta + 4);
  cell.tb_lo = pack(tb);
  cell.tb_hi = pack(tb + 4);
  cell.tc_lo = pack(tc);
  cell.tc_hi = pack(tc + 4);
}
}  // namespace lsec

using namespace lsec::eng;

extern "C" {

int nearest_prime(int w, int which) {
  static const int primes[55] = {2,   3,   5,   7,   11,  13,  17,  19,  23,  29,  31,  37,  41,  43,
                                 47,  53,  59,  61,  67,  71,  73,  79,  83,  89,  97,  101, 103, 107,
                                 109, 113, 127, 131, 137, 139, 149, 151, 157, 163, 167, 173, 179, 181,
                                 191, 193, 197, 199, 211, 223, 227, 229, 233, 239, 241, 251, 257};
  // first prime >= w among primes[1..54]; which>0 -> it, which<0 -> the one below,
  // which==0 -> the closer of the two (ties go up)  (erasure_tools.c:50-77)
  for (int i = 1; i < 55; ++i) {
    if (w > primes[i]) continue;
    if (which > 0) return primes[i];
    if (which < 0) return primes[i - 1];
    return (w - primes[i - 1] < primes[i] - w) ? primes[i - 1] : primes[i];
  }
  return primes[54];
}

int et_method_type(char *meth) {
  if (!meth) return -1;
  for (int i = 0; i < N_JE_METHODS; ++i)
    if (strcasecmp(meth, JE_method[i]) == 0) return i;
  return -1;
}

lio_erasure_plan_t *et_new_plan(int method, long long int strip_size, int data_strips, int parity_strips, int w,
                                int packet_size, int base_unit) {
  if (method < 0 || method >= N_JE_METHODS) {
    fail("et_new_plan: invalid method %d", method);
    return nullptr;
  }
  PlanExt *e = static_cast<PlanExt *>(calloc(1, sizeof(PlanExt)));
  if (!e) return nullptr;
  e->magic = kPlanMagic;
  e->impl = new PlanImpl();
  lio_erasure_plan_t *p = &e->pub;
  p->method = method;
  p->strip_size = strip_size;
  p->data_strips = data_strips;
  p->parity_strips = parity_strips;
  p->w = w;
  p->base_unit = base_unit;
  p->packet_size = packet_size;
  if (method == RAID4) {
    p->form_encoding_matrix = fp_dummy;
    p->form_decoding_matrix = fp_dummy;
  } else {
    p->form_encoding_matrix = fp_form_encoding;
    p->form_decoding_matrix = fp_form_decoding;
  }
  p->encode_block = fp_encode_block;
  p->decode_block = fp_decode_block;
  return p;
}

void et_destroy_plan(lio_erasure_plan_t *p) {
  if (!p) return;
  PlanExt *e = ext_of(p);
  free(p->encode_matrix);
  free(p->encode_bitmatrix);
  if (p->encode_schedule) {
    int i = 0;
    for (; p->encode_schedule[i][0] != -1; ++i) free(p->encode_schedule[i]);
    free(p->encode_schedule[i]);
    free(p->encode_schedule);
  }
  if (e) {
    int cur = -1;
    (void)hipGetDevice(&cur);
    for (auto &kv : e->impl->enc_cells) {
      lsec::jit::unbind(kv.second);  // before the address can be handed out again
      (void)hipSetDevice(kv.first);
      (void)hipFree(kv.second);
    }
    for (auto &kv : e->impl->enc_dev_masks) {
      lsec::jit::unbind(kv.second);
      (void)hipSetDevice(kv.first);
      (void)hipFree(kv.second);
    }
    for (auto &ent : e->impl->decode_cache) {
      for (auto &kv : ent.second.dev_cells) {
        lsec::jit::unbind(kv.second);
        (void)hipSetDevice(kv.first);
        (void)hipFree(kv.second);
      }
      for (auto &kv : ent.second.dev_masks) {
        lsec::jit::unbind(kv.second);
        (void)hipSetDevice(kv.first);
        (void)hipFree(kv.second);
      }
    }
    if (cur >= 0) (void)hipSetDevice(cur);
    delete e->impl;
    e->magic = 0;
  }
  free(e ? static_cast<void *>(e) : static_cast<void *>(p));
}

lio_erasure_plan_t *et_generate_plan(long long int file_size, int method, int data_strips, int parity_strips, int w,
                                     int packet_low, int packet_high) {
  int base_unit = 8;
  if (w == -1) {  // auto word size (erasure_tools.c:746-776)
    switch (method) {
      case REED_SOL_R6_OP: case REED_SOL_VAN: case CAUCHY_ORIG: case CAUCHY_GOOD: case LIBER8TION:
        w = 8;
        break;
      case BLAUM_ROTH: w = nearest_prime(data_strips + 1, 1) - 1; break;
      case LIBERATION: w = nearest_prime(data_strips, 1); break;
      case RAID4: w = 8; base_unit = 1; break;
      default:
        fail("et_generate_plan: invalid method %d", method);
        return nullptr;
    }
  }
  // search range (erasure_tools.c:779-796)
  const long long approx = file_size / (static_cast<long long>(w) * base_unit * data_strips);
  const int plow = approx < 4 * 1024 ? static_cast<int>(approx / 4) : 512;
  const int phigh = approx < 4 * 1024 ? static_cast<int>(approx) : 4096;
  if (packet_low < 0) packet_low = plow;
  if (packet_high < 0) packet_high = phigh;
  if (packet_low > packet_high) {
    fail("et_generate_plan: packet_low > packet_high (%d > %d)", packet_low, packet_high);
    return nullptr;
  }
  packet_low = (packet_low / base_unit) * base_unit;
  packet_high = (packet_high / base_unit) * base_unit;
  // validation (erasure_tools.c:801-872)
  switch (method) {
    case REED_SOL_R6_OP:
      if (parity_strips != 2) { fail("%s needs parity_strips == 2", JE_method[method]); return nullptr; }
      [[fallthrough]];
    case REED_SOL_VAN: case CAUCHY_ORIG: case CAUCHY_GOOD:
      if (w != 8 && w != 16 && w != 32) { fail("%s needs w in {8,16,32}", JE_method[method]); return nullptr; }
      break;
    case BLAUM_ROTH:
      if (data_strips > w || nearest_prime(w + 1, 0) != w + 1 || packet_high % 8 != 0) {
        fail("blaum_roth: need k <= w, w+1 prime, packet %% 8 == 0");
        return nullptr;
      }
      break;
    case LIBERATION:
      if (data_strips > w || nearest_prime(w, 0) != w || packet_high % 8 != 0) {
        fail("liberation: need k <= w, w prime, packet %% 8 == 0");
        return nullptr;
      }
      break;
    case LIBER8TION:
      if (w != 8 || parity_strips != 2 || data_strips > w) { fail("liber8tion: need w == 8, m == 2, k <= 8"); return nullptr; }
      break;
    case RAID4:
      if (parity_strips != 1) { fail("raid4 needs parity_strips == 1"); return nullptr; }
      base_unit = 1;
      packet_low = 0;
      packet_high = 1;
      break;
    default:
      fail("et_generate_plan: invalid method %d", method);
      return nullptr;
  }
  // packet search: least padding, ties to the smaller packet, stop below 1 % (erasure_tools.c:876-896)
  long long best_excess = 10 * file_size, best_size = 0;
  int best_packet = -1;
  for (int ps = packet_high; ps > packet_low; ps -= base_unit) {
    const long long unit = static_cast<long long>(data_strips) * w * ps * base_unit;
    long long size = file_size;
    const long long rem = size % unit;
    if (rem > 0) size += unit - rem;
    const int excess = static_cast<int>(size - file_size);
    if (excess <= best_excess) {
      best_excess = excess;
      best_packet = ps;
      best_size = size;
      // `float increase = (1.0*j) / file_size * 100`: double arithmetic, then stored to a
      // float, which is what the < 1 test sees (erasure_tools.c:741, :893-894)
      const float increase = static_cast<float>((1.0 * excess) / file_size * 100);
      if (increase < 1) break;
    }
  }
  // Refused at plan time instead of failing on every block later (the segment maps a NULL plan
  // to -7 at exnode load, segment/jerasure.c:2237-2240):
  //  * packet codes asked for k equal chunks (file_size = k*C, what the segment passes,
  //    :2236) whose C is not a multiple of w * packet_size: the reference builds them, and its
  //    schedule encode then runs past the chunks (jerasure.c:1193-1207 walks strip_size > C
  //    bytes).  A file_size that is not k equal chunks is a file-tool request (et_encode pads
  //    the last strip to strip_size, erasure_tools.c:339-436) and keeps its padded plan.
  //  * plans no GPU kernel serves (there is no CPU path)
  const int kind = kernel_kind(method, w);
  if (kind == KNONE) {
    fail("et_generate_plan: %s at w=%d has no GPU kernel in this build", JE_method[method], w);
    return nullptr;
  }
  if (data_strips < 1 || parity_strips < 1 || data_strips + parity_strips > max_devs(method, w)) {
    fail("et_generate_plan: k=%d m=%d: k+m outside the engine's 2..%d at w=%d", data_strips, parity_strips,
         max_devs(method, w), w);
    return nullptr;
  }
  if (packet_kind(kind) && best_size != file_size && file_size % data_strips == 0) {
    fail("et_generate_plan: %s chunk %lld is not a multiple of w*packet_size = %d (the search padded %lld to %lld)",
         JE_method[method], file_size / data_strips, w * best_packet, file_size, best_size);
    return nullptr;
  }
  return et_new_plan(method, best_size / data_strips, data_strips, parity_strips, w, best_packet, base_unit);
}

// ---- file tools (erasure_tools.c:339-600): same file layout and padding ('0' bytes past EOF)
static size_t bread(char *buf, size_t n, FILE *f) {
  const size_t got = fread(buf, 1, n, f);
  if (got < n) memset(buf + got, '0', n - got);  // BLANK_CHAR, erasure_tools.c:37
  return n;
}

static int file_block(const lio_erasure_plan_t *p, int buffer_size) {
  const int unit = (p->data_strips + p->parity_strips) * p->w * p->packet_size * p->base_unit;
  if (unit <= 0) return -1;
  if (buffer_size == 0) buffer_size = 10 * 1024 * 1024;
  int j = buffer_size / unit;
  if (j == 0) j = 1;
  return j * unit / (p->data_strips + p->parity_strips);
}

int et_encode(lio_erasure_plan_t *plan, const char *fname, long long int foffset, const char *pname,
              long long int poffset, int buffer_size) {
  if (!ext_of(plan)) return fail("not an lstore_ec plan"), 1;
  FILE *fd = fopen(fname, "r");
  if (!fd) return fail("et_encode: cannot open %s", fname), 1;
  FILE *fp = fopen(pname, "r+");
  if (!fp) fp = fopen(pname, "w");
  if (!fp) { fclose(fd); return fail("et_encode: cannot open %s", pname), 1; }
  plan->form_encoding_matrix(plan);
  const int k = plan->data_strips, m = plan->parity_strips;
  const int block = file_block(plan, buffer_size);
  std::vector<char> buf(static_cast<size_t>(block) * (k + m));
  std::vector<char *> ptr(k + m);
  for (int i = 0; i < k + m; ++i) ptr[i] = buf.data() + static_cast<size_t>(i) * block;
  int rc = 0;
  for (long long rpos = 0, apos = foffset, ppos = poffset; rpos < plan->strip_size && rc == 0;
       rpos += block, apos += block, ppos += block) {
    const int bsize = static_cast<int>(std::min<long long>(block, plan->strip_size - rpos));
    for (int i = 0; i < k; ++i) {
      fseek(fd, apos + i * plan->strip_size, SEEK_SET);
      bread(ptr[i], bsize, fd);
    }
    if (encode_stripes_impl(ext_of(plan), ptr.data(), 1, bsize)) { rc = 1; break; }
    for (int i = 0; i < m; ++i) {
      fseek(fp, ppos + i * plan->strip_size, SEEK_SET);
      if (fwrite(ptr[k + i], 1, bsize, fp) != static_cast<size_t>(bsize)) rc = 1;
    }
  }
  fclose(fd);
  fclose(fp);
  return rc;
}

int et_decode(lio_erasure_plan_t *plan, long long int fsize, const char *fname, long long int foffset,
              const char *pname, long long int poffset, int buffer_size, int *erasures) {
  if (!ext_of(plan)) return fail("not an lstore_ec plan"), 1;
  const int k = plan->data_strips, m = plan->parity_strips;
  std::vector<int> missing(k + m, 0);
  int n = 0;
  for (; erasures[n] != -1; ++n) {
    if (erasures[n] < 0 || erasures[n] >= k + m) return fail("erasure id out of range"), 1;
    missing[erasures[n]] = 1;
  }
  if (n == 0) return 0;
  FILE *fd = fopen(fname, "r+");
  if (!fd) return fail("et_decode: cannot open %s", fname), 1;
  FILE *fp = fopen(pname, "r+");
  if (!fp) { fclose(fd); return fail("et_decode: cannot open %s", pname), 1; }
  plan->form_decoding_matrix(plan);
  const int block = file_block(plan, buffer_size);
  std::vector<char> buf(static_cast<size_t>(block) * (k + m));
  std::vector<char *> ptr(k + m);
  for (int i = 0; i < k + m; ++i) ptr[i] = buf.data() + static_cast<size_t>(i) * block;
  int rc = 0;
  for (long long rpos = 0, apos = foffset, ppos = poffset; rpos < plan->strip_size && rc == 0;
       rpos += block, apos += block, ppos += block) {
    const int bsize = static_cast<int>(std::min<long long>(block, plan->strip_size - rpos));
    for (int i = 0; i < k; ++i)
      if (!missing[i]) {
        fseek(fd, apos + i * plan->strip_size, SEEK_SET);
        bread(ptr[i], bsize, fd);
      }
    for (int i = 0; i < m; ++i)
      if (!missing[k + i]) {
        fseek(fp, ppos + i * plan->strip_size, SEEK_SET);
        if (fread(ptr[k + i], 1, bsize, fp) != static_cast<size_t>(bsize)) { rc = 1; break; }
      }
    if (rc) break;
    if (decode_stripes_impl(ext_of(plan), ptr.data(), 1, bsize, erasures)) { rc = 1; break; }
    for (int i = 0; i < k; ++i) {
      if (!missing[i]) continue;
      const long long bpos = apos + i * plan->strip_size;
      fseek(fd, bpos, SEEK_SET);
      // the last data strip is truncated to the file size (erasure_tools.c:576-582)
      const long long len = (i == k - 1 && bpos + bsize > fsize) ? fsize - bpos : bsize;
      if (len > 0 && fwrite(ptr[i], 1, len, fd) != static_cast<size_t>(len)) rc = 1;
    }
  }
  fclose(fd);
  fclose(fp);
  return rc;
}


int lsec_prepare_decode(lio_erasure_plan_t *plan, const int *erasures) {
  PlanExt *e = ext_of(plan);
  if (!e) return fail("not an lstore_ec plan");
  std::vector<int> ids;
  const int pr = parse_erasures(plan, erasures, ids);
  if (pr != 0) return pr < 0 ? -1 : 0;
  DecodeEntry *ent = nullptr;
  const void *cells = nullptr;
  if (decode_entry(e, ids, &ent, &cells)) return -1;
  (void)lsec::jit::wait(cells, 30000);  // a wide code's XOR network, if it has one
  return 0;
}

int lsec_prepare_encode(lio_erasure_plan_t *plan) {
  PlanExt *e = ext_of(plan);
  if (!e) return fail("not an lstore_ec plan");
  const void *cells = nullptr;
  if (encode_cells(e, &cells)) return -1;
  (void)lsec::jit::wait(cells, 30000);
  return 0;
}

int lsec_plan_jit(lio_erasure_plan_t *plan, const int *erasures) {
  PlanExt *e = ext_of(plan);
  if (!e) return 0;
  const int kind = kernel_kind(e->pub.method, e->pub.w);
  if (kind == KBYTEWISE ? lsec::bytewise_variant() != 0
                        : (kind == KWORDWISE || kind == KBITMATRIX || kind == KBITSLICEDW || kind == KBITSLICED)
                            ? lsec::bitsliced_variant() != 0
                            : true)
    return 0;
  const void *cells = nullptr;
  int R = 0;
  if (!erasures) {
    if (encode_cells(e, &cells)) return 0;
    R = encode_rows(e);
  } else {
    std::vector<int> ids;
    DecodeEntry *ent = nullptr;
    if (parse_erasures(plan, erasures, ids) != 0 || decode_entry(e, ids, &ent, &cells)) return 0;
    R = static_cast<int>(ent->dp.erased.size());
  }
  // Cauchy w = 8 shapes the bit-sliced kernel serves (at the plan's chunk size) run no network
  if (kind == KBITSLICED && plan->w == 8 && cauchy8_bitsliced_dw(plan->data_strips, R, plan->strip_size) > 0) return 0;
  return lsec::jit::ready(cells, R, plan->data_strips) != nullptr ? 1 : 0;
}

int lsec_plan_kernel(lio_erasure_plan_t *plan) { return plan ? kernel_kind(plan->method, plan->w) : 0; }

void lsec_set_kernel_variant(int bytewise_variant, int bitsliced_variant) {
  lsec::set_kernel_variant(bytewise_variant, bitsliced_variant);
}

void lsec_set_tile_sharing(int mode) { lsec::set_tile_mode(mode); }

int lsec_tile_sharing(void) { return lsec::tile_mode(); }

// Test hook, not in include/: device buffer of n u64 for the bytewise kernels' per-workgroup end
// times (s_memrealtime) in the following launches, or NULL to stop (tools/xcd_stamps.py).
void lsec_test_set_stamps(void *dev_buf, unsigned n) {
  lsec::set_launch_stamps(static_cast<unsigned long long *>(dev_buf), n);
}

// Test hook, not in include/: 1 = Cauchy at w = 8 on its compiled packet network wherever one exists,
// 0 = by shape (cauchy8_bitsliced_dw, the default).
void lsec_test_set_cauchy8_policy(int mode) { g_c8_policy.store(mode == 1 ? 1 : 0, std::memory_order_relaxed); }

// Test hook, not in include/: the XCD tile phase for the following launches, bit 0 the tile loops,
// bit 1 the compiled networks (lsec::tile_phase_on; LSEC_TILE_PHASE sets the start value, 1), for
// A/B runs in one allocation.
void lsec_test_set_tile_phase(int mode) { lsec::set_tile_phase(mode); }


// Self-test of the bitmatrix decode planner (test hook, not in include/; no GPU): for the
// liberation-family plan (method, k, w) with m = 2, make_bit_decode's masks must equal those of
// the whole-bitmatrix inversion (make_bit_decode_dense) for every erasure pattern of one and two
// devices.  Returns the number of patterns compared, or -1 with a message.
int lsec_selftest_bit_decode(int method, int k, int w) {
  std::vector<int> bm = method == LIBERATION   ? lsec::gf8::liberation_bitmatrix(k, w)
                        : method == BLAUM_ROTH ? lsec::gf8::blaum_roth_bitmatrix(k, w)
                        : method == LIBER8TION ? lsec::gf8::liber8tion_bitmatrix(k)
                                               : std::vector<int>();
  if (bm.empty()) return fail("lsec_selftest_bit_decode: no %d bitmatrix for k=%d w=%d", method, k, w);
  const int m = 2;
  int n = 0;
  for (int a = 0; a < k + m; ++a)
    for (int b = a; b < k + m; ++b) {
      std::vector<int> ids = a == b ? std::vector<int>{a} : std::vector<int>{a, b};
      lsec::gf8::DecodePlan p1, p2;
      std::vector<uint32_t> m1, m2;
      const bool ok1 = lsec::gf8::make_bit_decode(k, m, w, bm, ids, p1, m1);
      const bool ok2 = lsec::gf8::make_bit_decode_dense(k, m, w, bm, ids, p2, m2);
      if (ok1 != ok2 || p1.survivors != p2.survivors || p1.erased != p2.erased || m1 != m2)
        return fail("lsec_selftest_bit_decode: erasures {%d, %d} differ (ok %d/%d)", a, b, ok1, ok2);
      ++n;
    }
  return n;
}

}  // extern "C"
