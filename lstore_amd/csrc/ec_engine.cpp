// ec_engine.cpp -- the C ABI of liblstore_ec.so (include/lstore_ec.h).
//
// Layers:
//   plan service     et_* entry points and the plan struct's fn-pointers, with the same
//                    arguments, return codes and struct contents as src/lio/erasure_tools.c
//   matrix images    per (plan, device) coefficient cells for the encode matrix and, per
//                    erasure pattern, for the decode matrix (built once, cached)
//   submission       device-resident calls enqueue one kernel per <=8 output shards on the
//                    caller's stream; host-memory calls go through a pooled, double-buffered
//                    pinned staging pipeline (pack -> H2D -> kernel -> D2H -> unpack)
//
// There is no CPU compute path: every byte of parity or recovered data is produced by the
// HIP kernels in ec_kernels.hip.  If the GPU is unavailable the calls fail (status -1, or
// abort() from the void encode_block fn-pointer).
#include <hip/hip_runtime.h>
#include <linux/futex.h>
#include <pthread.h>
#include <sched.h>
#include <strings.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdarg>
#include <climits>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <random>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/lstore_ec.h"
#include "ec_host.h"
#include "ec_jit.h"
#include "ec_numa.h"
#include "ec_kernels.h"
#include "ec_server.h"
#include "gf8.h"

using lsec::CoefCell;
using lsec::ShardRef;

extern "C" const char *JE_method[N_JE_METHODS] = {"reed_sol_van", "reed_sol_r6_op", "cauchy_orig", "cauchy_good",
                                                  "blaum_roth",   "liberation",     "liber8tion",  "raid4"};

namespace {

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

#define HIP_OK(expr)                                                                             \
  do {                                                                                           \
    hipError_t e_ = (expr);                                                                      \
    if (e_ != hipSuccess) return fail("%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, __LINE__); \
  } while (0)

enum KernelKind { KNONE = 0, KBYTEWISE = 1, KBITSLICED = 2, KBITMATRIX = 3, KWORDWISE = 4, KBITSLICEDW = 5 };

// devices per stripe: Jerasure takes k + m <= 2^w (reed_sol.c:247-248, cauchy.c:139), 256 at w = 8.
// The engine takes that at w = 8 and for the bitmatrix codes (LSEC_MAX_DEVS), and up to
// kMaxDevs = 1024 for the GF(2^16) / GF(2^32) matrix codes (RS, r6, Cauchy); the segment adapters
// keep LSEC_MAX_DEVS, which sizes their ABI structs.  Inputs beyond lsec::kMaxK per launch run as
// several launches over the grouped image layout (ec_kernels.h).
constexpr int kMaxDevs = LSEC_MAX_DEVS_WIDE;
int max_devs(int method, int w) {
  const bool matrix = method == REED_SOL_VAN || method == REED_SOL_R6_OP || method == CAUCHY_ORIG || method == CAUCHY_GOOD;
  return matrix && (w == 16 || w == 32) ? kMaxDevs : LSEC_MAX_DEVS;
}

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
  if (kernel_kind(e->pub.method, e->pub.w) == KBYTEWISE)  // wide codes: an XOR network, compiled in the background
    lsec::jit::bind(d, e->impl->coding.data(), rows, k);
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
    if (!ent.xor_only && kernel_kind(e->pub.method, e->pub.w) == KBYTEWISE)
      lsec::jit::bind(d, ent.dp.rows.data(), static_cast<int>(ent.dp.erased.size()), e->pub.data_strips);
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

// Enqueue out[r] = rows[r] . in  for every stripe, splitting R into launches of <= 8 rows
// (<= 2 for the bitmatrix kernel) and K into groups of <= lsec::kMaxK inputs.  `image` is the
// CoefCell[R][K] matrix image, the uint32 row masks [((r*w+l)*K + j)*NW + q] (KBITMATRIX) or the
// word products [(r*K + j)*w + b] (KWORDWISE / KBITSLICEDW), grouped when K > kMaxK.
int enqueue_apply(int kind, const void *image, int K, int R, const ShardRef *in, const ShardRef *out,
                  int nstripes, long long size, int packet, hipStream_t st, int w = 8) {
  const bool net = kind == KBYTEWISE   ? lsec::bytewise_variant() == 0 && lsec::jit::wants_xornet(R, K)
                   : kind == KWORDWISE ? lsec::bitsliced_variant() == 0 && lsec::jit::wants_gfw_net(R, K, w)
                                       : false;
  ShardRef tin[lsec::kMaxK], tout[lsec::kMaxR];  // a w = 16 / 32 network's ragged tail, below
  if (net) {
    if (hipFunction_t fn = lsec::jit::ready(image, R, K)) {  // the matrix's compiled XOR network
      // w = 16 / 32 networks take whole tiles only: the tail columns go to the generic kernel
      const long long whole = kind == KWORDWISE ? size / lsec::jit::gfw_tile(w) * lsec::jit::gfw_tile(w) : size;
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
                                                    : lsec::launch_bitsliced(b, st);
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

// ---------------------------------------------------------------- host copy pool
// Host-memory callers hand over pageable buffers (cache pages, parity on the stack,
// segment/jerasure.c:1315), so bytes must be packed into pinned staging before DMA.  One
// CPU thread copies ~10 GB/s, well below PCIe Gen5, so packing/unpacking is spread over a
// small process-wide worker pool (LSEC_COPY_THREADS, default min(8, cores)); the calling
// thread works too.
struct CopyJob {
  char *dst;
  const char *src;
  size_t bytes;
};

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

// LSEC_NT_COPY=0: plain memcpy instead of streaming stores for the host copies (A/B runs)
bool nt_copies() {
  static const bool on = [] {
    const char *v = getenv("LSEC_NT_COPY");
    return !v || *v != '0';
  }();
  return on;
}

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
    const char *s = getenv("LSEC_COPY_THREADS");
    const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
    const int n = s ? atoi(s) : static_cast<int>(std::min(8u, hw));
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
    if (hipGetDeviceCount(&n) != hipSuccess) (void)hipGetLastError();
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
    size_t cap = 0;
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

void release_staging(Staging *s) {
  std::lock_guard<std::mutex> lk(g_pool_mu);
  g_pool[s->dev].push_back(s);
}

size_t staging_budget() {
  static size_t b = [] {
    const char *s = getenv("LSEC_STAGING_MB");
    const long v = s ? atol(s) : 128;
    return static_cast<size_t>(std::max(1L, v)) << 20;
  }();
  return b;
}

// Slots are sized for a full batch (half the staging budget) the first time, so that a
// small first call does not leave them too small for the next one: re-pinning 64 MiB of
// host memory costs more than moving it over PCIe.  need_host = false (pinned callers, see
// below) allocates only the device half.
int ensure_slot(Staging::Slot &sl, size_t bytes, bool need_host = true) {
  if (sl.cap >= bytes && (sl.h || !need_host)) return 0;
  if (sl.d) (void)hipFree(sl.d);
  if (sl.h) (void)hipHostFree(sl.h);
  sl.d = nullptr;
  sl.h = nullptr;
  sl.cap = 0;
  const size_t cap = std::max(bytes, staging_budget() / 2);
  HIP_OK(hipMalloc(&sl.d, cap));
  if (need_host) HIP_OK(hipHostMalloc(reinterpret_cast<void **>(&sl.h), cap, hipHostMallocDefault));
  sl.cap = cap;
  return 0;
}

std::atomic<unsigned long long> g_st_queries{0};  // runtime pointer queries (LSEC_STATS)

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
thread_local int tl_memo_depth = 0;
thread_local std::vector<std::pair<const void *, PtrInfo>> tl_memo;

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

PtrInfo query_ptr(const void *ptr) {
  if (tl_memo_depth > 0)
    for (const auto &kv : tl_memo)
      if (kv.first == ptr) return kv.second;
  PtrInfo r;
  hipPointerAttribute_t attr;
  g_st_queries.fetch_add(1, std::memory_order_relaxed);
  if (hipPointerGetAttributes(&attr, ptr) == hipSuccess) {
    r.ok = true;
    r.type = attr.type;
    r.dev = attr.devicePointer;
  } else {
    (void)hipGetLastError();  // pageable host memory reports an error on some runtimes
  }
  if (tl_memo_depth > 0 && tl_memo.size() < 64) tl_memo.push_back({ptr, r});  // small: scanned linearly
  return r;
}

// Caller buffers that are already page-locked (hipHostMalloc'd, or hipHostRegister'ed by an
// allocator that pins its cache pages) need no packing: the DMA engines copy straight
// between them and the device slots, and the host copy pool stays idle.
bool is_pinned_host(const void *ptr) {
  const PtrInfo i = query_ptr(ptr);
  return i.ok && i.type == hipMemoryTypeHost;
}

// every staged shard of the first and last stripe pinned?  (a stray pageable pointer in
// between stays correct -- hipMemcpyAsync accepts pageable memory too, only slower)
// Ranges pinned in place by a running call (InPlacePin), page-rounded.  Another call that
// touches them must not take them for caller-pinned memory: the owner unregisters them when
// it returns, maybe while the other call's DMA is still queued.
std::mutex g_inplace_mu;
std::vector<std::pair<uintptr_t, uintptr_t>> g_inplace;

constexpr uintptr_t kPage = 4096;

bool inplace_overlaps_locked(uintptr_t lo, uintptr_t hi) {
  for (const auto &r : g_inplace)
    if (lo < r.second && r.first < hi) return true;
  return false;
}

// Caller page-locked buffers.  pinned: every staged chunk of the first and last stripe is
// page-locked (a stray pageable chunk in between stays correct -- hipMemcpyAsync accepts
// pageable memory too, only slower).  by_kernel (asked with kernel_ok): small runs, and EVERY
// chunk checked to have a device address -- see caller_pinned_aliases.  The whole decision is
// one pass under g_inplace_mu, with every chunk's page range checked against the in-flight
// in-place registrations first: a range a concurrent InPlacePin has claimed (it claims before
// it registers and releases after it unregisters) is never taken for caller-pinned memory,
// since its owner may unregister it while this call's DMA or copy kernel still reads it.
// A page-locked allocation a call has verified: [lo, hi) host bytes, device alias = host + delta.
// A chunk inside one needs no further runtime query (each takes a runtime lock; a page-locked
// per-stripe call made ~11 of them under g_inplace_mu: RS(6+3) 16 KiB at 128 threads spent
// 430 us of its 450 us in this set-up, profiles/r02_v45_zc_phases.txt).
struct PinnedAlloc {
  uintptr_t lo, hi;
  intptr_t delta;
};

// p..p+len inside one page-locked allocation with a device alias?  (its device address in *dev)
bool pinned_chunk(const char *p, size_t len, std::vector<PinnedAlloc> &seen, uint64_t *dev) {
  const uintptr_t u = reinterpret_cast<uintptr_t>(p);
  for (const PinnedAlloc &a : seen)
    if (u >= a.lo && u + len <= a.hi) {
      *dev = static_cast<uint64_t>(static_cast<intptr_t>(u) + a.delta);
      return true;
    }
  const PtrInfo i = query_ptr(p);
  if (!i.ok || i.type != hipMemoryTypeHost || !i.dev) return false;
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  if (hipMemGetAddressRange(&base, &size, reinterpret_cast<hipDeviceptr_t>(const_cast<char *>(p))) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  const uintptr_t lo = reinterpret_cast<uintptr_t>(base), hi = lo + size;
  if (u < lo || u + len > hi) return false;
  const intptr_t delta = reinterpret_cast<intptr_t>(i.dev) - static_cast<intptr_t>(u);
  seen.push_back({lo, hi, delta});
  *dev = reinterpret_cast<uint64_t>(i.dev);
  return true;
}

bool caller_pinned_aliases(char **ptrs, int nstripes, int km, const std::vector<int> &in_ids,
                           const std::vector<int> &out_ids, long long C, std::vector<PinnedAlloc> &seen,
                           std::vector<uint64_t> &dev);

struct CallerPinned {
  bool pinned = false, by_kernel = false;
  std::vector<uint64_t> dev;  // by_kernel: device address of every chunk (caller_pinned_aliases order)
};

CallerPinned caller_pinned(char **ptrs, int nstripes, int km, const std::vector<int> &in_ids, const std::vector<int> &out_ids,
                           long long C, bool kernel_ok) {
  CallerPinned r;
  // A first chunk that is not page-locked settles it, with no lock: every path below returns
  // "not pinned" for it too, and taking memory for pageable is always safe.  (Per-stripe calls
  // from hundreds of threads queued on this mutex.)
  if (nstripes >= 1 && tl_memo_depth > 0)
    for (const auto &kv : tl_memo)  // a chunk of this call already known not to be page-locked
      if (!kv.second.ok || kv.second.type != hipMemoryTypeHost)
        for (const std::vector<int> *ids : {&in_ids, &out_ids})
          for (int id : *ids)
            if (ptrs[id] == kv.first) return r;
  if (!in_ids.empty() && nstripes >= 1 && !is_pinned_host(ptrs[in_ids[0]])) return r;
  std::lock_guard<std::mutex> lk(g_inplace_mu);
  if (!g_inplace.empty()) {
    for (int s = 0; s < nstripes; ++s)
      for (const std::vector<int> *ids : {&in_ids, &out_ids})
        for (int id : *ids) {
          const uintptr_t a = reinterpret_cast<uintptr_t>(ptrs[static_cast<size_t>(s) * km + id]);
          if (inplace_overlaps_locked(a & ~(kPage - 1), (a + static_cast<uintptr_t>(C) + kPage - 1) & ~(kPage - 1))) return r;
        }
  }
  std::vector<PinnedAlloc> seen;
  uint64_t d = 0;
  for (int s : {0, nstripes - 1}) {
    for (int id : in_ids)
      if (!pinned_chunk(ptrs[static_cast<size_t>(s) * km + id], static_cast<size_t>(C), seen, &d)) return r;
    for (int id : out_ids)
      if (!pinned_chunk(ptrs[static_cast<size_t>(s) * km + id], static_cast<size_t>(C), seen, &d)) return r;
  }
  r.pinned = true;
  r.by_kernel = kernel_ok && caller_pinned_aliases(ptrs, nstripes, km, in_ids, out_ids, C, seen, r.dev);
  return r;
}

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
  bool pin(char **ptrs, int nstripes, int km, const std::vector<int> &in_ids, const std::vector<int> &out_ids,
           long long C) {
    static const bool off = getenv("LSEC_NO_HOST_REGISTER") != nullptr;
    if (off) return false;
    std::vector<std::pair<char *, char *>> pieces;
    pieces.reserve(static_cast<size_t>(nstripes) * (in_ids.size() + out_ids.size()));
    for (int s = 0; s < nstripes; ++s) {
      for (int id : in_ids) pieces.push_back({ptrs[static_cast<size_t>(s) * km + id], ptrs[static_cast<size_t>(s) * km + id] + C});
      for (int id : out_ids) pieces.push_back({ptrs[static_cast<size_t>(s) * km + id], ptrs[static_cast<size_t>(s) * km + id] + C});
    }
    std::sort(pieces.begin(), pieces.end());
    std::vector<std::pair<char *, char *>> regions;
    for (const auto &pc : pieces) {
      if (!regions.empty() && pc.first < regions.back().second) return false;  // overlapping chunks
      if (!regions.empty() && pc.first == regions.back().second)
        regions.back().second = pc.second;
      else
        regions.push_back(pc);
      if (regions.size() > kMaxRegions) return false;
    }
    size_t total = 0;
    for (const auto &r : regions) total += static_cast<size_t>(r.second - r.first);
    if (total < kMinBytes) return false;  // packing a small batch is cheaper than the syscalls
    // Each DMA from registered pageable memory has a fixed cost on top of the bytes, so pin
    // only when the copies the pinned path will issue (one per run of host-contiguous chunks,
    // stripe by stripe) average >= 2.5 MiB; smaller runs pack faster.  Round 1's 4 MiB had
    // every single-erasure decode below C = 2 MiB packing (RS(6+3) 1 MiB decode: 3.5 MiB runs,
    // 31 GiB/s packed, 37-46 pinned).  An in-process A/B (tools/pin_run_ab.py,
    // profiles/r02_v27_pin_run_ab.jsonl) put the break-even near 800 KiB, but the c5 sweep
    // with that threshold (r02_v38_sweep_c5.jsonl vs r02_v25) lost up to half the rate at
    // 1.5-2.25 MiB runs (RS(6+3) 256 KiB encode 32 -> 16, 512 KiB 29 -> 22.5) while runs of
    // 2.75 MiB and up gained (RS(10+4) 512 KiB decode 30 -> 40).
    size_t runs = 0;
    for (const std::vector<int> *ids : {&in_ids, &out_ids}) {
      const char *end = nullptr;
      for (int s = 0; s < nstripes; ++s)
        for (int id : *ids) {
          const char *b = ptrs[static_cast<size_t>(s) * km + id];
          if (b != end) ++runs;
          end = b + C;
        }
    }
    if (runs == 0) return false;
    if (total / runs < min_run()) return false;
    {
      // claim the page-rounded regions, so a concurrent call over the same pages packs
      std::lock_guard<std::mutex> lk(g_inplace_mu);
      for (const auto &r : regions) {
        const uintptr_t lo = reinterpret_cast<uintptr_t>(r.first) & ~(kPage - 1);
        const uintptr_t hi = (reinterpret_cast<uintptr_t>(r.second) + kPage - 1) & ~(kPage - 1);
        if (inplace_overlaps_locked(lo, hi)) {
          claimed_.clear();
          return false;
        }
        claimed_.push_back({lo, hi});
      }
      for (size_t i = 1; i < claimed_.size(); ++i)
        if (claimed_[i].first < claimed_[i - 1].second) {  // two (sorted) regions share a page
          claimed_.clear();
          return false;
        }
      g_inplace.insert(g_inplace.end(), claimed_.begin(), claimed_.end());
    }
    // whole pages (the claims above are page-rounded and disjoint)
    for (const auto &r : regions) {
      char *lo = reinterpret_cast<char *>(reinterpret_cast<uintptr_t>(r.first) & ~(kPage - 1));
      char *hi = reinterpret_cast<char *>((reinterpret_cast<uintptr_t>(r.second) + kPage - 1) & ~(kPage - 1));
      if (hipHostRegister(lo, static_cast<size_t>(hi - lo), hipHostRegisterPortable | hipHostRegisterMapped) != hipSuccess) {
        (void)hipGetLastError();
        release();
        return false;
      }
      held_.push_back(lo);
    }
    return true;
  }
  void release() {
    for (char *b : held_)
      if (hipHostUnregister(b) != hipSuccess) {
        (void)hipGetLastError();
        static std::atomic<bool> told{false};
        if (!told.exchange(true)) fprintf(stderr, "liblstore_ec: hipHostUnregister(%p) failed\n", static_cast<void *>(b));
      }
    held_.clear();
    if (claimed_.empty()) return;
    std::lock_guard<std::mutex> lk(g_inplace_mu);
    for (const auto &c : claimed_) {
      auto it = std::find(g_inplace.begin(), g_inplace.end(), c);
      if (it != g_inplace.end()) g_inplace.erase(it);
    }
    claimed_.clear();
  }

 private:
  static constexpr size_t kMaxRegions = 1024;
  static constexpr size_t kMinBytes = 8ull << 20;
  static constexpr size_t kMinRun = 2560ull << 10;
  // LSEC_PIN_MIN_RUN_KB overrides kMinRun (read per call: measurement A/B runs)
  static size_t min_run() {
    const char *s = getenv("LSEC_PIN_MIN_RUN_KB");
    return s && *s ? static_cast<size_t>(strtoull(s, nullptr, 10)) << 10 : kMinRun;
  }
  std::vector<char *> held_;
  std::vector<std::pair<uintptr_t, uintptr_t>> claimed_;
};

// DMA runs: pieces whose source and destination both continue the previous piece merge
// into one copy (LStore's k data chunks of a stripe sit back to back in one cache page, so
// a stripe's inputs usually become a single k*C transfer)
struct DmaRun {
  char *dst;
  const char *src;
  size_t bytes;
};

void add_run(std::vector<DmaRun> &v, char *dst, const char *src, size_t n) {
  if (!v.empty() && v.back().dst + v.back().bytes == dst && v.back().src + v.back().bytes == src)
    v.back().bytes += n;
  else
    v.push_back({dst, src, n});
}

// kernel transport pieces of one chunk (addresses already device-visible)
// (returns 0 when either address is 0 -- a host byte outside the pinned regions -- so the
// caller stops before launching)
size_t add_pieces(lsec::CopyPiece *pl, size_t n, uint64_t src, uint64_t dst, size_t len) {
  if (src == 0 || dst == 0) return 0;
  for (size_t o = 0; o < len; o += lsec::kPieceBytes) pl[n++] = {src + o, dst + o, std::min<uint64_t>(lsec::kPieceBytes, len - o)};
  return n;
}

// Kernel transport policy, LSEC_KERNEL_COPY read per call:
//   unset  caller page-locked buffers with small runs move by kernel (DMA of their 384 KiB runs
//          moves 17-20 GiB/s at C = 64 KiB, the kernel 30 / 38: profiles/r01_v28_kcopy_pinned.txt);
//          pageable batches with small runs are packed
//   0      never
// (Until round 3, `1` also pinned pageable batches in place for the copy kernel; kernels over
// per-call registrations of pageable pages are gone, see InPlacePin.)
enum class KernelCopy { kNever, kCallerPinned };
KernelCopy kernel_copy_policy() {
  const char *on = getenv("LSEC_KERNEL_COPY");
  return on && *on == '0' ? KernelCopy::kNever : KernelCopy::kCallerPinned;
}

// every transferred chunk (and column block) 16-byte aligned, as the copy-piece kernel needs
bool kernel_transport_aligned(char **ptrs, int nstripes, int km, const std::vector<int> &in_ids,
                              const std::vector<int> &out_ids, long long C, long long cb) {
  if (C % 16 != 0 || cb % 16 != 0) return false;
  for (int s = 0; s < nstripes; ++s)
    for (const std::vector<int> *ids : {&in_ids, &out_ids})
      for (int id : *ids)
        if (reinterpret_cast<uintptr_t>(ptrs[static_cast<size_t>(s) * km + id]) % 16 != 0) return false;
  return true;
}

// Caller page-locked buffers with small runs (average < 1 MiB: DMA of 384 KiB runs from
// hipHostMalloc memory moves ~20 GiB/s, profiles/r01_v27_kernel_copy_ab.txt) move by kernel,
// once EVERY chunk is checked: page-locked, inside one allocation, with a device address
// (a pageable chunk between pinned ones is harmless to a DMA but would fault a kernel).  The
// check costs ~0.06 us per chunk (tools/probes/pinned_attr_probe.cpp).  dev[i] gets the device
// address of chunk i, in the order stripe, then in_ids, then out_ids.
// (called by caller_pinned with g_inplace_mu held)
bool caller_pinned_aliases(char **ptrs, int nstripes, int km, const std::vector<int> &in_ids,
                           const std::vector<int> &out_ids, long long C, std::vector<PinnedAlloc> &seen,
                           std::vector<uint64_t> &dev) {
  size_t runs = 0, total = 0;
  for (const std::vector<int> *ids : {&in_ids, &out_ids}) {
    const char *end = nullptr;
    for (int s = 0; s < nstripes; ++s)
      for (int id : *ids) {
        const char *b = ptrs[static_cast<size_t>(s) * km + id];
        if (b != end) ++runs;
        end = b + C;
        total += static_cast<size_t>(C);
      }
  }
  if (runs == 0 || total / runs >= (1ull << 20)) return false;
  dev.clear();
  dev.reserve(static_cast<size_t>(nstripes) * (in_ids.size() + out_ids.size()));
  for (int s = 0; s < nstripes; ++s)
    for (const std::vector<int> *ids : {&in_ids, &out_ids})
      for (int id : *ids) {
        uint64_t d = 0;
        if (!pinned_chunk(ptrs[static_cast<size_t>(s) * km + id], static_cast<size_t>(C), seen, &d)) return false;
        dev.push_back(d);
      }
  return true;
}

void split_pieces(std::vector<lsec::CopyPiece> &v, uint64_t src, uint64_t dst, size_t len) {
  for (size_t o = 0; o < len; o += lsec::kPieceBytes) v.push_back({src + o, dst + o, std::min<uint64_t>(lsec::kPieceBytes, len - o)});
}

hipError_t issue_runs(const std::vector<DmaRun> &v, hipMemcpyKind kind, hipStream_t st) {
  for (const DmaRun &r : v) {
    const hipError_t e = hipMemcpyAsync(r.dst, r.src, r.bytes, kind, st);
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
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
             const std::vector<int> &out_ids, const void *cells, int kind, uint8_t *magic_host = nullptr) {
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
  const size_t budget = staging_budget();
  const size_t per_col = static_cast<size_t>(nin + nout);  // staging bytes per column byte
  long long cb = C;
  if (per_col * C > budget / 2) {
    // packet codes must cut at super-packet boundaries (w * P bytes)
    const long long align = packet_kind(kind) ? static_cast<long long>(p->w) * p->packet_size : 8192;
    cb = static_cast<long long>(budget / 2 / per_col) / align * align;
    if (cb < align) cb = align;
    if (cb >= C) cb = C;
  }
  const int nb_max = cb < C ? 1 : static_cast<int>(std::max<size_t>(1, std::min<size_t>(nstripes, budget / 2 / (per_col * C))));
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
  const bool pinned = caller_pinned || inplace.pin(ptrs, nstripes, km, in_ids, out_ids, C);
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
  const size_t slot_bytes = per_col * static_cast<size_t>(cb) * nb_max;
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
    CopyPool::get().run(jobs);
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
          if (hipHostMalloc(reinterpret_cast<void **>(&sl.pl), cap * sizeof(lsec::CopyPiece), hipHostMallocDefault) !=
              hipSuccess) {
            (void)hipGetLastError();
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
        err = lsec::launch_copy_pieces(sl.pl, static_cast<int>(npin), stg->s_in);
      } else if (pinned) {
        runs.clear();
        for (int s = 0; s < nb; ++s)
          for (int j = 0; j < nin; ++j)
            add_run(runs, sl.d + (static_cast<size_t>(s) * nin + j) * len, ptrs[static_cast<size_t>(s0 + s) * km + in_ids[j]] + c0,
                    len);
        err = issue_runs(runs, hipMemcpyHostToDevice, stg->s_in);
      } else {
        jobs.clear();
        for (int s = 0; s < nb; ++s)
          for (int j = 0; j < nin; ++j)
            jobs.push_back({sl.h + (static_cast<size_t>(s) * nin + j) * len,
                            ptrs[static_cast<size_t>(s0 + s) * km + in_ids[j]] + c0, len});
        CopyPool::get().run(jobs);
        err = hipMemcpyAsync(sl.d, sl.h, in_bytes, hipMemcpyHostToDevice, stg->s_in);
      }
      if (err == hipSuccess) err = hipEventRecord(sl.in_done, stg->s_in);
      if (err == hipSuccess) err = hipStreamWaitEvent(stg->s_out, sl.in_done, 0);
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
  if (trace && rc == 0) {  // every slot drained: no transfer still reads or writes the pins
    const auto t_rel0 = now();
    inplace.release();  // (the destructor would, after this print)
    const auto t_end = now();
    fprintf(stderr, "[lsec trace] host call %d stripes, %d in / %d out x %lld B (%s): pin %.2f ms, submit %.2f ms, "
                    "drain %.2f ms, unpin %.2f ms\n",
            nstripes, nin, nout, C, by_kernel ? "kernel transport" : pinned ? "pinned DMA" : "packed", ms(t_pin0, t_loop0),
            ms(t_loop0, t_drain0), ms(t_drain0, t_rel0), ms(t_rel0, t_end));
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

bool is_device_ptr(const void *ptr) {
  const PtrInfo i = query_ptr(ptr);
  return i.ok && (i.type == hipMemoryTypeDevice || i.type == hipMemoryTypeManaged);
}

// all k+m pointers of every stripe device memory?  then describe them as shard refs
// Returns 1 (device layout in sh), 0 (host memory), -1 (device and host pointers mixed, or an
// irregular device stride: refused rather than guessed).  A batch whose first chunk is device
// memory has every chunk of its first and last stripe checked; a multi-stripe batch whose first
// chunk is host memory has the last chunk of its first and last stripe checked, and a single
// stripe whose first chunk is host memory nothing more (each check is a query under a runtime
// lock that per-stripe calls contend on; a device pointer among host chunks faults the host
// copy, as it faults the reference's CPU code).
int device_layout(const lio_erasure_plan_t *p, char **ptrs, int nstripes, std::vector<lsec_shard_t> &sh) {
  const int km = p->data_strips + p->parity_strips;
  if (!is_device_ptr(ptrs[0])) {
    // A single-stripe call (LStore's per-stripe fn-pointer path) stops at its first chunk:
    // every extra query is a turn on a runtime lock that spins, and at 128 threads on 16 CPUs
    // one extra query per call cut 16 KiB decodes from 30.2 to 3.2-5.3 GiB/s with the CPU quota
    // spent spinning (profiles/r02_v32_zc_decode2.txt).
    if (nstripes == 1) return 0;
    for (int s : {0, nstripes - 1})
      for (int i : {0, km - 1})
        if (is_device_ptr(ptrs[static_cast<size_t>(s) * km + i])) return fail("stripe pointers mix device and host memory");
    return 0;
  }
  for (int s : {0, nstripes - 1})
    for (int i = 0; i < km; ++i)
      if (!is_device_ptr(ptrs[static_cast<size_t>(s) * km + i])) return fail("stripe pointers mix device and host memory");
  sh.resize(km);
  for (int i = 0; i < km; ++i) {
    sh[i].base = ptrs[i];
    sh[i].stride = nstripes > 1 ? static_cast<long long>(ptrs[km + i] - ptrs[i]) : 0;
  }
  for (int s = 2; s < nstripes; ++s)  // require a regular stride (one layout descriptor)
    for (int i = 0; i < km; ++i)
      if (ptrs[static_cast<size_t>(s) * km + i] != ptrs[i] + s * sh[i].stride)
        return fail("device stripe pointers are not regularly strided (stripe %d, shard %d)", s, i);
  return 1;
}

hipStream_t thread_stream() {
  // per-thread stream for the synchronous fn-pointer entry points, destroyed when the thread
  // exits (a caller that churns threads does not accumulate streams)
  struct Streams {
    std::map<int, hipStream_t> by_dev;
    ~Streams() {
      for (auto &kv : by_dev) (void)hipStreamDestroy(kv.second);
    }
  };
  static thread_local Streams streams;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  auto it = streams.by_dev.find(dev);
  if (it != streams.by_dev.end()) return it->second;
  hipStream_t s = nullptr;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return nullptr;
  streams.by_dev[dev] = s;
  return s;
}

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

size_t coalesce_limit() {  // per-request bytes below which calls go through the dispatcher
  static size_t b = [] {
    const char *s = getenv("LSEC_COALESCE_MB");
    return static_cast<size_t>(std::max(0L, s ? atol(s) : 16)) << 20;
  }();
  return b;
}

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

  static constexpr size_t kBatchBudget = 96u << 20;  // bytes packed per dispatcher batch

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
      CopyPool::get().run(jobs);
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
      const size_t cap = std::max({total, std::min(2 * sl.cap, kBatchBudget + (1u << 20)), size_t(32u << 20)});
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
    CopyPool::get().run(jobs);
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
        while (!q_.empty() && (batch.empty() || bytes + q_.front()->bytes() <= kBatchBudget)) {
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

// ---------------------------------------------------------------- zero-copy small calls
// LStore calls encode_block / decode_block once per stripe (16 KiB chunks by default,
// cjerase_16k.ex3:46) from many pool threads.  For such calls the DMA round trip (H2D, kernel,
// D2H, each a queue operation with its own fixed cost, plus the hops through a dispatcher
// thread) dominates: 78 us per 16 KiB Cauchy(6+3) call at one thread in round 1.  Here the
// calling thread copies its chunks into its own page-locked slot and the coding kernel reads
// and writes that slot over PCIe directly (zero-copy): one launch on the thread's stream and
// one synchronisation per call, no DMA and no other thread.  Chunks the caller already holds
// in page-locked memory are read and written in place, with no copies at all.
// Per-call bytes (inputs + outputs) served this way; LSEC_ZEROCOPY_KB.  4 MiB: calls of 1-4 MiB
// (RS(6+3) at 128 / 256 KiB chunks) ran 1.3-2.5x faster zero-copy than through the dispatcher
// at 1-128 threads (profiles/r02_v42_route_mid.jsonl).  Each thread keeps a page-locked slot as
// large as its largest such call.
size_t zerocopy_limit() {
  static size_t b = [] {
    const char *s = getenv("LSEC_ZEROCOPY_KB");
    return static_cast<size_t>(std::max(0L, s ? atol(s) : 4096L)) << 10;
  }();
  return b;
}

// Completion signals of zero-copy calls (flag in coherent page-locked memory, arrival counter
// in device memory) are pooled per device and never freed: a poller (FlagWaits) may read a flag
// just as the thread that owned it exits.
struct SignalBlock {
  unsigned *flag, *dflag, *counter;
};
std::mutex g_signal_mu;
std::map<int, std::vector<SignalBlock>> &signal_pool() {
  static auto *p = new std::map<int, std::vector<SignalBlock>>();  // leaked with the blocks
  return *p;
}

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
    static PinnedBudget *b = [] {
      const char *s = getenv("LSEC_ZC_SLOTS_MB");
      return new PinnedBudget(static_cast<size_t>(std::max(0L, s ? atol(s) : 1024L)) << 20);  // leaked: slots outlive statics
    }();
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

struct ZcSlot {  // one calling thread's page-locked slot on one device
  char *h = nullptr;
  uint64_t d = 0;  // its device address
  size_t cap = 0;
  // completion: flag in coherent page-locked memory (the host spins on it), the signal
  // kernel's arrival counter in device memory, and the value the next call waits for
  unsigned *flag = nullptr, *dflag = nullptr, *counter = nullptr;
  unsigned seq = 0;
  int dev = -1;
  bool clean = true;  // every signal launched was seen: the block can serve another thread
  ZcSlot() = default;
  ZcSlot(const ZcSlot &) = delete;
  ZcSlot &operator=(const ZcSlot &) = delete;
  ~ZcSlot() {
    if (h) {
      (void)hipHostFree(h);
      PinnedBudget::global().release_slot(dev, cap);
    }
    if (flag && clean) {
      std::lock_guard<std::mutex> lk(g_signal_mu);
      signal_pool()[dev].push_back({flag, dflag, counter});
    }
  }
  int init_signal() {
    if (flag) return 0;
    HIP_OK(hipGetDevice(&dev));
    {
      std::lock_guard<std::mutex> lk(g_signal_mu);
      std::vector<SignalBlock> &pool = signal_pool()[dev];
      if (!pool.empty()) {
        flag = pool.back().flag;
        dflag = pool.back().dflag;
        counter = pool.back().counter;
        pool.pop_back();
        seq = __atomic_load_n(flag, __ATOMIC_ACQUIRE);  // continue the sequence the flag holds
        return 0;
      }
    }
    HIP_OK(hipHostMalloc(reinterpret_cast<void **>(&flag), 64, hipHostMallocCoherent));
    *flag = 0;
    void *d = nullptr;
    HIP_OK(hipHostGetDevicePointer(&d, flag, 0));
    dflag = static_cast<unsigned *>(d);
    HIP_OK(hipMalloc(reinterpret_cast<void **>(&counter), 64));
    HIP_OK(hipMemset(counter, 0, 64));
    return 0;
  }
};

// Completes a zero-copy call: the signal kernel behind the coding kernel on `st`, then a spin
// on the flag (a flag seen ~8 us sooner than hipStreamSynchronize returns:
// tools/probes/zc_probe.hip, profiles/r02_v3_zc_probe.txt).  A call whose flag has not come
// after a second falls back to the stream's own status, so a failed launch is reported.
bool wait_flag(const unsigned *flag, unsigned v, hipStream_t st, int *rc);

int zc_complete(ZcSlot &sl, hipStream_t st) {
  const unsigned v = ++sl.seq == 0 ? ++sl.seq : sl.seq;
  const hipError_t e = lsec::launch_signal(sl.counter, sl.dflag, v, st);
  if (e != hipSuccess) return fail("signal launch: %s", hipGetErrorString(e));
  int rc = 0;
  if (!wait_flag(sl.flag, v, st, &rc)) sl.clean = false;
  return rc;
}

// regular stripe stride of device addresses a[s * per + i] (i < per): shard i of stripe s at
// a[i] + s * stride[i]; false if irregular
bool regular_refs(const std::vector<uint64_t> &a, int nstripes, size_t per, std::vector<int64_t> &stride) {
  stride.assign(per, 0);
  if (nstripes < 2) return true;
  for (size_t i = 0; i < per; ++i) stride[i] = static_cast<int64_t>(a[per + i] - a[i]);
  for (int s = 2; s < nstripes; ++s)
    for (size_t i = 0; i < per; ++i)
      if (a[s * per + i] != a[i] + static_cast<uint64_t>(s * stride[i])) return false;
  return true;
}

// ---------------------------------------------------------------- waiting for completion flags
// CPUs this process may keep busy: the affinity mask, capped by the cgroup CPU quota (a GPU box
// may show the whole machine's CPUs and grant a share of them).
int usable_cpus() {
  static const int n = [] {
    int c = 1;
    cpu_set_t set;
    if (sched_getaffinity(0, sizeof(set), &set) == 0) c = std::max(1, CPU_COUNT(&set));
    if (FILE *f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
      char q[32] = {0};
      long long period = 0;
      if (fscanf(f, "%31s %lld", q, &period) == 2 && strcmp(q, "max") != 0 && period > 0)
        c = std::min<long long>(c, std::max(1LL, (atoll(q) + period - 1) / period));
      fclose(f);
    }
    return c;
  }();
  return n;
}

// Completion waits.  LStore calls encode_block from up to 300 pool threads; a waiter that spins
// (or yields) holds a CPU, and with more waiters than CPUs the spinning starves the threads whose
// calls are done -- on a cgroup quota it also burns the quota and gets the whole process
// throttled.  So at most a quarter of the usable CPUs spin; every other waiter parks on a futex
// word of its own, and poller threads watch the parked waiters' flags (written by the GPU, which
// cannot wake a thread) and wake them.
//
// Parking is lock-free: each thread owns a record in a static table (its flags and wanted values
// copied in, published under a sequence lock), and the pollers scan the table.  An earlier form
// (one poller holding one mutex over a list of condition variables while it scanned and
// notified) capped per-stripe calls at ~150k/s: at 32 and 128 threads an RS(6+3) 16 KiB encode
// ran 12.5-13.7 GiB/s against 20.9 at 8 threads, with CPUs to spare
// (profiles/r02_v28_zc_routes.txt).  Every flag a record can name stays mapped for the life of
// the process (server done lines; zero-copy flags come from a pool that is never freed), so a
// poller that reads a record just as its waiter leaves reads valid memory.
// LSEC_STATS counters of the waiting machinery (printed with ZcStats at exit)
std::atomic<unsigned long long> g_st_parks{0}, g_st_spin_hits{0}, g_st_claim_misses{0}, g_st_claim_spins{0},
    g_st_wakes{0}, g_st_slices{0};

class FlagWaits {
 public:
  static constexpr int kMaxFlags = 16;  // flags one wait covers (StripeServer::kMaxParts)

  static FlagWaits &get() {
    static FlagWaits *w = new FlagWaits();  // leaked: the poller threads outlive static destruction
    return *w;
  }

  // Waits until every flags[i] reaches wants[i] (wrapping u32 sequences: wants[i] - *flags[i] <= 0),
  // or up to `slice`; true when all are reached.  Callers loop, doing their own checks between
  // slices.  One wait covers all the parts of a call: the parts land on different server
  // workgroups and finish in any order (a wait per part could park and wake its thread once
  // per part under load).
  bool wait(const unsigned *const *flags, const unsigned *wants, int n, std::chrono::microseconds slice) {
    int from = 0;
    if (reached_all(flags, wants, n, from)) return true;
    Record *rec = n <= kMaxFlags ? my_record() : nullptr;
    if (!rec) {  // no record: spin, then yield, then nap
      const auto t0 = std::chrono::steady_clock::now();
      for (unsigned i = 0;; ++i) {
        if (reached_all(flags, wants, n, from)) return true;
        if (i < 500) {
          __builtin_ia32_pause();
          continue;
        }
        const auto dt = std::chrono::steady_clock::now() - t0;
        if (dt > slice) return false;
        if (dt < std::chrono::microseconds(200)) std::this_thread::yield();
        else std::this_thread::sleep_for(std::chrono::microseconds(20));
      }
    }
    const auto t0 = std::chrono::steady_clock::now();
    // spin only while waits are short: under load (waits of 100s of us) a spinner holds a CPU
    // for nothing that the callers' copies need
    const bool short_waits = recent_us_.load(std::memory_order_relaxed) < 2 * spin_.count();
    const int active = spinners_.fetch_add(1, std::memory_order_relaxed) + 1;
    if (short_waits && active <= spin_limit_) {
      for (unsigned i = 1;; ++i) {
        if (reached_all(flags, wants, n, from)) {
          spinners_.fetch_sub(1, std::memory_order_relaxed);
          note(t0);
          g_st_spin_hits.fetch_add(1, std::memory_order_relaxed);
          return true;
        }
        __builtin_ia32_pause();
        if ((i & 63) == 0 && std::chrono::steady_clock::now() - t0 > spin_) break;
      }
    }
    spinners_.fetch_sub(1, std::memory_order_relaxed);
    // park: publish the flags still outstanding, then sleep on the record's futex word
    const int m = n - from;
    rec->seq.fetch_add(1, std::memory_order_relaxed);  // odd: fields changing
    std::atomic_thread_fence(std::memory_order_release);
    for (int i = 0; i < m; ++i) {
      rec->flags[i].store(flags[from + i], std::memory_order_relaxed);
      rec->wants[i].store(wants[from + i], std::memory_order_relaxed);
    }
    rec->n.store(m, std::memory_order_relaxed);
    rec->word.store(0, std::memory_order_relaxed);
    rec->seq.fetch_add(1, std::memory_order_release);  // even: published
    rec->active.store(1, std::memory_order_seq_cst);
    g_st_parks.fetch_add(1, std::memory_order_relaxed);
    if (sleeping_.load(std::memory_order_seq_cst) > 0) {  // a poller sleeps: new work for it
      epoch_.fetch_add(1, std::memory_order_seq_cst);
      futex_wake(&epoch_, INT32_MAX);
    }
    const auto deadline = t0 + slice;
    while (rec->word.load(std::memory_order_acquire) == 0 && !reached_all(flags, wants, n, from)) {
      const auto now = std::chrono::steady_clock::now();
      if (now >= deadline) break;
      futex_wait(&rec->word, 0, std::chrono::duration_cast<std::chrono::nanoseconds>(deadline - now));
    }
    rec->active.store(0, std::memory_order_release);
    if (!reached_all(flags, wants, n, from)) {
      g_st_slices.fetch_add(1, std::memory_order_relaxed);
      return false;
    }
    note(t0);
    return true;
  }
  bool wait(const unsigned *flag, unsigned want, std::chrono::microseconds slice) {
    return wait(&flag, &want, 1, slice);
  }

 private:
  static constexpr int kMaxRecords = 4096;  // threads that have parked at least once

  struct alignas(64) Record {
    std::atomic<uint32_t> seq{0};   // sequence lock over n / flags / wants (odd while writing)
    std::atomic<uint32_t> word{0};  // futex word: set to 1 by the poller that wakes the waiter
    std::atomic<int> active{0};     // 1 while the waiter is parked
    std::atomic<int> n{0};
    std::atomic<const unsigned *> flags[kMaxFlags];
    std::atomic<unsigned> wants[kMaxFlags];
  };

  // this thread's record; a thread that exits returns it for reuse
  Record *my_record() {
    struct Owner {
      int idx = -1;
      ~Owner() {
        if (idx >= 0) FlagWaits::get().free_record(idx);
      }
    };
    static thread_local Owner own;
    if (own.idx < 0) own.idx = alloc_record();
    return own.idx < 0 ? nullptr : &records_[own.idx];
  }
  int alloc_record() {
    std::lock_guard<std::mutex> lk(free_mu_);
    if (!free_.empty()) {
      const int i = free_.back();
      free_.pop_back();
      return i;
    }
    const int i = used_.load(std::memory_order_relaxed);
    if (i >= kMaxRecords) return -1;
    used_.store(i + 1, std::memory_order_release);
    return i;
  }
  void free_record(int i) {
    records_[i].active.store(0, std::memory_order_release);
    std::lock_guard<std::mutex> lk(free_mu_);
    free_.push_back(i);
  }

  static void futex_wait(std::atomic<uint32_t> *w, uint32_t v, std::chrono::nanoseconds t) {
    struct timespec ts;
    ts.tv_sec = static_cast<time_t>(t.count() / 1000000000);
    ts.tv_nsec = static_cast<long>(t.count() % 1000000000);
    syscall(SYS_futex, reinterpret_cast<uint32_t *>(w), FUTEX_WAIT_PRIVATE, v, &ts, nullptr, 0);
  }
  static void futex_wake(std::atomic<uint32_t> *w, int n) {
    syscall(SYS_futex, reinterpret_cast<uint32_t *>(w), FUTEX_WAKE_PRIVATE, n, nullptr, nullptr, 0);
  }

  // moving average of completed waits (us), 1/8 weight per sample
  void note(std::chrono::steady_clock::time_point t0) {
    const long us = static_cast<long>(
        std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0).count());
    const long old = recent_us_.load(std::memory_order_relaxed);
    recent_us_.store(old + (us - old) / 8, std::memory_order_relaxed);
  }

  static bool reached(const unsigned *flag, unsigned want) {
    return static_cast<int>(__atomic_load_n(flag, __ATOMIC_ACQUIRE) - want) >= 0;
  }
  // all of flags[from, n) reached; advances `from` past the ones that are
  static bool reached_all(const unsigned *const *flags, const unsigned *wants, int n, int &from) {
    while (from < n && reached(flags[from], wants[from])) ++from;
    return from == n;
  }

  FlagWaits() {
    // from a sweep of both (profiles/r02_v22_wait_sweep.jsonl): a quarter of the usable CPUs
    // spin, for up to 30 us (an unloaded call completes in 14-20 us)
    spin_limit_ = std::max(1, usable_cpus() / 4);
    spin_ = std::chrono::microseconds(30);
    // pollers: one per 8 usable CPUs, at most 4
    npollers_ = std::max(1, std::min(4, usable_cpus() / 8));
    for (int p = 0; p < npollers_; ++p) std::thread([this, p] { poll(p); }).detach();
  }

  // poller p scans records p, p + npollers, ...: wakes every parked waiter whose flags have all
  // come; sleeps on epoch_ while none of its records is parked
  void poll(int p) {
    const unsigned *f[kMaxFlags];
    unsigned wv[kMaxFlags];
    for (;;) {
      bool any = false;
      const int hi = used_.load(std::memory_order_acquire);
      for (int i = p; i < hi; i += npollers_) {
        Record &r = records_[i];
        if (!r.active.load(std::memory_order_acquire)) continue;
        any = true;
        const uint32_t s1 = r.seq.load(std::memory_order_acquire);
        if (s1 & 1u) continue;
        const int m = r.n.load(std::memory_order_relaxed);
        if (m < 1 || m > kMaxFlags) continue;
        for (int j = 0; j < m; ++j) {
          f[j] = r.flags[j].load(std::memory_order_relaxed);
          wv[j] = r.wants[j].load(std::memory_order_relaxed);
        }
        std::atomic_thread_fence(std::memory_order_acquire);
        if (r.seq.load(std::memory_order_relaxed) != s1) continue;  // rewritten meanwhile
        int from = 0;
        if (!reached_all(f, wv, m, from)) continue;
        if (r.word.exchange(1, std::memory_order_acq_rel) == 0) {
          futex_wake(&r.word, 1);
          g_st_wakes.fetch_add(1, std::memory_order_relaxed);
        }
      }
      if (any) {  // flags are written by the GPU: poll, a few us apart
        for (int i = 0; i < 32; ++i) __builtin_ia32_pause();
        std::this_thread::yield();
        continue;
      }
      // nothing parked here: sleep until a waiter parks (it bumps epoch_ when it sees a sleeper)
      const uint32_t e = epoch_.load(std::memory_order_seq_cst);
      sleeping_.fetch_add(1, std::memory_order_seq_cst);
      bool now_any = false;
      const int hi2 = used_.load(std::memory_order_acquire);
      for (int i = p; i < hi2 && !now_any; i += npollers_) now_any = records_[i].active.load(std::memory_order_seq_cst) != 0;
      if (!now_any) futex_wait(&epoch_, e, std::chrono::milliseconds(10));
      sleeping_.fetch_sub(1, std::memory_order_seq_cst);
    }
  }

  int spin_limit_ = 1;                   // waiters allowed to spin at once (LSEC_WAIT_SPINNERS)
  std::chrono::microseconds spin_{100};  // how long one spins before parking (LSEC_WAIT_SPIN_US)
  int npollers_ = 1;
  std::atomic<int> spinners_{0};
  std::atomic<long> recent_us_{0};
  std::atomic<uint32_t> epoch_{0};
  std::atomic<int> sleeping_{0};
  std::atomic<int> used_{0};
  Record records_[kMaxRecords];
  std::mutex free_mu_;
  std::vector<int> free_;
};

// Waits until flag reaches v (wrapping u32 sequence) through FlagWaits.  Bounded: after 2 s
// the caller checks its stream for an error.
bool wait_flag(const unsigned *flag, unsigned v, hipStream_t st, int *rc) {
  const auto t0 = std::chrono::steady_clock::now();
  while (!FlagWaits::get().wait(flag, v, std::chrono::milliseconds(1))) {
    if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
      const hipError_t e = hipStreamSynchronize(st);
      if (static_cast<int>(__atomic_load_n(flag, __ATOMIC_ACQUIRE) - v) >= 0) return true;
      *rc = fail("zero-copy call: completion flag never came (%s)", hipGetErrorString(e));
      return false;
    }
  }
  return true;
}

// Routes taken by zero-copy calls, printed at exit with LSEC_STATS=1: served by the stripe
// server, refused by it (no free slots: claim failed, or not servable), then run as their own
// launch (kernel over the caller's page-locked chunks, or over this thread's slot)
thread_local std::chrono::steady_clock::time_point tl_call_t0;  // fn-pointer entry (LSEC_STATS)
thread_local std::chrono::steady_clock::time_point tl_zc_t0;    // run_zerocopy entry (LSEC_STATS)
thread_local long long tl_call_cpu0 = 0, tl_zc_cpu0 = 0;           // this thread's CPU ns at both

long long thread_cpu_ns() {
  struct timespec ts;
  clock_gettime(CLOCK_THREAD_CPUTIME_ID, &ts);
  return static_cast<long long>(ts.tv_sec) * 1000000000LL + ts.tv_nsec;
}

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

// ---------------------------------------------------------------- stripe server (host side)
// Per-stripe calls up to kSlotBytes per part are served by the persistent stripe server
// (ec_server.hip): the calling thread claims slots, copies its chunks' column blocks into them
// (or, for page-locked caller chunks, just names their device addresses), posts one descriptor
// per part and spins on the parts' done flags.  No launch, no DMA and no other host thread per
// call; the server's workgroups serve the parts of many callers in parallel.  The server exits
// after 2 ms without work and is relaunched by the next caller (or by a waiting one that finds
// it gone).  LSEC_SERVER=0 turns it off.
// the stripe server's answer time limit (LSEC test hook lsec_test_server_hold) and its hold
std::atomic<int> g_srv_timeout_ms{5000};
std::atomic<int> g_srv_hold{0};
std::atomic<unsigned long long> g_st_srv_timeouts{0};

class StripeServer {
 public:
  static StripeServer *for_device(int dev) {
    // every per-stripe call asks: a lock-free read once the device's server exists
    static std::atomic<StripeServer *> fast[64] = {};
    if (dev >= 0 && dev < 64)
      if (StripeServer *f = fast[dev].load(std::memory_order_acquire)) return f;
    static std::mutex m;
    static std::map<int, StripeServer *> all;  // intentionally leaked: lives until exit
    std::lock_guard<std::mutex> lk(m);
    StripeServer *&r = all[dev];
    if (!r) {
      r = new StripeServer(dev);
      registry().push_back(r);
      static std::once_flag once;
      std::call_once(once, [] { atexit(stop_all); });
    }
    if (dev >= 0 && dev < 64) fast[dev].store(r, std::memory_order_release);
    return r;
  }

  // 0 served, -1 error, 1 not servable here (the caller takes another path)
  int run(PlanExt *e, char **ptrs, long long C, const std::vector<int> &in_ids, const std::vector<int> &out_ids,
          const void *image, int kind, const CallerPinned *cp) {
    const auto t_enter = std::chrono::steady_clock::now();
    const bool stats = ZcStats::on();
    const long long c_enter = stats ? thread_cpu_ns() : 0;
    long long c_post = 0, c_waited = 0;
    const size_t nin = in_ids.size(), nout = out_ids.size(), nio = nin + nout;
    const auto refuse = [] {
      ZcStats::get().not_servable.fetch_add(1, std::memory_order_relaxed);
      return 1;
    };
    if (nin < 1 || nout < 1 || nin > lsec::kSrvMaxK || nout > lsec::kSrvMaxR) return refuse();
    if (kind != KBYTEWISE && kind != KBITSLICED) return refuse();
    // a server that cannot be set up or launched is never posted to: the call takes its own
    // zero-copy launch or the dispatcher (a post nobody will serve would strand its slots)
    if (broken_.load(std::memory_order_acquire)) return refuse();
    if (init_once()) {
      broken_ = true;
      return refuse();
    }
    const lio_erasure_plan_t *p = &e->pub;
    const bool direct = cp && cp->by_kernel;
    // calls whose parts the server reads and writes in the caller's own buffers: a server that
    // cannot be stopped while any is in flight ends the process (stop_and_settle)
    struct DirectCall {
      std::atomic<int> *n;
      explicit DirectCall(std::atomic<int> *c) : n(c) {
        if (n) n->fetch_add(1, std::memory_order_acq_rel);
      }
      ~DirectCall() {
        if (n) n->fetch_sub(1, std::memory_order_acq_rel);
      }
    } direct_call(direct ? &direct_inflight_ : nullptr);
    // parts: column blocks of about 4 KiB per shard (one 256-lane x 16 B pass), whole
    // super-packets for the bit-sliced layout, at most kMaxParts of them
    const long long unit = kind == KBITSLICED ? 8LL * p->packet_size : 16;
    const long long max_len = direct ? C : static_cast<long long>(kSlotBytes / nio) / unit * unit;
    if (max_len < std::min<long long>(unit, C)) return refuse();
    // column bytes per part: 4 KiB (4-16 KiB parts measured level, profiles/r02_v22_server_part_ab.jsonl)
    constexpr long long target = 4096;
    long long len = std::min(std::max<long long>(unit, target / unit * unit), max_len);
    if ((C + len - 1) / len > kMaxParts) {
      len = ((C + kMaxParts - 1) / kMaxParts + unit - 1) / unit * unit;
      if (len > max_len) return refuse();
    }
    if (len > C) len = C;
    int nparts = static_cast<int>((C + len - 1) / len);
    int slot[kMaxParts];
    if (!claim(nparts, slot)) {
      // under load: fewer, larger parts (as many columns as a slot holds), then a short wait for
      // slots to come free -- the other route, a launch of this call's own, costs the host far
      // more CPU per call than a wait (profiles/r02_v28_zc_routes.txt)
      bool got = false;
      g_st_claim_misses.fetch_add(1, std::memory_order_relaxed);
      if (len < std::min(max_len, C)) {
        len = std::min(max_len, C);
        nparts = static_cast<int>((C + len - 1) / len);
        got = claim(nparts, slot);
      }
      const auto t0 = std::chrono::steady_clock::now();
      while (!got && std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(50)) {
        std::this_thread::yield();
        g_st_claim_spins.fetch_add(1, std::memory_order_relaxed);
        got = claim(nparts, slot);
      }
      if (!got) {
        ZcStats::get().no_slots.fetch_add(1, std::memory_order_relaxed);
        return 1;
      }
    }
    uint32_t want[kMaxParts];
    for (int q = 0; q < nparts; ++q) {
      const int sl = slot[q];
      const long long c0 = static_cast<long long>(q) * len, n = std::min(len, C - c0);
      lsec::SrvDesc &d = sh_->desc[sl];
      d.kind = kind == KBITSLICED ? lsec::kSrvBitsliced : lsec::kSrvBytewise;
      d.K = static_cast<uint32_t>(nin);
      d.R = static_cast<uint32_t>(nout);
      d.packet = static_cast<uint32_t>(p->packet_size);
      d.size = static_cast<uint64_t>(n);
      d.cells = reinterpret_cast<uint64_t>(image);
      d.cstride = static_cast<uint32_t>(nin);
      if (direct) {
        for (size_t j = 0; j < nin; ++j) d.in[j] = cp->dev[j] + static_cast<uint64_t>(c0);
        for (size_t r = 0; r < nout; ++r) d.out[r] = cp->dev[nin + r] + static_cast<uint64_t>(c0);
      } else {
        char *region = data_ + static_cast<size_t>(sl) * kSlotBytes;
        const uint64_t dregion = data_dev_ + static_cast<uint64_t>(sl) * kSlotBytes;
        for (size_t j = 0; j < nin; ++j) {
          // plain stores: for these 4 KiB pieces streaming ones cost 15 -> 18 us p50 at one
          // thread (the server reads them back from DRAM instead of the host's caches;
          // profiles/r03_v27_fnptr_fair.jsonl)
          std::memcpy(region + j * n, ptrs[in_ids[j]] + c0, static_cast<size_t>(n));
          d.in[j] = dregion + j * n;
        }
        for (size_t r = 0; r < nout; ++r) d.out[r] = dregion + (nin + r) * n;
      }
      want[q] = ++seq_[sl] == 0 ? ++seq_[sl] : seq_[sl];
      __atomic_store_n(&sh_->post[lsec::srv_wg(sl)][lsec::srv_word(sl)], want[q], __ATOMIC_RELEASE);
    }
    const auto t_post = std::chrono::steady_clock::now();
    if (stats) c_post = thread_cpu_ns();
    int rc = ensure_running(false);
    const auto t0 = std::chrono::steady_clock::now();
    auto last_check = t0;
    const unsigned *flags[kMaxParts];
    for (int q = 0; q < nparts; ++q) flags[q] = &sh_->done[slot[q]][0];
    const auto timeout = std::chrono::milliseconds(g_srv_timeout_ms.load(std::memory_order_relaxed));
    bool late = false;
    // spin or park (FlagWaits) until every part is done, checking every 500 us that the server
    // has not retired meanwhile (it retires only after 2 ms without work; at 100 us slices a
    // loaded box woke 1.5 parked waiters per call just to check, profiles/r02_v30_zc_phases3.txt)
    while (rc == 0 && !FlagWaits::get().wait(flags, want, nparts, std::chrono::microseconds(500))) {
      const auto now = std::chrono::steady_clock::now();
      if (now - last_check > std::chrono::microseconds(500)) {
        last_check = now;
        if ((rc = ensure_running(true))) break;
      }
      if (now - t0 > timeout) {
        late = true;
        break;
      }
    }
    if (rc != 0 || late) {
      // No answer in time (a throttled box, a stuck server) or no server: stop it and wait until
      // it has left, so no post of this call can be served after the call returns -- for
      // page-locked callers the server writes the caller's own buffers.  Parts served meanwhile
      // count; the others are cancelled and the call takes another route (return 1).
      g_st_srv_timeouts.fetch_add(1, std::memory_order_relaxed);
      std::lock_guard<std::mutex> lk(mu_);
      const int served = stop_and_settle(nparts, slot, want);
      if (served < 0) return 1;  // a server that would not stop: its slots stay claimed for good
      if (served != nparts) {
        release(nparts, slot);
        return 1;
      }
      rc = 0;
    }
    const auto t_waited = std::chrono::steady_clock::now();
    if (stats) c_waited = thread_cpu_ns();
    static const bool trace = getenv("LSEC_TRACE") != nullptr;
    if (trace) {  // calls slower than 1 ms: where the time went
      const auto t_end = std::chrono::steady_clock::now();
      const auto us = [](std::chrono::steady_clock::duration d) { return std::chrono::duration<double, std::micro>(d).count(); };
      if (t_end - t_post > std::chrono::milliseconds(1))
        fprintf(stderr, "[lsec trace] server call %d parts (slots %d..): ensure %.1f us, wait %.1f us, rc %d\n", nparts, slot[0],
                us(t0 - t_post), us(t_end - t0), rc);
    }
    if (rc == 0)
      last_seen_us_.store(std::chrono::duration_cast<std::chrono::microseconds>(
                              std::chrono::steady_clock::now().time_since_epoch()).count(),
                          std::memory_order_relaxed);
    if (rc == 0 && !direct)
      for (int q = 0; q < nparts; ++q) {
        const long long c0 = static_cast<long long>(q) * len, n = std::min(len, C - c0);
        const char *region = data_ + static_cast<size_t>(slot[q]) * kSlotBytes;
        for (size_t r = 0; r < nout; ++r) std::memcpy(ptrs[out_ids[r]] + c0, region + (nin + r) * n, static_cast<size_t>(n));
      }
    release(nparts, slot);
    if (rc == 0 && stats) {
      ZcStats &z = ZcStats::get();
      const auto ns = [](std::chrono::steady_clock::duration d) {
        return static_cast<unsigned long long>(std::chrono::duration_cast<std::chrono::nanoseconds>(d).count());
      };
      const auto t_done = std::chrono::steady_clock::now();
      if (tl_call_t0.time_since_epoch().count() && t_enter > tl_call_t0) z.t_setup.fetch_add(ns(t_enter - tl_call_t0), std::memory_order_relaxed);
      if (tl_zc_t0.time_since_epoch().count() && t_enter > tl_zc_t0) z.t_zc.fetch_add(ns(t_enter - tl_zc_t0), std::memory_order_relaxed);
      z.t_post.fetch_add(ns(t_post - t_enter), std::memory_order_relaxed);
      z.t_wait.fetch_add(ns(t_waited - t_post), std::memory_order_relaxed);
      z.t_out.fetch_add(ns(t_done - t_waited), std::memory_order_relaxed);
      const long long c_done = thread_cpu_ns();
      if (tl_call_cpu0 && c_enter > tl_call_cpu0) z.c_setup.fetch_add(c_enter - tl_call_cpu0, std::memory_order_relaxed);
      if (tl_zc_cpu0 && c_enter > tl_zc_cpu0) z.c_zc.fetch_add(c_enter - tl_zc_cpu0, std::memory_order_relaxed);
      z.c_post.fetch_add(c_post - c_enter, std::memory_order_relaxed);
      z.c_wait.fetch_add(c_waited - c_post, std::memory_order_relaxed);
      z.c_out.fetch_add(c_done - c_waited, std::memory_order_relaxed);
    }
    return rc;
  }

 private:
  static constexpr size_t kSlotBytes = lsec::kSrvSlotBytes;  // chunk bytes of one part (inputs + outputs)
  static constexpr int kMaxParts = 16;

  explicit StripeServer(int dev) : dev_(dev) {
    for (auto &b : busy_) b.store(0);
    for (auto &q : seq_) q = 0;
  }

  static std::vector<StripeServer *> &registry() {
    // leaked: stop_all runs from atexit and must find it intact (a function-local static
    // constructed after the atexit registration would be destroyed before stop_all runs)
    static std::vector<StripeServer *> *r = new std::vector<StripeServer *>();
    return *r;
  }
  // at exit: stop every running server and let it drain (its stop word is read on every idle poll)
  static void stop_all() {
    for (StripeServer *s : registry()) {
      std::lock_guard<std::mutex> lk(s->mu_);
      if (s->sh_) s->stop_and_settle(0, nullptr, nullptr);
    }
  }

 public:
  // test hook (lsec_test_server_hold): stop every server, so the next launch takes the new hold
  static void restart_all() { stop_all(); }

 private:
  // Stop the running server and wait (bounded) until it has left.  The stop word is final (the
  // kernel picks nothing after it sees it, ec_server.hip), so the launch leaves after the parts
  // its workgroups are serving; afterwards nothing can serve a post until the next launch, which
  // takes served[] from done[].  Of this call's parts, those served count; the rest are
  // cancelled by setting done to the posted value, so no later launch serves them.  Returns
  // the number served.  mu_ held.
  // A server still there after 30 s (a hung device) may yet write whatever it was serving.  If
  // any call in flight has the server write the caller's own page-locked buffers in place
  // (direct_inflight_), the process ends: those buffers may not be handed back while a kernel can
  // write them.  Otherwise it writes only its own slot region: the server is marked broken (no
  // call posts to it again), the caller abandons its slots, and -1 is returned.
  int stop_and_settle(int nparts, const int *slot, const uint32_t *want) {
    if (zombie_) return -1;
    if (running_) {
      for (int g = 0; g < lsec::kSrvWG; ++g) __atomic_store_n(&sh_->post[g][lsec::kSrvSlotsPerWG], 1u, __ATOMIC_RELEASE);
      const auto t0 = std::chrono::steady_clock::now();
      for (;;) {
        const hipError_t q = hipEventQuery(ev_);
        if (q == hipSuccess) break;
        if (q != hipErrorNotReady) {  // the device failed: nothing runs there any more
          (void)hipGetLastError();
          broken_ = true;
          break;
        }
        if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(kStopWaitS)) {
          if (direct_inflight_.load(std::memory_order_acquire) > 0)
            fatal("the stripe server on device %d did not stop within %d s while it serves page-locked caller "
                  "buffers in place", dev_, kStopWaitS);
          broken_ = true;
          zombie_ = true;
          fprintf(stderr, "liblstore_ec: the stripe server on device %d did not stop within %d s; its slots are "
                  "abandoned and this device's per-stripe calls take other routes\n", dev_, kStopWaitS);
          return -1;
        }
        std::this_thread::sleep_for(std::chrono::microseconds(100));
      }
      running_ = false;
    }
    int served = 0;
    for (int q = 0; q < nparts; ++q) {
      unsigned *d = &sh_->done[slot[q]][0];
      if (__atomic_load_n(d, __ATOMIC_ACQUIRE) == want[q]) ++served;
      else __atomic_store_n(d, want[q], __ATOMIC_RELEASE);
    }
    return served;
  }

  bool claim(int n, int *slot) {
    static std::atomic<unsigned> next{0};
    thread_local unsigned base = next.fetch_add(7919) % lsec::kSrvSlots;
    int got = 0;
    for (int k = 0; k < lsec::kSrvSlots && got < n; ++k) {
      const int s = static_cast<int>((base + k) % lsec::kSrvSlots);
      uint8_t z = 0;
      // look before the locked exchange: under load most slots are busy, and a failed
      // exchange on every one of them from every thread kept the flag lines bouncing
      if (busy_[s].load(std::memory_order_relaxed) == 0 && busy_[s].compare_exchange_strong(z, 1)) slot[got++] = s;
    }
    if (got < n) {
      release(got, slot);
      return false;
    }
    return true;
  }
  void release(int n, const int *slot) {
    for (int q = 0; q < n; ++q) busy_[slot[q]].store(0, std::memory_order_release);
  }

  int init_once() {
    if (ready_.load(std::memory_order_acquire)) return 0;
    std::lock_guard<std::mutex> lk(mu_);
    if (ready_.load()) return 0;
    DeviceGuardLite g(dev_);
    int lo = 0, hi = 0;
    HIP_OK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    HIP_OK(hipStreamCreateWithPriority(&st_, hipStreamNonBlocking, hi));  // a hardware queue of its own
    HIP_OK(hipEventCreateWithFlags(&ev_, hipEventDisableTiming));
    HIP_OK(hipMalloc(reinterpret_cast<void **>(&votes_), 64));
    HIP_OK(hipMemset(votes_, 0, 64));
    HIP_OK(hipHostMalloc(reinterpret_cast<void **>(&sh_), sizeof(lsec::SrvShared), hipHostMallocCoherent));
    std::memset(static_cast<void *>(sh_), 0, sizeof(lsec::SrvShared));
    void *p = nullptr;
    HIP_OK(hipHostGetDevicePointer(&p, sh_, 0));
    sh_dev_ = reinterpret_cast<uint64_t>(p);
    // the slot region: about 93 MiB per device, accounted as the device's server memory, apart
    // from the threads' slot budget (PinnedBudget)
    const size_t region = kSlotBytes * lsec::kSrvSlots;
    if (hipHostMalloc(reinterpret_cast<void **>(&data_), region, hipHostMallocCoherent) != hipSuccess) {
      (void)hipGetLastError();
      return fail("stripe server: cannot allocate its slots");
    }
    PinnedBudget::global().add_server(dev_, region);
    HIP_OK(hipHostGetDevicePointer(&p, data_, 0));
    data_dev_ = reinterpret_cast<uint64_t>(p);
    ready_.store(true, std::memory_order_release);
    return 0;
  }

  int ensure_running(bool check) {
    // the server retires after 2 ms without work: past 1.5 ms since a part was last seen done,
    // ask the runtime whether it is still there before relying on it
    const int64_t now = std::chrono::duration_cast<std::chrono::microseconds>(
                            std::chrono::steady_clock::now().time_since_epoch()).count();
    if (!check && now - last_seen_us_.load(std::memory_order_relaxed) > 1500) check = true;
    if (!check && running_.load(std::memory_order_acquire)) return 0;
    if (running_.load(std::memory_order_acquire)) {
      // one liveness query per 200 us for all threads: after the cgroup throttles the process
      // every waiter's slice expires at once, and each asking the runtime (under mu_) kept a
      // 128-thread process throttled (profiles/r02_v32_zc_decode2.txt)
      int64_t prev = last_check_us_.load(std::memory_order_relaxed);
      if (now - prev < 200 || !last_check_us_.compare_exchange_strong(prev, now)) return 0;
    }
    std::lock_guard<std::mutex> lk(mu_);
    if (broken_) return fail("stripe server: unusable after an earlier failure");
    if (running_ && check) {
      const hipError_t q = hipEventQuery(ev_);
      if (q == hipSuccess) running_ = false;
      else if (q != hipErrorNotReady) {
        broken_ = true;
        return fail("stripe server: %s", hipGetErrorString(q));
      }
    }
    if (running_) return 0;
    for (int g = 0; g < lsec::kSrvWG; ++g) sh_->post[g][lsec::kSrvSlotsPerWG] = 0;  // stop word
    lsec::SrvArgs a;
    a.shared = reinterpret_cast<lsec::SrvShared *>(sh_dev_);
    a.votes = votes_;
    a.idle_ticks = 200000;  // 2 ms at the 100 MHz wall clock
    a.hold = g_srv_hold.load(std::memory_order_relaxed) ? 1u : 0u;
    a.pad = 0;
    DeviceGuardLite g(dev_);
    hipError_t err = hipMemsetAsync(votes_, 0, sizeof(int), st_);
    if (err == hipSuccess) err = lsec::launch_stripe_server(a, st_);
    if (err == hipSuccess) err = hipEventRecord(ev_, st_);
    if (err != hipSuccess) {
      broken_ = true;
      return fail("stripe server launch: %s", hipGetErrorString(err));
    }
    running_ = true;
    return 0;
  }

  struct DeviceGuardLite {  // (DeviceGuard is defined further down)
    int prev = -1;
    explicit DeviceGuardLite(int dev) {
      if (hipGetDevice(&prev) != hipSuccess) prev = -1;
      if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuardLite() {
      if (prev >= 0) (void)hipSetDevice(prev);
    }
  };

  int dev_;
  lsec::SrvShared *sh_ = nullptr;
  uint64_t sh_dev_ = 0;
  char *data_ = nullptr;
  uint64_t data_dev_ = 0;
  std::atomic<uint8_t> busy_[lsec::kSrvSlots];
  uint32_t seq_[lsec::kSrvSlots];
  std::atomic<bool> ready_{false};
  std::mutex mu_;
  hipStream_t st_ = nullptr;
  hipEvent_t ev_ = nullptr;
  int *votes_ = nullptr;
  std::atomic<bool> running_{false};
  std::atomic<bool> broken_{false};
  bool zombie_ = false;                 // a launch that would not stop (mu_)
  std::atomic<int> direct_inflight_{0};  // calls whose parts the server serves in the caller's buffers
  static constexpr int kStopWaitS = 30;  // how long stop_and_settle waits for a launch to leave
  std::atomic<int64_t> last_seen_us_{0};
  std::atomic<int64_t> last_check_us_{0};
};

bool server_enabled() {
  static const bool on = [] {
    const char *s = getenv("LSEC_SERVER");
    return !s || *s != '0';
  }();
  return on;
}

ZcSlot &thread_zc_slot(int dev);

int run_zerocopy(PlanExt *e, char **ptrs, int nstripes, long long C, const std::vector<int> &in_ids,
                 const std::vector<int> &out_ids, const void *image, int kind) {
  if (ZcStats::on()) {
    tl_zc_t0 = std::chrono::steady_clock::now();
    tl_zc_cpu0 = thread_cpu_ns();
  }
  int dev = 0;
  HIP_OK(hipGetDevice(&dev));
  hipStream_t st = thread_stream();
  if (!st) return fail("no HIP stream");
  const lio_erasure_plan_t *p = &e->pub;
  const int km = p->data_strips + p->parity_strips;
  const size_t nin = in_ids.size(), nout = out_ids.size(), nio = nin + nout;
  ShardRef in[kMaxDevs], out[kMaxDevs];
  const bool aligned = kernel_transport_aligned(ptrs, nstripes, km, in_ids, out_ids, C, C);
  ZcSlot *slot = &thread_zc_slot(dev);
  if (slot->init_signal()) return -1;
  CallerPinned cp = caller_pinned(ptrs, nstripes, km, in_ids, out_ids, C, aligned);
  if (nstripes == 1 && server_enabled()) {
    const int rc = StripeServer::for_device(dev)->run(e, ptrs, C, in_ids, out_ids, image, kind, &cp);
    if (rc != 1) {
      if (rc == 0) ZcStats::get().server.fetch_add(1, std::memory_order_relaxed);
      return rc;
    }
  }
  std::vector<int64_t> stride;
  if (cp.by_kernel && regular_refs(cp.dev, nstripes, nio, stride)) {
    // caller page-locked chunks: read and written in place over PCIe
    for (size_t j = 0; j < nin; ++j) in[j] = {cp.dev[j], stride[j]};
    for (size_t r = 0; r < nout; ++r) out[r] = {cp.dev[nin + r], stride[nin + r]};
    ZcStats::get().launch_direct.fetch_add(1, std::memory_order_relaxed);
    if (enqueue_apply(kind, image, static_cast<int>(nin), static_cast<int>(nout), in, out, nstripes, C, p->packet_size, st, p->w))
      return -1;
    return zc_complete(*slot, st);
  }
  const size_t need = static_cast<size_t>(nstripes) * nio * static_cast<size_t>(C);
  if (slot->cap < need) {
    const size_t cap = std::max<size_t>(need, 256u << 10);
    // all threads' slots on this device together stay within LSEC_ZC_SLOTS_MB (default 1 GiB of
    // page-locked memory per device, PinnedBudget); a call whose slot would pass it goes to the
    // dispatcher's shared staging instead
    if (!PinnedBudget::global().grow_slot(dev, slot->cap, cap)) return 1;
    if (slot->h) (void)hipHostFree(slot->h);
    slot->h = nullptr;
    slot->cap = 0;
    slot->d = 0;
    // coherent: the kernel's reads and writes of the slot go straight over PCIe, none stays in an L2
    char *h = nullptr;
    void *d = nullptr;
    if (hipHostMalloc(reinterpret_cast<void **>(&h), cap, hipHostMallocCoherent) != hipSuccess) {
      (void)hipGetLastError();
      PinnedBudget::global().release_slot(dev, cap);
      return fail("zero-copy slot: cannot allocate %zu bytes of page-locked memory", cap);
    }
    if (hipHostGetDevicePointer(&d, h, 0) != hipSuccess || !d) {
      (void)hipGetLastError();
      (void)hipHostFree(h);
      PinnedBudget::global().release_slot(dev, cap);
      return fail("zero-copy slot: no device address");
    }
    slot->h = h;
    slot->d = reinterpret_cast<uint64_t>(d);
    slot->cap = cap;
  }
  ZcStats::get().launch_slot.fetch_add(1, std::memory_order_relaxed);
  const bool stats = ZcStats::on();
  const auto tnow = [] { return std::chrono::steady_clock::now(); };
  const auto tns = [](std::chrono::steady_clock::time_point a, std::chrono::steady_clock::time_point b) {
    return static_cast<unsigned long long>(std::chrono::duration_cast<std::chrono::nanoseconds>(b - a).count());
  };
  auto t_last = stats ? tnow() : std::chrono::steady_clock::time_point{};
  // Packing: a call running alone (with at most one other) copies its own chunks -- one thread
  // packed a 1 MiB Cauchy(6+3) decode's 6 MiB in 164 us against 200 us on the 8-thread copy pool,
  // at a quarter of the CPU (profiles/r03_v20_slot_phases.txt; 1 MiB decodes at one thread
  // 19.1 -> 22.6 GiB/s, RS(6+3) 1 MiB encodes 12.9 -> 16.1).  Under concurrency the pool, whose
  // workers sit on the GPU's NUMA node, packs faster (8 threads: 46.0 pool vs 34.8 inline;
  // profiles/r03_v21_fnptr_fair.jsonl).  LSEC_ZC_POOL=1 / 0 forces either (A/B runs).
  static const int pool_mode = [] {
    const char *v = getenv("LSEC_ZC_POOL");
    return v && *v ? (*v == '1' ? 1 : 0) : -1;
  }();
  static std::atomic<int> slot_calls{0};
  struct InFlight {
    std::atomic<int> &n;
    const int at;
    explicit InFlight(std::atomic<int> &c) : n(c), at(c.fetch_add(1, std::memory_order_acq_rel) + 1) {}
    ~InFlight() { n.fetch_sub(1, std::memory_order_acq_rel); }
  } inflight(slot_calls);
  const bool pool = pool_mode >= 0 ? pool_mode == 1 : inflight.at > 2;
  const auto pack = [&](std::vector<CopyJob> &js) {
    if (pool) {
      CopyPool::get().run(js, 64 << 10);
      return;
    }
    for (const CopyJob &j : js) host_copy(j.dst, j.src, j.bytes);
    _mm_sfence();  // the streamed bytes are visible before the launch (or the return) that follows
  };
  if (stats) ZcStats::get().s_alloc.fetch_add(tns(tl_zc_t0, t_last), std::memory_order_relaxed);
  const auto lap = [&](std::atomic<unsigned long long> &acc) {
    if (!stats) return;
    const auto t = tnow();
    acc.fetch_add(tns(t_last, t), std::memory_order_relaxed);
    t_last = t;
  };
  // slot layout: inputs [s][nin][C], then outputs [s][nout][C].  Calls of 1 MiB and more are
  // packed and computed in blocks of about 1 MiB (groups of stripes, or column blocks of a
  // single stripe): the copy pool packs block b+1 while the kernel of block b reads the slot over
  // PCIe, and a 7 MiB call no longer waits for all its packing before the GPU starts.
  const size_t in_bytes = static_cast<size_t>(nstripes) * nin * C;
  const int nblk = static_cast<int>(std::min<size_t>(16, std::max<size_t>(1, need >> 20)));
  const long long unit = packet_kind(kind) ? static_cast<long long>(p->w) * p->packet_size : 16;
  const bool by_cols = nstripes == 1 && nblk > 1 && C > unit;
  const int sg = by_cols ? 1 : (nstripes + nblk - 1) / nblk;                       // stripes per block
  const long long cl = by_cols ? ((C + nblk - 1) / nblk + unit - 1) / unit * unit : C;  // columns per block
  std::vector<CopyJob> jobs;
  for (int s0 = 0; s0 < nstripes; s0 += sg) {
    const int n = std::min(sg, nstripes - s0);
    for (long long c0 = 0; c0 < C; c0 += cl) {
      const long long len = std::min(cl, C - c0);
      jobs.clear();
      for (int s = s0; s < s0 + n; ++s)
        for (size_t j = 0; j < nin; ++j)
          jobs.push_back({slot->h + (s * nin + j) * C + c0, ptrs[static_cast<size_t>(s) * km + in_ids[j]] + c0,
                          static_cast<size_t>(len)});
      pack(jobs);
      lap(ZcStats::get().s_pack);
      for (size_t j = 0; j < nin; ++j) in[j] = {slot->d + (s0 * nin + j) * C + c0, static_cast<int64_t>(nin * C)};
      for (size_t r = 0; r < nout; ++r)
        out[r] = {slot->d + in_bytes + (s0 * nout + r) * C + c0, static_cast<int64_t>(nout * C)};
      if (enqueue_apply(kind, image, static_cast<int>(nin), static_cast<int>(nout), in, out, n, len, p->packet_size, st, p->w))
        return -1;
      lap(ZcStats::get().s_enq);
    }
  }
  if (zc_complete(*slot, st)) return -1;
  lap(ZcStats::get().s_wait);
  jobs.clear();
  for (int s = 0; s < nstripes; ++s)
    for (size_t r = 0; r < nout; ++r)
      jobs.push_back({ptrs[static_cast<size_t>(s) * km + out_ids[r]], slot->h + in_bytes + (s * nout + r) * C, static_cast<size_t>(C)});
  pack(jobs);
  lap(ZcStats::get().s_out);
  return 0;
}

ZcSlot &thread_zc_slot(int dev) {
  static thread_local std::map<int, std::unique_ptr<ZcSlot>> slots;
  std::unique_ptr<ZcSlot> &slot = slots[dev];
  if (!slot) slot.reset(new ZcSlot());
  return *slot;
}

// host-memory batches: small ones are served zero-copy by the calling thread (or coalesced
// with concurrent callers), large ones stream through their own staging pipeline
//
// Between the zero-copy and coalescing limits (LStore's 1 MiB chunks: 9 MiB per RS(6+3)
// stripe), a call of at least 4 MiB takes its own pipeline (in-place pinned from 8 MiB, else
// packed on the copy pool) while few
// such calls run at once: no packing copies (RS(6+3) 1 MiB encode at one thread 15 -> 27 GiB/s,
// Cauchy at 8 threads 19-23 -> 35-36); with many, the registrations contend on the runtime and
// the dispatcher's packed batches win (decode at 32 threads 38 vs 17 GiB/s;
// profiles/r02_v36_route_1m.jsonl; gated vs dispatcher-only in r02_v36_route_1m2.jsonl).
int run_host_auto(PlanExt *e, char **ptrs, int nstripes, long long C, const std::vector<int> &in_ids,
                  const std::vector<int> &out_ids, const void *image, int kind) {
  const size_t bytes = static_cast<size_t>(nstripes) * (in_ids.size() + out_ids.size()) * C;
  static const int own_max = [] {  // LSEC_OWN_PIPELINE_MAX: A/B runs (0: always the dispatcher)
    const char *v = getenv("LSEC_OWN_PIPELINE_MAX");
    return v ? std::max(0, atoi(v)) : std::max(2, usable_cpus() / 2);
  }();
  static std::atomic<int> own_inflight{0};
  if (bytes <= zerocopy_limit()) {
    const int rc = run_zerocopy(e, ptrs, nstripes, C, in_ids, out_ids, image, kind);
    if (rc != 1) return rc;  // 1: its slot would pass the page-locked budget
  }
  if (bytes <= coalesce_limit()) {
    if (bytes >= (4u << 20) && own_max > 0) {
      if (own_inflight.fetch_add(1, std::memory_order_acq_rel) < own_max) {
        static const bool zc_big = [] {  // LSEC_ZC_BIG=0: 4-16 MiB calls on their own staging pipeline (A/B runs)
          const char *v = getenv("LSEC_ZC_BIG");
          return !v || *v != '0';
        }();
        int rc = zc_big ? run_zerocopy(e, ptrs, nstripes, C, in_ids, out_ids, image, kind) : 1;
        if (rc == 1) rc = run_host(e, ptrs, nstripes, C, in_ids, out_ids, image, kind);
        own_inflight.fetch_sub(1, std::memory_order_acq_rel);
        return rc;
      }
      own_inflight.fetch_sub(1, std::memory_order_acq_rel);
    }
    return run_coalesced(e, ptrs, nstripes, C, in_ids, out_ids, image, kind);
  }
  return run_host(e, ptrs, nstripes, C, in_ids, out_ids, image, kind);
}

// Last resort of the per-stripe fn-pointers after a failed call (a pinned allocation or a
// registration refused, a dispatcher error): plain synchronous copies of the caller's chunks
// into per-thread device scratch, the kernel, and synchronous copies back -- no page-locked
// memory, no dispatcher, no kernel transport.  Still the GPU kernels: there is no CPU path.
int run_direct(PlanExt *e, char **ptrs, long long C, const std::vector<int> &in_ids, const std::vector<int> &out_ids,
               const void *image, int kind) {
  struct Scratch {
    int dev = -1;
    char *d = nullptr;
    size_t cap = 0;
    ~Scratch() {
      if (d) (void)hipFree(d);
    }
  };
  static thread_local Scratch sc;
  int dev = 0;
  HIP_OK(hipGetDevice(&dev));
  const size_t nin = in_ids.size(), nout = out_ids.size(), need = (nin + nout) * static_cast<size_t>(C);
  if (sc.dev != dev || sc.cap < need) {
    if (sc.d) {
      (void)hipSetDevice(sc.dev);
      (void)hipFree(sc.d);
      (void)hipSetDevice(dev);
    }
    sc.d = nullptr;
    sc.cap = 0;
    sc.dev = dev;
    HIP_OK(hipMalloc(&sc.d, need));
    sc.cap = need;
  }
  hipStream_t st = thread_stream();
  if (!st) return fail("no HIP stream");
  ShardRef in[kMaxDevs], out[kMaxDevs];
  for (size_t j = 0; j < nin; ++j) {
    HIP_OK(hipMemcpyAsync(sc.d + j * C, ptrs[in_ids[j]], C, hipMemcpyHostToDevice, st));
    in[j] = {reinterpret_cast<uint64_t>(sc.d) + j * C, 0};
  }
  for (size_t r = 0; r < nout; ++r) out[r] = {reinterpret_cast<uint64_t>(sc.d) + (nin + r) * C, 0};
  if (enqueue_apply(kind, image, static_cast<int>(nin), static_cast<int>(nout), in, out, 1, C, e->pub.packet_size, st, e->pub.w))
    return -1;
  for (size_t r = 0; r < nout; ++r) HIP_OK(hipMemcpyAsync(ptrs[out_ids[r]], sc.d + (nin + r) * C, C, hipMemcpyDeviceToHost, st));
  HIP_OK(hipStreamSynchronize(st));
  return 0;
}

// ---------------------------------------------------------------- host-path device set
// Host-memory calls run on the caller's current device unless lsec_set_host_devices() named a
// device set.  Then a batch above the coalescing limit is cut into contiguous stripe ranges,
// one per device, each driven by its own thread through that device's staging pipeline and
// PCIe link -- SURVEY §8e's static partition inside one LStore process -- and smaller calls go
// to the devices' dispatchers in turn.  Matrix images are per device (encode_cells /
// decode_entry are called on the device that runs the range).
std::mutex g_devs_mu;
std::vector<int> g_host_devs;  // empty: the caller's current device

std::atomic<unsigned> g_devs_version{0};  // bumped under g_devs_mu by every change

// the device set, as a per-thread copy refreshed only when lsec_set_host_devices changed it
// (no lock on the per-stripe path)
const std::vector<int> &host_devices() {
  thread_local std::vector<int> mine;
  thread_local unsigned seen = ~0u;
  const unsigned v = g_devs_version.load(std::memory_order_acquire);
  if (v != seen) {
    std::lock_guard<std::mutex> lk(g_devs_mu);
    mine = g_host_devs;
    seen = g_devs_version.load(std::memory_order_relaxed);
  }
  return mine;
}

struct DeviceGuard {
  int prev = -1;
  bool ok = true;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (dev != prev) ok = hipSetDevice(dev) == hipSuccess;
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

template <typename F>
int on_host_devices(int nstripes, size_t bytes, F &&fn) {
  const std::vector<int> devs = host_devices();
  if (devs.empty()) return fn(0, nstripes);
  if (devs.size() == 1 || nstripes < 2 || bytes <= coalesce_limit()) {
    static std::atomic<unsigned> rr{0};
    const int dev = devs[rr.fetch_add(1) % devs.size()];
    DeviceGuard g(dev);
    if (!g.ok) return fail("cannot select device %d", dev);
    return fn(0, nstripes);
  }
  const int G = std::min(static_cast<int>(devs.size()), nstripes);
  std::vector<int> rc(G, 0);
  std::vector<std::string> err(G);
  auto work = [&](int g) {
    const int base = nstripes / G, extra = nstripes % G;
    const int s0 = g * base + std::min(g, extra), n = base + (g < extra ? 1 : 0);
    DeviceGuard dg(devs[g]);
    // each range packs with its device's node-local copy pool (ec_numa.h)
    const int node0 = tl_copy_node;
    tl_copy_node = lsec::numa::of_device(devs[g]).node;
    rc[g] = dg.ok ? fn(s0, n) : fail("cannot select device %d", devs[g]);
    tl_copy_node = node0;
    if (rc[g]) err[g] = tl_err;  // tl_err is per thread
  };
  std::vector<std::thread> th;
  for (int g = 1; g < G; ++g)
    th.emplace_back([&work, &devs, g] {
      lsec::numa::bind_this_thread(devs[g]);  // a range thread of its own: on its device's node
      work(g);
    });
  work(0);
  for (auto &t : th) t.join();
  for (int g = 0; g < G; ++g)
    if (rc[g]) return fail("device %d: %s", devs[g], err[g].c_str());
  return 0;
}


int encode_stripes_impl(PlanExt *e, char **ptrs, int nstripes, long long C) {
  PtrMemo memo;
  lio_erasure_plan_t *p = &e->pub;
  if (!ptrs) return fail("ptrs is NULL");
  if (check_geometry(p, C)) return -1;
  if (nstripes <= 0 || C == 0) return 0;
  std::vector<lsec_shard_t> sh;
  const int dl = device_layout(p, ptrs, nstripes, sh);
  if (dl < 0) return -1;
  if (dl) {
    hipStream_t st = thread_stream();
    if (!st) return fail("no HIP stream");
    if (encode_dev(e, sh.data(), nstripes, C, st)) return -1;
    HIP_OK(hipStreamSynchronize(st));
    return 0;
  }
  if (ensure_coding(e)) return -1;
  const int k = p->data_strips, km = k + p->parity_strips;
  const int R = encode_rows(e);
  std::vector<int> in_ids(k), out_ids(R);
  for (int j = 0; j < k; ++j) in_ids[j] = j;
  for (int r = 0; r < R; ++r) out_ids[r] = k + r;
  return on_host_devices(nstripes, static_cast<size_t>(nstripes) * (k + R) * C, [&](int s0, int n) {
    const void *cells = nullptr;
    if (encode_cells(e, &cells)) return -1;
    return run_host_auto(e, ptrs + static_cast<size_t>(s0) * km, n, C, in_ids, out_ids, cells, kernel_kind(p->method, p->w));
  });
}

int decode_stripes_impl(PlanExt *e, char **ptrs, int nstripes, long long C, const int *erasures) {
  PtrMemo memo;
  lio_erasure_plan_t *p = &e->pub;
  if (!ptrs) return fail("ptrs is NULL");
  std::vector<int> ids;
  const int pr = parse_erasures(p, erasures, ids);
  if (pr < 0) return -1;
  if (pr == 1) return 0;
  if (check_geometry(p, C)) return -1;
  if (p->method == RAID4 && ids[0] >= p->data_strips) return 0;
  if (nstripes <= 0 || C == 0) return 0;
  std::vector<lsec_shard_t> sh;
  const int dl = device_layout(p, ptrs, nstripes, sh);
  if (dl < 0) return -1;
  if (dl) {
    hipStream_t st = thread_stream();
    if (!st) return fail("no HIP stream");
    if (decode_dev(e, sh.data(), nstripes, C, erasures, st)) return -1;
    HIP_OK(hipStreamSynchronize(st));
    return 0;
  }
  const int km = p->data_strips + p->parity_strips;
  return on_host_devices(nstripes, static_cast<size_t>(nstripes) * (p->data_strips + ids.size()) * C, [&](int s0, int n) {
    DecodeEntry *ent = nullptr;
    const void *cells = nullptr;
    if (decode_entry(e, ids, &ent, &cells)) return -1;
    return run_host_auto(e, ptrs + static_cast<size_t>(s0) * km, n, C, ent->dp.survivors, ent->dp.erased, cells,
                         decode_kind(e, ent));
  });
}

int encode_stripes_magic_impl(PlanExt *e, char **ptrs, int nstripes, long long C, uint8_t *magic) {
  lio_erasure_plan_t *p = &e->pub;
  if (!ptrs || !magic) return fail("ptrs / magic is NULL");
  if (check_geometry(p, C)) return -1;
  if (nstripes <= 0 || C == 0) return 0;
  if (ensure_coding(e)) return -1;
  const int k = p->data_strips, km = k + p->parity_strips;
  const int R = encode_rows(e);
  if (R != p->parity_strips) return fail("stripe magic needs m parity rows");
  std::vector<int> in_ids(k), out_ids(R);
  for (int j = 0; j < k; ++j) in_ids[j] = j;
  for (int r = 0; r < R; ++r) out_ids[r] = k + r;
  return on_host_devices(nstripes, static_cast<size_t>(nstripes) * km * C, [&](int s0, int n) {
    const void *cells = nullptr;
    if (encode_cells(e, &cells)) return -1;
    return run_host(e, ptrs + static_cast<size_t>(s0) * km, n, C, in_ids, out_ids, cells, kernel_kind(p->method, p->w),
                    magic + 4 * static_cast<size_t>(s0));
  });
}

int stripes_magic_impl(PlanExt *e, char **ptrs, int nstripes, long long C, uint8_t *magic) {
  lio_erasure_plan_t *p = &e->pub;
  if (!ptrs || !magic) return fail("ptrs / magic is NULL");
  if (C < 0 || C % 8 != 0) return fail("block_size %lld is not a multiple of 8", C);
  if (nstripes <= 0 || C == 0) return 0;
  const int km = p->data_strips + p->parity_strips;
  std::vector<int> in_ids(km), none;
  for (int i = 0; i < km; ++i) in_ids[i] = i;
  return on_host_devices(nstripes, static_cast<size_t>(nstripes) * km * C, [&](int s0, int n) {
    return run_host(e, ptrs + static_cast<size_t>(s0) * km, n, C, in_ids, none, nullptr, KBYTEWISE,
                    magic + 4 * static_cast<size_t>(s0));
  });
}

int magic_dev_impl(PlanExt *e, const lsec_shard_t *sh, int nstripes, long long C, uint8_t *magic, hipStream_t st) {
  lio_erasure_plan_t *p = &e->pub;
  const int km = p->data_strips + p->parity_strips;
  if (km > kMaxDevs) return fail("stripe magic supports at most %d chunks", kMaxDevs);
  if (C < 0 || C % 8 != 0) return fail("block_size %lld is not a multiple of 8", C);
  if (nstripes <= 0 || C == 0) return 0;
  unsigned long long *acc = nullptr;
  HIP_OK(hipMallocAsync(reinterpret_cast<void **>(&acc), 16ull * nstripes, st));
  HIP_OK(hipMemsetAsync(acc, 0, 16ull * nstripes, st));
  lsec::MagicArgs ma;
  std::memset(&ma, 0, sizeof(ma));
  ma.size = C;
  ma.col0 = 0;
  ma.chunk = C;
  const int per = static_cast<int>(std::max(1LL, (1LL << 30) / std::max(1LL, C / 8192 + 1)));
  ShardRef msh[kMaxDevs];
  for (int s0 = 0; s0 < nstripes; s0 += per) {
    ma.nstripes = std::min(per, nstripes - s0);
    ma.acc = acc + 2ull * s0;
    for (int i = 0; i < km; ++i)
      msh[i] = {reinterpret_cast<uint64_t>(sh[i].base) + static_cast<uint64_t>(s0) * sh[i].stride, sh[i].stride};
    HIP_OK(launch_magic_groups(ma, msh, km, st));
  }
  HIP_OK(lsec::launch_magic_finalize(acc, nstripes, static_cast<int64_t>(km) * C, magic, st));
  HIP_OK(hipFreeAsync(acc, st));
  return 0;
}

// plan->encode_block / plan->decode_block
// Retry of a failed host-memory fn-pointer call through run_direct.  Geometry errors are not
// retried (they would fail again); a plan from et_generate_plan never has them.
int retry_direct(PlanExt *e, char **ptr, long long C, const std::vector<int> &ids) {
  const std::string first = tl_err;
  lio_erasure_plan_t *p = &e->pub;
  if (check_geometry(p, C) != 0) return -1;
  std::vector<lsec_shard_t> sh;
  if (device_layout(p, ptr, 1, sh) != 0) {
    tl_err = first;  // device pointers (or mixed): nothing to retry with another transport
    return -1;
  }
  int rc;
  if (ids.empty()) {  // encode
    const int k = p->data_strips;
    const void *cells = nullptr;
    rc = encode_cells(e, &cells);
    if (rc == 0) {
      const int R = encode_rows(e);
      std::vector<int> in_ids(k), out_ids(R);
      for (int j = 0; j < k; ++j) in_ids[j] = j;
      for (int r = 0; r < R; ++r) out_ids[r] = k + r;
      rc = run_direct(e, ptr, C, in_ids, out_ids, cells, kernel_kind(p->method, p->w));
    }
  } else {
    DecodeEntry *ent = nullptr;
    const void *cells = nullptr;
    rc = decode_entry(e, ids, &ent, &cells);
    if (rc == 0) rc = run_direct(e, ptr, C, ent->dp.survivors, ent->dp.erased, cells, decode_kind(e, ent));
  }
  if (rc == 0) {
    static std::atomic<bool> warned{false};
    if (!warned.exchange(true))
      fprintf(stderr, "lstore_ec: a stripe call failed (%s); retried with direct copies\n", first.c_str());
    return 0;
  }
  tl_err = first + "; direct retry: " + tl_err;
  return -1;
}

void fp_encode_block(lio_erasure_plan_t *p, char **ptr, int block_size) {
  if (ZcStats::on()) {
    tl_call_t0 = std::chrono::steady_clock::now();
    tl_call_cpu0 = thread_cpu_ns();
  }
  PlanExt *e = ext_of(p);
  if (!e) fatal("encode_block on a plan not created by this library");
  if (encode_stripes_impl(e, ptr, 1, block_size) == 0) return;
  // encode_block cannot report a status, and writing no (or stale) parity would be stamped with
  // a matching stripe magic by the caller (segment/jerasure.c:1850): retry once, then abort as
  // Jerasure exits on errors (jerasure.c:306-310).  tl_err then holds both attempts' reasons
  // ("<first>; direct retry: <second>", retry_direct).
  if (retry_direct(e, ptr, block_size, {}) == 0) return;
  fatal("encode_block (k=%d m=%d w=%d C=%d) failed: %s", p->data_strips, p->parity_strips, p->w, block_size,
        tl_err.c_str());
}

int fp_decode_block(lio_erasure_plan_t *p, char **ptr, int block_size, int *erasures) {
  if (ZcStats::on()) {
    tl_call_t0 = std::chrono::steady_clock::now();
    tl_call_cpu0 = thread_cpu_ns();
  }
  PlanExt *e = ext_of(p);
  if (!e) return fail("not an lstore_ec plan");
  if (decode_stripes_impl(e, ptr, 1, block_size, erasures) == 0) return 0;
  std::vector<int> ids;
  if (parse_erasures(p, erasures, ids) != 0) return -1;
  if (p->method == RAID4 && ids[0] >= p->data_strips) return 0;
  return retry_direct(e, ptr, block_size, ids);
}

int fp_dummy(lio_erasure_plan_t *) { return 0; }

}  // namespace

namespace lsec {

int set_error(const char *fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  tl_err = buf;
  return -1;
}

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
        if (hipMemGetAddressRange(&b, &sz, d) != hipSuccess) {
          (void)hipGetLastError();
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

// ==================================================================== C ABI
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

// ---- extensions
int et_encode_stripes(lio_erasure_plan_t *plan, char **ptrs, int nstripes, int block_size) {
  PlanExt *e = ext_of(plan);
  if (!e) return fail("not an lstore_ec plan");
  return encode_stripes_impl(e, ptrs, nstripes, block_size);
}

int et_decode_stripes(lio_erasure_plan_t *plan, char **ptrs, int nstripes, int block_size, int *erasures) {
  PlanExt *e = ext_of(plan);
  if (!e) return fail("not an lstore_ec plan");
  return decode_stripes_impl(e, ptrs, nstripes, block_size, erasures);
}

int lsec_encode_dev(lio_erasure_plan_t *plan, const lsec_shard_t *shards, int nstripes, long long block_size,
                    void *stream) {
  PlanExt *e = ext_of(plan);
  if (!e) return fail("not an lstore_ec plan");
  if (!shards) return fail("shards is NULL");
  return encode_dev(e, shards, nstripes, block_size, static_cast<hipStream_t>(stream));
}

int lsec_decode_dev(lio_erasure_plan_t *plan, const lsec_shard_t *shards, int nstripes, long long block_size,
                    const int *erasures, void *stream) {
  PlanExt *e = ext_of(plan);
  if (!e) return fail("not an lstore_ec plan");
  if (!shards) return fail("shards is NULL");
  return decode_dev(e, shards, nstripes, block_size, erasures, static_cast<hipStream_t>(stream));
}

int et_encode_stripes_magic(lio_erasure_plan_t *plan, char **ptrs, int nstripes, int block_size, char *magic) {
  PlanExt *e = ext_of(plan);
  if (!e) return fail("not an lstore_ec plan");
  return encode_stripes_magic_impl(e, ptrs, nstripes, block_size, reinterpret_cast<uint8_t *>(magic));
}

int et_stripes_magic(lio_erasure_plan_t *plan, char **ptrs, int nstripes, int block_size, char *magic) {
  PlanExt *e = ext_of(plan);
  if (!e) return fail("not an lstore_ec plan");
  return stripes_magic_impl(e, ptrs, nstripes, block_size, reinterpret_cast<uint8_t *>(magic));
}

int lsec_stripe_magic_dev(lio_erasure_plan_t *plan, const lsec_shard_t *shards, int nstripes, long long block_size,
                          void *magic, void *stream) {
  PlanExt *e = ext_of(plan);
  if (!e) return fail("not an lstore_ec plan");
  if (!shards || !magic) return fail("shards / magic is NULL");
  return magic_dev_impl(e, shards, nstripes, block_size, static_cast<uint8_t *>(magic), static_cast<hipStream_t>(stream));
}

int lsec_encode_magic_dev(lio_erasure_plan_t *plan, const lsec_shard_t *shards, int nstripes, long long block_size,
                          void *magic, void *stream) {
  PlanExt *e = ext_of(plan);
  if (!e) return fail("not an lstore_ec plan");
  if (!shards || !magic) return fail("shards / magic is NULL");
  hipStream_t st = static_cast<hipStream_t>(stream);
  const int k = plan->data_strips, m = plan->parity_strips;
  // One pass: the encode kernel also accumulates the magic of the k inputs and m outputs.
  // Each lane keeps it in 32-bit dot-product chains (MagicLane, ec_kernels_impl.h), about
  // 3 VALU ops per data dword, so fusing wins at every k, m a single launch takes (m <= 8):
  // RS 12+4 5.9 ms fused vs 5.7 + 5.2 ms as two passes, Cauchy 6+3 5.9 vs 5.9 + 6.2 ms
  // (profiles/r01_v12_kbench_fused_magic.txt).
  const int kind = kernel_kind(plan->method, plan->w);
  const bool fuse = kind == KBYTEWISE || kind == KBITSLICED;
  if (fuse && m <= 8 && k <= lsec::kMaxK && !check_geometry(plan, block_size) && k + m <= lsec::kMaxMagicShards) {
    if (nstripes <= 0 || block_size == 0) return 0;
    const void *cells = nullptr;
    if (encode_cells(e, &cells)) return -1;
    if (encode_rows(e) != m) return fail("stripe magic needs m parity rows");
    unsigned long long *acc = nullptr;
    HIP_OK(hipMallocAsync(reinterpret_cast<void **>(&acc), 16ull * nstripes, st));
    HIP_OK(hipMemsetAsync(acc, 0, 16ull * nstripes, st));
    lsec::ApplyArgs a;
    std::memset(&a, 0, sizeof(a));
    a.cells = static_cast<const CoefCell *>(cells);
    a.K = k;
    a.R = m;
    a.size = block_size;
    a.packet = plan->packet_size;
    const int per = static_cast<int>(std::max(1LL, (1LL << 30) / std::max(1LL, block_size / 8192 + 1)));
    for (int s0 = 0; s0 < nstripes; s0 += per) {
      a.nstripes = std::min(per, nstripes - s0);
      a.magic_acc = acc + 2ull * s0;
      for (int j = 0; j < k; ++j)
        a.in[j] = {reinterpret_cast<uint64_t>(shards[j].base) + static_cast<uint64_t>(s0) * shards[j].stride, shards[j].stride};
      for (int r = 0; r < m; ++r)
        a.out[r] = {reinterpret_cast<uint64_t>(shards[k + r].base) + static_cast<uint64_t>(s0) * shards[k + r].stride,
                    shards[k + r].stride};
      HIP_OK(kind == KBITSLICED ? lsec::launch_bitsliced(a, st) : lsec::launch_bytewise_magic(a, st));
    }
    HIP_OK(lsec::launch_magic_finalize(acc, nstripes, static_cast<int64_t>(k + m) * block_size,
                                       static_cast<uint8_t *>(magic), st));
    HIP_OK(hipFreeAsync(acc, st));
    return 0;
  }
  if (encode_dev(e, shards, nstripes, block_size, st)) return -1;
  return magic_dev_impl(e, shards, nstripes, block_size, static_cast<uint8_t *>(magic), st);
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
  if (kind == KBYTEWISE ? lsec::bytewise_variant() != 0 : kind == KWORDWISE ? lsec::bitsliced_variant() != 0 : true)
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
  return lsec::jit::ready(cells, R, plan->data_strips) != nullptr ? 1 : 0;
}

int lsec_set_host_devices(const int *devices, int n) {
  std::vector<int> v;
  if (n > 0) {
    if (!devices) return fail("devices is NULL");
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess) {
      (void)hipGetLastError();
      return fail("no HIP device");
    }
    for (int i = 0; i < n; ++i) {
      if (devices[i] < 0 || devices[i] >= count) return fail("device %d outside 0..%d", devices[i], count - 1);
      v.push_back(devices[i]);
    }
  }
  std::lock_guard<std::mutex> lk(g_devs_mu);
  g_host_devs.swap(v);
  g_devs_version.fetch_add(1, std::memory_order_release);
  return 0;
}

int lsec_abi_version(void) { return LSEC_ABI_VERSION; }

int lsec_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    return 0;
  }
  return n;
}

const char *lsec_last_error(void) { return tl_err.c_str(); }

int lsec_plan_kernel(lio_erasure_plan_t *plan) { return plan ? kernel_kind(plan->method, plan->w) : 0; }

void lsec_set_kernel_variant(int bytewise_variant, int bitsliced_variant) {
  lsec::set_kernel_variant(bytewise_variant, bitsliced_variant);
}

int lsec_hbm_copy_dev(void *dst, const void *src, unsigned long long bytes, void *stream) {
  const hipError_t e = lsec::launch_hbm_copy(dst, src, bytes, static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return fail("lsec_hbm_copy_dev: %s", hipGetErrorString(e));
  return 0;
}

int lsec_hbm_mix_dev(const lsec_shard_t *shards, int k, int m, int nstripes, long long block_size, void *stream) {
  if (!shards || k < 1 || k > lsec::kMaxK || m < 1 || m > lsec::kMaxR || nstripes < 0 || block_size < 0 ||
      block_size % 8 != 0)
    return fail("lsec_hbm_mix_dev: bad arguments (k=%d m=%d nstripes=%d block_size=%lld)", k, m, nstripes, block_size);
  lsec::ApplyArgs a;
  std::memset(&a, 0, sizeof(a));
  a.K = k;
  a.R = m;
  a.nstripes = nstripes;
  a.size = block_size;
  for (int j = 0; j < k; ++j) a.in[j] = {reinterpret_cast<uint64_t>(shards[j].base), shards[j].stride};
  for (int r = 0; r < m; ++r) a.out[r] = {reinterpret_cast<uint64_t>(shards[k + r].base), shards[k + r].stride};
  const hipError_t e = lsec::launch_hbm_mix(a, static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return fail("lsec_hbm_mix_dev: %s", hipGetErrorString(e));
  return 0;
}

// Self-test of the completion waits (FlagWaits: spinners, lock-free parking, pollers) with the
// flags written by host threads instead of the GPU: `threads` waiters, each with a producer that
// sets its 1..16 flags in random order after a random delay of 0-300 us, `iters` rounds.  Every
// wait must end with all its flags set and within 2 s.  Test hook, not part of include/*.h;
// needs no GPU.  Returns 0, or -1 with a message.
// Test hook, not part of include/*.h: hold = 1 makes stripe servers launched from now on poll
// but serve nothing (a server that never answers); timeout_ms sets how long a call waits for
// its parts (default 5000).  Running servers are stopped so the next launch takes the setting.
// Returns the number of server calls that have timed out (or lost their server) so far.
int lsec_device_numa(int dev, int *node, int *cpus, int max_cpus) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) {
    (void)hipGetLastError();
    n = 0;
  }
  if (dev < 0 || dev >= n) return fail("lsec_device_numa: no device %d", dev);
  const lsec::numa::Placement &pl = lsec::numa::of_device(dev);
  if (node) *node = pl.node;
  for (int i = 0; cpus && i < max_cpus && i < static_cast<int>(pl.cpus.size()); ++i) cpus[i] = pl.cpus[i];
  return static_cast<int>(pl.cpus.size());
}

// Test hook, not part of include/*.h: the placement of PCI function `bus` under the sysfs tree
// `root` (a fake tree in tests/test_numa.py), unfiltered by this process's affinity.
int lsec_test_numa_for_bus(const char *root, const char *bus, int *node, int *cpus, int max_cpus) {
  if (!root || !bus) return fail("lsec_test_numa_for_bus: NULL argument");
  const lsec::numa::Placement pl = lsec::numa::for_bus(root, bus, {});
  if (node) *node = pl.node;
  for (int i = 0; cpus && i < max_cpus && i < static_cast<int>(pl.cpus.size()); ++i) cpus[i] = pl.cpus[i];
  return static_cast<int>(pl.cpus.size());
}

long long lsec_test_server_hold(int hold, int timeout_ms) {
  if (hold >= 0) g_srv_hold.store(hold ? 1 : 0);
  if (timeout_ms > 0) g_srv_timeout_ms.store(timeout_ms);
  if (hold >= 0) StripeServer::restart_all();
  return static_cast<long long>(g_st_srv_timeouts.load());
}

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

// Test hook, not in include/ (no GPU): the zero-copy page-locked accounting (PinnedBudget) on a
// fresh instance with a slot budget of budget_mb per device: `ndev` devices each start their
// stripe server, every device but 0 fills its threads' slots with slot_mb slots, then device 0
// takes slot_mb slots until refused.  Returns how many it got; *server_mb = the servers' total.
long long lsec_test_pinned_budget(int ndev, long long budget_mb, long long slot_mb, long long *server_mb) {
  if (ndev < 1 || ndev > PinnedBudget::kDevs || budget_mb < 0 || slot_mb < 1) return fail("lsec_test_pinned_budget: bad arguments");
  PinnedBudget b(static_cast<size_t>(budget_mb) << 20);
  const size_t region = lsec::kSrvSlotBytes * lsec::kSrvSlots, slot = static_cast<size_t>(slot_mb) << 20;
  for (int d = 0; d < ndev; ++d) b.add_server(d, region);
  for (int d = 1; d < ndev; ++d)
    while (b.grow_slot(d, 0, slot)) {
    }
  long long n = 0;
  while (b.grow_slot(0, 0, slot)) ++n;
  size_t total = 0;
  for (int d = 0; d < ndev; ++d) total += b.server_bytes(d);
  if (server_mb) *server_mb = static_cast<long long>(total >> 20);
  return n;
}

int lsec_selftest_waits(int threads, int iters) {
  if (threads < 1 || threads > 512 || iters < 1) return fail("lsec_selftest_waits: bad arguments");
  struct alignas(64) Pair {
    unsigned flags[16][16];  // one 64-byte line per flag, as the server's done lines
    std::atomic<int> ready{-1};
    int n = 1;
  };
  std::vector<std::unique_ptr<Pair>> pairs;
  for (int t = 0; t < threads; ++t) {
    pairs.emplace_back(new Pair());
    std::memset(pairs.back()->flags, 0, sizeof(pairs.back()->flags));
    pairs.back()->n = 1 + (t * 7) % 16;
  }
  std::atomic<int> bad{0};
  const unsigned long long parks0 = g_st_parks.load(), wakes0 = g_st_wakes.load();
  std::vector<std::thread> th;
  for (int t = 0; t < threads; ++t) {
    th.emplace_back([&, t] {  // producer
      Pair &p = *pairs[t];
      uint64_t x = 0x9E3779B97F4A7C15ull * (t + 1);
      for (int it = 0; it < iters && !bad.load(); ++it) {
        while (p.ready.load(std::memory_order_acquire) < it && !bad.load()) std::this_thread::yield();
        x ^= x << 13, x ^= x >> 7, x ^= x << 17;
        std::this_thread::sleep_for(std::chrono::microseconds(x % 300));
        int order[16];
        for (int i = 0; i < p.n; ++i) order[i] = i;
        for (int i = p.n - 1; i > 0; --i) std::swap(order[i], order[(x >> (i % 48)) % (i + 1)]);
        for (int i = 0; i < p.n; ++i) __atomic_store_n(&p.flags[order[i]][0], static_cast<unsigned>(it + 1), __ATOMIC_RELEASE);
      }
    });
    th.emplace_back([&, t] {  // waiter
      Pair &p = *pairs[t];
      const unsigned *f[16];
      unsigned want[16];
      for (int i = 0; i < p.n; ++i) f[i] = &p.flags[i][0];
      for (int it = 0; it < iters && !bad.load(); ++it) {
        for (int i = 0; i < p.n; ++i) want[i] = static_cast<unsigned>(it + 1);
        p.ready.store(it, std::memory_order_release);
        const auto t0 = std::chrono::steady_clock::now();
        while (!FlagWaits::get().wait(f, want, p.n, std::chrono::microseconds(500))) {
          if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
            bad.store(1);
            return;
          }
        }
        for (int i = 0; i < p.n; ++i)
          if (static_cast<int>(__atomic_load_n(f[i], __ATOMIC_ACQUIRE) - want[i]) < 0) {
            bad.store(2);
            return;
          }
      }
    });
  }
  for (auto &x : th) x.join();
  if (bad.load() == 1) return fail("lsec_selftest_waits: a wait did not end within 2 s of its flags");
  if (bad.load() == 2) return fail("lsec_selftest_waits: a wait returned before all its flags were set");
  // delays up to 300 us against a 30 us spin: long runs must have parked and been woken
  if (static_cast<long long>(threads) * iters >= 200 && (g_st_parks.load() == parks0 || g_st_wakes.load() == wakes0))
    return fail("lsec_selftest_waits: no waiter parked or was woken by a poller");
  return 0;
}

}  // extern "C"
