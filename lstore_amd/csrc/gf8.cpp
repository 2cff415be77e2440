// gf8.cpp -- host-side GF(2^8) algebra for the plan service.  See gf8.h.
#include "gf8.h"

#include <algorithm>
#include <cstring>

namespace lsec {
namespace gf8 {

namespace {

struct Tables {
  uint8_t exp[512];
  int16_t log[256];
  uint8_t prod[256][256];
  Tables() {
    unsigned x = 1;
    for (int i = 0; i < 255; ++i) {
      exp[i] = exp[i + 255] = static_cast<uint8_t>(x);
      log[x] = static_cast<int16_t>(i);
      x <<= 1;
      if (x & 0x100) x ^= 0x11D;
    }
    exp[510] = exp[511] = exp[0];
    log[0] = -1;
    for (int a = 0; a < 256; ++a)
      for (int b = 0; b < 256; ++b)
        prod[a][b] = (a && b) ? exp[log[a] + log[b]] : 0;
  }
};

const Tables &T() {
  static const Tables t;  // thread-safe static init (C++11)
  return t;
}

}  // namespace

uint8_t mul(uint8_t a, uint8_t b) { return T().prod[a][b]; }
uint8_t div(uint8_t a, uint8_t b) { return a ? T().exp[T().log[a] + 255 - T().log[b]] : 0; }
uint8_t inv(uint8_t a) { return T().exp[255 - T().log[a]]; }

// ---------------------------------------------------------------- Reed-Solomon
// The systematic Vandermonde "distribution matrix" of Jerasure (reed_sol.c:242-367):
// start from the extended Vandermonde matrix V[(k+m) x k] (row 0 = e0, last row = e_{k-1},
// row i = powers of i), column-reduce the top k x k block to the identity, scale every
// column so that row k is all ones, then scale each later row so its column 0 is one.
bool reed_sol_vandermonde(int k, int m, Mat &out) {
  const int rows = k + m;
  if (k < 1 || m < 1 || rows > 256) return false;
  std::vector<uint8_t> v(static_cast<size_t>(rows) * k, 0);
  auto at = [&](int r, int c) -> uint8_t & { return v[static_cast<size_t>(r) * k + c]; };
  at(0, 0) = 1;
  at(rows - 1, k - 1) = 1;
  for (int r = 1; r < rows - 1; ++r) {
    uint8_t p = 1;
    for (int c = 0; c < k; ++c) { at(r, c) = p; p = mul(p, static_cast<uint8_t>(r)); }
  }
  for (int piv = 1; piv < k; ++piv) {
    int r = piv;
    while (r < rows && at(r, piv) == 0) ++r;
    if (r == rows) return false;
    if (r != piv)
      for (int c = 0; c < k; ++c) std::swap(at(r, c), at(piv, c));
    if (at(piv, piv) != 1) {
      const uint8_t s = inv(at(piv, piv));
      for (int rr = 0; rr < rows; ++rr) at(rr, piv) = mul(s, at(rr, piv));
    }
    for (int c = 0; c < k; ++c) {
      const uint8_t e = at(piv, c);
      if (c == piv || e == 0) continue;
      for (int rr = 0; rr < rows; ++rr) at(rr, c) ^= mul(e, at(rr, piv));
    }
  }
  for (int c = 0; c < k; ++c) {
    const uint8_t e = at(k, c);
    if (e == 1) continue;
    const uint8_t s = inv(e);
    for (int rr = k; rr < rows; ++rr) at(rr, c) = mul(s, at(rr, c));
  }
  for (int rr = k + 1; rr < rows; ++rr) {
    const uint8_t e = at(rr, 0);
    if (e == 1) continue;
    const uint8_t s = inv(e);
    for (int c = 0; c < k; ++c) at(rr, c) = mul(at(rr, c), s);
  }
  out.assign(v.begin() + static_cast<size_t>(k) * k, v.end());
  return true;
}

bool reed_sol_r6(int k, Mat &out) {
  if (k < 1 || k > 255) return false;
  out.assign(2 * static_cast<size_t>(k), 1);
  uint8_t p = 1;
  for (int j = 0; j < k; ++j) { out[k + j] = p; p = mul(p, 2); }
  return true;
}

// ---------------------------------------------------------------- Cauchy
int bit_block_ones(uint8_t e) {
  int n = 0;
  for (int x = 0; x < 8; ++x) { n += __builtin_popcount(e); e = mul(e, 2); }
  return n;
}

bool cauchy_original(int k, int m, Mat &out) {
  if (k < 1 || m < 1 || k + m > 256) return false;
  out.resize(static_cast<size_t>(k) * m);
  for (int i = 0; i < m; ++i)
    for (int j = 0; j < k; ++j) out[i * k + j] = inv(static_cast<uint8_t>(i ^ (m + j)));
  return true;
}

void cauchy_improve(int k, int m, Mat &a) {
  for (int j = 0; j < k; ++j) {           // make row 0 all ones (column scaling)
    if (a[j] == 1) continue;
    const uint8_t s = inv(a[j]);
    for (int i = 0; i < m; ++i) a[i * k + j] = mul(a[i * k + j], s);
  }
  for (int i = 1; i < m; ++i) {           // then pick, per row, the scaling with fewest ones
    uint8_t *row = &a[static_cast<size_t>(i) * k];
    int best = 0, best_col = -1;
    for (int j = 0; j < k; ++j) best += bit_block_ones(row[j]);
    for (int j = 0; j < k; ++j) {
      if (row[j] == 1) continue;
      const uint8_t s = inv(row[j]);
      int ones = 0;
      for (int x = 0; x < k; ++x) ones += bit_block_ones(mul(row[x], s));
      if (ones < best) { best = ones; best_col = j; }
    }
    if (best_col >= 0) {
      const uint8_t s = inv(row[best_col]);
      for (int j = 0; j < k; ++j) row[j] = mul(row[j], s);
    }
  }
}

// Second rows of the optimal m = 2 Cauchy matrices for w = 8: a table of constants from
// vendor/jerasure/src/cauchy.c:262-274 (cbest_8), indexed by data column.
static const uint8_t kCauchyBestW8[255] = {
    1,   2,   142, 4,   71,  8,   70,  173, 3,   35,  143, 16,  17,  67,  134, 140, 172, 6,   34,
    69,  201, 216, 5,   33,  86,  12,  65,  138, 158, 159, 175, 10,  32,  43,  66,  108, 130, 193,
    234, 9,   24,  25,  50,  68,  79,  100, 132, 174, 200, 217, 20,  21,  42,  48,  87,  169, 41,
    54,  64,  84,  96,  117, 154, 155, 165, 226, 77,  82,  135, 136, 141, 168, 192, 218, 238, 7,
    18,  19,  39,  40,  78,  113, 116, 128, 164, 180, 195, 205, 220, 232, 14,  26,  27,  58,  109,
    156, 157, 203, 235, 13,  28,  29,  38,  51,  56,  75,  85,  90,  101, 110, 112, 139, 171, 11,
    37,  49,  52,  76,  83,  102, 119, 131, 150, 151, 167, 182, 184, 188, 197, 219, 224, 45,  55,
    80,  94,  97,  133, 170, 194, 204, 221, 227, 236, 36,  47,  73,  92,  98,  104, 118, 152, 153,
    166, 202, 207, 239, 251, 22,  23,  44,  74,  91,  148, 149, 161, 181, 190, 233, 46,  59,  88,
    137, 146, 147, 163, 196, 208, 212, 222, 250, 57,  81,  95,  106, 111, 129, 160, 176, 199, 243,
    249, 15,  53,  72,  93,  103, 115, 125, 162, 183, 185, 189, 206, 225, 255, 186, 210, 230, 237,
    242, 248, 30,  31,  62,  89,  99,  105, 114, 121, 124, 178, 209, 213, 223, 228, 241, 254, 60,
    191, 198, 247, 120, 240, 107, 127, 144, 145, 177, 211, 214, 246, 245, 123, 126, 187, 231, 253,
    63,  179, 229, 244, 61,  122, 215, 252};

bool cauchy_good(int k, int m, Mat &out) {
  if (m == 2 && k >= 1 && k <= 255) {
    out.assign(2 * static_cast<size_t>(k), 1);
    std::memcpy(&out[k], kCauchyBestW8, k);
    return true;
  }
  if (!cauchy_original(k, m, out)) return false;
  cauchy_improve(k, m, out);
  return true;
}

std::vector<int> to_bitmatrix(int k, int m, const Mat &a) {
  const int cols = k * 8;
  std::vector<int> bm(static_cast<size_t>(m) * 8 * cols, 0);
  for (int i = 0; i < m; ++i)
    for (int j = 0; j < k; ++j) {
      uint8_t e = a[i * k + j];
      for (int x = 0; x < 8; ++x, e = mul(e, 2))
        for (int l = 0; l < 8; ++l) bm[static_cast<size_t>(i * 8 + l) * cols + j * 8 + x] = (e >> l) & 1;
    }
  return bm;
}

// ---------------------------------------------------------------- schedule
// Greedy "smart" scheduling of Jerasure (jerasure.c:1241-1360): emit output rows in
// order of fewest remaining XORs; a row may start from a copy of an already emitted
// row (from[]) when that is cheaper than starting from scratch.  Reproduced op for op
// because plan->encode_schedule is part of the ABI the segment layer can see.
std::vector<std::array<int, 5>> smart_schedule(int k, int m, int w, const std::vector<int> &bm) {
  const int rows = m * w, cols = k * w;
  std::vector<std::array<int, 5>> ops;
  std::vector<int> diff(rows), from(rows, -1), next(rows), prev(rows);
  int best_row = -1, best = cols + 1;
  for (int r = 0; r < rows; ++r) {
    int ones = 0;
    for (int c = 0; c < cols; ++c) ones += bm[static_cast<size_t>(r) * cols + c];
    diff[r] = ones;
    next[r] = r + 1;
    prev[r] = r - 1;
    if (ones < best) { best = ones; best_row = r; }
  }
  next[rows - 1] = -1;
  int head = 0;
  while (head != -1) {
    const int row = best_row;
    if (prev[row] == -1) {                        // unlink row
      head = next[row];
      if (head != -1) prev[head] = -1;
    } else {
      next[prev[row]] = next[row];
      if (next[row] != -1) prev[next[row]] = prev[row];
    }
    const int *cur = &bm[static_cast<size_t>(row) * cols];
    if (from[row] == -1) {
      int x = 0;
      for (int c = 0; c < cols; ++c)
        if (cur[c]) { ops.push_back({c / w, c % w, k + row / w, row % w, x}); x = 1; }
    } else {
      ops.push_back({k + from[row] / w, from[row] % w, k + row / w, row % w, 0});
      const int *base = &bm[static_cast<size_t>(from[row]) * cols];
      for (int c = 0; c < cols; ++c)
        if (cur[c] ^ base[c]) ops.push_back({c / w, c % w, k + row / w, row % w, 1});
    }
    best = cols + 1;
    for (int r = head; r != -1; r = next[r]) {
      const int *other = &bm[static_cast<size_t>(r) * cols];
      int d = 1;
      for (int c = 0; c < cols; ++c) d += cur[c] ^ other[c];
      if (d < diff[r]) { from[r] = row; diff[r] = d; }
      if (diff[r] < best) { best = diff[r]; best_row = r; }
    }
  }
  return ops;
}

// ---------------------------------------------------------------- inversion / decode
bool invert(int n, Mat a, Mat &out) {
  out.assign(static_cast<size_t>(n) * n, 0);
  for (int i = 0; i < n; ++i) out[i * n + i] = 1;
  for (int c = 0; c < n; ++c) {
    int p = c;
    while (p < n && a[p * n + c] == 0) ++p;
    if (p == n) return false;
    if (p != c)
      for (int x = 0; x < n; ++x) { std::swap(a[p * n + x], a[c * n + x]); std::swap(out[p * n + x], out[c * n + x]); }
    const uint8_t s = inv(a[c * n + c]);
    for (int x = 0; x < n; ++x) { a[c * n + x] = mul(a[c * n + x], s); out[c * n + x] = mul(out[c * n + x], s); }
    for (int r = 0; r < n; ++r) {
      const uint8_t f = a[r * n + c];
      if (r == c || f == 0) continue;
      for (int x = 0; x < n; ++x) { a[r * n + x] ^= mul(f, a[c * n + x]); out[r * n + x] ^= mul(f, out[c * n + x]); }
    }
  }
  return true;
}

bool make_decode(int k, int m, const Mat &coding, const std::vector<int> &erased_ids, DecodePlan &dp) {
  std::vector<char> lost(k + m, 0);
  for (int e : erased_ids) {
    if (e < 0 || e >= k + m) return false;
    lost[e] = 1;
  }
  dp.erased.clear();
  dp.survivors.clear();
  for (int i = 0; i < k + m; ++i) {
    if (lost[i]) dp.erased.push_back(i);
    else if (static_cast<int>(dp.survivors.size()) < k) dp.survivors.push_back(i);
  }
  if (static_cast<int>(dp.survivors.size()) < k) return false;
  // S (k x k): row j expresses survivor j in terms of the data devices
  Mat s(static_cast<size_t>(k) * k, 0), sinv;
  for (int j = 0; j < k; ++j) {
    const int id = dp.survivors[j];
    if (id < k) s[j * k + id] = 1;
    else std::memcpy(&s[static_cast<size_t>(j) * k], &coding[static_cast<size_t>(id - k) * k], k);
  }
  if (!invert(k, s, sinv)) return false;
  // data_i = row i of S^-1 . survivors;  coding_i = C_i . data = (C_i . S^-1) . survivors
  dp.rows.assign(dp.erased.size() * k, 0);
  for (size_t r = 0; r < dp.erased.size(); ++r) {
    const int id = dp.erased[r];
    uint8_t *dst = &dp.rows[r * k];
    if (id < k) {
      std::memcpy(dst, &sinv[static_cast<size_t>(id) * k], k);
    } else {
      const uint8_t *crow = &coding[static_cast<size_t>(id - k) * k];
      for (int j = 0; j < k; ++j) {
        uint8_t acc = 0;
        for (int t = 0; t < k; ++t) acc ^= mul(crow[t], sinv[t * k + j]);
        dst[j] = acc;
      }
    }
  }
  return true;
}

namespace {

using BitRow = std::vector<uint64_t>;

bool bit_at(const BitRow &r, int c) { return (r[c / 64] >> (c % 64)) & 1; }
void set_bit(BitRow &r, int c) { r[c / 64] |= 1ull << (c % 64); }
void xor_into(BitRow &dst, const BitRow &src) {
  for (size_t x = 0; x < dst.size(); ++x) dst[x] ^= src[x];
}

// survivors / erased as make_decode (first k surviving ids, jerasure.c:100-128)
bool pick_survivors(int k, int m, const std::vector<int> &erased_ids, DecodePlan &dp) {
  std::vector<char> lost(k + m, 0);
  for (int e : erased_ids) {
    if (e < 0 || e >= k + m) return false;
    lost[e] = 1;
  }
  dp.erased.clear();
  dp.survivors.clear();
  for (int i = 0; i < k + m; ++i) {
    if (lost[i]) dp.erased.push_back(i);
    else if (static_cast<int>(dp.survivors.size()) < k) dp.survivors.push_back(i);
  }
  return static_cast<int>(dp.survivors.size()) == k;
}

// rows[(r*w + l)] over survivor bit columns -> the kernels' mask layout
void rows_to_masks(int k, int w, const std::vector<BitRow> &rows, std::vector<uint32_t> &masks) {
  const int nw = (w + 31) / 32;  // mask words per (bit-row, input), as lsec::mask_words
  const int n = k * w;
  masks.assign(rows.size() * k * nw, 0u);
  for (size_t rl = 0; rl < rows.size(); ++rl)
    for (int c = 0; c < n; ++c)
      if (bit_at(rows[rl], c)) masks[(rl * k + c / w) * nw + (c % w) / 32] |= 1u << (c % w % 32);
}

}  // namespace

// Solves only for the lost data bits.  With d data strips lost, the survivors are the k - d
// surviving data strips plus d coding strips (pick_survivors), so the unknowns are the d*w lost
// data bits and the equations the d*w bit-rows of those coding strips:
//   B_L . data_L = coding_P + B_D . data_D        (GF(2): minus is plus)
// A = B_L is (d*w) x (d*w); data_L = A^-1 . (coding_P + B_D . data_D), written over survivor bit
// columns.  A lost coding strip is re-encoded from data expressed the same way.  This is the
// decoding matrix jerasure_generate_decoding_schedule builds (jerasure.c:823-951) without its
// (k*w) x (k*w) inversion: O((d*w)^3 + (d*w)^2 * k*w / 64) word operations instead of
// O((k*w)^3 / 64), so liberation plans up to k = 254, w = 257 decode in well under a second.
// Decoded bytes are unique (the codes are MDS), so the rows equal make_bit_decode_dense's.
bool make_bit_decode(int k, int m, int w, const std::vector<int> &bm, const std::vector<int> &erased_ids,
                     DecodePlan &dp, std::vector<uint32_t> &masks) {
  if (!pick_survivors(k, m, erased_ids, dp)) return false;
  const int n = k * w;
  const int words = (n + 63) / 64;
  std::vector<int> pos(k + m, -1);  // survivor index of a device id
  for (int j = 0; j < k; ++j) pos[dp.survivors[j]] = j;
  std::vector<int> lost_data, used_coding;
  for (int id : dp.erased)
    if (id < k) lost_data.push_back(id);
  for (int id : dp.survivors)
    if (id >= k) used_coding.push_back(id);
  const int d = static_cast<int>(lost_data.size());
  if (static_cast<int>(used_coding.size()) != d) return false;
  const auto brow = [&](int id, int l) { return &bm[static_cast<size_t>((id - k) * w + l) * n]; };
  // known part of a coding bit-row over survivor columns: the row's surviving-data bits
  const auto data_part = [&](int id, int l, BitRow &row) {
    const int *src = brow(id, l);
    for (int j = 0; j < k; ++j) {
      if (pos[j] < 0) continue;
      for (int x = 0; x < w; ++x)
        if (src[j * w + x]) set_bit(row, pos[j] * w + x);
    }
  };
  std::vector<BitRow> lost_rows(static_cast<size_t>(d) * w, BitRow(words, 0));  // lost data bit (u, x)
  if (d > 0) {
    const int dw = d * w, aw = (dw + 63) / 64;
    std::vector<BitRow> a(dw, BitRow(aw, 0)), ainv(dw, BitRow(aw, 0));
    std::vector<BitRow> rhs(dw, BitRow(words, 0));  // coding_P + B_D . data_D over survivor columns
    for (int t = 0; t < d; ++t)
      for (int l = 0; l < w; ++l) {
        const int row = t * w + l;
        const int *src = brow(used_coding[t], l);
        for (int u = 0; u < d; ++u)
          for (int x = 0; x < w; ++x)
            if (src[lost_data[u] * w + x]) set_bit(a[row], u * w + x);
        set_bit(rhs[row], pos[used_coding[t]] * w + l);
        data_part(used_coding[t], l, rhs[row]);
      }
    for (int i = 0; i < dw; ++i) set_bit(ainv[i], i);
    for (int c = 0; c < dw; ++c) {  // Gauss-Jordan over GF(2)
      int p = c;
      while (p < dw && !bit_at(a[p], c)) ++p;
      if (p == dw) return false;
      std::swap(a[p], a[c]);
      std::swap(ainv[p], ainv[c]);
      for (int r = 0; r < dw; ++r)
        if (r != c && bit_at(a[r], c)) {
          xor_into(a[r], a[c]);
          xor_into(ainv[r], ainv[c]);
        }
    }
    for (int r = 0; r < dw; ++r)
      for (int c = 0; c < dw; ++c)
        if (bit_at(ainv[r], c)) xor_into(lost_rows[r], rhs[c]);
  }
  std::vector<int> lost_index(k, -1);
  for (int u = 0; u < d; ++u) lost_index[lost_data[u]] = u;
  std::vector<BitRow> out;
  out.reserve(dp.erased.size() * w);
  for (int id : dp.erased)
    for (int l = 0; l < w; ++l) {
      if (id < k) {
        out.push_back(lost_rows[static_cast<size_t>(lost_index[id]) * w + l]);
        continue;
      }
      BitRow row(words, 0);
      data_part(id, l, row);
      const int *src = brow(id, l);
      for (int u = 0; u < d; ++u)
        for (int x = 0; x < w; ++x)
          if (src[lost_data[u] * w + x]) xor_into(row, lost_rows[static_cast<size_t>(u) * w + x]);
      out.push_back(std::move(row));
    }
  rows_to_masks(k, w, out, masks);
  return true;
}

// The whole (k*w) x (k*w) survivor bitmatrix inverted, as jerasure_invert_bitmatrix does
// (jerasure.c:1049-1104).  Test comparator of make_bit_decode (lsec_selftest_bit_decode).
bool make_bit_decode_dense(int k, int m, int w, const std::vector<int> &bm, const std::vector<int> &erased_ids,
                           DecodePlan &dp, std::vector<uint32_t> &masks) {
  std::vector<char> lost(k + m, 0);
  for (int e : erased_ids) {
    if (e < 0 || e >= k + m) return false;
    lost[e] = 1;
  }
  dp.erased.clear();
  dp.survivors.clear();
  for (int i = 0; i < k + m; ++i) {
    if (lost[i]) dp.erased.push_back(i);
    else if (static_cast<int>(dp.survivors.size()) < k) dp.survivors.push_back(i);
  }
  if (static_cast<int>(dp.survivors.size()) < k) return false;
  const int n = k * w;
  // S: survivor bit-rows in terms of the data bits; rows packed as bitsets of n bits
  const int words = (n + 63) / 64;
  auto bit = [&](std::vector<uint64_t> &row, int c) { row[c / 64] |= 1ull << (c % 64); };
  std::vector<std::vector<uint64_t>> a(n, std::vector<uint64_t>(words, 0)), inv(n, std::vector<uint64_t>(words, 0));
  for (int j = 0; j < k; ++j) {
    const int id = dp.survivors[j];
    for (int l = 0; l < w; ++l) {
      auto &row = a[j * w + l];
      if (id < k) {
        bit(row, id * w + l);
      } else {
        const int *src = &bm[static_cast<size_t>((id - k) * w + l) * n];
        for (int c = 0; c < n; ++c)
          if (src[c]) bit(row, c);
      }
    }
  }
  for (int i = 0; i < n; ++i) bit(inv[i], i);
  for (int c = 0; c < n; ++c) {  // Gauss-Jordan over GF(2)
    int p = c;
    while (p < n && !((a[p][c / 64] >> (c % 64)) & 1)) ++p;
    if (p == n) return false;
    std::swap(a[p], a[c]);
    std::swap(inv[p], inv[c]);
    for (int r = 0; r < n; ++r)
      if (r != c && ((a[r][c / 64] >> (c % 64)) & 1))
        for (int x = 0; x < words; ++x) { a[r][x] ^= a[c][x]; inv[r][x] ^= inv[c][x]; }
  }
  // output bit-rows: erased data i -> inv rows i*w..; erased coding c -> B_c x inv
  const int e = static_cast<int>(dp.erased.size());
  const int nw = (w + 31) / 32;  // mask words per (bit-row, input), as lsec::mask_words
  masks.assign(static_cast<size_t>(e) * w * k * nw, 0u);
  for (int r = 0; r < e; ++r) {
    const int id = dp.erased[r];
    for (int l = 0; l < w; ++l) {
      std::vector<uint64_t> row(words, 0);
      if (id < k) {
        row = inv[id * w + l];
      } else {
        const int *src = &bm[static_cast<size_t>((id - k) * w + l) * n];
        for (int c = 0; c < n; ++c)
          if (src[c])
            for (int x = 0; x < words; ++x) row[x] ^= inv[c][x];
      }
      for (int c = 0; c < n; ++c)
        if ((row[c / 64] >> (c % 64)) & 1)
          masks[(static_cast<size_t>(r * w + l) * k + c / w) * nw + (c % w) / 32] |= 1u << (c % w % 32);
    }
  }
  return true;
}

// ---------------------------------------------------------------- liberation family
// Layout helper: a (2w) x (kw) bitmatrix whose first w rows are [I I ... I].
static std::vector<int> identity_top(int k, int w) {
  std::vector<int> bm(2 * static_cast<size_t>(k) * w * w, 0);
  for (int i = 0; i < w; ++i)
    for (int j = 0; j < k; ++j) bm[static_cast<size_t>(i) * k * w + j * w + i] = 1;
  return bm;
}

std::vector<int> liberation_bitmatrix(int k, int w) {
  if (k > w) return {};
  std::vector<int> bm = identity_top(k, w);
  const size_t q = static_cast<size_t>(k) * w * w;  // start of the Q block row
  const int kw = k * w;
  for (int j = 0; j < k; ++j) {
    for (int i = 0; i < w; ++i) bm[q + static_cast<size_t>(i) * kw + j * w + (j + i) % w] = 1;
    if (j > 0) {
      const int i = (j * ((w - 1) / 2)) % w;
      bm[q + static_cast<size_t>(i) * kw + j * w + (i + j - 1) % w] = 1;
    }
  }
  return bm;
}

// liber8tion Q block (liberation.c:167-265, constants): for data column j, row r of the
// 8x8 block has a one at column kLib8Perm[j][r]; plus one extra bit kLib8Extra[j] =
// {row, col} for j >= 1.
static const int8_t kLib8Perm[8][8] = {
    {0, 1, 2, 3, 4, 5, 6, 7}, {7, 3, 0, 2, 6, 1, 5, 4}, {6, 2, 4, 0, 7, 3, 1, 5},
    {2, 5, 7, 6, 0, 3, 4, 1}, {5, 6, 1, 7, 2, 4, 3, 0}, {1, 2, 3, 4, 5, 6, 7, 0},
    {3, 0, 6, 5, 1, 7, 4, 2}, {4, 7, 1, 5, 3, 2, 0, 6}};
static const int8_t kLib8Extra[8][2] = {{-1, -1}, {4, 7}, {1, 3}, {5, 4}, {2, 0}, {7, 2}, {6, 5}, {3, 1}};

std::vector<int> liber8tion_bitmatrix(int k) {
  const int w = 8;
  if (k > w) return {};
  std::vector<int> bm = identity_top(k, w);
  const size_t q = static_cast<size_t>(k) * w * w;
  const int kw = k * w;
  for (int j = 0; j < k; ++j) {
    for (int r = 0; r < 8; ++r) bm[q + static_cast<size_t>(r) * kw + j * w + kLib8Perm[j][r]] = 1;
    if (kLib8Extra[j][0] >= 0) bm[q + static_cast<size_t>(kLib8Extra[j][0]) * kw + j * w + kLib8Extra[j][1]] = 1;
  }
  return bm;
}

std::vector<int> blaum_roth_bitmatrix(int k, int w) {
  if (k > w) return {};
  std::vector<int> bm = identity_top(k, w);
  const size_t q = static_cast<size_t>(k) * w * w;
  const int kw = k * w, p = w + 1;
  for (int j = 0; j < k; ++j) {
    for (int l = 1; l <= w; ++l) {
      int *row = &bm[q + static_cast<size_t>(l - 1) * kw + j * w];
      if (j == 0) { row[l - 1] = 1; continue; }
      if (l != p - j) {
        int c = l + j;
        if (c >= p) c -= p;
        row[c - 1] = 1;
      } else {
        row[j - 1] = 1;
        const int c = (j % 2 == 0) ? j / 2 : (p / 2) + 1 + (j / 2);
        row[c - 1] = 1;
      }
    }
  }
  return bm;
}

}  // namespace gf8

// ==================================================================== GF(2^16) / GF(2^32)
namespace gfw {

namespace {
uint64_t full_poly(int w) { return w == 16 ? 0x1100Bull : (1ull << 32) | 0x400007ull; }
uint32_t field_mask(int w) { return w == 32 ? 0xFFFFFFFFu : (1u << w) - 1; }
}  // namespace

uint32_t mul(uint32_t a, uint32_t b, int w) {
  if (w == 8) return gf8::mul(static_cast<uint8_t>(a), static_cast<uint8_t>(b));
  uint64_t p = 0;  // carry-less product, then reduce from the top bit down
  for (int i = 0; i < w; ++i)
    if ((b >> i) & 1u) p ^= static_cast<uint64_t>(a) << i;
  const uint64_t f = full_poly(w);
  for (int i = 2 * w - 2; i >= w; --i)
    if ((p >> i) & 1u) p ^= f << (i - w);
  return static_cast<uint32_t>(p) & field_mask(w);
}

uint32_t times_x(uint32_t a, int w) { return mul(a, 2, w); }

uint32_t inv(uint32_t a, int w) {
  if (w == 8) return gf8::inv(static_cast<uint8_t>(a));
  // a^(2^w - 2): square-and-multiply over the exponent bits 1..w-1
  uint32_t r = 1, sq = a;
  for (int i = 1; i < w; ++i) {
    sq = mul(sq, sq, w);
    r = mul(r, sq, w);
  }
  return r;
}

bool reed_sol_vandermonde(int k, int m, int w, Mat &out) {
  const int rows = k + m;
  if (k < 1 || m < 1 || (w < 30 && (1 << w) < rows)) return false;
  Mat v(static_cast<size_t>(rows) * k, 0);
  auto at = [&](int r, int c) -> uint32_t & { return v[static_cast<size_t>(r) * k + c]; };
  at(0, 0) = 1;
  at(rows - 1, k - 1) = 1;
  for (int r = 1; r < rows - 1; ++r) {
    uint32_t p = 1;
    for (int c = 0; c < k; ++c) { at(r, c) = p; p = mul(p, static_cast<uint32_t>(r), w); }
  }
  for (int piv = 1; piv < k; ++piv) {
    int r = piv;
    while (r < rows && at(r, piv) == 0) ++r;
    if (r == rows) return false;
    if (r != piv)
      for (int c = 0; c < k; ++c) std::swap(at(r, c), at(piv, c));
    if (at(piv, piv) != 1) {
      const uint32_t s = inv(at(piv, piv), w);
      for (int rr = 0; rr < rows; ++rr) at(rr, piv) = mul(s, at(rr, piv), w);
    }
    for (int c = 0; c < k; ++c) {
      const uint32_t e = at(piv, c);
      if (c == piv || e == 0) continue;
      for (int rr = 0; rr < rows; ++rr) at(rr, c) ^= mul(e, at(rr, piv), w);
    }
  }
  for (int c = 0; c < k; ++c) {
    const uint32_t e = at(k, c);
    if (e == 1) continue;
    const uint32_t s = inv(e, w);
    for (int rr = k; rr < rows; ++rr) at(rr, c) = mul(s, at(rr, c), w);
  }
  for (int rr = k + 1; rr < rows; ++rr) {
    const uint32_t e = at(rr, 0);
    if (e == 1) continue;
    const uint32_t s = inv(e, w);
    for (int c = 0; c < k; ++c) at(rr, c) = mul(at(rr, c), s, w);
  }
  out.assign(v.begin() + static_cast<size_t>(k) * k, v.end());
  return true;
}

bool reed_sol_r6(int k, int w, Mat &out) {
  if (k < 1) return false;
  out.assign(2 * static_cast<size_t>(k), 1);
  uint32_t p = 1;
  for (int j = 0; j < k; ++j) { out[k + j] = p; p = times_x(p, w); }
  return true;
}

int bit_block_ones(uint32_t e, int w) {
  int n = 0;
  for (int x = 0; x < w; ++x) { n += __builtin_popcount(e); e = times_x(e, w); }
  return n;
}

bool cauchy_original(int k, int m, int w, Mat &out) {
  if (k < 1 || m < 1 || (w < 31 && k + m > (1 << w))) return false;
  out.resize(static_cast<size_t>(k) * m);
  for (int i = 0; i < m; ++i)
    for (int j = 0; j < k; ++j) out[static_cast<size_t>(i) * k + j] = inv(static_cast<uint32_t>(i ^ (m + j)), w);
  return true;
}

void cauchy_improve(int k, int m, int w, Mat &a) {
  for (int j = 0; j < k; ++j) {
    if (a[j] == 1) continue;
    const uint32_t s = inv(a[j], w);
    for (int i = 0; i < m; ++i) a[static_cast<size_t>(i) * k + j] = mul(a[static_cast<size_t>(i) * k + j], s, w);
  }
  for (int i = 1; i < m; ++i) {
    uint32_t *row = &a[static_cast<size_t>(i) * k];
    int best = 0, best_col = -1;
    for (int j = 0; j < k; ++j) best += bit_block_ones(row[j], w);
    for (int j = 0; j < k; ++j) {
      if (row[j] == 1) continue;
      const uint32_t s = inv(row[j], w);
      int ones = 0;
      for (int x = 0; x < k; ++x) ones += bit_block_ones(mul(row[x], s, w), w);
      if (ones < best) { best = ones; best_col = j; }
    }
    if (best_col >= 0) {
      const uint32_t s = inv(row[best_col], w);
      for (int j = 0; j < k; ++j) row[j] = mul(row[j], s, w);
    }
  }
}

bool cauchy_good(int k, int m, int w, Mat &out) {
  if (!cauchy_original(k, m, w, out)) return false;
  cauchy_improve(k, m, w, out);
  return true;
}

std::vector<int> to_bitmatrix(int k, int m, int w, const Mat &a) {
  const int cols = k * w;
  std::vector<int> bm(static_cast<size_t>(m) * w * cols, 0);
  for (int i = 0; i < m; ++i)
    for (int j = 0; j < k; ++j) {
      uint32_t e = a[static_cast<size_t>(i) * k + j];
      for (int x = 0; x < w; ++x, e = times_x(e, w))
        for (int l = 0; l < w; ++l) bm[static_cast<size_t>(i * w + l) * cols + j * w + x] = (e >> l) & 1;
    }
  return bm;
}

namespace {
bool invert(int n, int w, Mat a, Mat &out) {
  out.assign(static_cast<size_t>(n) * n, 0);
  for (int i = 0; i < n; ++i) out[static_cast<size_t>(i) * n + i] = 1;
  for (int c = 0; c < n; ++c) {
    int p = c;
    while (p < n && a[static_cast<size_t>(p) * n + c] == 0) ++p;
    if (p == n) return false;
    if (p != c)
      for (int x = 0; x < n; ++x) {
        std::swap(a[static_cast<size_t>(p) * n + x], a[static_cast<size_t>(c) * n + x]);
        std::swap(out[static_cast<size_t>(p) * n + x], out[static_cast<size_t>(c) * n + x]);
      }
    const uint32_t s = inv(a[static_cast<size_t>(c) * n + c], w);
    for (int x = 0; x < n; ++x) {
      a[static_cast<size_t>(c) * n + x] = mul(a[static_cast<size_t>(c) * n + x], s, w);
      out[static_cast<size_t>(c) * n + x] = mul(out[static_cast<size_t>(c) * n + x], s, w);
    }
    for (int r = 0; r < n; ++r) {
      const uint32_t f = a[static_cast<size_t>(r) * n + c];
      if (r == c || f == 0) continue;
      for (int x = 0; x < n; ++x) {
        a[static_cast<size_t>(r) * n + x] ^= mul(f, a[static_cast<size_t>(c) * n + x], w);
        out[static_cast<size_t>(r) * n + x] ^= mul(f, out[static_cast<size_t>(c) * n + x], w);
      }
    }
  }
  return true;
}
}  // namespace

bool make_decode(int k, int m, int w, const Mat &coding, const std::vector<int> &erased_ids, DecodePlan &dp) {
  std::vector<char> lost(k + m, 0);
  for (int e : erased_ids) {
    if (e < 0 || e >= k + m) return false;
    lost[e] = 1;
  }
  dp.erased.clear();
  dp.survivors.clear();
  for (int i = 0; i < k + m; ++i) {
    if (lost[i]) dp.erased.push_back(i);
    else if (static_cast<int>(dp.survivors.size()) < k) dp.survivors.push_back(i);
  }
  if (static_cast<int>(dp.survivors.size()) < k) return false;
  Mat s(static_cast<size_t>(k) * k, 0), sinv;
  for (int j = 0; j < k; ++j) {
    const int id = dp.survivors[j];
    if (id < k) s[static_cast<size_t>(j) * k + id] = 1;
    else std::copy_n(&coding[static_cast<size_t>(id - k) * k], k, &s[static_cast<size_t>(j) * k]);
  }
  if (!invert(k, w, s, sinv)) return false;
  dp.rows.assign(dp.erased.size() * k, 0);
  for (size_t r = 0; r < dp.erased.size(); ++r) {
    const int id = dp.erased[r];
    uint32_t *dst = &dp.rows[r * k];
    if (id < k) {
      std::copy_n(&sinv[static_cast<size_t>(id) * k], k, dst);
    } else {
      const uint32_t *crow = &coding[static_cast<size_t>(id - k) * k];
      for (int j = 0; j < k; ++j) {
        uint32_t acc = 0;
        for (int t = 0; t < k; ++t) acc ^= mul(crow[t], sinv[static_cast<size_t>(t) * k + j], w);
        dst[j] = acc;
      }
    }
  }
  return true;
}

}  // namespace gfw
}  // namespace lsec
