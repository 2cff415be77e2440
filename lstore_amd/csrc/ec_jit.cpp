// ec_jit.cpp -- per-matrix XOR networks for wide GF(2^8) matrix codes, compiled at run time
// with hipRTC for gfx950.
//
// The bytewise kernel (ec_kernels_impl.h) multiplies by a coefficient with three v_perm_b32
// table lookups per 4 bytes, about 5 VALU ops per (output, input) pair and dword.  Wide codes
// are VALU-bound that way: RS(20+6) encode ran at 0.61-0.65 of 8 TB/s, 97 % VALU-busy
// (DESIGN.md §3).  With the matrix known when the kernel is compiled, output r is a fixed
// network evaluated in Horner form over the coefficient bits,
//     out_r = x(...x(x S_r7 + S_r6)...) + S_r0,   S_rt = XOR of the inputs j whose A[r][j] has
//     bit t set,
// on 4 packed bytes per dword: multiplying by x is a shift plus 0x1D times the bit-7 flags (a
// packed 16-bit multiply; 5 VALU ops), the S_rt are 3-input XORs (v_bitop3) -- straight-line
// code, no table lookups, no branches.  For RS(20+6), with the 6-op shift-and-subtract doubling
// (variant bit 1), that is 469 VALU instructions per dword column against 634 for the table
// kernel (SQ_INSTS_VALU per wave 1875 vs 2537, profiles/r02_v14_pmc_valu_rs206.txt); the
// packed multiply takes 7 % more off (offline count, tools/jit_variants.py).  Encode goes from
// 0.67 to 0.73-0.74 of 8 TB/s.
// (A bit-sliced form of the same Horner chains needs 8 x 8 bit transposes, 150 ops per dword,
// and 300 VGPRs; it lost: profiles/r02_kbench_jit_v1.txt.)  Used for R * K >= 96 only: on
// narrower codes the table kernel is already at the memory-bound rate.  The generated kernel
// computes the same GF(2^8) products as the table kernel, bit for bit; it is used once its
// compile has finished (in the background), and the table kernel serves until then.
// LSEC_JIT=0 turns it off.
//
// RS / r6 at w = 16 / 32 (Jerasure's word layout, galois.c:527-604, :730-810) get the same
// treatment in the bit-sliced domain of k_gfw_transposed: each lane transposes W words of an
// input so that word x holds bit x of 32 elements, and output slice b of row r is the XOR of the
// input slices x whose product c_rj * x^x has bit b set -- the 32 x 32 (16 x 16) bitmatrix block
// of the coefficient, known at compile time, so every slice is a straight chain of 3-input XORs
// (about w/4 per output slice per input) instead of the generic kernel's popcount(c) sweeps of
// w XORs plus w-1 doublings.  gfw_source below.
#include <dlfcn.h>
#include <fcntl.h>
#include <hip/hip_runtime.h>
#include <signal.h>
#include <spawn.h>
#include <sys/socket.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "ec_hiperr.h"
#include "ec_host.h"
#include "ec_jit.h"

namespace lsec {
namespace jit {

namespace {

// a balanced left fold of terms with 3-input XORs (ceil((n-1)/2) ops)
std::string xor_chain(std::vector<std::string> t) {
  if (t.empty()) return "0u";
  while (t.size() > 1) {
    std::vector<std::string> n;
    size_t i = 0;
    for (; i + 3 <= t.size(); i += 3) n.push_back("X3(" + t[i] + "," + t[i + 1] + "," + t[i + 2] + ")");
    if (t.size() - i == 2) n.push_back("(" + t[i] + "^" + t[i + 1] + ")");
    else if (t.size() - i == 1) n.push_back(t[i]);
    t.swap(n);
  }
  return t[0];
}

// How a network reads its shard table (struct Args { ...; Ref in[K]; Ref out[R]; }): "a." for the
// kernel argument, or -- from 24 shards -- "ap->", an opaque pointer to the kernarg segment
// re-read in every tile, so that the table's 4 (K + R) SGPRs are not hoisted out of the tile loop
// and spilled to VGPR lanes (RS(24+8): 65 SGPRs spilled, 2661 -> 2339 VALU ops a tile, encode
// 0.65 -> 0.71, 8-loss decode 0.62 -> 0.69; RS(12+8) spills 7 and loses 3 % with it:
// profiles/r04_v18_xornet_reload.txt).  LSEC_JIT_VARIANT bit 28 forces it on, bit 30 off
std::string shard_table(std::ostringstream &s, int K, int R, const char *ind) {
  const int var = jit_variant();
  if (((var >> 30) & 1) || !(((var >> 28) & 1) || K + R >= 24)) return "a.";
  s << ind << "const __attribute__((address_space(4))) Args *ap = (const __attribute__((address_space(4))) Args *)"
            "__builtin_amdgcn_kernarg_segment_ptr();\n"
    << ind << "asm volatile(\"\" : \"+s\"(ap));\n";
  return "ap->";
}

}  // namespace

bool jit_on() {
  static const bool on = [] {
    const char *s = getenv("LSEC_JIT");
    return !s || *s != '0';
  }();
  return on;
}

bool wants_gfw_net(int R, int K, int w) {
  // every non-trivial w = 16 / 32 matrix (XOR-only ones take the plain-XOR path); at w = 32 the
  // R x 32 accumulator slices limit the one-wave form to 4 rows, the wave-pair split (half the
  // slices per wave) to 6 (8 rows spill at 2 waves per SIMD)
  const int max_w32 = gfw_rowsplit(32, 4) ? 6 : 4;
  return jit_on() && (w == 16 || w == 32) && R >= 1 && R <= (w == 32 ? max_w32 : kMaxRows) && K >= 1 && K <= kMaxCols;
}

bool wants_pktnet(int R, int K, int w) {
  // liberation-family bitmatrices (one mask word per bit-row and input) of modest width, two
  // outputs (encodes, double erasures): single-erasure decodes measured 0.72 on a network against
  // 0.76 on k_bitmatrix (profiles/r04_v12_pktnet.txt).  R * w <= 128: the measured shapes (4 rows
  // at w = 32, Cauchy-good(10+4) 0.80, r04_v13_pktnet_cauchy.txt); 8 rows at w = 32 hold 256
  // accumulator dwords per lane, and hipRTC took 320 s over one such network on the build host
  // (6 s at 4 rows), so wider shapes stay on the generic kernels
  return jit_on() && w >= 2 && w <= 32 && R >= 2 && R <= kMaxRows && K >= 1 && K <= kMaxCols && R * w <= 128;
}

bool wants_xornet(int R, int K) {
  const bool on = jit_on();
  // R * K >= 96 only: narrower codes are memory-bound on the table kernel already (RS(16+4) /
  // RS(12+4) level within noise on a network, profiles/r02_v15_jit_ab.txt)
  return on && R >= 2 && R <= kMaxRows && K >= 2 && K <= kMaxCols && R * K >= 96;
}

// Code shape knobs (LSEC_JIT_VARIANT, read once; A/B runs): bit 0 = uncapped common-pair
// elimination, bit 3 = none (the default caps it by registers, xornet_source), bit 1 = doubling by
// shift-and-subtract instead of a packed 16-bit multiply, bits 4-7 = dwords per lane (1, 2, 4;
// 0 = xornet_dwords).  Round 2 measured the shapes on RS(20+6) encode within 70.6-74.3 % of 8 TB/s
// (profiles/r02_v15_jit_ab.txt); round 4 capped pairs (r04_v15_xornet_ab.txt).  w = 16 / 32 networks: bits
// 8-15 shared-pair cap, 16 unfenced loads, 17-18 inputs ahead, 21 serial XOR folds (gfw_source);
// 19 turns the wave-pair split of 4-row w = 32 networks off, 20-23 shape it
// (gfw_rowsplit_source; profiles/r04_v7_gfw_w32_ab.md, r04_v9_gfw_w32_split.txt).
// The first tile of a block (one tile per block, XCD x taking a contiguous eighth of the tiles in
// dispatch order), as the generated kernels compute it.  Args::phase > 0 (the XCD tile phase,
// lsec::tile_phase_net_on, ec_kernels.h; off by default for the networks): XCD x starts its eighth
// x * phase tiles further on and wraps around inside it.
std::string tile_start() {
  return "  const unsigned sz_ = per + (xcd < rem ? 1u : 0u);\n"
         "  const unsigned ph_ = (nb == nt && sz_) ? (xcd * a.phase) % sz_ : 0u;\n"
         "  const unsigned t0 = xcd * per + (xcd < rem ? xcd : rem) + (ph_ ? ((blockIdx.x >> 3) + ph_) % sz_ : (blockIdx.x >> 3));\n";
}

int jit_variant() {
  static const int v = [] {
    const char *s = getenv("LSEC_JIT_VARIANT");
    return s ? atoi(s) : 0;
  }();
  return v;
}

namespace {

// One Horner step's XOR set: the inputs (or shared pairs) whose coefficient has bit t set.
struct Step {
  bool doubled;            // h = x * h first (every step after the top one)
  std::vector<int> terms;  // symbol ids: 0..K-1 inputs, K.. shared pairs
};

// Greedy common-pair elimination over all steps of all rows (Paar's heuristic): the pair of
// symbols that occurs together in the most XOR sets becomes a new symbol while it occurs in at
// least 3 (one 2-input XOR then saves a term in each of them).
void share_pairs(std::vector<std::vector<Step>> &rows, int K, std::vector<std::pair<int, int>> &pairs,
                 int max_pairs = 1 << 30) {
  while (static_cast<int>(pairs.size()) < max_pairs) {
    std::map<std::pair<int, int>, int> count;
    for (auto &row : rows)
      for (auto &st : row) {
        std::vector<int> t = st.terms;
        std::sort(t.begin(), t.end());
        for (size_t i = 0; i < t.size(); ++i)
          for (size_t j = i + 1; j < t.size(); ++j) ++count[{t[i], t[j]}];
      }
    std::pair<int, int> best{-1, -1};
    int n = 0;
    for (auto &kv : count)
      if (kv.second > n) {
        n = kv.second;
        best = kv.first;
      }
    if (n < 3) return;
    const int sym = K + static_cast<int>(pairs.size());
    pairs.push_back(best);
    for (auto &row : rows)
      for (auto &st : row) {
        auto a = std::find(st.terms.begin(), st.terms.end(), best.first);
        auto b = std::find(st.terms.begin(), st.terms.end(), best.second);
        if (a == st.terms.end() || b == st.terms.end()) continue;
        st.terms.erase(std::remove_if(st.terms.begin(), st.terms.end(),
                                      [&](int x) { return x == best.first || x == best.second; }),
                       st.terms.end());
        st.terms.push_back(sym);
      }
  }
}

}  // namespace

// dwords per lane: 16 B loads by default, 8 B for many-row networks over few inputs (R >= 8,
// K <= 13, where 16 B would be two pieces per lane: RS(12+8) encode 0.67 -> 0.70,
// profiles/r04_v15_xornet_ab.txt); LSEC_JIT_VARIANT bits 4-7 force 1 / 2 / 4
int xornet_dwords(int R, int K) {
  const int v = (jit_variant() >> 4) & 15;
  if (v == 1 || v == 2 || v == 4) return v;
  return R >= 8 && K * 8 <= 104 ? 2 : 4;
}

std::string xornet_source(const uint8_t *mat, int R, int K) {
  const int var = jit_variant();
  const int D = xornet_dwords(R, K);
  const int IT = D == 4 && K * 8 <= 104 ? 2 : 1;  // 16 B pieces per lane per shard (D = 4)
  const int lane_bytes = 4 * D * IT;
  const int tile = 256 * lane_bytes;
  // the Horner steps of every row, then the shared pairs
  std::vector<std::vector<Step>> rows(R);
  for (int r = 0; r < R; ++r) {
    int top = -1;
    for (int t = 7; t >= 0 && top < 0; --t)
      for (int j = 0; j < K; ++j)
        if ((mat[r * K + j] >> t) & 1) top = t;
    for (int t = top; t >= 0; --t) {
      Step st;
      st.doubled = t != top;
      for (int j = 0; j < K; ++j)
        if ((mat[r * K + j] >> t) & 1) st.terms.push_back(j);
      rows[r].push_back(st);
    }
  }
  std::vector<std::pair<int, int>> pairs;
  // common-pair elimination, capped so that the inputs and the pairs (D*IT registers each) stay
  // within about 128 registers: RS(20+6) encode 0.70 -> 0.74 and its 6-loss decode 0.65 -> 0.73,
  // RS(24+8) encode 0.60 -> 0.66, RS(12+8) 0.68 -> 0.72 (profiles/r04_v15_xornet_ab.txt; uncapped,
  // the pairs cost occupancy).  LSEC_JIT_VARIANT bit 0: no cap; bit 3: no pairs (the round-3 form)
  if (var & 1) share_pairs(rows, K, pairs);
  else if (!(var & 8)) share_pairs(rows, K, pairs, std::max(0, (128 - K * D * IT) / (D * IT)));
  auto sym = [&](int x) { return (x < K ? "e" : "p") + std::to_string(x < K ? x : x - K) + "[d]"; };

  std::ostringstream s;
  s << "typedef unsigned int u32;\n"
       "typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));\n"
       "typedef u32 u32x4 __attribute__((ext_vector_type(4)));\n"
       "typedef u32 u32x2 __attribute__((ext_vector_type(2)));\n"
       "struct Ref { unsigned long long base; long long stride; };\n"
    << "struct Args { long long size; int nstripes; int pad; Ref in[" << K << "]; Ref out[" << R << "]; unsigned phase; };\n"
    << "#define X3(a,b,c) __builtin_amdgcn_bitop3_b32((a),(b),(c),0x96)\n";
  if (!(var & 2)) {
    // x * (4 packed GF(2^8) elements), polynomial 0x11D: shift, and 0x1D times the bit-7 flags
    // by a packed 16-bit multiply (each 16-bit half holds two flags, 0x1D1D at most)
    s << "__device__ static inline u32 XT(u32 a) {\n"
         "  const u16x2 f = __builtin_bit_cast(u16x2, (a >> 7) & 0x01010101u) * (u16x2){0x1D, 0x1D};\n"
         "  return ((a << 1) & 0xFEFEFEFEu) ^ __builtin_bit_cast(u32, f);\n"
         "}\n";
  } else {
    // x * (4 packed GF(2^8) elements), polynomial 0x11D: shift the low 7 bits of every byte,
    // and XOR the taps 0x1D into the bytes whose bit 7 was set (t - (t >> 7) is 0x7F in exactly
    // those bytes, borrow-free).  A 24-bit multiply of the bit-7 flags by 0x1D would drop byte 3.
    s << "__device__ static inline u32 XT(u32 a) {\n"
         "  const u32 t = a & 0x80808080u;\n"
         "  return ((a ^ t) << 1) ^ ((t - (t >> 7)) & 0x1D1D1D1Du);\n"
         "}\n";
  }
  s << "#define G(a) ((const __attribute__((address_space(1))) u32x4 *)(a))\n"
       "#define GW(a) ((__attribute__((address_space(1))) u32x4 *)(a))\n"
       "#define G2(a) ((const __attribute__((address_space(1))) u32x2 *)(a))\n"
       "#define GW2(a) ((__attribute__((address_space(1))) u32x2 *)(a))\n"
       "#define G1(a) ((const __attribute__((address_space(1))) u32 *)(a))\n"
       "#define GW1(a) ((__attribute__((address_space(1))) u32 *)(a))\n"
       // a lane's D dwords at byte o of a shard of C bytes (C % 8 == 0: tails are whole 8 B)
       "__device__ static inline void ld4(u32 *e, unsigned long long p, long long o, long long C) {\n"
       "  if (o + 16 <= C) { const u32x4 v = __builtin_nontemporal_load(G(p + o)); e[0] = v.x; e[1] = v.y; e[2] = v.z; e[3] = v.w; return; }\n"
       "  e[0] = e[1] = e[2] = e[3] = 0u;\n"
       "  if (o + 8 <= C) { const u32x2 h = *G2(p + o); e[0] = h.x; e[1] = h.y; }\n"
       "}\n"
       "__device__ static inline void st4(const u32 *h, unsigned long long p, long long o, long long C) {\n"
       "  if (o + 16 <= C) __builtin_nontemporal_store((u32x4){h[0], h[1], h[2], h[3]}, GW(p + o));\n"
       "  else if (o + 8 <= C) *GW2(p + o) = (u32x2){h[0], h[1]};\n"
       "}\n"
       "__device__ static inline void ld2(u32 *e, unsigned long long p, long long o, long long C) {\n"
       "  if (o + 8 <= C) { const u32x2 v = __builtin_nontemporal_load(G2(p + o)); e[0] = v.x; e[1] = v.y; return; }\n"
       "  e[0] = e[1] = 0u;\n"
       "}\n"
       "__device__ static inline void st2(const u32 *h, unsigned long long p, long long o, long long C) {\n"
       "  if (o + 8 <= C) __builtin_nontemporal_store((u32x2){h[0], h[1]}, GW2(p + o));\n"
       "}\n"
       // D = 1: a lane owns 4 B; a chunk ends on 8 B, so its last 4 B are in range too
       "__device__ static inline void ld1(u32 *e, unsigned long long p, long long o, long long C) {\n"
       "  e[0] = o + 4 <= C ? __builtin_nontemporal_load(G1(p + o)) : 0u;\n"
       "}\n"
       "__device__ static inline void st1(const u32 *h, unsigned long long p, long long o, long long C) {\n"
       "  if (o + 4 <= C) __builtin_nontemporal_store(h[0], GW1(p + o));\n"
       "}\n"
       "extern \"C\" __global__ __launch_bounds__(256) void lsec_xornet(Args a) {\n"
       "  const long long C = a.size;\n"
    << "  const unsigned tps = (unsigned)((C + " << tile - 1 << ") / " << tile << ");\n"
    << "  const unsigned nt = tps * (unsigned)a.nstripes;\n"
       "  const unsigned nb = gridDim.x, per = nb >> 3, rem = nb & 7, xcd = blockIdx.x & 7;\n"
    << tile_start() <<
       "  for (unsigned t = t0; t < nt; t += nb) {\n"
       "    const unsigned s = t / tps;\n"
    << "    const long long o0 = (long long)(t - s * tps) * " << tile << " + threadIdx.x * " << 4 * D << ";\n";
  const std::string A = shard_table(s, K, R, "    ");
  const int DL = D * IT;  // dwords per lane per shard
  for (int j = 0; j < K; ++j) {
    s << "    u32 e" << j << "[" << DL << "];\n    { const unsigned long long p = " << A << "in[" << j
      << "].base + (unsigned long long)s * " << A << "in[" << j << "].stride;\n";
    for (int it = 0; it < IT; ++it)
      s << "      ld" << D << "(e" << j << " + " << D * it << ", p, o0 + " << 256 * 4 * D * it << ", C);\n";
    s << "    }\n";
  }
  for (size_t i = 0; i < pairs.size(); ++i)
    s << "    u32 p" << i << "[" << DL << "];\n    for (int d = 0; d < " << DL << "; ++d) p" << i << "[d] = " << sym(pairs[i].first)
      << " ^ " << sym(pairs[i].second) << ";\n";
  for (int r = 0; r < R; ++r) {
    s << "    { u32 h[" << DL << "];\n";
    if (rows[r].empty()) s << "      for (int d = 0; d < " << DL << "; ++d) h[d] = 0u;\n";
    // Horner over the coefficient bits: h = x(...x(S_top) + ...) + S_0
    for (const Step &st : rows[r]) {
      s << "      for (int d = 0; d < " << DL << "; ++d) {\n";
      std::vector<std::string> terms;
      if (st.doubled) {
        s << "        const u32 x = XT(h[d]);\n";
        terms.push_back("x");
      }
      for (int x : st.terms) terms.push_back(sym(x));
      s << "        h[d] = " << xor_chain(terms) << ";\n      }\n";
    }
    s << "      const unsigned long long q = " << A << "out[" << r << "].base + (unsigned long long)s * " << A << "out[" << r
      << "].stride;\n";
    for (int it = 0; it < IT; ++it) s << "      st" << D << "(h + " << D * it << ", q, o0 + " << 256 * 4 * D * it << ", C);\n";
    s << "    }\n";
  }
  s << "  }\n}\n";
  return s.str();
}

// ---- GF(2^16) / GF(2^32): bit-sliced networks over Jerasure's word layout
namespace {

// c * x in GF(2^w), Jerasure's polynomials (galois.c:65-98: 0210013, 020000007)
uint32_t gfw_times_x(uint32_t c, int w) {
  if (w == 8) {  // Jerasure's GF(2^8), x^8 = x^4+x^3+x^2+1 (0x11D)
    c <<= 1;
    return (c & 0x100u) ? (c ^ 0x11Du) & 0xFFu : c;
  }
  if (w == 16) {
    c <<= 1;
    return (c & 0x10000u) ? (c ^ 0x1100Bu) & 0xFFFFu : c;
  }
  const bool top = c >> 31;
  return (c << 1) ^ (top ? 0x400007u : 0u);
}

// Greedy common-pair elimination (Paar) over one input's rows (sets of slice ids 0..W-1):
// at most `cap` shared pairs, each used by at least 3 rows.  New symbols are W, W+1, ...
void share_slice_pairs(std::vector<std::vector<int>> &rows, int W, int cap, std::vector<std::pair<int, int>> &pairs) {
  while (static_cast<int>(pairs.size()) < cap) {
    const int nsym = W + static_cast<int>(pairs.size());
    std::vector<int> count(static_cast<size_t>(nsym) * nsym, 0);
    for (auto &row : rows)
      for (size_t i = 0; i < row.size(); ++i)
        for (size_t j = i + 1; j < row.size(); ++j) {
          const int a = std::min(row[i], row[j]), b = std::max(row[i], row[j]);
          ++count[static_cast<size_t>(a) * nsym + b];
        }
    int best = -1, n = 0;
    for (size_t i = 0; i < count.size(); ++i)
      if (count[i] > n) {
        n = count[i];
        best = static_cast<int>(i);
      }
    if (n < 3) return;
    const int a = best / nsym, b = best % nsym;
    pairs.push_back({a, b});
    for (auto &row : rows) {
      auto ia = std::find(row.begin(), row.end(), a), ib = std::find(row.begin(), row.end(), b);
      if (ia == row.end() || ib == row.end()) continue;
      row.erase(std::remove_if(row.begin(), row.end(), [&](int x) { return x == a || x == b; }), row.end());
      row.push_back(nsym);
    }
  }
}

}  // namespace

bool gfw_rowsplit(int w, int R) {
  // the wave-pair split below for networks of 4+ rows at w = 32, where the one-wave form holds one
  // wave per SIMD (RS(10+4) encode 0.66 -> 0.76; at 3 rows the one-wave form holds two and the
  // split gains nothing: profiles/r04_v9_gfw_w32_split.txt).  LSEC_JIT_VARIANT bit 19 turns it off
  // and from 5 rows at w = 16 (RS(20+6) 0.68 -> 0.72; bit 24 turns that off)
  if ((jit_variant() >> 19) & 1) return false;
  return (w == 32 && R >= 4) || (w == 16 && R >= 5 && !((jit_variant() >> 24) & 1));
}

int gfw_tile(int w, int R) { return gfw_rowsplit(w, R) ? 128 * 4 * w : 256 * 4 * w; }

namespace {

// Types, the bit transpose and the whole-tile loads / stores shared by both network shapes: a
// lane's W dwords of a shard are W/4 pieces of 16 B, `stride` bytes apart
void gfw_prelude(std::ostringstream &s, int R, int K, int W, int stride) {
  s << "typedef unsigned int u32;\n"
       "typedef u32 u32x4 __attribute__((ext_vector_type(4)));\n"
       "typedef u32 u32x2 __attribute__((ext_vector_type(2)));\n"
       "struct Ref { unsigned long long base; long long stride; };\n"
    << "struct Args { long long size; int nstripes; int pad; Ref in[" << K << "]; Ref out[" << R << "]; unsigned phase; };\n"
    << "#define W " << W << "\n"
    << "#define PIECE " << stride << "\n"
       "#define X3(a,b,c) __builtin_amdgcn_bitop3_b32((a),(b),(c),0x96)\n"
       "#define G(a) ((const __attribute__((address_space(1))) u32x4 *)(a))\n"
       "#define GW(a) ((__attribute__((address_space(1))) u32x4 *)(a))\n"
       // the W x W bit transpose of k_gfw_transposed (ec_kernels_impl.h, transpose_units)
       "template <int d> __device__ static inline void tb(u32 (&D)[W], u32 m) {\n"
       "#pragma unroll\n"
       "  for (int r = 0; r < W; ++r) { if (r & d) continue; const u32 x = D[r], y = D[r + d];\n"
       "    D[r] = (x & m) | ((y << d) & ~m); D[r + d] = ((x >> d) & m) | (y & ~m); }\n"
       "}\n"
       "__device__ static inline void tr(u32 (&D)[W]) {\n"
       "#if W == 32\n"
       "#pragma unroll\n"
       "  for (int r = 0; r < 16; ++r) { const u32 x = D[r], y = D[r + 16];\n"
       "    D[r] = __builtin_amdgcn_perm(y, x, 0x05040100u); D[r + 16] = __builtin_amdgcn_perm(y, x, 0x07060302u); }\n"
       "#endif\n"
       "#pragma unroll\n"
       "  for (int r = 0; r < W; ++r) { if (r & 8) continue; const u32 x = D[r], y = D[r + 8];\n"
       "    D[r] = __builtin_amdgcn_perm(y, x, 0x06020400u); D[r + 8] = __builtin_amdgcn_perm(y, x, 0x07030501u); }\n"
       "  tb<4>(D, 0x0F0F0F0Fu); tb<2>(D, 0x33333333u); tb<1>(D, 0x55555555u);\n"
       "}\n"
       // whole tiles only: the launcher hands a ragged tail to the generic kernel, so loads are
       // unconditional and each tile is one basic block for the scheduler
       "__device__ static inline void ld(u32 (&e)[W], unsigned long long p) {\n"
       "#pragma unroll\n"
       "  for (int q = 0; q < W / 4; ++q) { const u32x4 v = __builtin_nontemporal_load(G(p + q * PIECE));\n"
       "    e[4 * q] = v.x; e[4 * q + 1] = v.y; e[4 * q + 2] = v.z; e[4 * q + 3] = v.w; }\n"
       "}\n"
       "__device__ static inline void st(const u32 (&h)[W], unsigned long long p) {\n"
       "#pragma unroll\n"
       "  for (int q = 0; q < W / 4; ++q)\n"
       "    __builtin_nontemporal_store((u32x4){h[4 * q], h[4 * q + 1], h[4 * q + 2], h[4 * q + 3]}, GW(p + q * PIECE));\n"
       "}\n";
}

// Input j's contribution to output rows `rows` (accumulators acc[i] of row rows[i]): slice b of
// row r takes the input slices x (in array `e`, transposed) with bit b of c_rj * x^x set -- the
// bitmatrix block of the coefficient -- after common-pair elimination over those rows
void gfw_net(std::ostringstream &s, const uint32_t *mat, int K, int W, int j, const std::vector<int> &rows,
             const std::vector<std::string> &acc, std::vector<std::vector<bool>> &live, int cap, const std::string &e,
             const char *ind, bool linear, int b0 = 0, int b1 = -1) {
  // output slices b0 .. b1-1 only (accumulator element b - b0); linear: serial folds into the
  // accumulator instead of balanced 3-input XOR trees
  if (b1 < 0) b1 = W;
  std::vector<std::vector<int>> sl(rows.size() * W);
  bool any = false;
  for (size_t i = 0; i < rows.size(); ++i) {
    uint32_t cx = mat[rows[i] * K + j];
    any |= cx != 0;
    for (int x = 0; x < W && cx; ++x) {
      for (int b = b0; b < b1; ++b)
        if ((cx >> b) & 1u) sl[i * W + b].push_back(x);
      cx = gfw_times_x(cx, W);
    }
  }
  if (!any) return;
  std::vector<std::pair<int, int>> pairs;
  if (cap > 0) share_slice_pairs(sl, W, cap, pairs);
  auto nm = [&](int x) { return x < W ? e + "[" + std::to_string(x) + "]" : "p" + std::to_string(x - W); };
  s << ind << "{\n";
  for (size_t i = 0; i < pairs.size(); ++i)
    s << ind << "  const u32 p" << i << " = " << nm(pairs[i].first) << " ^ " << nm(pairs[i].second) << ";\n";
  for (size_t i = 0; i < rows.size(); ++i)
    for (int b = b0; b < b1; ++b) {
      const auto &row = sl[i * W + b];
      if (row.empty()) continue;
      std::vector<std::string> t;
      const std::string a = acc[i] + "[" + std::to_string(b - b0) + "]";
      if (live[i][b - b0]) t.push_back(a);
      for (int x : row) t.push_back(nm(x));
      if (linear) {
        // a serial fold into the accumulator: no partial sums of the inputs alone for the
        // scheduler to hoist (each is a VGPR live until its fold)
        std::string v = t[0];
        size_t k = 1;
        for (; k + 2 <= t.size(); k += 2) {
          s << ind << "  " << a << " = X3(" << v << ", " << t[k] << ", " << t[k + 1] << ");\n";
          v = a;
        }
        if (k < t.size()) s << ind << "  " << a << " = " << v << " ^ " << t[k] << ";\n";
        else if (v != a) s << ind << "  " << a << " = " << v << ";\n";
      } else {
        s << ind << "  " << a << " = " << xor_chain(t) << ";\n";
      }
      live[i][b - b0] = true;
    }
  s << ind << "}\n";
}

// the inputs with a non-zero coefficient in some row
std::vector<int> gfw_used(const uint32_t *mat, int R, int K) {
  std::vector<int> used;
  for (int j = 0; j < K; ++j)
    for (int r = 0; r < R; ++r)
      if (mat[r * K + j]) {
        used.push_back(j);
        break;
      }
  return used;
}

// Wave-pair split of the w = 32 (4-6 rows) and w = 16 (5-8 rows) networks.  The one-wave form keeps R x 32
// accumulator slices per lane (128 VGPRs at 4 rows) plus two inputs' 32 slices: at 4 rows its code
// object takes 273 registers, one wave per SIMD.  Here the 4 waves of a block form 2 pairs; the two waves of a pair cover the same 64 lane
// columns and each computes half of every output row's bit slices (role 0 slices 0-15, role 1
// 16-31; balanced for any R).  Per step each wave loads and transposes one input (role 0 the even
// used inputs, role 1 the odd), writes its 32 slices to LDS, XORs them into its half slices, and
// after a barrier reads its partner's input slices from LDS into the same registers and XORs
// those in: every input is still loaded and transposed once and the accumulators halve (64 VGPRs
// at 4 rows).  At the end the halves meet through LDS: role 0 transposes and stores rows
// 0 .. ceil(R/2)-1, role 1 the rest.  Tile: 128 lane columns x 16 B x 8 pieces, 2 KiB apart
// (16 KiB per shard); LDS 2 pairs x 2 roles x 8 KiB (12 KiB at 5-6 rows).  The roles' code sits
// in two consecutive `if (role == r)` blocks, never in if / else: at an if / else join the
// compiler kept both branches' accumulators apart (294 registers at RS(10+4) even with identical
// branches; 139 as consecutive ifs, profiles/r04_v9_gfw_w32_split.txt).
std::string gfw_rowsplit_source(const uint32_t *mat, int R, int K, int W) {
  const int capv = (jit_variant() >> 8) & 255;
  const int cap = capv == 0 ? 32 : capv == 255 ? 0 : capv;
  const int tile = gfw_tile(W, R), HW = W / 2;
  const int n0 = (R + 1) / 2;  // output rows of role 0: 0 .. n0-1; role 1: n0 .. R-1
  // quads (64 lanes x 16 B) of a wave's LDS slot: one transposed input (W / 4), or the half
  // slices of the rows it hands its partner at the end (at most n0 rows of HW / 4)
  const int lq = std::max(W / 4, n0 * (HW / 4));
  std::vector<int> rows;
  std::vector<std::string> acc;
  for (int r = 0; r < R; ++r) {
    rows.push_back(r);
    acc.push_back("h" + std::to_string(r));
  }
  std::vector<std::vector<bool>> live0(R, std::vector<bool>(HW, false)), live1(R, std::vector<bool>(HW, false));
  const std::vector<int> used = gfw_used(mat, R, K);
  const int n = static_cast<int>(used.size()), steps = (n + 1) / 2;
  std::ostringstream s;
  // defaults measured best (profiles/r04_v9_gfw_w32_split.txt): serial folds (LSEC_JIT_VARIANT
  // bit 21: trees instead), one input prefetched (bit 20: none), and an occupancy target of 3
  // waves per SIMD for the register allocator (bits 22-23: 1 none, 2 four, 3 two), which RS(10+4)
  // meets at 167 registers without spills
  const bool linear = !((jit_variant() >> 21) & 1);
  const int wv_opt = (jit_variant() >> 22) & 3, wpe = wv_opt == 0 ? (R <= 4 ? 3 : 2) : wv_opt == 1 ? 0 : wv_opt == 2 ? 4 : 2;
  gfw_prelude(s, R, K, W, 128 * 16);
  s << "extern \"C\" __global__ __launch_bounds__(256) ";
  if (wpe) s << "__attribute__((amdgpu_waves_per_eu(" << wpe << "))) ";
  s << "void lsec_xornet(Args a) {\n"
    << "  __shared__ u32x4 L[2][2][" << lq << "][64];\n"
       "  const unsigned wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;\n"
       "  const unsigned pair = wv >> 1, role = wv & 1;\n"
       "  u32x4 (*const mine)[64] = L[pair][role];\n"
       "  u32x4 (*const theirs)[64] = L[pair][role ^ 1];\n"
       "  const long long C = a.size;\n"
    << "  const unsigned tps = (unsigned)(C / " << tile << ");\n"
    << "  const unsigned nt = tps * (unsigned)a.nstripes;\n"
       "  const unsigned nb = gridDim.x, per = nb >> 3, rem = nb & 7, xcd = blockIdx.x & 7;\n"
    << tile_start() <<
       "  for (unsigned t = t0; t < nt; t += nb) {\n"
       "    const unsigned s = t / tps;\n"
    << "    const long long base = (long long)(t - s * tps) * " << tile << " + (pair * 64 + lane) * 16;\n";
  const std::string A = shard_table(s, K, R, "    ");
  for (int r = 0; r < R; ++r) s << "    u32 h" << r << "[" << HW << "];\n";
  s << "    u32 e0[W], e1[W];\n";
  auto ptr = [&](int j) {
    return A + "in[" + std::to_string(j) + "].base + (unsigned long long)s * " + A + "in[" + std::to_string(j) + "].stride + base";
  };
  // step u's own inputs into buffer b: used[2u] (role 0) and used[2u+1] (role 1)
  auto load = [&](int u, int b) {
    if (2 * u >= n) return;
    if (2 * u + 1 < n)
      s << "    ld(e" << b << ", role ? " << ptr(used[2 * u + 1]) << " : " << ptr(used[2 * u]) << ");\n";
    else
      s << "    if (role == 0) ld(e" << b << ", " << ptr(used[2 * u]) << ");\n";
  };
  // bit 20: no prefetch -- each step loads its own input at its top (32 fewer VGPRs live; the
  // other waves of the SIMD hide the latency)
  const bool ahead = !((jit_variant() >> 20) & 1);
  if (ahead) load(0, 0);
  for (int u = 0; u < steps; ++u) {
    const int b = ahead ? u & 1 : 0;
    const std::string e = "e" + std::to_string(b);
    const bool pairB = 2 * u + 1 < n;
    load(ahead ? u + 1 : u, ahead ? b ^ 1 : 0);
    // own input: transpose, publish, accumulate.  A lone last input (odd count) is role 0's:
    // role 1 then only reads it
    if (pairB) {
      s << "    tr(" << e << ");\n";
    } else {
      s << "    if (role == 0) tr(" << e << ");\n";
    }
    s << "    " << (pairB ? "" : "if (role == 0) ") << "{\n"
      << "#pragma unroll\n      for (int q = 0; q < W / 4; ++q) mine[q][lane] = (u32x4){" << e << "[4 * q], " << e
      << "[4 * q + 1], " << e << "[4 * q + 2], " << e << "[4 * q + 3]};\n    }\n";
    if (pairB) {
      s << "    if (role == 0) {\n";
      gfw_net(s, mat, K, W, used[2 * u], rows, acc, live0, cap, e, "      ", linear, 0, HW);
      s << "    }\n    if (role == 1) {\n";
      gfw_net(s, mat, K, W, used[2 * u + 1], rows, acc, live1, cap, e, "      ", linear, HW, W);
      s << "    }\n";
    } else {
      s << "    if (role == 0) {\n";
      gfw_net(s, mat, K, W, used[2 * u], rows, acc, live0, cap, e, "      ", linear, 0, HW);
      s << "    }\n";
    }
    s << "    __builtin_amdgcn_sched_barrier(0);\n    __syncthreads();\n";
    // the partner's input from LDS, into the same registers
    const std::string rd = "#pragma unroll\n      for (int q = 0; q < W / 4; ++q) { const u32x4 v = theirs[q][lane]; " + e + "[4 * q] = v.x; " + e +
                           "[4 * q + 1] = v.y; " + e + "[4 * q + 2] = v.z; " + e + "[4 * q + 3] = v.w; }\n";
    if (pairB) {
      s << "    {\n" << rd << "    }\n    if (role == 0) {\n";
      gfw_net(s, mat, K, W, used[2 * u + 1], rows, acc, live0, cap, e, "      ", linear, 0, HW);
      s << "    }\n    if (role == 1) {\n";
      gfw_net(s, mat, K, W, used[2 * u], rows, acc, live1, cap, e, "      ", linear, HW, W);
      s << "    }\n";
    } else {
      s << "    if (role == 1) {\n" << rd;
      gfw_net(s, mat, K, W, used[2 * u], rows, acc, live1, cap, e, "      ", linear, HW, W);
      s << "    }\n";
    }
    s << "    __builtin_amdgcn_sched_barrier(0);\n    __syncthreads();\n";
  }
  // the halves meet: each role publishes its slices of the rows the other stores (slot k = the
  // k-th of those rows, 4 quads each), then completes its own rows from the partner's slots
  auto zero = [&](const std::vector<std::vector<bool>> &live) {
    for (int r = 0; r < R; ++r)
      for (int b = 0; b < HW; ++b)
        if (!live[r][b]) s << "      h" << r << "[" << b << "] = 0u;\n";
  };
  auto publish = [&](int lo, int hi) {
    for (int r = lo; r < hi; ++r)
      for (int q = 0; q < HW / 4; ++q)
        s << "      mine[" << (r - lo) * (HW / 4) + q << "][lane] = (u32x4){h" << r << "[" << 4 * q << "], h" << r << "["
          << 4 * q + 1 << "], h" << r << "[" << 4 * q + 2 << "], h" << r << "[" << 4 * q + 3 << "]};\n";
  };
  auto complete = [&](int lo, int hi, bool low_half_mine) {
    for (int r = lo; r < hi; ++r) {
      s << "      { u32 f[W];\n";
      for (int q = 0; q < HW / 4; ++q) {
        const int mo = low_half_mine ? 4 * q : HW + 4 * q, po = low_half_mine ? HW + 4 * q : 4 * q;
        s << "        { const u32x4 v = theirs[" << (r - lo) * (HW / 4) + q << "][lane]; f[" << po << "] = v.x; f[" << po + 1
          << "] = v.y; f[" << po + 2 << "] = v.z; f[" << po + 3 << "] = v.w; }\n";
        for (int d = 0; d < 4; ++d) s << "        f[" << mo + d << "] = h" << r << "[" << 4 * q + d << "];\n";
      }
      s << "        tr(f);\n        st(f, " << A << "out[" << r << "].base + (unsigned long long)s * " << A << "out[" << r
        << "].stride + base);\n      }\n";
    }
  };
  s << "    if (role == 0) {\n";
  zero(live0);
  publish(n0, R);
  s << "    }\n    if (role == 1) {\n";
  zero(live1);
  publish(0, n0);
  s << "    }\n    __syncthreads();\n    if (role == 0) {\n";
  complete(0, n0, true);
  s << "    }\n    if (role == 1) {\n";
  complete(n0, R, false);
  s << "    }\n    __syncthreads();\n  }\n}\n";
  return s.str();
}

}  // namespace

// Packet networks for bitmatrix codes (liberation / blaum_roth / liber8tion; jerasure_bitmatrix_dotprod,
// jerasure.c:317-362) and for Cauchy codes at w = 16 / 32 (the bitmatrix of each GF(2^w)
// coefficient): a super-packet is w packets of P bytes per shard; packet l of output r is the XOR
// of the input packets (j, x) whose bit B[r*w+l][j*w+x] is set.  With the bitmatrix known when the
// kernel is compiled every output packet is a straight XOR chain (shared pairs per input, as
// gfw_net), where k_bitmatrix tests R*w*w mask bits per input under uniform branches and moves 4 B
// per lane, and k_gfw_bitsliced XORs w slices per set coefficient bit.  A lane owns D dwords (16 B
// at P % 16 == 0) of one packet column; it loads the packets of that column each input needs (one
// input ahead, fenced) and stores its output packets.  With S > 1 groups (an A/B knob; slower)
// the output packets (r, l) are split by l into S groups, tile t computing group t % S of column
// tile t / S: the groups of one column run side by side on one XCD and re-read the inputs from its
// L2.  Lanes past the last column redo the last column: no divergent branch.
// masks[((r*w + l)*K + j)] bit x = B[r*w+l][j*w+x] (w <= 32).
std::string pktnet_source(const uint32_t *masks, int R, int K, int W, int D, int S) {
  const int capv = (jit_variant() >> 8) & 255;
  const int cap = capv == 0 ? 32 : capv == 255 ? 0 : capv;
  const int tile = 256 * 4 * D;
  const char *vt = D == 4 ? "u32x4" : D == 2 ? "u32x2" : "u32";
  std::ostringstream s;
  s << "typedef unsigned int u32;\n"
       "typedef u32 u32x4 __attribute__((ext_vector_type(4)));\n"
       "typedef u32 u32x2 __attribute__((ext_vector_type(2)));\n"
       "struct Ref { unsigned long long base; long long stride; };\n"
    << "struct Args { long long size; int nstripes; int packet; Ref in[" << K << "]; Ref out[" << R << "]; unsigned phase; };\n"
    << "typedef " << vt << " V;\n"
       "#define X3(a,b,c) __builtin_amdgcn_bitop3_b32((a),(b),(c),0x96)\n"
       "#define G(a) ((const __attribute__((address_space(1))) V *)(a))\n"
       "#define GW(a) ((__attribute__((address_space(1))) V *)(a))\n"
    << "#define D " << D << "\n"
       "__device__ static inline void ld(u32 (&e)[D], unsigned long long p) {\n"
       "  const V v = __builtin_nontemporal_load(G(p));\n"
    << (D == 1 ? "  e[0] = v;\n" : D == 2 ? "  e[0] = v.x; e[1] = v.y;\n" : "  e[0] = v.x; e[1] = v.y; e[2] = v.z; e[3] = v.w;\n")
    << "}\n"
       "__device__ static inline void st(const u32 (&h)[D], unsigned long long p) {\n"
    << (D == 1 ? "  __builtin_nontemporal_store(h[0], GW(p));\n"
               : D == 2 ? "  __builtin_nontemporal_store((u32x2){h[0], h[1]}, GW(p));\n"
                        : "  __builtin_nontemporal_store((u32x4){h[0], h[1], h[2], h[3]}, GW(p));\n")
    << "}\n"
       "extern \"C\" __global__ __launch_bounds__(256) void lsec_xornet(Args a) {\n"
       "  const unsigned P = (unsigned)a.packet;\n"
    << "  const unsigned cols = (unsigned)(a.size / " << W << ");\n"
    << "  const unsigned tps = (cols + " << tile - 1 << ") / " << tile << ";\n"
    << "  const unsigned nt = tps * (unsigned)a.nstripes * " << S << "u;\n"
       "  const unsigned nb = gridDim.x, per = nb >> 3, rem = nb & 7, xcd = blockIdx.x & 7;\n"
    << tile_start() <<
       "  for (unsigned t = t0; t < nt; t += nb) {\n"
    << "    const unsigned g = t % " << S << "u, ct = t / " << S << "u;\n"
       "    const unsigned s = ct / tps;\n"
    // lanes past the last column redo the last column (same loads, same bytes stored)
    << "    const unsigned colb = min((ct - s * tps) * " << tile << " + threadIdx.x * " << 4 * D << ", cols - " << 4 * D << "u);\n"
       "    const unsigned sp = colb / P;\n"
    << "    const long long off = (long long)sp * " << W << " * P + (colb - sp * P);\n";
  const std::string A = shard_table(s, K, R, "    ");
  const int per_g = (W + S - 1) / S;
  // accumulators and input buffers declared once, shared by the groups' blocks (each group's
  // packet l uses slot l - l0): the compiler then gives the blocks the same registers
  for (int r = 0; r < R; ++r)
    for (int i = 0; i < per_g; ++i) s << "    u32 h" << r << "_" << i << "[D];\n";
  for (int b2 = 0; b2 < 2; ++b2)
    for (int x = 0; x < W; ++x) s << "    u32 e" << b2 << "_" << x << "[D];\n";
  for (int grp = 0; grp < S; ++grp) {
    const int l0 = grp * per_g, l1 = std::min(W, l0 + per_g);
    if (l0 >= l1) continue;
    std::vector<int> rl_of;  // this group's output packets, as r*W + l
    for (int r = 0; r < R; ++r)
      for (int l = l0; l < l1; ++l) rl_of.push_back(r * W + l);
    s << "    if (g == " << grp << "u) {\n";
    std::vector<bool> live(static_cast<size_t>(R) * W, false);
    // inputs and their packets this group reads
    std::vector<int> used;
    std::vector<uint32_t> need;
    for (int j = 0; j < K; ++j) {
      uint32_t nm_ = 0;
      for (int rl : rl_of) nm_ |= masks[static_cast<size_t>(rl) * K + j];
      if (nm_) {
        used.push_back(j);
        need.push_back(nm_);
      }
    }
    auto load = [&](size_t u) {
      const int j = used[u];
      s << "      { const unsigned long long p = " << A << "in[" << j << "].base + (unsigned long long)s * " << A << "in[" << j
        << "].stride + off;\n";
      for (int x = 0; x < W; ++x)
        if ((need[u] >> x) & 1u) s << "        ld(e" << u % 2 << "_" << x << ", p + " << x << "ull * P);\n";
      s << "      }\n";
    };
    if (!used.empty()) load(0);
    for (size_t u = 0; u < used.size(); ++u) {
      const int j = used[u];
      if (u + 1 < used.size()) load(u + 1);
      std::vector<std::vector<int>> rows(rl_of.size());
      for (size_t i = 0; i < rl_of.size(); ++i) {
        const uint32_t m = masks[static_cast<size_t>(rl_of[i]) * K + j];
        for (int x = 0; x < W; ++x)
          if ((m >> x) & 1u) rows[i].push_back(x);
      }
      std::vector<std::pair<int, int>> pairs;
      if (cap > 0) share_slice_pairs(rows, W, cap, pairs);
      const std::string eb = "e" + std::to_string(u % 2) + "_";
      auto nm = [&](int x) { return x < W ? eb + std::to_string(x) + "[d]" : "p" + std::to_string(x - W); };
      s << "      for (int d = 0; d < D; ++d) {\n";
      for (size_t i = 0; i < pairs.size(); ++i)
        s << "        const u32 p" << i << " = " << nm(pairs[i].first) << " ^ " << nm(pairs[i].second) << ";\n";
      for (size_t i = 0; i < rl_of.size(); ++i) {
        if (rows[i].empty()) continue;
        const int rl = rl_of[i];
        const std::string acc = "h" + std::to_string(rl / W) + "_" + std::to_string(rl % W - l0) + "[d]";
        std::vector<std::string> t;
        if (live[rl]) t.push_back(acc);
        for (int x : rows[i]) t.push_back(nm(x));
        s << "        " << acc << " = " << xor_chain(t) << ";\n";
        live[rl] = true;
      }
      s << "      }\n      __builtin_amdgcn_sched_barrier(0);\n";
    }
    for (int r = 0; r < R; ++r) {
      s << "      { const unsigned long long q = " << A << "out[" << r << "].base + (unsigned long long)s * " << A << "out[" << r
        << "].stride + off;\n";
      for (int l = l0; l < l1; ++l) {
        if (!live[static_cast<size_t>(r) * W + l]) s << "        for (int d = 0; d < D; ++d) h" << r << "_" << l - l0 << "[d] = 0u;\n";
        s << "        st(h" << r << "_" << l - l0 << ", q + " << l << "ull * P);\n";
      }
      s << "      }\n";
    }
    s << "    }\n";
  }
  s << "  }\n}\n";
  return s.str();
}

std::string gfw_source(const uint32_t *mat, int R, int K, int W) {
  if (gfw_rowsplit(W, R)) return gfw_rowsplit_source(mat, R, K, W);
  // LSEC_JIT_VARIANT bits 8-15: most shared pairs per input (0: the default 32, 255: none);
  // bit 16: let the compiler schedule loads freely (no one-input-ahead prefetch fenced by sched
  // barriers: it then hoists every input's loads and spills at 10+4, w = 32)
  const int capv = (jit_variant() >> 8) & 255;
  const int cap = capv == 0 ? 32 : capv == 255 ? 0 : capv;
  const bool fenced = !((jit_variant() >> 16) & 1);
  // bits 17-18: inputs loaded ahead of their use (0: the default 1); bit 21: serial XOR folds
  const int ahead = std::max(1, (jit_variant() >> 17) & 3);
  const bool linear = (jit_variant() >> 21) & 1;
  const int tile = gfw_tile(W, R);  // the launch covers whole tiles only
  std::ostringstream s;
  gfw_prelude(s, R, K, W, 4096);
  s << "extern \"C\" __global__ __launch_bounds__(256) void lsec_xornet(Args a) {\n"
       "  const long long C = a.size;\n"
    << "  const unsigned tps = (unsigned)(C / " << tile << ");\n"
    << "  const unsigned nt = tps * (unsigned)a.nstripes;\n"
       "  const unsigned nb = gridDim.x, per = nb >> 3, rem = nb & 7, xcd = blockIdx.x & 7;\n"
    << tile_start() <<
       "  for (unsigned t = t0; t < nt; t += nb) {\n"
       "    const unsigned s = t / tps;\n"
    << "    const long long base = (long long)(t - s * tps) * " << tile << " + threadIdx.x * 16;\n";
  const std::string A = shard_table(s, K, R, "    ");
  std::vector<std::string> acc;
  std::vector<int> rows;
  for (int r = 0; r < R; ++r) {
    s << "    u32 h" << r << "[W];\n";
    acc.push_back("h" + std::to_string(r));
    rows.push_back(r);
  }
  std::vector<std::vector<bool>> live(R, std::vector<bool>(W, false));
  // inputs with a non-zero coefficient in some row, each loaded one input ahead of its use: the
  // scheduler would otherwise hoist every input's loads to the top (K x W registers live: spills
  // at 10+4, w = 32), so sched barriers fence each input's arithmetic
  const std::vector<int> used = gfw_used(mat, R, K);
  const size_t nbuf = static_cast<size_t>(ahead) + 1;
  auto load = [&](size_t u) {
    const int j = used[u];
    s << "    ld(e" << u % nbuf << ", " << A << "in[" << j << "].base + (unsigned long long)s * " << A << "in[" << j
      << "].stride + base);\n";
  };
  for (size_t b = 0; b < nbuf; ++b) s << "    u32 e" << b << "[W];\n";
  for (size_t u = 0; u < used.size() && u < static_cast<size_t>(ahead); ++u) load(u);
  for (size_t u = 0; u < used.size(); ++u) {
    if (u + ahead < used.size()) load(u + ahead);
    const std::string e = "e" + std::to_string(u % nbuf);
    s << "    tr(" << e << ");\n";
    gfw_net(s, mat, K, W, used[u], rows, acc, live, cap, e, "    ", linear);
    if (fenced) s << "    __builtin_amdgcn_sched_barrier(0);\n";
  }
  for (int r = 0; r < R; ++r) {
    for (int b = 0; b < W; ++b)
      if (!live[r][b]) s << "    h" << r << "[" << b << "] = 0u;\n";
    s << "    tr(h" << r << ");\n    st(h" << r << ", " << A << "out[" << r << "].base + (unsigned long long)s * " << A << "out[" << r
      << "].stride + base);\n";
  }
  s << "  }\n}\n";
  return s.str();
}

int xornet_tile(int K, int R) {
  const int D = xornet_dwords(R, K);
  const int IT = D == 4 && K * 8 <= 104 ? 2 : 1;
  return 256 * 4 * D * IT;
}

namespace {

struct Entry {
  std::vector<uint32_t> mat;  // R x K coefficients (GF(2^w) elements)
  int R = 0, K = 0, w = 8;
  int D = 0;  // packet networks (pktnet_source): dwords per lane per packet; 0 = a matrix network
  int S = 1;  // packet networks: output groups
  enum State { kCompiling, kReady, kFailed } state = kCompiling;
  std::vector<char> code;                 // code object
  std::map<int, hipModule_t> modules;     // device -> module
  std::map<int, hipFunction_t> functions; // device -> kernel
  std::string err;
  std::vector<uint32_t> key;  // its g_by_matrix key
};

// leaked on purpose: a compile worker still waiting on its compiler when the process exits may
// touch them
std::mutex &g_mu = *new std::mutex();
std::condition_variable &g_cv = *new std::condition_variable();
// Compiles run in child processes (lsec_jitc, ec_jitc.cpp), started by at most kWorkers threads
// fed from a queue.  hipRTC never runs in this process: its compiler's global state, destroyed
// by the process's exit under a compile still running, corrupted the heap in round 4, and the
// wait for running compiles that fixed it held exit for as long as a compile takes (30 s for the
// widest w = 32 networks on the build host).  At exit no queued compile starts and the running
// compilers are killed; nothing is waited for (tests/test_jit_queue.py).
constexpr int kWorkers = 2;
auto &g_queue = *new std::deque<std::shared_ptr<struct Entry>>();
int g_running = 0, g_workers = 0;
bool g_exiting = false;
// bumped whenever an image is bound or unbound: invalidates the threads' ready() caches
std::atomic<uint64_t> g_gen{1};
// the compiler processes running now (their own lock: the exit handler may run while a worker
// holds g_mu)
std::mutex &g_child_mu = *new std::mutex();
auto &g_children = *new std::set<pid_t>();
bool g_children_killed = false;

void stop_compiles() {
  {
    std::lock_guard<std::mutex> lk(g_child_mu);
    g_children_killed = true;
    for (pid_t p : g_children) kill(p, SIGKILL);
  }
  std::lock_guard<std::mutex> lk(g_mu);
  g_exiting = true;
  g_cv.notify_all();
}
auto &g_by_matrix = *new std::map<std::vector<uint32_t>, std::shared_ptr<Entry>>();  // key: R, K, w, matrix
auto &g_by_image = *new std::map<const void *, std::shared_ptr<Entry>>();           // device image -> entry

std::vector<uint32_t> key_of(const uint32_t *mat, int R, int K, int w) {
  std::vector<uint32_t> k(3 + static_cast<size_t>(R) * K);
  k[0] = static_cast<uint32_t>(R);
  k[1] = static_cast<uint32_t>(K);
  k[2] = static_cast<uint32_t>(w);
  std::memcpy(k.data() + 3, mat, sizeof(uint32_t) * R * K);
  return k;
}

// lsec_jitc beside this library (LSEC_JITC overrides)
const std::string &compiler_path() {
  // leaked: a compile worker may still report a failure while the process exits
  static const std::string &path = *new std::string([] {
    if (const char *e = getenv("LSEC_JITC")) return std::string(e);
    Dl_info info;
    if (dladdr(reinterpret_cast<void *>(&compiler_path), &info) && info.dli_fname) {
      std::string f(info.dli_fname);
      const size_t slash = f.rfind('/');
      return (slash == std::string::npos ? std::string(".") : f.substr(0, slash)) + "/lsec_jitc";
    }
    return std::string("lsec_jitc");
  }());
  return path;
}

// The exit handler is registered by the first compile (a handler that runs while no compile
// exists has nothing to do).
void register_exit_handler() {
  static std::once_flag once;
  std::call_once(once, [] { atexit(stop_compiles); });
}

// gfx950 code object of `src` from a compiler process (protocol in ec_jitc.cpp), or the reason in
// err.  Sockets, not pipes: a write to a compiler that died must return EPIPE, not raise SIGPIPE
// in the caller's process.
void compile_source(const std::string &src, std::string &err, std::vector<char> &code) {
  register_exit_handler();
  int in[2], out[2];
  if (socketpair(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0, in) != 0) {
    err = "socketpair failed";
    return;
  }
  if (socketpair(AF_UNIX, SOCK_STREAM | SOCK_CLOEXEC, 0, out) != 0) {
    close(in[0]);
    close(in[1]);
    err = "socketpair failed";
    return;
  }
  posix_spawn_file_actions_t fa;
  posix_spawn_file_actions_init(&fa);
  posix_spawn_file_actions_adddup2(&fa, in[1], 0);
  posix_spawn_file_actions_adddup2(&fa, out[1], 1);
  posix_spawn_file_actions_addopen(&fa, 2, "/dev/null", O_WRONLY, 0);
  const std::string ppid = std::to_string(getpid());
  char *argv[] = {const_cast<char *>(compiler_path().c_str()), const_cast<char *>(ppid.c_str()), nullptr};
  pid_t pid = -1;
  int rc;
  {
    std::lock_guard<std::mutex> lk(g_child_mu);
    rc = g_children_killed ? -1 : posix_spawn(&pid, argv[0], &fa, nullptr, argv, ::environ);
    if (rc == 0) g_children.insert(pid);
  }
  posix_spawn_file_actions_destroy(&fa);
  close(in[1]);
  close(out[1]);
  if (rc != 0) {
    close(in[0]);
    close(out[0]);
    err = rc < 0 ? "exiting" : "cannot start the network compiler " + compiler_path() + ": " + strerror(rc);
    return;
  }
  for (size_t o = 0; o < src.size();) {
    const ssize_t w = send(in[0], src.data() + o, src.size() - o, MSG_NOSIGNAL);
    if (w <= 0) break;  // the compiler died: its missing reply says so below
    o += static_cast<size_t>(w);
  }
  close(in[0]);
  std::vector<char> reply;
  char buf[1 << 16];
  for (;;) {
    const ssize_t r = read(out[0], buf, sizeof(buf));
    if (r <= 0) break;
    reply.insert(reply.end(), buf, buf + r);
  }
  close(out[0]);
  // Wait for the exit without reaping (WNOWAIT), take the pid out of g_children, and only then
  // reap: until the reap the pid stays a zombie of ours, so stop_compiles can never SIGKILL a pid
  // the system has already handed to another process
  siginfo_t si;
  while (waitid(P_PID, static_cast<id_t>(pid), &si, WEXITED | WNOWAIT) < 0 && errno == EINTR) {
  }
  {
    std::lock_guard<std::mutex> lk(g_child_mu);
    g_children.erase(pid);
  }
  int status = 0;
  while (waitpid(pid, &status, 0) < 0 && errno == EINTR) {
  }
  uint64_t n = 0;
  if (reply.size() >= 13)
    for (int i = 0; i < 8; ++i) n |= static_cast<uint64_t>(static_cast<uint8_t>(reply[5 + i])) << (8 * i);
  if (reply.size() < 13 || std::memcmp(reply.data(), "LSJC", 4) != 0 || reply.size() != 13 + n) {
    std::lock_guard<std::mutex> lk(g_child_mu);
    err = g_children_killed ? "exiting" : "the network compiler " + compiler_path() + " gave no answer";
    return;
  }
  if (reply[4] != 0) {
    err.assign(reply.begin() + 13, reply.end());
    return;
  }
  code.assign(reply.begin() + 13, reply.end());
}

void compile(std::shared_ptr<Entry> e) {
  const auto t0 = std::chrono::steady_clock::now();
  std::string src;
  if (e->D > 0) {
    src = pktnet_source(e->mat.data(), e->R, e->K, e->w, e->D, e->S);
  } else if (e->w == 8) {
    std::vector<uint8_t> m8(e->mat.begin(), e->mat.end());
    src = xornet_source(m8.data(), e->R, e->K);
  } else {
    src = gfw_source(e->mat.data(), e->R, e->K, e->w);
  }
  std::string err;
  std::vector<char> code;
  compile_source(src, err, code);
  static const bool trace = getenv("LSEC_TRACE") != nullptr;
  if ((trace || !err.empty()) && err != "exiting")
    fprintf(stderr, "[lsec jit] %dx%d w=%d xor network: %s (%.2f s)\n", e->R, e->K, e->w, err.empty() ? "compiled" : err.c_str(),
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
  std::lock_guard<std::mutex> lk(g_mu);
  e->code.swap(code);
  e->err = err;
  e->state = err.empty() ? Entry::kReady : Entry::kFailed;
  --g_running;
  g_cv.notify_all();
}

void compile_worker() {
  for (;;) {
    std::shared_ptr<Entry> e;
    {
      std::unique_lock<std::mutex> lk(g_mu);
      g_cv.wait(lk, [] { return g_exiting || !g_queue.empty(); });
      if (g_exiting) return;
      e = g_queue.front();
      g_queue.pop_front();
      // a network whose every image was unbound (its plans destroyed before the compile started)
      // is dropped: a later bind of the same matrix queues it afresh
      bool bound = false;
      for (const auto &kv : g_by_image)
        if (kv.second == e) {
          bound = true;
          break;
        }
      if (!bound) {
        g_by_matrix.erase(e->key);
        e->state = Entry::kFailed;
        e->err = "dropped: no longer bound";
        g_cv.notify_all();
        continue;
      }
      ++g_running;
    }
    compile(e);
  }
}

// the kernel of a ready entry on device `dev` (loads the module once per device; under g_mu)
hipFunction_t function_locked(Entry &e, int dev) {
  if (e.state != Entry::kReady) return nullptr;
  auto it = e.functions.find(dev);
  if (it != e.functions.end()) return it->second;
  hipModule_t mod = nullptr;
  hipFunction_t fn = nullptr;
  if (quiet([&] {
        const hipError_t r = hipModuleLoadData(&mod, e.code.data());
        return r != hipSuccess ? r : hipModuleGetFunction(&fn, mod, "lsec_xornet");
      }) != hipSuccess) {
    e.state = Entry::kFailed;
    e.err = "module load failed";
    return nullptr;
  }
  e.modules[dev] = mod;
  e.functions[dev] = fn;
  return fn;
}

}  // namespace

void bind(const void *image, const uint8_t *mat, int R, int K) {
  if (!image || !wants_xornet(R, K)) return;
  std::vector<uint32_t> m32(mat, mat + static_cast<size_t>(R) * K);
  bind_entry(image, m32.data(), R, K, 8);
}

void bind_w(const void *image, const uint32_t *mat, int R, int K, int w) {
  if (!image || !wants_gfw_net(R, K, w)) return;
  bind_entry(image, mat, R, K, w);
}

void bind_entry(const void *image, const uint32_t *mat, int R, int K, int w) {
  bind_key(image, key_of(mat, R, K, w), mat, static_cast<size_t>(R) * K, R, K, w, 0, 1);
}

void bind_pkt(const void *image, const uint32_t *masks, int R, int K, int w, int packet) {
  if (!image || !wants_pktnet(R, K, w)) return;
  int D = 0, S = 1;
  pkt_shape(R, w, packet, &D, &S);
  if (D == 0) return;
  const size_t n = static_cast<size_t>(R) * w * K;  // one mask word per (bit-row, input): w <= 32
  std::vector<uint32_t> key = {static_cast<uint32_t>(R), static_cast<uint32_t>(K), 1000u + static_cast<uint32_t>(w),
                               static_cast<uint32_t>(D), static_cast<uint32_t>(S)};
  key.insert(key.end(), masks, masks + n);
  bind_key(image, key, masks, n, R, K, w, D, S);
}

void bind_pkt_field(const void *image, const uint32_t *coef, int R, int K, int w, int packet) {
  // the bitmatrix of each GF(2^w) coefficient: output packet l takes input packet x where bit l
  // of c * x^x is set (Cauchy's packet layout, k_gfw_bitsliced)
  if (!image || !wants_pktnet(R, K, w) || (w != 8 && w != 16 && w != 32)) return;
  // w = 8: Cauchy's bit-sliced GF(2^8) (k_gf8_bitsliced's layout): Cauchy-good(10+4) at 4 MiB
  // 0.72 -> 0.74, (6+3) level (profiles/r04_v17_pktnet_cauchy8.txt); LSEC_JIT_VARIANT bit 27: off
  if (w == 8 && ((jit_variant() >> 27) & 1)) return;
  std::vector<uint32_t> masks(static_cast<size_t>(R) * w * K, 0u);
  for (int r = 0; r < R; ++r)
    for (int j = 0; j < K; ++j) {
      uint32_t cx = coef[r * K + j] & (w == 8 ? 0xFFu : w == 16 ? 0xFFFFu : 0xFFFFFFFFu);
      for (int x = 0; x < w && cx; ++x) {
        for (int l = 0; l < w; ++l)
          if ((cx >> l) & 1u) masks[(static_cast<size_t>(r) * w + l) * K + j] |= 1u << x;
        cx = gfw_times_x(cx, w);
      }
    }
  bind_pkt(image, masks.data(), R, K, w, packet);
}

void bind_key(const void *image, const std::vector<uint32_t> &key, const uint32_t *mat, size_t n, int R, int K, int w,
              int D, int S) {
  std::shared_ptr<Entry> e;
  bool start = false;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_by_matrix.find(key);
    if (it == g_by_matrix.end()) {
      e = std::make_shared<Entry>();
      e->mat.assign(mat, mat + n);
      e->R = R;
      e->K = K;
      e->w = w;
      e->D = D;
      e->S = S;
      e->key = key;
      g_by_matrix.emplace(key, e);
      start = true;
      g_queue.push_back(e);
      if (g_workers < kWorkers) {
        ++g_workers;
        std::thread(compile_worker).detach();
      }

    } else {
      e = it->second;
    }
    g_by_image[image] = e;
    g_gen.fetch_add(1, std::memory_order_acq_rel);
  }
  if (start) g_cv.notify_all();
}

void unbind(const void *image) {
  std::lock_guard<std::mutex> lk(g_mu);
  g_by_image.erase(image);
  g_gen.fetch_add(1, std::memory_order_acq_rel);
}

int wait(const void *image, int timeout_ms) {
  std::unique_lock<std::mutex> lk(g_mu);
  auto it = g_by_image.find(image);
  if (it == g_by_image.end()) return 0;
  std::shared_ptr<Entry> e = it->second;
  // a network someone waits for compiles next
  auto q = std::find(g_queue.begin(), g_queue.end(), e);
  if (q != g_queue.end() && q != g_queue.begin()) {
    g_queue.erase(q);
    g_queue.push_front(e);
  }
  g_cv.wait_for(lk, std::chrono::milliseconds(timeout_ms), [&] { return e->state != Entry::kCompiling; });
  return e->state == Entry::kReady ? 1 : 0;
}

hipFunction_t ready(const void *image, int R, int K) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  // per-thread cache of ready kernels: per-stripe launches from hundreds of pool threads take no
  // lock once their network is loaded (a bind or unbind anywhere empties every cache)
  struct Key {
    const void *image;
    int dev, R, K;
    bool operator<(const Key &o) const {
      return image != o.image ? image < o.image : dev != o.dev ? dev < o.dev : R != o.R ? R < o.R : K < o.K;
    }
  };
  thread_local std::map<Key, hipFunction_t> cache;
  thread_local uint64_t cache_gen = 0;
  const uint64_t gen = g_gen.load(std::memory_order_acquire);
  if (cache_gen != gen) {
    cache.clear();
    cache_gen = gen;
  }
  const Key key{image, dev, R, K};
  auto c = cache.find(key);
  if (c != cache.end()) return c->second;
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_by_image.find(image);
  if (it == g_by_image.end() || it->second->R != R || it->second->K != K) return nullptr;
  hipFunction_t fn = function_locked(*it->second, dev);
  if (fn && g_gen.load(std::memory_order_acquire) == gen) cache[key] = fn;  // not yet ready: ask again next time
  return fn;
}

hipError_t launch(hipFunction_t fn, int R, int K, const ShardRef *in, const ShardRef *out, int nstripes, int64_t size,
                  hipStream_t st, int w) {
  // struct Args { long long size; int nstripes; int pad; Ref in[K]; Ref out[R]; }
  // struct Args { ...; Ref out[R]; unsigned phase; } (8-byte aligned size)
  std::vector<uint8_t> args(16 + sizeof(ShardRef) * (K + R) + 8, 0);
  std::memcpy(args.data(), &size, 8);
  std::memcpy(args.data() + 8, &nstripes, 4);
  std::memcpy(args.data() + 16, in, sizeof(ShardRef) * K);
  std::memcpy(args.data() + 16 + sizeof(ShardRef) * K, out, sizeof(ShardRef) * R);
  const int64_t tile = w == 8 ? xornet_tile(K, R) : gfw_tile(w, R);  // as xornet_source / gfw_source
  const uint64_t tps = w == 8 ? static_cast<uint64_t>((size + tile - 1) / tile) : static_cast<uint64_t>(size / tile);
  const uint32_t phase = lsec::tile_phase_net_on() ? static_cast<uint32_t>(tps / 8) : 0;
  std::memcpy(args.data() + 16 + sizeof(ShardRef) * (K + R), &phase, 4);
  size_t bytes = args.size();
  void *cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, args.data(), HIP_LAUNCH_PARAM_BUFFER_SIZE, &bytes, HIP_LAUNCH_PARAM_END};
  const uint64_t ntiles = static_cast<uint64_t>((size + tile - 1) / tile) * static_cast<uint64_t>(nstripes);
  if (ntiles == 0) return hipSuccess;
  if (ntiles >= (1ull << 31)) return hipErrorInvalidValue;
  return hipModuleLaunchKernel(fn, static_cast<unsigned>(ntiles), 1, 1, 256, 1, 1,
                               static_cast<unsigned>(lsec::occupancy_lds_bytes(size)), st, nullptr, cfg);
}

hipError_t launch_pkt(hipFunction_t fn, int R, int K, const ShardRef *in, const ShardRef *out, int nstripes, int64_t size,
                      int packet, int w, hipStream_t st) {
  // struct Args { long long size; int nstripes; int packet; Ref in[K]; Ref out[R]; }
  std::vector<uint8_t> args(16 + sizeof(ShardRef) * (K + R) + 8, 0);  // (+ unsigned phase, 8-byte aligned)
  std::memcpy(args.data(), &size, 8);
  std::memcpy(args.data() + 8, &nstripes, 4);
  std::memcpy(args.data() + 12, &packet, 4);
  std::memcpy(args.data() + 16, in, sizeof(ShardRef) * K);
  std::memcpy(args.data() + 16 + sizeof(ShardRef) * K, out, sizeof(ShardRef) * R);
  int D = 0, S = 1;
  pkt_shape(R, w, packet, &D, &S);  // as bind_pkt
  const int64_t tile = 256 * 4 * D, cols = size / w;  // column bytes of a stripe: nsuper * packet
  const uint64_t tps = static_cast<uint64_t>((cols + tile - 1) / tile) * S;  // tiles per stripe
  const uint32_t phase = lsec::tile_phase_net_on() ? static_cast<uint32_t>(tps / 8) : 0;
  std::memcpy(args.data() + 16 + sizeof(ShardRef) * (K + R), &phase, 4);
  size_t bytes = args.size();
  void *cfg[] = {HIP_LAUNCH_PARAM_BUFFER_POINTER, args.data(), HIP_LAUNCH_PARAM_BUFFER_SIZE, &bytes, HIP_LAUNCH_PARAM_END};
  const uint64_t ntiles = tps * static_cast<uint64_t>(nstripes);
  if (ntiles == 0) return hipSuccess;
  if (ntiles >= (1ull << 31)) return hipErrorInvalidValue;
  return hipModuleLaunchKernel(fn, static_cast<unsigned>(ntiles), 1, 1, 256, 1, 1,
                               static_cast<unsigned>(lsec::occupancy_lds_bytes(size)), st, nullptr, cfg);
}

void pkt_shape(int R, int w, int packet, int *D, int *S) {
  // 16 B per lane where the packet allows, fewer where the R*w accumulator packets would pass 64
  // dwords (w = 7 / 8 at R = 2: 4 dwords, ~120 registers).  One output group: Cauchy(10+4) at
  // w = 32 (128 accumulators, one wave per SIMD) encodes at 0.80 that way, 0.61 / 0.41 in 2 / 4
  // groups (profiles/r04_v13_pktnet_cauchy.txt); LSEC_JIT_VARIANT bits 25-26 force 1 / 2 / 4
  int d = packet % 16 == 0 ? 4 : packet % 8 == 0 ? 2 : packet % 4 == 0 ? 1 : 0;
  while (d > 1 && R * w * d > 64) d /= 2;
  const int fv = (jit_variant() >> 25) & 3;
  *D = d;
  *S = fv ? 1 << (fv - 1) : 1;
}

bool pkt_aligned(const ShardRef *in, int K, const ShardRef *out, int R, int w, int packet) {
  int d = 0, g = 1;
  pkt_shape(R, w, packet, &d, &g);
  if (d == 0) return false;
  const uint64_t a = 4u * static_cast<uint64_t>(d);
  for (int j = 0; j < K; ++j)
    if (in[j].base % a || static_cast<uint64_t>(in[j].stride) % a) return false;
  for (int r = 0; r < R; ++r)
    if (out[r].base % a || static_cast<uint64_t>(out[r].stride) % a) return false;
  return true;
}

}  // namespace jit
}  // namespace lsec

extern "C" {

// Test hook, not in include/ (no GPU): generate and compile, synchronously (lsec_jitc), the
// network of a pseudo-random matrix for each generator shape -- shape 0: w = 8 XOR network
// (R x K bytes), 1: w = 16 / 32 bit-sliced network (one wave, or the wave-pair split from 4 rows
// at w = 32 / 5 rows at w = 16), 2: packet network over bitmatrix masks (w <= 32), 3: packet
// network over GF(2^w) coefficients.  Returns 0, or -1 with the compiler's reason.
int lsec_test_jit_compile(int shape, int R, int K, int w, int packet, unsigned seed) {
  if (R < 1 || R > 8 || K < 1 || K > 32 || shape < 0 || shape > 3) return lsec::set_error("lsec_test_jit_compile: bad arguments");
  unsigned x = seed * 2654435761u + 12345u;
  auto rnd = [&x] {
    x = x * 1103515245u + 12345u;
    return x >> 7;
  };
  std::string src;
  if (shape == 0) {
    std::vector<uint8_t> m(static_cast<size_t>(R) * K);
    for (auto &v : m) v = static_cast<uint8_t>(rnd() | 1u);
    src = lsec::jit::xornet_source(m.data(), R, K);
  } else if (shape == 1) {
    if (w != 16 && w != 32) return lsec::set_error("lsec_test_jit_compile: w %d", w);
    std::vector<uint32_t> m(static_cast<size_t>(R) * K);
    for (auto &v : m) v = (rnd() ^ (rnd() << 16)) & (w == 16 ? 0xFFFFu : 0xFFFFFFFFu);
    src = lsec::jit::gfw_source(m.data(), R, K, w);
  } else {
    if (w < 2 || w > 32 || packet < 4) return lsec::set_error("lsec_test_jit_compile: w %d packet %d", w, packet);
    std::vector<uint32_t> masks(static_cast<size_t>(R) * w * K);
    if (shape == 2) {
      for (auto &v : masks) v = rnd() & rnd() & (w == 32 ? 0xFFFFFFFFu : (1u << w) - 1u);
    } else {
      if (w != 16 && w != 32) return lsec::set_error("lsec_test_jit_compile: w %d", w);
      std::vector<uint32_t> coef(static_cast<size_t>(R) * K);
      for (auto &v : coef) v = (rnd() ^ (rnd() << 16)) & (w == 16 ? 0xFFFFu : 0xFFFFFFFFu);
      for (int r = 0; r < R; ++r)
        for (int j = 0; j < K; ++j) {
          uint32_t cx = coef[r * K + j];
          for (int b = 0; b < w && cx; ++b) {
            for (int l = 0; l < w; ++l)
              if ((cx >> l) & 1u) masks[(static_cast<size_t>(r) * w + l) * K + j] |= 1u << b;
            cx = lsec::jit::gfw_times_x(cx, w);
          }
        }
    }
    int D = 0, S = 1;
    lsec::jit::pkt_shape(R, w, packet, &D, &S);
    if (D == 0) return lsec::set_error("lsec_test_jit_compile: packet %d", packet);
    src = lsec::jit::pktnet_source(masks.data(), R, K, w, D, S);
  }
  std::string err;
  std::vector<char> code;
  lsec::jit::compile_source(src, err, code);
  if (!err.empty()) return lsec::set_error("lsec_test_jit_compile: %s", err.c_str());
  return code.empty() ? lsec::set_error("lsec_test_jit_compile: no code object") : 0;
}

// Test hook, not in include/ (no GPU; the compiler runs on the host): bind n distinct pseudo-random
// R x K GF(2^w) matrices (w = 16 / 32) to stand-in image addresses (never dereferenced), wait up to
// wait_ms for the first compile, unbind them all, and return how many compiles were ready by then.
// A process that returns right after leaves compiles queued and running at its exit
// (tests/test_jit_queue.py).
int lsec_test_jit_queue(int n, int wait_ms, int R, int K, int w, unsigned seed) {
  if (n < 1 || n > 64 || wait_ms < 0 || R < 1 || R > 8 || K < 1 || K > 32 || (w != 16 && w != 32)) return -1;
  static char stand_in[64];
  std::vector<uint32_t> mat(static_cast<size_t>(R) * K);
  unsigned x = seed * 2654435761u + 777u;
  for (int i = 0; i < n; ++i) {
    for (auto &c : mat) {
      x = x * 1103515245u + 12345u;
      c = ((x >> 5) ^ (x << 11)) & (w == 16 ? 0xFFFFu : 0xFFFFFFFFu);
      c |= 2u;  // not an XOR-only row
    }
    lsec::jit::bind_entry(stand_in + i, mat.data(), R, K, w);
  }
  (void)lsec::jit::wait(stand_in, wait_ms);
  int ready = 0;
  {
    std::lock_guard<std::mutex> lk(lsec::jit::g_mu);
    for (int i = 0; i < n; ++i) {
      auto it = lsec::jit::g_by_image.find(stand_in + i);
      if (it != lsec::jit::g_by_image.end() && it->second->state == lsec::jit::Entry::kReady) ++ready;
    }
  }
  for (int i = 0; i < n; ++i) lsec::jit::unbind(stand_in + i);
  return ready;
}

}  // extern "C"
