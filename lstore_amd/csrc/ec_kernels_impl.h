// ec_kernels_impl.h -- gfx950 (CDNA4) erasure-coding kernels (device templates).
// Instantiated per output-row count R in ec_kernels_inst.hip (one translation unit per R, so
// the many (R, K, tile) specialisations compile in parallel); launched from ec_kernels.hip.
// See ec_kernels.h for the contract.
//
// The path is HBM-bound byte/bit arithmetic (no MFMA):
//   encode  reads K*C, writes R*C bytes per stripe
//   decode  reads K survivors, writes R = #erased shards
// Both kernels stream every input byte exactly once from HBM and write every output byte
// exactly once; all GF(2^8) work happens in VGPRs.
//
// gf8_bytewise (Reed-Solomon / matrix codes).  Multiply-by-constant c of a byte v is split
// over three bit fields of v:  c*v = c*(v & 7) ^ c*(v & 0x38) ^ c*(v & 0xC0).  Each field
// has at most 8 values, so each partial product is ONE v_perm_b32 that selects bytes out of
// an 8-byte table {c*0..c*7}, {c*0,c*8,..,c*56} or {c*0,c*64,c*128,c*192} -- four bytes of
// the word at once.  The three field extractions are shared by all R outputs of an input
// shard; per (output, input) pair a word costs 3 perms + 2 xors (one of them gfx950's
// 3-input v_bitop3), versus a 64 KiB table walk per byte on the CPU (galois.c:471-525).
//
// gf8_bitsliced (Cauchy / bitmatrix codes).  In Jerasure's packet layout the 8 bits of a
// field element live in 8 different packets, so a 32-bit lane word of each packet carries
// bit x of 32 independent elements.  Multiplying all of them by 2 is then a renaming of
// the 8 packet words plus 3 XORs (x^8 = x^4+x^3+x^2+1), and c*e = sum_{t: c_t=1} 2^t e.
// Per input shard: 7 doublings (21 xors per 8 words), then 8 xors per set coefficient bit,
// under wave-uniform branches.  Identical result to running the smart XOR schedule over
// the bitmatrix (jerasure.c:1168-1191), but every packet is read once and all
// intermediates stay in registers instead of streaming P-byte XORs through memory.
#pragma once
#include "ec_kernels.h"

#include <algorithm>

namespace lsec {

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int N> struct VecT;
template <> struct VecT<1> { typedef uint32_t type; };
template <> struct VecT<2> { typedef u32x2 type; };
template <> struct VecT<4> { typedef u32x4 type; };

constexpr int kBlock = 256;

// The coefficient image is read-only and every lane of a wave reads the same cell, so read
// it through the constant address space: uniform addresses there become s_load (SGPRs),
// leaving the VALU and the vector memory pipe to the shard bytes.
typedef const __attribute__((address_space(4))) CoefCell ConstCell;

__device__ __forceinline__ ConstCell *const_cells(const CoefCell *p) {
  return reinterpret_cast<ConstCell *>(reinterpret_cast<uintptr_t>(p));
}

// Shard addresses arrive as integers; give them the global address space explicitly so
// loads/stores are global_* (vmcnt only) rather than flat_* (vmcnt + lgkmcnt).
#define LSEC_GLOBAL __attribute__((address_space(1)))
template <typename T>
__device__ __forceinline__ const LSEC_GLOBAL T *gptr(uint64_t addr) {
  return reinterpret_cast<const LSEC_GLOBAL T *>(addr);
}
template <typename T>
__device__ __forceinline__ LSEC_GLOBAL T *gptr_w(uint64_t addr) {
  return reinterpret_cast<LSEC_GLOBAL T *>(addr);
}

// ------------------------------------------------------------------ bytewise
// 3-input XOR in one VALU op (gfx950 v_bitop3_b32, truth table 0x96)
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// acc ^= c * word (4 bytes in parallel): 3 byte-permutes over the cell's tables + 2 xors
__device__ __forceinline__ uint32_t gf_mul_acc(uint32_t acc, uint32_t ia, uint32_t ib, uint32_t ic,
                                               const uint32_t (&t)[6]) {
  return xor3(acc, __builtin_amdgcn_perm(t[1], t[0], ia), __builtin_amdgcn_perm(t[3], t[2], ib)) ^
         __builtin_amdgcn_perm(t[5], t[4], ic);
}

// Spread the grid so that each XCD (blocks b, b+8, b+16, ... are dealt to one XCD) gets a
// contiguous run of tiles instead of every 8th tile: measured +2-3% HBM throughput on this
// streaming pattern (tools/kprobe.hip).  Bijective for any grid size; placement is only a
// speed hint, correctness never depends on it.
__device__ __forceinline__ uint32_t xcd_remap(uint32_t b, uint32_t nb) {
  const uint32_t per = nb >> 3, rem = nb & 7, xcd = b & 7;
  return xcd * per + min(xcd, rem) + (b >> 3);
}

// Per-lane work unit of the bytewise kernel: VW dwords (16 B for VW = 4, 8 B for VW = 2) per
// step, IT steps kBlock*4*VW bytes apart; a tile is kBlock*4*VW*IT bytes of every shard.
template <int IT, int VW>
struct BwTile {
  static constexpr int kStep = kBlock * 4 * VW;
  static constexpr int kBytes = kStep * IT;
};

template <int R, int IT, int VW>
__device__ __forceinline__ void bw_accumulate(typename VecT<VW>::type (&acc)[IT][R],
                                              const typename VecT<VW>::type (&v)[IT], ConstCell *cells, int K,
                                              int j) {
  typedef typename VecT<VW>::type V;
  V ia[IT], ib[IT], ic[IT];
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    ia[it] = v[it] & 0x07070707u;
    ib[it] = (v[it] >> 3) & 0x07070707u;
    ic[it] = (v[it] >> 6) & 0x03030303u;
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    ConstCell *cell = cells + r * K + j;  // wave-uniform -> scalar loads
    const uint32_t c = cell->coef;
    if (c == 0) continue;
    if (c == 1) {
#pragma unroll
      for (int it = 0; it < IT; ++it) acc[it][r] ^= v[it];
      continue;
    }
    const uint32_t t[6] = {cell->ta_lo, cell->ta_hi, cell->tb_lo, cell->tb_hi, cell->tc_lo, cell->tc_hi};
#pragma unroll
    for (int it = 0; it < IT; ++it)
#pragma unroll
      for (int e = 0; e < VW; ++e) acc[it][r][e] = gf_mul_acc(acc[it][r][e], ia[it][e], ib[it][e], ic[it][e], t);
  }
}

// MINW = minimum waves per SIMD the register allocation must allow (1 = unconstrained).
template <int R, int KC, int IT, int MINW, int VW>
__global__ __launch_bounds__(kBlock, MINW) void k_gf8_bytewise(ApplyArgs a) {
  typedef typename VecT<VW>::type V;
  constexpr int kStep = BwTile<IT, VW>::kStep;
  constexpr int kTile = BwTile<IT, VW>::kBytes;
  constexpr int kLane = 4 * VW;
  const int K = KC ? KC : a.K;
  const int64_t C = a.size;
  const uint32_t tiles_per_stripe = static_cast<uint32_t>((C + kTile - 1) / kTile);
  const uint32_t ntiles = tiles_per_stripe * static_cast<uint32_t>(a.nstripes);
  ConstCell *cells = const_cells(a.cells);

  for (uint32_t t = xcd_remap(blockIdx.x, gridDim.x); t < ntiles; t += gridDim.x) {
    const uint32_t s = t / tiles_per_stripe;
    const int64_t off0 = static_cast<int64_t>(t - s * tiles_per_stripe) * kTile + threadIdx.x * kLane;
    const bool full = (static_cast<int64_t>(t - s * tiles_per_stripe) + 1) * kTile <= C;  // wave-uniform

    V acc[IT][R];
#pragma unroll
    for (int it = 0; it < IT; ++it)
#pragma unroll
      for (int r = 0; r < R; ++r) acc[it][r] = 0u;

    if (full) {
      if constexpr (KC > 0) {
        // all K*IT loads in flight before any arithmetic
        V v[KC][IT];
#pragma unroll
        for (int j = 0; j < KC; ++j) {
          const uint64_t p = a.in[j].base + s * a.in[j].stride + off0;
#pragma unroll
          for (int it = 0; it < IT; ++it) v[j][it] = __builtin_nontemporal_load(gptr<V>(p + it * kStep));
        }
#pragma unroll
        for (int j = 0; j < KC; ++j) bw_accumulate<R, IT, VW>(acc, v[j], cells, K, j);
      } else {
        for (int j0 = 0; j0 < K; j0 += 4) {
          V v[4][IT];
          const int nj = min(4, K - j0);
#pragma unroll
          for (int jj = 0; jj < 4; ++jj) {
            if (jj < nj) {
              const uint64_t p = a.in[j0 + jj].base + s * a.in[j0 + jj].stride + off0;
#pragma unroll
              for (int it = 0; it < IT; ++it) v[jj][it] = __builtin_nontemporal_load(gptr<V>(p + it * kStep));
            }
          }
#pragma unroll
          for (int jj = 0; jj < 4; ++jj)
            if (jj < nj) bw_accumulate<R, IT, VW>(acc, v[jj], cells, K, j0 + jj);
        }
      }
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const uint64_t q = a.out[r].base + s * a.out[r].stride + off0;
#pragma unroll
        for (int it = 0; it < IT; ++it) __builtin_nontemporal_store(acc[it][r], gptr_w<V>(q + it * kStep));
      }
    } else {
      // ragged last tile: C is a multiple of 8, so a 16-byte lane unit may be half full
      for (int j = 0; j < K; ++j) {
        const uint64_t p = a.in[j].base + s * a.in[j].stride;
        V v[IT];
#pragma unroll
        for (int it = 0; it < IT; ++it) {
          const int64_t o = off0 + it * kStep;
          v[it] = 0u;
          if (o + kLane <= C) {
            v[it] = *gptr<V>(p + o);
          } else if (o < C) {
            const u32x2 h = *gptr<u32x2>(p + o);
            v[it][0] = h.x;
            v[it][1] = h.y;
          }
        }
        bw_accumulate<R, IT, VW>(acc, v, cells, K, j);
      }
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const uint64_t q = a.out[r].base + s * a.out[r].stride;
#pragma unroll
        for (int it = 0; it < IT; ++it) {
          const int64_t o = off0 + it * kStep;
          if (o + kLane <= C) {
            *gptr_w<V>(q + o) = acc[it][r];
          } else if (o < C) {
            u32x2 h;
            h.x = acc[it][r][0];
            h.y = acc[it][r][1];
            *gptr_w<u32x2>(q + o) = h;
          }
        }
      }
    }
  }
}

// ------------------------------------------------------------------ bitsliced
// A lane owns DW consecutive dwords of packet-column space in one super-packet and reads
// the same columns of all 8 packets of every input shard.
template <int R, int KC, int DW>
__global__ __launch_bounds__(kBlock) void k_gf8_bitsliced(ApplyArgs a) {
  typedef typename VecT<DW>::type V;
  const int K = KC ? KC : a.K;
  const uint32_t P = static_cast<uint32_t>(a.packet);
  const uint32_t col_bytes = static_cast<uint32_t>(a.size / 8);  // nsuper * P
  constexpr uint32_t kTile = kBlock * 4 * DW;
  const uint32_t tiles_per_stripe = (col_bytes + kTile - 1) / kTile;
  const uint32_t ntiles = tiles_per_stripe * static_cast<uint32_t>(a.nstripes);
  ConstCell *cells = const_cells(a.cells);

  for (uint32_t t = xcd_remap(blockIdx.x, gridDim.x); t < ntiles; t += gridDim.x) {
    const uint32_t s = t / tiles_per_stripe;
    const uint32_t colb = (t - s * tiles_per_stripe) * kTile + threadIdx.x * (4 * DW);
    if (colb >= col_bytes) continue;  // only in a ragged last tile (P % 16 == 0 keeps a lane's DW dwords inside one packet)
    const uint32_t sp = colb / P;
    const int64_t off = static_cast<int64_t>(sp) * 8 * P + (colb - sp * P);

    V acc[R][8];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int x = 0; x < 8; ++x) acc[r][x] = 0u;

    for (int j = 0; j < K; ++j) {
      const uint64_t p = a.in[j].base + s * a.in[j].stride + off;
      V e[8];
#pragma unroll
      for (int x = 0; x < 8; ++x) e[x] = __builtin_nontemporal_load(gptr<V>(p + x * P));
      uint32_t c[R];
#pragma unroll
      for (int r = 0; r < R; ++r) c[r] = cells[r * K + j].coef;
#pragma unroll
      for (int b = 0; b < 8; ++b) {
#pragma unroll
        for (int r = 0; r < R; ++r)
          if ((c[r] >> b) & 1u) {
#pragma unroll
            for (int x = 0; x < 8; ++x) acc[r][x] ^= e[x];
          }
        if (b < 7) {  // e <- 2*e in bit-sliced form
          const V top = e[7];
          e[7] = e[6];
          e[6] = e[5];
          e[5] = e[4];
          e[4] = e[3] ^ top;
          e[3] = e[2] ^ top;
          e[2] = e[1] ^ top;
          e[1] = e[0];
          e[0] = top;
        }
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint64_t q = a.out[r].base + s * a.out[r].stride + off;
#pragma unroll
      for (int x = 0; x < 8; ++x) __builtin_nontemporal_store(acc[r][x], gptr_w<V>(q + x * P));
    }
  }
}

// ------------------------------------------------------------------ generic bitmatrix
// Bitmatrix codes that are not GF(2^8)-linear per byte (liberation / blaum_roth / liber8tion,
// vendor/jerasure/src/liberation.c): packet l of output r = XOR of the input packets (j, x)
// whose bit B[r*w+l][j*w+x] is set (jerasure_bitmatrix_dotprod, jerasure.c:317-362).  A lane
// owns one dword column of a super-packet and applies the bitmatrix under wave-uniform
// branches (the row masks live in the constant address space).
typedef const __attribute__((address_space(4))) uint32_t ConstU32;

template <int R, int W>
__global__ __launch_bounds__(kBlock) void k_bitmatrix(ApplyArgs a) {
  const int K = a.K;
  const uint32_t P = static_cast<uint32_t>(a.packet);
  const uint32_t col_bytes = static_cast<uint32_t>(a.size / W);  // nsuper * P
  constexpr uint32_t kTile = kBlock * 4;
  const uint32_t tiles_per_stripe = (col_bytes + kTile - 1) / kTile;
  const uint32_t ntiles = tiles_per_stripe * static_cast<uint32_t>(a.nstripes);
  ConstU32 *masks = reinterpret_cast<ConstU32 *>(reinterpret_cast<uintptr_t>(a.masks));
  for (uint32_t t = xcd_remap(blockIdx.x, gridDim.x); t < ntiles; t += gridDim.x) {
    const uint32_t s = t / tiles_per_stripe;
    const uint32_t colb = (t - s * tiles_per_stripe) * kTile + threadIdx.x * 4;
    if (colb >= col_bytes) continue;
    const uint32_t sp = colb / P;
    const int64_t off = static_cast<int64_t>(sp) * W * P + (colb - sp * P);
    uint32_t acc[R][W];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int l = 0; l < W; ++l) acc[r][l] = 0u;
    for (int j = 0; j < K; ++j) {
      const uint64_t p = a.in[j].base + s * a.in[j].stride + off;
      uint32_t e[W];
#pragma unroll
      for (int x = 0; x < W; ++x) e[x] = __builtin_nontemporal_load(gptr<uint32_t>(p + x * P));
#pragma unroll
      for (int r = 0; r < R; ++r)
#pragma unroll
        for (int l = 0; l < W; ++l) {
          const uint32_t mask = masks[(r * W + l) * K + j];
          uint32_t v = 0;
#pragma unroll
          for (int x = 0; x < W; ++x)
            if ((mask >> x) & 1u) v ^= e[x];
          acc[r][l] ^= v;
        }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint64_t q = a.out[r].base + s * a.out[r].stride + off;
#pragma unroll
      for (int l = 0; l < W; ++l) __builtin_nontemporal_store(acc[r][l], gptr_w<uint32_t>(q + l * P));
    }
  }
}

// word sizes the liberation family can produce: primes (liberation), p-1 for prime p
// (blaum_roth), 8 (liber8tion)
#define LSEC_BITMATRIX_W(X) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(10) X(11) X(12) X(13) X(16) X(17) \
                            X(18) X(19) X(22) X(23) X(28) X(29) X(30) X(31)

// ------------------------------------------------------------------ per-R dispatch
template <int R, int IT, int MINW, int VW>
hipError_t bytewise_k(const ApplyArgs &a, hipStream_t st, int grid) {
  switch (a.K) {
#define LSEC_BW_K(KK) \
  case KK: hipLaunchKernelGGL((k_gf8_bytewise<R, KK, IT, MINW, VW>), dim3(grid), dim3(kBlock), 0, st, a); break;
    LSEC_BW_K(4) LSEC_BW_K(6) LSEC_BW_K(8) LSEC_BW_K(10) LSEC_BW_K(12) LSEC_BW_K(16) LSEC_BW_K(20)
#undef LSEC_BW_K
    default: hipLaunchKernelGGL((k_gf8_bytewise<R, 0, IT, MINW, VW>), dim3(grid), dim3(kBlock), 0, st, a); break;
  }
  return hipGetLastError();
}

// Bytewise launch shapes (tile per lane):  code -> (IT, VW)   [all MINW = 1]
//   0 -> (2, 4) 32 B/lane    1 -> (1, 4) 16 B/lane    2 -> (2, 2) 16 B/lane in 8 B pieces
//   3 -> (1, 2)  8 B/lane
constexpr int kBwShapes = 4;
inline int bw_shape_it(int shape) { return (shape == 0 || shape == 2) ? 2 : 1; }
inline int bw_shape_vw(int shape) { return shape <= 1 ? 4 : 2; }

template <int R>
hipError_t dispatch_bytewise(const ApplyArgs &a, hipStream_t st, int grid, int shape) {
  switch (shape) {
    case 1: return bytewise_k<R, 1, 1, 4>(a, st, grid);
    case 2: return bytewise_k<R, 2, 1, 2>(a, st, grid);
    case 3: return bytewise_k<R, 1, 1, 2>(a, st, grid);
    default: return bytewise_k<R, 2, 1, 4>(a, st, grid);
  }
}

template <int R>
hipError_t dispatch_bitsliced(const ApplyArgs &a, hipStream_t st, int grid, int dw) {
  switch (dw) {
    case 4: hipLaunchKernelGGL((k_gf8_bitsliced<R, 0, 4>), dim3(grid), dim3(kBlock), 0, st, a); break;
    case 2: hipLaunchKernelGGL((k_gf8_bitsliced<R, 0, 2>), dim3(grid), dim3(kBlock), 0, st, a); break;
    default: hipLaunchKernelGGL((k_gf8_bitsliced<R, 0, 1>), dim3(grid), dim3(kBlock), 0, st, a); break;
  }
  return hipGetLastError();
}

template <int R>
hipError_t dispatch_bitmatrix(const ApplyArgs &a, hipStream_t st, int grid) {
  if constexpr (R <= 2) {
    switch (a.w) {
#define LSEC_BM_W(WW) \
  case WW: hipLaunchKernelGGL((k_bitmatrix<R, WW>), dim3(grid), dim3(kBlock), 0, st, a); break;
      LSEC_BITMATRIX_W(LSEC_BM_W)
#undef LSEC_BM_W
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  } else {
    return hipErrorInvalidValue;
  }
}

#define LSEC_DECLARE_R(RR)                                                                         \
  extern template hipError_t dispatch_bytewise<RR>(const ApplyArgs &, hipStream_t, int, int);      \
  extern template hipError_t dispatch_bitsliced<RR>(const ApplyArgs &, hipStream_t, int, int);         \
  extern template hipError_t dispatch_bitmatrix<RR>(const ApplyArgs &, hipStream_t, int);
#ifndef LSEC_INSTANTIATING
LSEC_DECLARE_R(1) LSEC_DECLARE_R(2) LSEC_DECLARE_R(3) LSEC_DECLARE_R(4)
LSEC_DECLARE_R(5) LSEC_DECLARE_R(6) LSEC_DECLARE_R(7) LSEC_DECLARE_R(8)
#endif

}  // namespace lsec
