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

// Output stores.  ACC XORs the result into what the output holds: the second and later input
// groups of a stripe wider than kMaxK inputs (ApplyArgs::accumulate), launched on separate
// ACC instantiations -- a run-time branch at the stores cost the hot kernels registers (RS
// 10+4: 155 -> 268 VGPRs, occupancy 3 -> 1, 0.77 -> 0.55 of 8 TB/s).
template <bool ACC, typename V>
__device__ __forceinline__ void put_nt(uint64_t q, V v) {
  if constexpr (ACC) v ^= *gptr<V>(q);
  __builtin_nontemporal_store(v, gptr_w<V>(q));
}
template <bool ACC, typename V>
__device__ __forceinline__ void put(uint64_t q, V v) {
  if constexpr (ACC) v ^= *gptr<V>(q);
  *gptr_w<V>(q) = v;
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

// Every tile t < ntiles to body(t) exactly once, body's t uniform over the workgroup.
//   q null: the grid strides over the tiles from its XCD-contiguous start (one tile per block
//   when the grid is the tile count): each XCD its static eighth.
//   q a tile queue slot (ec_kernels.h, "Work-sharing tiles"): each eighth's first `pre` tiles go
//   one per block to blocks 0 .. 8*pre-1 (block b on XCD b % 8, as the static form), and the
//   blocks after those share the rest: each takes G consecutive tiles at a time (a grab) from its
//   own XCD's remainder, then from the other eighths'.  pre = 0: all tiles are shared.  Thread 0
//   issues the atomic for the next grab as soon as it has the current one, so the counter's round
//   trip hides behind the grab's tiles; it posts the grab in one of two LDS words (never one a wave
//   has yet to read: that wave has not passed the barrier after its read), and readfirstlane keeps
//   the loop uniform.  One call site of body for every form: the kernels' code is not repeated.
//   phase > 0 (ApplyArgs::tile_phase): XCD / eighth x visits its tiles starting x * phase tiles in,
//   wrapping around inside its own range (a bijection; the static form only when the grid is the
//   tile count).
template <int G = 1, typename Body>
__device__ __forceinline__ void for_tiles(uint32_t ntiles, unsigned *q, uint32_t pre, Body &&body, uint32_t phase = 0) {
  __shared__ uint32_t next[2];
  const uint32_t per = (ntiles + 7) >> 3, xcd = blockIdx.x & 7;
  // the phase's map of a queue-form tile index: eighth e = t / per, rotated inside its own range
  const auto rot = [&](uint32_t t) -> uint32_t {
    const uint32_t e = t / per, base = e * per, size = min(per, ntiles - base);
    return base + ((t - base) + (e * phase) % size) % size;
  };
  const bool sharing = q != nullptr && blockIdx.x >= 8 * pre;  // block-uniform
  const uint32_t rest = per - pre, grabs = (rest + G - 1) / G;  // each eighth's shared tiles, grabs
  uint32_t k = 0, pend = 0, it = 0;  // thread 0: eighths done, the counter value in flight
  const auto take = [&]() -> uint32_t {  // thread 0: first tile of the grab `pend` names, or ntiles
    for (;;) {
      const uint32_t t = ((xcd + k) & 7) * per + pre + pend * G;
      if (pend < grabs && t < ntiles) return t;
      if (++k == 8) return ntiles;
      pend = atomicAdd(q + kTileQueueLine * ((xcd + k) & 7), 1u);
    }
  };
  uint32_t t, end, step = 1;
  if (q == nullptr) {
    t = xcd_remap(blockIdx.x, gridDim.x);
    if (phase && gridDim.x == ntiles) {  // one tile per block: rotate inside this XCD's contiguous run
      const uint32_t nb = gridDim.x, p8 = nb >> 3, rem = nb & 7;
      const uint32_t size = p8 + (xcd < rem ? 1u : 0u), start = xcd * p8 + min(xcd, rem);
      t = start + ((blockIdx.x >> 3) + (xcd * phase) % size) % size;
    }
    end = ntiles;
    step = gridDim.x;
  } else if (!sharing) {  // the static prefix: one tile
    t = xcd * per + (blockIdx.x >> 3);
    end = min(ntiles, t + 1);
  } else {
    t = end = 0;  // the first grab comes below
  }
  for (;;) {
    if (t >= end) {
      if (!sharing) break;
      if (threadIdx.x == 0) {
        if (it == 0) pend = atomicAdd(q + kTileQueueLine * xcd, 1u);
        next[it & 1] = take();
      }
      __syncthreads();
      t = __builtin_amdgcn_readfirstlane(next[it & 1]);
      ++it;
      if (t >= ntiles) break;
      end = min(min(ntiles, (t / per + 1) * per), t + G);  // a grab stays inside its eighth
      if (threadIdx.x == 0) pend = atomicAdd(q + kTileQueueLine * ((xcd + k) & 7), 1u);  // the next grab
    }
    body(q != nullptr && phase ? rot(t) : t);
    t += step;
  }
  // the launch's last sharing block leaves the slot zeroed for its next taker
  if (sharing && threadIdx.x == 0 && atomicAdd(q + kTileQueueLine * 8, 1u) == gridDim.x - 8 * pre - 1)
    for (int e = 0; e <= 8; ++e) atomicExch(q + kTileQueueLine * e, 0u);
}

// A tile-loop kernel over ApplyArgs, launched with a work-sharing tile queue slot and its
// persistent grid when tile sharing is on (ec_kernels.h), else on `grid` blocks over static eighths.
template <typename Kern>
hipError_t launch_tiled(Kern *k, int grid, hipStream_t st, ApplyArgs a) {
  a.stamps = launch_stamps(&a.nstamps);
  // `grid` is the tile count here: tiles per stripe = grid / nstripes
  a.tile_phase = tile_phase_on() && a.nstripes > 0 && grid % a.nstripes == 0 ? static_cast<uint32_t>(grid / a.nstripes / 8) : 0;
  unsigned *slot = tile_queue_slot(st, static_cast<uint64_t>(grid));
  a.tiles = nullptr;
  a.tiles_pre = 0;
  if (slot) {
    const int pg = persistent_grid(reinterpret_cast<const void *>(k), grid, st);
    if (pg > 0) {
      // `grid` is the tile count here (one tile per block in the static form)
      a.tiles = slot;
      a.tiles_pre = tiles_prefix(static_cast<uint32_t>(grid));
      grid = static_cast<int>(8 * a.tiles_pre) + pg;
    }
  }
  const hipError_t e = launch_kernel_shm(k, dim3(grid), dim3(kBlock), occupancy_lds_bytes(a.size), st, a);
  tile_queue_release(st, slot);
  return e;
}

// ------------------------------------------------------------------ adler32 partial sums
constexpr uint32_t kAdlerMod = 65521;

template <typename V>
__device__ __forceinline__ void adler_add(V v, uint64_t len_minus_pos, uint64_t &a_sum, uint64_t &b_sum) {
  // S = sum of the 16 bytes, U = sum t*b_t (t = 0..15) via packed byte dot products
  constexpr int N = sizeof(V) / 4;
  uint32_t S = 0, U = 0;
#pragma unroll
  for (int e = 0; e < N; ++e) {
    const uint32_t x = reinterpret_cast<const uint32_t *>(&v)[e];
    S = __builtin_amdgcn_udot4(x, 0x01010101u, S, false);
    U = __builtin_amdgcn_udot4(x, 0x03020100u + 0x04040404u * e, U, false);
  }
  a_sum += S;
  b_sum += len_minus_pos * S - U;   // sum_t (L - p - t) b_t, every term >= 0
}

__device__ __forceinline__ uint32_t block_sum(uint32_t v, uint32_t *lds) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  if ((threadIdx.x & 63) == 0) lds[threadIdx.x >> 6] = v;
  __syncthreads();
  uint32_t t = 0;
  if (threadIdx.x == 0)
    for (int w = 0; w < kBlock / 64; ++w) t += lds[w];
  __syncthreads();
  return t;
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

// Branch-free variant: every coefficient takes the 3-perm path (the tables of 0 and 1 give 0
// and the identity), so there are no per-cell branches (whose merges cost register copies
// and serialise the cell loads), and inputs are taken two at a time so three 3-input XORs
// fold six partial products.  The c*(v>>6) table has 4 entries: one dword, so that perm
// takes an inline 0 as its high half and needs no VGPR copy of the table.
template <int IT, int VW>
__device__ __forceinline__ void bw_fields(const typename VecT<VW>::type (&v)[IT], typename VecT<VW>::type (&fa)[IT],
                                          typename VecT<VW>::type (&fb)[IT], typename VecT<VW>::type (&fc)[IT]) {
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    fa[it] = v[it] & 0x07070707u;
    fb[it] = (v[it] >> 3) & 0x07070707u;
    fc[it] = (v[it] >> 6) & 0x03030303u;
  }
}

//
// X0: output row 0 is the plain XOR of the inputs (every coefficient 1 -- P0 of RS / Cauchy
// encodes, and decode rows that re-encode P0), flagged by the host in the row's first cell.
// That row then costs one 3-input XOR per input pair instead of 6 perms + 3 XORs, which
// is what the VALU-bound wide codes pay for it otherwise (RS 20+6: 20 of 120 cells).
template <int R, int IT, int VW, bool TWO, bool X0 = false>
__device__ __forceinline__ void bw_accumulate_bf(typename VecT<VW>::type (&acc)[IT][R],
                                                 const typename VecT<VW>::type (&va)[IT],
                                                 const typename VecT<VW>::type (&vb)[IT], ConstCell *cells, int K, int j) {
  typedef typename VecT<VW>::type V;
  V ia[IT], ib[IT], ic[IT], ja[IT], jb[IT], jc[IT];
  bw_fields<IT, VW>(va, ia, ib, ic);
  if constexpr (TWO) bw_fields<IT, VW>(vb, ja, jb, jc);
#pragma unroll
  for (int r = 0; r < R; ++r) {
    if constexpr (X0) {
      if (r == 0) {
#pragma unroll
        for (int it = 0; it < IT; ++it)
#pragma unroll
          for (int e = 0; e < VW; ++e) acc[it][0][e] = TWO ? xor3(acc[it][0][e], va[it][e], vb[it][e]) : acc[it][0][e] ^ va[it][e];
        continue;
      }
    }
    ConstCell *ca = cells + r * K + j;  // wave-uniform -> scalar loads
    const uint32_t a0 = ca->ta_lo, a1 = ca->ta_hi, a2 = ca->tb_lo, a3 = ca->tb_hi, a4 = ca->tc_lo;
    uint32_t b0 = 0, b1 = 0, b2 = 0, b3 = 0, b4 = 0;
    if constexpr (TWO) {
      ConstCell *cb = ca + 1;
      b0 = cb->ta_lo, b1 = cb->ta_hi, b2 = cb->tb_lo, b3 = cb->tb_hi, b4 = cb->tc_lo;
    }
#pragma unroll
    for (int it = 0; it < IT; ++it)
#pragma unroll
      for (int e = 0; e < VW; ++e) {
        uint32_t x = acc[it][r][e];
        const uint32_t p1 = __builtin_amdgcn_perm(a1, a0, ia[it][e]);
        const uint32_t p2 = __builtin_amdgcn_perm(a3, a2, ib[it][e]);
        const uint32_t p3 = __builtin_amdgcn_perm(0u, a4, ic[it][e]);
        if constexpr (TWO) {
          const uint32_t q1 = __builtin_amdgcn_perm(b1, b0, ja[it][e]);
          const uint32_t q2 = __builtin_amdgcn_perm(b3, b2, jb[it][e]);
          const uint32_t q3 = __builtin_amdgcn_perm(0u, b4, jc[it][e]);
          x = xor3(x, p1, p2);
          x = xor3(x, p3, q1);
          x = xor3(x, q2, q3);
        } else {
          x = xor3(x, p1, p2) ^ p3;
        }
        acc[it][r][e] = x;
      }
  }
}

// one input (BF = false: branchy per-cell path; true: branch-free)
template <int R, int IT, int VW, bool BF, bool X0>
__device__ __forceinline__ void bw_acc1(typename VecT<VW>::type (&acc)[IT][R], const typename VecT<VW>::type (&v)[IT],
                                       ConstCell *cells, int K, int j) {
  if constexpr (BF) bw_accumulate_bf<R, IT, VW, false, X0>(acc, v, v, cells, K, j);
  else bw_accumulate<R, IT, VW>(acc, v, cells, K, j);
}

__device__ __forceinline__ void magic_commit(unsigned long long *acc, uint32_t s, uint64_t as, uint64_t bs, uint32_t *red) {
  const uint32_t am = block_sum(static_cast<uint32_t>(as % kAdlerMod), red);
  const uint32_t bm = block_sum(static_cast<uint32_t>(bs % kAdlerMod), red);
  if (threadIdx.x == 0) {
    atomicAdd(acc + 2 * s, static_cast<unsigned long long>(am));
    atomicAdd(acc + 2 * s + 1, static_cast<unsigned long long>(bm));
  }
}

// Per-lane partial sums of the fused stripe magic.  A lane's byte at stripe position
//   p = sh*C + off + x*X + 4d + t
// (shard sh, the lane's first byte `off`, its x-th word group X bytes further on -- the
// iteration of the bytewise kernel, the packet of the bit-sliced one -- dword d, byte t)
// contributes (L - p)*b to adler32's B, so over the lane's bytes
//   sum (L - p) b = L*A - (C*JS + off*A + X*XS + W)
// with A = sum b, JS = sum sh*b, XS = sum x*b, W = sum (4d+t)*b: 32-bit v_dot4 chains,
// no 64-bit arithmetic until the lane's tile is done.
struct MagicLane {
  uint32_t a = 0, js = 0, xs = 0, w = 0;
};

__device__ __forceinline__ void ml_commit(const MagicLane &m, unsigned long long *acc, uint32_t s, int nsh, uint64_t C,
                                          uint64_t off, uint64_t X, uint32_t *red) {
  const uint64_t A = m.a;
  const uint64_t B = static_cast<uint64_t>(nsh) * C * A - (C * m.js + off * A + X * m.xs + m.w);
  magic_commit(acc, s, A, B, red);
}

// one shard's words of a lane: e[x] = VW dwords, x = 0..NX-1
template <int NX, int VW>
__device__ __forceinline__ void ml_add(MagicLane &m, const typename VecT<VW>::type (&e)[NX], uint32_t sh) {
  uint32_t sum = 0;
#pragma unroll
  for (int x = 0; x < NX; ++x)
#pragma unroll
    for (int d = 0; d < VW; ++d) {
      const uint32_t v = reinterpret_cast<const uint32_t *>(&e[x])[d];
      sum = __builtin_amdgcn_udot4(v, 0x01010101u, sum, false);
      if (NX > 1) m.xs = __builtin_amdgcn_udot4(v, 0x01010101u * x, m.xs, false);
      m.w = __builtin_amdgcn_udot4(v, 0x03020100u + 0x04040404u * d, m.w, false);
    }
  m.a += sum;
  m.js += sh * sum;
}

// fused stripe magic (bytewise kernel): lane words are the IT steps kStep bytes apart
template <int R, int IT, int VW>
__device__ __forceinline__ void bw_magic(MagicLane &ml, const typename VecT<VW>::type (*v)[IT], int nv, int j0) {
  for (int jj = 0; jj < nv; ++jj) ml_add<IT, VW>(ml, v[jj], static_cast<uint32_t>(j0 + jj));
}

template <int R, int IT, int VW>
__device__ __forceinline__ void bw_magic_out(MagicLane &ml, int K, const typename VecT<VW>::type (&acc)[IT][R]) {
  typedef typename VecT<VW>::type V;
#pragma unroll
  for (int r = 0; r < R; ++r) {
    V o[IT];
#pragma unroll
    for (int it = 0; it < IT; ++it) o[it] = acc[it][r];
    ml_add<IT, VW>(ml, o, static_cast<uint32_t>(K + r));
  }
}

// BF = branch-free coefficient path (bw_accumulate_bf).
// MG = also accumulate the stripe magic of inputs + outputs (encode + je_cksum_calc fused).
// X0 = row 0 is a plain XOR (see bw_accumulate_bf).
template <int R, int KC, int IT, bool BF, int VW, bool MG, bool X0, bool ACC>
__device__ __forceinline__ void bytewise_tiles(const ApplyArgs &a) {
  typedef typename VecT<VW>::type V;
  __shared__ uint32_t red[MG ? kBlock / 64 : 1];
  constexpr int kStep = BwTile<IT, VW>::kStep;
  constexpr int kTile = BwTile<IT, VW>::kBytes;
  constexpr int kLane = 4 * VW;
  const int K = KC ? KC : a.K;
  const int64_t C = a.size;
  const uint32_t tiles_per_stripe = static_cast<uint32_t>((C + kTile - 1) / kTile);
  const uint32_t ntiles = tiles_per_stripe * static_cast<uint32_t>(a.nstripes);
  ConstCell *cells = const_cells(a.cells);

  // grabs of about 8 KiB per shard (the single-erasure decode's 2 KiB tiles go 4 at a time)
  for_tiles<(kTile >= 8192 ? 1 : 8192 / kTile)>(ntiles, a.tiles, a.tiles_pre, [&](uint32_t t) {
    const uint32_t s = t / tiles_per_stripe;
    const int64_t off0 = static_cast<int64_t>(t - s * tiles_per_stripe) * kTile + threadIdx.x * kLane;
    const bool full = (static_cast<int64_t>(t - s * tiles_per_stripe) + 1) * kTile <= C;  // wave-uniform

    V acc[IT][R];
#pragma unroll
    for (int it = 0; it < IT; ++it)
#pragma unroll
      for (int r = 0; r < R; ++r) acc[it][r] = 0u;
    MagicLane ml;  // fused magic partial sums (MG only)

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
        if constexpr (BF) {
#pragma unroll
          for (int j = 0; j + 1 < KC; j += 2) bw_accumulate_bf<R, IT, VW, true, X0>(acc, v[j], v[j + 1], cells, K, j);
          if constexpr (KC % 2) bw_accumulate_bf<R, IT, VW, false, X0>(acc, v[KC - 1], v[KC - 1], cells, K, KC - 1);
        } else {
#pragma unroll
          for (int j = 0; j < KC; ++j) bw_accumulate<R, IT, VW>(acc, v[j], cells, K, j);
        }
        if constexpr (MG) bw_magic<R, IT, VW>(ml, v, KC, 0);
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
          if constexpr (BF) {
            if (nj >= 2) bw_accumulate_bf<R, IT, VW, true, X0>(acc, v[0], v[1], cells, K, j0);
            if (nj == 4) bw_accumulate_bf<R, IT, VW, true, X0>(acc, v[2], v[3], cells, K, j0 + 2);
            if (nj == 1 || nj == 3) bw_accumulate_bf<R, IT, VW, false, X0>(acc, v[nj - 1], v[nj - 1], cells, K, j0 + nj - 1);
          } else {
#pragma unroll
            for (int jj = 0; jj < 4; ++jj)
              if (jj < nj) bw_accumulate<R, IT, VW>(acc, v[jj], cells, K, j0 + jj);
          }
          if constexpr (MG) bw_magic<R, IT, VW>(ml, v, nj, j0);
        }
      }
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const uint64_t q = a.out[r].base + s * a.out[r].stride + off0;
#pragma unroll
        for (int it = 0; it < IT; ++it) put_nt<ACC, V>(q + it * kStep, acc[it][r]);
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
        bw_acc1<R, IT, VW, BF, X0>(acc, v, cells, K, j);
        if constexpr (MG) {
          const V(*vv)[IT] = &v;
          bw_magic<R, IT, VW>(ml, vv, 1, j);
        }
      }
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const uint64_t q = a.out[r].base + s * a.out[r].stride;
#pragma unroll
        for (int it = 0; it < IT; ++it) {
          const int64_t o = off0 + it * kStep;
          if (o + kLane <= C) {
            put<ACC, V>(q + o, acc[it][r]);
          } else if (o < C) {
            u32x2 h;
            h.x = acc[it][r][0];
            h.y = acc[it][r][1];
            put<ACC, u32x2>(q + o, h);
          }
        }
      }
    }
    if constexpr (MG) {
      bw_magic_out<R, IT, VW>(ml, K, acc);
      ml_commit(ml, a.magic_acc, s, K + R, static_cast<uint64_t>(a.size), static_cast<uint64_t>(off0), kStep, red);
    }
  }, a.tile_phase);
}

// The XOR-row flag (CoefCell::pad bit 0 of the launch's first cell) picks one of two whole
// instantiations once per wave: a uniform branch outside the tile loop, no merges inside it.
// Only codes with K*R >= 40 cells take the dual form: narrow codes are HBM-bound, and the
// second path would only raise the kernel's register allocation (RS 6+3: 56 -> 108 VGPRs).
template <int R, int KC, int IT, bool BF, int VW, bool MG = false, bool ACC = false>
__global__ __launch_bounds__(kBlock) void k_gf8_bytewise(ApplyArgs a) {
  if constexpr (BF && R >= 2 && (KC == 0 || KC * R >= 40)) {
    if (const_cells(a.cells)->pad & kCellXorRow) {
      bytewise_tiles<R, KC, IT, BF, VW, MG, true, ACC>(a);
      return;
    }
  }
  bytewise_tiles<R, KC, IT, BF, VW, MG, false, ACC>(a);
  if (a.stamps) {  // measurement only: when this workgroup finished (s_memrealtime, 100 MHz)
    __syncthreads();
    if (threadIdx.x == 0 && blockIdx.x < a.nstamps) a.stamps[blockIdx.x] = __builtin_amdgcn_s_memrealtime();
  }
}

// ------------------------------------------------------------------ bitsliced
// A lane owns DW consecutive dwords of packet-column space in one super-packet and reads
// the same columns of all 8 packets of every input shard.  MG: also the stripe magic of the
// inputs and outputs (encode + je_cksum_calc in one pass, as the bytewise kernel does).
template <int R, int KC, int DW, bool MG = false, bool ACC = false>
__global__ __launch_bounds__(kBlock) void k_gf8_bitsliced(ApplyArgs a) {
  typedef typename VecT<DW>::type V;
  __shared__ uint32_t red[MG ? kBlock / 64 : 1];
  const int K = KC ? KC : a.K;
  const uint32_t P = static_cast<uint32_t>(a.packet);
  const uint32_t col_bytes = static_cast<uint32_t>(a.size / 8);  // nsuper * P
  constexpr uint32_t kTile = kBlock * 4 * DW;
  const uint32_t tiles_per_stripe = (col_bytes + kTile - 1) / kTile;
  const uint32_t ntiles = tiles_per_stripe * static_cast<uint32_t>(a.nstripes);
  ConstCell *cells = const_cells(a.cells);

  for_tiles(ntiles, a.tiles, a.tiles_pre, [&](uint32_t t) {
    const uint32_t s = t / tiles_per_stripe;
    const uint32_t colb = (t - s * tiles_per_stripe) * kTile + threadIdx.x * (4 * DW);
    // lanes past the end occur only in a ragged last tile (P % 16 == 0 keeps a lane's DW
    // dwords inside one packet); with MG they still join the block's magic reduction
    const bool valid = colb < col_bytes;
    if (!MG && !valid) return;
    const uint32_t sp = colb / P;
    const int64_t off = static_cast<int64_t>(sp) * 8 * P + (colb - sp * P);
    MagicLane ml;

    V acc[R][8];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int x = 0; x < 8; ++x) acc[r][x] = 0u;

    for (int j = 0; j < K && valid; ++j) {
      const uint64_t p = a.in[j].base + s * a.in[j].stride + off;
      V e[8];
#pragma unroll
      for (int x = 0; x < 8; ++x) e[x] = __builtin_nontemporal_load(gptr<V>(p + x * P));
      if constexpr (MG) ml_add<8, DW>(ml, e, static_cast<uint32_t>(j));
      uint32_t c[R];
      uint32_t cm = 0;  // bits used by any output: no doublings past the highest one
#pragma unroll
      for (int r = 0; r < R; ++r) {
        c[r] = cells[r * K + j].coef;
        cm |= c[r];
      }
#pragma unroll
      for (int b = 0; b < 8; ++b) {
#pragma unroll
        for (int r = 0; r < R; ++r)
          if ((c[r] >> b) & 1u) {
#pragma unroll
            for (int x = 0; x < 8; ++x) acc[r][x] ^= e[x];
          }
        if ((cm >> (b + 1)) == 0) break;  // e.g. the XOR rows of a single-erasure decode
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
    if (valid) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const uint64_t q = a.out[r].base + s * a.out[r].stride + off;
#pragma unroll
        for (int x = 0; x < 8; ++x) put_nt<ACC, V>(q + x * P, acc[r][x]);
        if constexpr (MG) ml_add<8, DW>(ml, acc[r], static_cast<uint32_t>(K + r));
      }
    }
    if constexpr (MG) ml_commit(ml, a.magic_acc, s, K + R, static_cast<uint64_t>(a.size), static_cast<uint64_t>(off), P, red);
  }, a.tile_phase);
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
      for (int l = 0; l < W; ++l) put_nt<false, uint32_t>(q + l * P, acc[r][l]);
    }
  }
}

// ------------------------------------------------------------------ bitmatrix, any w
// Word sizes outside LSEC_BITMATRIX_W: a liberation plan with k > 31 gets the next prime w >= k
// (37, 41, ..; erasure_tools.c:756-757), blaum_roth w = p - 1.  Per-w register tiles do not
// scale there (acc[2][w] + e[w] registers), so a block stages its inputs in LDS instead.  A block
// owns 1 KiB of packet-column space (4 B per lane); for each input it stages the words of up to
// 64 packets of that column in LDS, and each of up to 64 output packets (registers) XORs the
// staged words its mask selects: a loop over the mask's set bits (wave-uniform scalar mask
// words), one LDS read per bit -- liberation rows have one or two bits per input block.  Output
// packets beyond 64 take another pass over the inputs (w <= 64: one pass).
template <int R>
__global__ __launch_bounds__(kBlock) void k_bitmatrix_any(ApplyArgs a) {
  constexpr int kChunk = 64;
  __shared__ uint32_t stage[kChunk][kBlock];  // 64 KiB
  const int K = a.K, W = a.w, NW = mask_words(a.w);
  const uint32_t P = static_cast<uint32_t>(a.packet);
  const uint32_t col_bytes = static_cast<uint32_t>(a.size / W);  // nsuper * P
  constexpr uint32_t kTile = kBlock * 4;
  const uint32_t tiles_per_stripe = (col_bytes + kTile - 1) / kTile;
  const uint32_t ntiles = tiles_per_stripe * static_cast<uint32_t>(a.nstripes);
  ConstU32 *masks = reinterpret_cast<ConstU32 *>(reinterpret_cast<uintptr_t>(a.masks));
  for (uint32_t t = xcd_remap(blockIdx.x, gridDim.x); t < ntiles; t += gridDim.x) {  // block-uniform
    const uint32_t s = t / tiles_per_stripe;
    const uint32_t colb = (t - s * tiles_per_stripe) * kTile + threadIdx.x * 4;
    const bool valid = colb < col_bytes;  // lanes past the end still join the barriers
    const uint32_t sp = valid ? colb / P : 0;
    const int64_t off = static_cast<int64_t>(sp) * W * P + (colb - sp * P);
    for (int l0 = 0; l0 < W; l0 += kChunk) {
      const int nl = min(kChunk, W - l0);
      uint32_t acc[R][kChunk];
#pragma unroll
      for (int r = 0; r < R; ++r)
#pragma unroll
        for (int l = 0; l < kChunk; ++l) acc[r][l] = 0u;
      for (int j = 0; j < K; ++j) {
        const uint64_t p = a.in[j].base + s * a.in[j].stride + off;
        for (int x0 = 0; x0 < W; x0 += kChunk) {
          const int nx = min(kChunk, W - x0);
          __syncthreads();  // the previous chunk's readers are done
          for (int x = 0; x < nx; ++x)
            stage[x][threadIdx.x] = valid ? __builtin_nontemporal_load(gptr<uint32_t>(p + static_cast<uint64_t>(x0 + x) * P)) : 0u;
          __syncthreads();
#pragma unroll
          for (int r = 0; r < R; ++r)
#pragma unroll
            for (int l = 0; l < kChunk; ++l) {
              if (l >= nl) continue;  // uniform; `continue` keeps the loop fully unrolled (acc in VGPRs)
              const uint32_t mi = static_cast<uint32_t>(((r * W + l0 + l) * K + j) * NW + (x0 >> 5));
              uint64_t m = masks[mi];
              if (nx > 32) m |= static_cast<uint64_t>(masks[mi + 1]) << 32;
              uint32_t v = 0;
              while (m) {
                v ^= stage[__builtin_ctzll(m)][threadIdx.x];
                m &= m - 1;
              }
              acc[r][l] ^= v;
            }
        }
      }
      if (valid) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const uint64_t q = a.out[r].base + s * a.out[r].stride + off;
#pragma unroll
          for (int l = 0; l < kChunk; ++l) {
            if (l >= nl) continue;
            if (a.accumulate) put_nt<true, uint32_t>(q + static_cast<uint64_t>(l0 + l) * P, acc[r][l]);
            else put_nt<false, uint32_t>(q + static_cast<uint64_t>(l0 + l) * P, acc[r][l]);
          }
        }
      }
    }
  }
}

// ------------------------------------------------------------------ wordwise GF(2^16) / GF(2^32)
// Reed-Solomon at w = 16 / 32 (jerasure_matrix_dotprod -> galois_w16/w32_region_multiply,
// galois.c:527-604, :730-810): element t of a shard is the little-endian uint16 / uint32 at
// byte 2t / 4t.  c*v = XOR_{b: v_b = 1} (c * x^b), so with the W products P_b = c*x^b of a
// cell in SGPRs (image [(r*K + j)*W + b], replicated into both halves of the dword for
// W = 16), each input dword yields W bit masks (bit b of each element smeared over the
// element: v_pk_lshlrev_b16 + v_pk_ashrrev_i16 for two uint16 elements, v_bfe_i32 for one
// uint32) shared by all R outputs, and each (output, input, bit) costs one v_bitop3_b32
// (acc ^ (mask & P_b), truth table 0x78).  VALU-bound by design at W ops per dword per
// (output, input) pair; these word sizes are off the headline configs.
typedef short s16x2 __attribute__((ext_vector_type(2)));

template <int W>
__device__ __forceinline__ uint32_t bit_smear(uint32_t x, int b) {
  if constexpr (W == 32) {
    return static_cast<uint32_t>(static_cast<int32_t>(x << (31 - b)) >> 31);
  } else {
    const s16x2 v = __builtin_bit_cast(s16x2, x);
    const s16x2 m = (v << static_cast<short>(15 - b)) >> static_cast<short>(15);
    return __builtin_bit_cast(uint32_t, m);
  }
}

template <int R, int W, bool ACC = false>
__global__ __launch_bounds__(kBlock) void k_gfw_wordwise(ApplyArgs a) {
  constexpr int VW = W == 16 ? 4 : 2;
  typedef typename VecT<VW>::type V;
  constexpr int kLane = 4 * VW;
  constexpr int kTile = kBlock * kLane;
  constexpr uint32_t kOne = W == 16 ? 0x00010001u : 1u;
  const int K = a.K;
  const int64_t C = a.size;
  const uint32_t tiles_per_stripe = static_cast<uint32_t>((C + kTile - 1) / kTile);
  const uint32_t ntiles = tiles_per_stripe * static_cast<uint32_t>(a.nstripes);
  ConstU32 *prod = reinterpret_cast<ConstU32 *>(reinterpret_cast<uintptr_t>(a.masks));
  for (uint32_t t = xcd_remap(blockIdx.x, gridDim.x); t < ntiles; t += gridDim.x) {
    const uint32_t s = t / tiles_per_stripe;
    const int64_t off = static_cast<int64_t>(t - s * tiles_per_stripe) * kTile + threadIdx.x * kLane;
    if (off >= C) continue;
    const bool whole = off + kLane <= C;  // C % 8 == 0: otherwise exactly 8 bytes remain
    V acc[R];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = 0u;
    for (int j = 0; j < K; ++j) {
      const uint64_t p = a.in[j].base + s * a.in[j].stride + off;
      V v = 0u;
      if (whole) {
        v = __builtin_nontemporal_load(gptr<V>(p));
      } else {
        const u32x2 h = *gptr<u32x2>(p);
        v[0] = h.x;
        v[1] = h.y;
      }
      V mk[W];
#pragma unroll
      for (int b = 0; b < W; ++b)
#pragma unroll
        for (int e = 0; e < VW; ++e) mk[b][e] = bit_smear<W>(v[e], b);
#pragma unroll
      for (int r = 0; r < R; ++r) {
        ConstU32 *pc = prod + (r * K + j) * W;  // wave-uniform -> scalar loads
        const uint32_t c0 = pc[0];
        if (c0 == 0) continue;
        if (c0 == kOne) {
          acc[r] ^= v;
          continue;
        }
#pragma unroll
        for (int b = 0; b < W; ++b) {
          const uint32_t pb = pc[b];
#pragma unroll
          for (int e = 0; e < VW; ++e) acc[r][e] = __builtin_amdgcn_bitop3_b32(acc[r][e], mk[b][e], pb, 0x78);
        }
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint64_t q = a.out[r].base + s * a.out[r].stride + off;
      if (whole) {
        put_nt<ACC, V>(q, acc[r]);
      } else {
        u32x2 h;
        h.x = acc[r][0];
        h.y = acc[r][1];
        put<ACC, u32x2>(q, h);
      }
    }
  }
}

// ------------------------------------------------------------------ bit-sliced GF(2^16) / GF(2^32)
// Cauchy codes at w = 16 / 32 in Jerasure's packet layout: a super-packet is W packets of P
// bytes, and bit x of element (t, b) is bit b of byte t of packet x, so a 32-bit word of each
// of the W packets holds bit x of 32 elements -- the w = 8 bit-sliced scheme with W slices.
// Multiplying all 32 elements by x renames the slices and XORs the top slice into the
// polynomial's taps (Jerasure's fields, galois.c:65-98: x^16 = x^12+x^3+x+1, x^32 =
// x^22+x^2+x+1), and c*e = sum_{t: c_t = 1} x^t e.  Identical bytes to the bitmatrix of the
// GF(2^W) coefficient matrix (what jerasure_bitmatrix_encode applies), in W XORs per set
// coefficient bit instead of one per set bitmatrix bit, under R*W uniform branches per input
// instead of R*W*W.  Coefficients come from the wordwise image (product b = 0 of a cell).
template <int W>
__device__ __forceinline__ void times_x_sliced(uint32_t (&e)[W]) {
  const uint32_t top = e[W - 1];
#pragma unroll
  for (int i = W - 1; i > 0; --i) e[i] = e[i - 1];
  e[0] = top;
  if constexpr (W == 16) {
    e[1] ^= top;
    e[3] ^= top;
    e[12] ^= top;
  } else {
    e[1] ^= top;
    e[2] ^= top;
    e[22] ^= top;
  }
}

template <int R, int W, bool ACC = false>
__global__ __launch_bounds__(kBlock) void k_gfw_bitsliced(ApplyArgs a) {
  const int K = a.K;
  const uint32_t P = static_cast<uint32_t>(a.packet);
  const uint32_t col_bytes = static_cast<uint32_t>(a.size / W);  // nsuper * P
  constexpr uint32_t kTile = kBlock * 4;
  constexpr uint32_t kCoefMask = W == 16 ? 0xFFFFu : 0xFFFFFFFFu;
  const uint32_t tiles_per_stripe = (col_bytes + kTile - 1) / kTile;
  const uint32_t ntiles = tiles_per_stripe * static_cast<uint32_t>(a.nstripes);
  ConstU32 *prod = reinterpret_cast<ConstU32 *>(reinterpret_cast<uintptr_t>(a.masks));
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
      uint32_t c[R], cm = 0;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        c[r] = prod[(r * K + j) * W] & kCoefMask;  // wave-uniform -> scalar loads
        cm |= c[r];
      }
#pragma unroll
      for (int b = 0; b < W; ++b) {
#pragma unroll
        for (int r = 0; r < R; ++r)
          if ((c[r] >> b) & 1u) {
#pragma unroll
            for (int x = 0; x < W; ++x) acc[r][x] ^= e[x];
          }
        if (b == W - 1 || (cm >> (b + 1)) == 0) break;
        times_x_sliced<W>(e);
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint64_t q = a.out[r].base + s * a.out[r].stride + off;
#pragma unroll
      for (int l = 0; l < W; ++l) put_nt<ACC, uint32_t>(q + l * P, acc[r][l]);
    }
  }
}

// ------------------------------------------------------------------ transposed GF(2^16) / GF(2^32)
// RS / r6 at w = 16 / 32 keep Jerasure's word layout (element t = little-endian uint16/uint32
// at byte 2t / 4t, galois.c:527-604, :730-810).  Each lane loads W dwords of a shard (32
// elements: W/4 coalesced 16 B pieces), transposes the W x W bit blocks in registers so that
// word x holds bit x of all 32 elements, runs k_gfw_bitsliced's arithmetic (one XOR per slice
// per set coefficient bit), and transposes back.  A W x W transpose is log2(W) swap stages:
// byte and halfword stages are two v_perm_b32 per pair of words, bit stages two shifts and two
// v_bfi_b32.  Elements never mix, so a zero-filled tail produces zeros that are not stored.
template <int W, int d>
__device__ __forceinline__ void transpose_bits(uint32_t (&D)[W], uint32_t m) {
#pragma unroll
  for (int r = 0; r < W; ++r) {
    if (r & d) continue;
    const uint32_t x = D[r], y = D[r + d];
    D[r] = (x & m) | ((y << d) & ~m);
    D[r + d] = ((x >> d) & m) | (y & ~m);
  }
}

template <int W>
__device__ __forceinline__ void transpose_units(uint32_t (&D)[W]) {
  if constexpr (W == 32) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const uint32_t x = D[r], y = D[r + 16];
      D[r] = __builtin_amdgcn_perm(y, x, 0x05040100u);       // (x.lo, y.lo)
      D[r + 16] = __builtin_amdgcn_perm(y, x, 0x07060302u);  // (x.hi, y.hi)
    }
  }
#pragma unroll
  for (int r = 0; r < W; ++r) {
    if (r & 8) continue;
    const uint32_t x = D[r], y = D[r + 8];
    D[r] = __builtin_amdgcn_perm(y, x, 0x06020400u);      // (x.b0, y.b0, x.b2, y.b2)
    D[r + 8] = __builtin_amdgcn_perm(y, x, 0x07030501u);  // (x.b1, y.b1, x.b3, y.b3)
  }
  transpose_bits<W, 4>(D, 0x0F0F0F0Fu);
  transpose_bits<W, 2>(D, 0x33333333u);
  transpose_bits<W, 1>(D, 0x55555555u);
}

template <int R, int W, bool xor_only, bool ACC>
__device__ __forceinline__ void gfw_transposed_tiles(const ApplyArgs &a) {
  constexpr int kPieces = W / 4;  // 16 B pieces per lane per shard
  constexpr uint32_t kTile = kBlock * 4 * W;
  constexpr uint32_t kCoefMask = W == 16 ? 0xFFFFu : 0xFFFFFFFFu;
  const int K = a.K;
  const int64_t C = a.size;
  const uint32_t tiles_per_stripe = static_cast<uint32_t>((C + kTile - 1) / kTile);
  const uint32_t ntiles = tiles_per_stripe * static_cast<uint32_t>(a.nstripes);
  ConstU32 *prod = reinterpret_cast<ConstU32 *>(reinterpret_cast<uintptr_t>(a.masks));
  for (uint32_t t = xcd_remap(blockIdx.x, gridDim.x); t < ntiles; t += gridDim.x) {
    const uint32_t s = t / tiles_per_stripe;
    const int64_t base = static_cast<int64_t>(t - s * tiles_per_stripe) * kTile + threadIdx.x * 16;
    if (base >= C) continue;
    // whole tile in range: every piece is a full 16 B; otherwise per piece (C % 8 == 0)
    const bool whole = static_cast<int64_t>(t - s * tiles_per_stripe) * kTile + kTile <= C;
    uint32_t acc[R][W];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
      for (int l = 0; l < W; ++l) acc[r][l] = 0u;
    for (int j = 0; j < K; ++j) {
      const uint64_t p = a.in[j].base + s * a.in[j].stride;
      uint32_t e[W];
#pragma unroll
      for (int q = 0; q < kPieces; ++q) {
        const int64_t o = base + static_cast<int64_t>(q) * kBlock * 16;
        u32x4 v = {0u, 0u, 0u, 0u};
        if (whole || o + 16 <= C) {
          v = __builtin_nontemporal_load(gptr<u32x4>(p + o));
        } else if (o + 8 <= C) {
          const u32x2 h = *gptr<u32x2>(p + o);
          v.x = h.x;
          v.y = h.y;
        }
        e[4 * q] = v.x;
        e[4 * q + 1] = v.y;
        e[4 * q + 2] = v.z;
        e[4 * q + 3] = v.w;
      }
      uint32_t c[R], cm = 0;
#pragma unroll
      for (int r = 0; r < R; ++r) {
        c[r] = prod[(r * K + j) * W] & kCoefMask;  // wave-uniform -> scalar loads
        cm |= c[r];
      }
      if (cm == 0) continue;
      if constexpr (xor_only) {  // coefficients 0 / 1: plain XOR, no transposes
#pragma unroll
        for (int r = 0; r < R; ++r)
          if (c[r])
#pragma unroll
            for (int x = 0; x < W; ++x) acc[r][x] ^= e[x];
        continue;
      }
      transpose_units<W>(e);
#pragma unroll
      for (int b = 0; b < W; ++b) {
#pragma unroll
        for (int r = 0; r < R; ++r)
          if ((c[r] >> b) & 1u) {
#pragma unroll
            for (int x = 0; x < W; ++x) acc[r][x] ^= e[x];
          }
        if (b == W - 1 || (cm >> (b + 1)) == 0) break;
        times_x_sliced<W>(e);
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if constexpr (!xor_only) transpose_units<W>(acc[r]);
      const uint64_t q0 = a.out[r].base + s * a.out[r].stride;
#pragma unroll
      for (int q = 0; q < kPieces; ++q) {
        const int64_t o = base + static_cast<int64_t>(q) * kBlock * 16;
        const u32x4 v = {acc[r][4 * q], acc[r][4 * q + 1], acc[r][4 * q + 2], acc[r][4 * q + 3]};
        if (whole || o + 16 <= C) {
          put_nt<ACC, u32x4>(q0 + o, v);
        } else if (o + 8 <= C) {
          u32x2 h;
          h.x = v.x;
          h.y = v.y;
          put<ACC, u32x2>(q0 + o, h);
        }
      }
    }
  }
}

// One kernel, two whole tile loops chosen by a uniform branch: a launch whose coefficients are
// all 0 / 1 (XOR-of-survivors decodes) is plain XOR and skips the bit slicing.
template <int R, int W, bool ACC = false>
__global__ __launch_bounds__(kBlock) void k_gfw_transposed(ApplyArgs a) {
  constexpr uint32_t kCoefMask = W == 16 ? 0xFFFFu : 0xFFFFFFFFu;
  ConstU32 *prod = reinterpret_cast<ConstU32 *>(reinterpret_cast<uintptr_t>(a.masks));
  bool xor_only = true;
  for (int i = 0; i < R * a.K && xor_only; ++i) xor_only = (prod[i * W] & kCoefMask) <= 1u;
  if (xor_only)
    gfw_transposed_tiles<R, W, true, ACC>(a);
  else
    gfw_transposed_tiles<R, W, false, ACC>(a);
}

// word sizes the liberation family can produce: primes (liberation), p-1 for prime p
// (blaum_roth), 8 (liber8tion); 16 and 32 for Cauchy at those word sizes
#define LSEC_BITMATRIX_W(X) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(10) X(11) X(12) X(13) X(16) X(17) \
                            X(18) X(19) X(22) X(23) X(28) X(29) X(30) X(31) X(32)

// ------------------------------------------------------------------ per-R dispatch
template <int R, int IT, bool BF, int VW>
hipError_t bytewise_k(const ApplyArgs &a, hipStream_t st, int grid) {
  switch (a.K) {
#define LSEC_BW_K(KK) \
  case KK: return launch_tiled(&k_gf8_bytewise<R, KK, IT, BF, VW>, grid, st, a);
    LSEC_BW_K(4) LSEC_BW_K(6) LSEC_BW_K(8) LSEC_BW_K(10) LSEC_BW_K(12) LSEC_BW_K(16) LSEC_BW_K(20)
#undef LSEC_BW_K
    default: return launch_tiled(&k_gf8_bytewise<R, 0, IT, BF, VW>, grid, st, a);
  }
}

// Bytewise launch shapes (tile per lane):  code -> (IT, VW, coefficient path)
//   0 -> (2, 4) 32 B/lane, branch-free   1 -> (1, 4) 16 B/lane, branch-free
//   2 -> (2, 2) 16 B/lane in 8 B pieces, branch-free   3 -> (1, 2) 8 B/lane, branch-free
//   4 -> (1, 2) 8 B/lane, per-cell branches (single-output decodes: mostly XORs of
//        coefficient-1 inputs, which the branch turns into one v_xor instead of 3 perms)
constexpr int kBwShapes = 5;
inline int bw_shape_it(int shape) { return (shape == 0 || shape == 2) ? 2 : 1; }
inline int bw_shape_vw(int shape) { return shape <= 1 ? 4 : 2; }

template <int R>
hipError_t dispatch_bytewise(const ApplyArgs &a, hipStream_t st, int grid, int shape) {
  if (a.accumulate) {  // a later input group of a wide stripe: generic K, 16 B per lane (shape 1)
    return launch_tiled(&k_gf8_bytewise<R, 0, 1, true, 4, false, true>, grid, st, a);
  }
  switch (shape) {
    case 1: return bytewise_k<R, 1, true, 4>(a, st, grid);
    case 2: return bytewise_k<R, 2, true, 2>(a, st, grid);
    case 3: return bytewise_k<R, 1, true, 2>(a, st, grid);
    case 4: return bytewise_k<R, 1, false, 2>(a, st, grid);
    default: return bytewise_k<R, 2, true, 4>(a, st, grid);
  }
}

// encode + magic: 2 x 16 B per lane, 16 B for K >= 16 (as bytewise_shape; keep in step with
// bytewise_magic_it in ec_kernels.hip)
template <int R>
hipError_t dispatch_bytewise_magic(const ApplyArgs &a, hipStream_t st, int grid) {
  switch (a.K) {
#define LSEC_BWM_K(KK, IT) \
  case KK: return launch_tiled(&k_gf8_bytewise<R, KK, IT, true, 4, true>, grid, st, a);
    LSEC_BWM_K(4, 2) LSEC_BWM_K(6, 2) LSEC_BWM_K(8, 2) LSEC_BWM_K(10, 2) LSEC_BWM_K(12, 2) LSEC_BWM_K(16, 1) LSEC_BWM_K(20, 1)
#undef LSEC_BWM_K
    default:
      if (a.K >= 16) return launch_tiled(&k_gf8_bytewise<R, 0, 1, true, 4, true>, grid, st, a);
      else return launch_tiled(&k_gf8_bytewise<R, 0, 2, true, 4, true>, grid, st, a);
      break;
  }
}

template <int R>
hipError_t dispatch_bitsliced(const ApplyArgs &a, hipStream_t st, int grid, int dw) {
  if (a.magic_acc) {  // encode + stripe magic, one lane dword wide
    return launch_tiled(&k_gf8_bitsliced<R, 0, 1, true>, grid, st, a);
  }
  if (a.accumulate) {  // a later input group of a wide stripe, one lane dword wide
    return launch_tiled(&k_gf8_bitsliced<R, 0, 1, false, true>, grid, st, a);
  }
  switch (dw) {
    case 4: return launch_tiled(&k_gf8_bitsliced<R, 0, 4>, grid, st, a);
    case 2: return launch_tiled(&k_gf8_bitsliced<R, 0, 2>, grid, st, a);
    default: return launch_tiled(&k_gf8_bitsliced<R, 0, 1>, grid, st, a);
  }
}

template <int R>
hipError_t dispatch_bitmatrix(const ApplyArgs &a, hipStream_t st, int grid) {
  if constexpr (R <= 2) {
    if (a.accumulate) {  // wide stripes (k > 64) only occur at w > 64: the any-w kernel
      return launch_kernel(&k_bitmatrix_any<R>, dim3(grid), dim3(kBlock), st, a);
    }
    switch (a.w) {
#define LSEC_BM_W(WW) \
  case WW: return launch_kernel(&k_bitmatrix<R, WW>, dim3(grid), dim3(kBlock), st, a);
      LSEC_BITMATRIX_W(LSEC_BM_W)
#undef LSEC_BM_W
      default: return launch_kernel(&k_bitmatrix_any<R>, dim3(grid), dim3(kBlock), st, a);
    }
  } else {
    return hipErrorInvalidValue;
  }
}

template <int R>
hipError_t dispatch_wordwise(const ApplyArgs &a, hipStream_t st, int grid) {
  switch (a.w * 2 + (a.accumulate ? 1 : 0)) {
    case 32: return launch_kernel(&k_gfw_wordwise<R, 16>, dim3(grid), dim3(kBlock), st, a);
    case 33: return launch_kernel(&k_gfw_wordwise<R, 16, true>, dim3(grid), dim3(kBlock), st, a);
    case 64: return launch_kernel(&k_gfw_wordwise<R, 32>, dim3(grid), dim3(kBlock), st, a);
    case 65: return launch_kernel(&k_gfw_wordwise<R, 32, true>, dim3(grid), dim3(kBlock), st, a);
    default: return hipErrorInvalidValue;
  }
}

// at most 8 rows per launch at w = 16, 4 at w = 32 (acc[R][W] lives in VGPRs)
template <int R>
hipError_t dispatch_gfw_transposed(const ApplyArgs &a, hipStream_t st, int grid) {
  if (a.w == 16) {
    if (a.accumulate) return launch_kernel(&k_gfw_transposed<R, 16, true>, dim3(grid), dim3(kBlock), st, a);
    else return launch_kernel(&k_gfw_transposed<R, 16>, dim3(grid), dim3(kBlock), st, a);
  } else if constexpr (R <= 4) {
    if (a.w != 32) return hipErrorInvalidValue;
    if (a.accumulate) return launch_kernel(&k_gfw_transposed<R, 32, true>, dim3(grid), dim3(kBlock), st, a);
    else return launch_kernel(&k_gfw_transposed<R, 32>, dim3(grid), dim3(kBlock), st, a);
  } else {
    return hipErrorInvalidValue;
  }
}

template <int R>
hipError_t dispatch_gfw_bitsliced(const ApplyArgs &a, hipStream_t st, int grid) {
  if (a.w == 16) {
    if (a.accumulate) return launch_kernel(&k_gfw_bitsliced<R, 16, true>, dim3(grid), dim3(kBlock), st, a);
    else return launch_kernel(&k_gfw_bitsliced<R, 16>, dim3(grid), dim3(kBlock), st, a);
  } else if constexpr (R <= 4) {
    if (a.w != 32) return hipErrorInvalidValue;
    if (a.accumulate) return launch_kernel(&k_gfw_bitsliced<R, 32, true>, dim3(grid), dim3(kBlock), st, a);
    else return launch_kernel(&k_gfw_bitsliced<R, 32>, dim3(grid), dim3(kBlock), st, a);
  } else {
    return hipErrorInvalidValue;
  }
}

#define LSEC_DECLARE_R(RR)                                                                         \
  extern template hipError_t dispatch_bytewise<RR>(const ApplyArgs &, hipStream_t, int, int);      \
  extern template hipError_t dispatch_bitsliced<RR>(const ApplyArgs &, hipStream_t, int, int);         \
  extern template hipError_t dispatch_bitmatrix<RR>(const ApplyArgs &, hipStream_t, int);           \
  extern template hipError_t dispatch_bytewise_magic<RR>(const ApplyArgs &, hipStream_t, int);          \
  extern template hipError_t dispatch_wordwise<RR>(const ApplyArgs &, hipStream_t, int);         \
  extern template hipError_t dispatch_gfw_bitsliced<RR>(const ApplyArgs &, hipStream_t, int);      \
  extern template hipError_t dispatch_gfw_transposed<RR>(const ApplyArgs &, hipStream_t, int);
#ifndef LSEC_INSTANTIATING
LSEC_DECLARE_R(1) LSEC_DECLARE_R(2) LSEC_DECLARE_R(3) LSEC_DECLARE_R(4)
LSEC_DECLARE_R(5) LSEC_DECLARE_R(6) LSEC_DECLARE_R(7) LSEC_DECLARE_R(8)
#endif

}  // namespace lsec
