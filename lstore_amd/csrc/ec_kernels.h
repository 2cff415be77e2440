// ec_kernels.h -- launch interface of the gfx950 erasure kernels (internal to liblstore_ec).
//
// Both kernels compute the same thing -- R output shards as GF(2^8)-linear combinations
// of K input shards, out_r = sum_j A[r][j] * in_j -- for every stripe of a batch.  They
// differ in how a shard's bytes map onto field elements:
//
//   gf8_bytewise   each byte is one element (Reed-Solomon "matrix" codes:
//                  jerasure_matrix_encode/_decode, jerasure.c:301, :169)
//   gf8_bitsliced  each shard is a sequence of super-packets of 8 packets of P bytes;
//                  bit b of byte t of packet x is bit x of element (t, b) (Cauchy
//                  "bitmatrix/schedule" codes: jerasure_schedule_encode, jerasure.c:1193,
//                  jerasure_schedule_decode_lazy, :953)
//
// Shard addressing per stripe s:  in_j = in[j].base + s * in[j].stride  (same for out),
// so a batch can describe LStore's layout (k data chunks back to back in one cache page,
// m parity chunks in a parity buffer) or any other strided layout without a pointer table.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <tuple>
#include <utility>

namespace lsec {

// Launches kernel k and returns the launch's own status (hipLaunchKernel's return value).  The
// engine never reads the runtime's per-thread last error to learn about its launches: that error
// is sticky until read, so a read would both take a caller's pending error for the engine's and
// clear it from under the caller.
template <typename T, size_t... I>
hipError_t launch_packed(const void *k, dim3 grid, dim3 block, hipStream_t st, T &args, std::index_sequence<I...>) {
  void *ptrs[] = {static_cast<void *>(&std::get<I>(args))..., nullptr};
  return hipLaunchKernel(k, grid, block, ptrs, 0, st);
}
template <typename... KArgs, typename... Args>
hipError_t launch_kernel(void (*k)(KArgs...), dim3 grid, dim3 block, hipStream_t st, const Args &...args) {
  static_assert(sizeof...(KArgs) == sizeof...(Args), "argument count");
  std::tuple<std::decay_t<KArgs>...> t(static_cast<std::decay_t<KArgs>>(args)...);
  return launch_packed(reinterpret_cast<const void *>(k), grid, block, st, t, std::index_sequence_for<KArgs...>{});
}

// Occupancy cap of the streaming launches (launch_tiled's kernels and the compiled networks), as
// unused dynamic LDS per workgroup: with it at most n workgroups share a CU's 160 KiB.  0 (the
// default, or n = 0): no cap.  n from LSEC_WGS_CAP for launches whose shards are at least
// LSEC_WGS_CAP_MIN_KB apart (A/B runs of the C = 8 MiB encode dip).
size_t occupancy_lds_bytes(int64_t shard_bytes);
template <typename T, size_t... I>
hipError_t launch_packed_shm(const void *k, dim3 grid, dim3 block, size_t shm, hipStream_t st, T &args,
                             std::index_sequence<I...>) {
  void *ptrs[] = {static_cast<void *>(&std::get<I>(args))..., nullptr};
  return hipLaunchKernel(k, grid, block, ptrs, shm, st);
}
template <typename... KArgs, typename... Args>
hipError_t launch_kernel_shm(void (*k)(KArgs...), dim3 grid, dim3 block, size_t shm, hipStream_t st, const Args &...args) {
  static_assert(sizeof...(KArgs) == sizeof...(Args), "argument count");
  std::tuple<std::decay_t<KArgs>...> t(static_cast<std::decay_t<KArgs>>(args)...);
  return launch_packed_shm(reinterpret_cast<const void *>(k), grid, block, shm, st, t, std::index_sequence_for<KArgs...>{});
}

constexpr int kMaxK = 64;   // input shards per launch (wider stripes: several launches, the later ones with
                            // ApplyArgs::accumulate, over images in the grouped layout below)
constexpr int kMaxR = 16;   // output shards per launch
constexpr int kMaxW = 257;  // bitmatrix word size w (packets per super-packet) the kernels accept:
                             // every liberation-family plan with k + m <= 256 (liberation k = 252..254
                             // gets w = 257, erasure_tools.c:756-757)

// Matrix images of stripes wider than kMaxK inputs are stored in groups of kMaxK input columns:
// group g (inputs g*kMaxK ..) holds every row's cells / masks / products for its columns, rows in
// order, so one launch per group reads a plain row-major image of its K_g columns.
__host__ __device__ inline int image_groups(int K) { return (K + kMaxK - 1) / kMaxK; }
// 32-bit words per bitmatrix mask: bit x of mask word q covers packet 32q + x of an input
__host__ __device__ inline int mask_words(int w) { return (w + 31) / 32; }

struct ShardRef {
  uint64_t base;    // device address of this shard in stripe 0
  int64_t stride;   // bytes between consecutive stripes
};

// One coefficient cell of the device "matrix image": 8 dwords, 32-byte aligned so a
// wave fetches it with one scalar load.  For bytewise kernels the three 8-entry
// product tables implement  c*v = Ta[v & 7] ^ Tb[(v >> 3) & 7] ^ Tc[v >> 6]  with one
// v_perm_b32 each (v_perm selects bytes from an 8-byte table).
constexpr uint32_t kCellXorRow = 1;  // CoefCell::pad of a row's first cell: every coefficient of the row is 1

struct CoefCell {
  uint32_t coef;        // A[r][j] (0..255)
  uint32_t pad;         // flags (kCellXorRow in the first cell of a row)
  uint32_t ta_lo, ta_hi;  // c * {0..7}
  uint32_t tb_lo, tb_hi;  // c * {0,8,..,56}
  uint32_t tc_lo, tc_hi;  // c * {0,64,128,192}, upper 4 bytes unused
};
static_assert(sizeof(CoefCell) == 32, "CoefCell must be 32 bytes");

struct ApplyArgs {
  const CoefCell *cells;  // R x K, row-major (device memory)
  int K, R;
  int nstripes;
  int packet;             // bitsliced / bitmatrix: packet size P (bytes)
  int64_t size;           // bytes per shard (chunk C)
  const uint32_t *masks;  // bitmatrix: (R*w) x K x mask_words(w) words, bit x of [((r*w+l)*K + j)*NW + q]
                          //   = B[r*w+l][j*w + 32q + x]
                          // wordwise: R x K x w products, [(r*K + j)*w + b] = c_rj * x^b
  int w;                  // bitmatrix: packets per super-packet; wordwise: field width (16 / 32)
  int accumulate;         // 1: out[r] ^= the result (the second and later input groups of a wide stripe)
  unsigned long long *magic_acc;  // encode only (bytewise, bitsliced): fused stripe magic over the K inputs then the
                                  // R outputs (2 x u64 per stripe, zeroed), see MagicArgs
  unsigned *tiles;        // work-sharing tile queue slot (tile_queue_slot), or null: each XCD its static eighth
  uint32_t tiles_pre;     // with a slot: the tiles of each eighth dealt statically before the sharing starts
  unsigned long long *stamps;  // measurement only (lsec_test_set_stamps): each workgroup's end time, or null
  uint32_t nstamps;
  uint32_t tile_phase;    // XCD tile phase (tile_phase_on): XCD x starts its eighth x * tile_phase tiles on, 0 = off
  ShardRef in[kMaxK];
  ShardRef out[kMaxR];
};

// Work-sharing tiles.  The streaming kernels deal each XCD a contiguous eighth of the tiles
// (xcd_remap), but the XCDs do not run at one rate: on the headline's memory shape the odd ones
// take ~15 % longer per tile, every launch, so the even ones idle for the last 6-8 % of it
// (tools/probes/xcd_balance.hip, profiles/r05_v2_xcd_balance.jsonl).  With a queue slot the grid
// is persistent (the kernel's resident workgroups) and each workgroup takes tiles from its own
// XCD's eighth through an atomic counter, then from the other eighths once its own is done, so
// the XCDs finish within microseconds of each other.  A slot is kTileQueueWords counters on
// lines of their own: one per eighth, then a done counter; the launch's last workgroup zeroes
// them, and slots rotate over a ring per device; a slot is taken again only after an event
// recorded behind its last launch has completed.  LSEC_TILES=static turns it off (A/B).
constexpr int kTileQueueLine = 32;  // unsigned words per counter (a 128-B line each)
constexpr int kTileQueueWords = 9 * kTileQueueLine;
constexpr int kTileQueueRing = 4096;
// a slot on the device of stream st for a launch of ntiles tiles; null: tile sharing off, the
// launch small (fewer than kTileQueueMinTiles), or no slot available (the static eighths serve)
constexpr uint64_t kTileQueueMinTiles = 16384;
unsigned *tile_queue_slot(hipStream_t st, uint64_t ntiles);
// XCD tile phase: every XCD's eighth of the tiles starts 1/8 of a stripe later than the previous
// XCD's (wrapping around inside the eighth), so the eight XCDs stream from different column offsets
// of their stripes at any moment.  On for launch_tiled's kernels (tile_phase_on), off for the
// compiled networks (tile_phase_net_on); LSEC_TILE_PHASE = bit 0 | bit 1 << 1 overrides (default 1)
bool tile_phase_on();
bool tile_phase_net_on();
void set_tile_phase(int mode);  // (lsec_test_set_tile_phase: A/B runs in one process)
// after the launch that took `slot` is queued on st: records the slot's event and frees it for a
// later taker (who waits for that event first: a slot is never shared by two unfinished launches)
void tile_queue_release(hipStream_t st, unsigned *slot);
// with tile sharing on, the tiles of each eighth (of ntiles) dealt statically, one per block,
// before the sharing blocks take the rest (LSEC_TILES=shared: none; the default keeps 7/8)
uint32_t tiles_prefix(uint32_t ntiles);
// measurement hook: the buffer launch_tiled hands its kernels for per-workgroup end times
unsigned long long *launch_stamps(uint32_t *n);
void set_launch_stamps(unsigned long long *p, uint32_t n);
// the persistent grid of `kernel` on st's device (its resident workgroups of kBlock threads,
// times the CUs), at most `grid`; 0 when the runtime cannot say
int persistent_grid(const void *kernel, int grid, hipStream_t st);

// Per-stripe adler32 "magic" of LStore's erasure segment (je_cksum_calc,
// src/lio/segment/jerasure.c:169-182): zlib adler32 (RFC 1950) over the concatenation of all
// k+m chunks of a stripe, stored as 4 little-endian bytes.  Computed with position-weighted
// partial sums: over bytes b_i at positions i of a stream of length L,
//   A = 1 + sum b_i,  B = L + sum (L - i) b_i   (mod 65521)
// so any tile of any shard contributes independently (S = sum b, U = sum (i - p0) b via
// v_dot4_u32_u8), blocks add their reduced partials into 2 x u64 per stripe (acc), and a
// finalize kernel folds them into the magic.
constexpr int kMaxMagicShards = kMaxK + kMaxR;

struct MagicArgs {
  int nshards;            // shards of this launch, in checksum order (LStore: data 0..k-1, parity 0..m-1)
  int shard0;             // checksum index of sh[0] (wide stripes: one launch per kMaxMagicShards shards)
  int total_shards;       // shards per stripe (0: nshards)
  int nstripes;
  int64_t size;           // bytes of each shard covered by this launch
  int64_t col0;           // column offset of those bytes inside the chunk (column-block staging)
  int64_t chunk;          // full chunk size C (checksum positions are i*C + col0 + o)
  unsigned long long *acc;  // 2 per stripe: sum A, sum B (zeroed before the first launch)
  ShardRef sh[kMaxMagicShards];
};

hipError_t launch_stripe_magic(const MagicArgs &a, hipStream_t stream);
// magic[s*4 .. s*4+3] from acc (total_len = shards * C)
hipError_t launch_magic_finalize(const unsigned long long *acc, int nstripes, int64_t total_len, uint8_t *magic,
                                 hipStream_t stream);

// Chunk comparison for the control-chunk check of jerase_control_check (segment/jerasure.c:
// 202-269): flags[s] = 1 when any byte of a[p] and b[p] (p < npairs) differs in stripe s
// (flags zeroed by the caller).
struct DiffArgs {
  int npairs;
  int nstripes;
  int64_t size;
  int *flags;
  ShardRef a[kMaxR];
  ShardRef b[kMaxR];
};
hipError_t launch_chunk_diff(const DiffArgs &a, hipStream_t stream);

// Device-side gather of scattered byte ranges into one contiguous buffer (so a scattered
// device -> host transfer becomes one DMA): dst + dst_off[i] <- src[i], bytes[i] (multiples of
// 8, 8-byte aligned).  `list` is in device memory; one block per piece.
struct GatherPiece {
  uint64_t src;
  uint64_t dst_off;
  uint64_t bytes;
};
hipError_t launch_gather(const GatherPiece *list, int n, char *dst, hipStream_t stream);

// Host-memory transport by kernel: piece i copies bytes[i] (a multiple of 16, <= kPieceBytes)
// from src to dst, both 16-byte aligned, one block per piece.  Either side may be the device
// alias of page-locked host memory, so one launch moves many small host runs over PCIe
// without a DMA command per run.  `list` must be device-readable (page-locked host is).
constexpr uint32_t kPieceBytes = 16384;
struct CopyPiece {
  uint64_t src;
  uint64_t dst;
  uint64_t bytes;
};
hipError_t launch_copy_pieces(const CopyPiece *list, int n, hipStream_t stream);

// Completion signal of a zero-copy call: every block writes back its XCD's L2 at system scope
// (a call's kernel may have left dirty lines of page-locked host memory in any XCD's L2), the
// last block to arrive (agent-scope counter in device memory, reset by it) stores `value` to
// `flag` (page-locked host memory) with system-scope release.  Launched on the call's stream
// right after its coding kernel, so stream order puts every byte the call wrote before the flag.
hipError_t launch_signal(unsigned *counter, unsigned *flag, unsigned value, hipStream_t stream);

// HBM probe (measurement only): dst <- src, bytes a multiple of 16, both 16-byte aligned.
hipError_t launch_hbm_copy(void *dst, const void *src, uint64_t bytes, hipStream_t stream);
// HBM probe (measurement only): out[r] = XOR of the K inputs for every stripe (a.K, a.R <= kMaxR,
// a.in / a.out / a.nstripes / a.size): the encode's K-read : R-write traffic without its arithmetic.
hipError_t launch_hbm_mix(const ApplyArgs &a, hipStream_t stream);
// HBM probe (measurement only): out = XOR of the K inputs for every stripe, in a kernel that shares
// no code with the coding kernels (the decode's K-read : 1-write shape); variant = IT | G << 4 |
// REMAP << 8: IT 16-byte steps per lane, G tiles per block, XCD-contiguous grabs (ec_kernels.hip).
hipError_t launch_probe_xor(const ShardRef *in, int K, ShardRef out, int nstripes, int64_t size, int variant,
                            hipStream_t stream);

// Host helper: fill one cell for coefficient c.
void make_cell(uint8_t c, CoefCell &cell);

// Launchers (return hipError_t of the launch).  grid_blocks <= 0 picks a default.
hipError_t launch_bytewise(const ApplyArgs &a, hipStream_t stream, int grid_blocks = 0);
// encode + stripe magic in one pass (a.magic_acc != nullptr; checksum order = inputs, outputs)
hipError_t launch_bytewise_magic(const ApplyArgs &a, hipStream_t stream, int grid_blocks = 0);
// dw_pref: dwords per lane (1, 2, 4; 0 = 1) unless an A/B variant is set (lsec_set_kernel_variant)
hipError_t launch_bitsliced(const ApplyArgs &a, hipStream_t stream, int grid_blocks = 0, int dw_pref = 0);
// generic GF(2) bitmatrix codes (liberation / blaum_roth / liber8tion, liberation.c; Cauchy at
// w = 16 / 32): w in LSEC_BITMATRIX_W by a kernel per w, any other 2 <= w <= kMaxW by the
// LDS-staged kernel; R <= 2 per launch
hipError_t launch_bitmatrix(const ApplyArgs &a, hipStream_t stream, int grid_blocks = 0);
bool bitmatrix_w_supported(int w);
// matrix codes over GF(2^16) / GF(2^32) (a.w), little-endian words, R <= 8: bit-sliced after
// an in-register transpose (R <= 4 at w = 32), per-bit masks beyond that
hipError_t launch_wordwise(const ApplyArgs &a, hipStream_t stream, int grid_blocks = 0);
// Cauchy codes at w = 16 / 32 in the packet layout, bit-sliced over GF(2^w): the wordwise
// image supplies the coefficients; R <= 8 per launch at w = 16, <= 4 at w = 32
hipError_t launch_gfw_bitsliced(const ApplyArgs &a, hipStream_t stream, int grid_blocks = 0);
// host helper: the w products c * x^b (b = 0..w-1) of a wordwise cell, replicated for w = 16
void make_word_cell(uint32_t c, int w, uint32_t *out);

// Variant selection knobs for experiments: 0 = default
void set_kernel_variant(int bytewise_variant, int bitsliced_variant);
void set_tile_mode(int mode);  // lsec_set_tile_sharing: 0 static, 1 shared, 2 static prefix + shared tail
int tile_mode();
int bytewise_variant();  // != 0: a forced bytewise shape (also keeps wide codes off their XOR networks)
int bitsliced_variant();  // != 0: a forced bit-sliced / wordwise variant (also keeps w = 16 / 32 RS off its XOR network)

}  // namespace lsec
