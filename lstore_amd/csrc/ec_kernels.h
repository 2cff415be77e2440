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

namespace lsec {

constexpr int kMaxK = 32;   // data devices per stripe the kernels accept
constexpr int kMaxR = 16;   // output shards per launch

struct ShardRef {
  uint64_t base;    // device address of this shard in stripe 0
  int64_t stride;   // bytes between consecutive stripes
};

// One coefficient cell of the device "matrix image": 8 dwords, 32-byte aligned so a
// wave fetches it with one scalar load.  For bytewise kernels the three 8-entry
// product tables implement  c*v = Ta[v & 7] ^ Tb[(v >> 3) & 7] ^ Tc[v >> 6]  with one
// v_perm_b32 each (v_perm selects bytes from an 8-byte table).
struct CoefCell {
  uint32_t coef;        // A[r][j] (0..255)
  uint32_t pad;
  uint32_t ta_lo, ta_hi;  // c * {0..7}
  uint32_t tb_lo, tb_hi;  // c * {0,8,..,56}
  uint32_t tc_lo, tc_hi;  // c * {0,64,128,192}, upper 4 bytes unused
};
static_assert(sizeof(CoefCell) == 32, "CoefCell must be 32 bytes");

struct ApplyArgs {
  const CoefCell *cells;  // R x K, row-major (device memory)
  int K, R;
  int nstripes;
  int packet;             // bitsliced only: packet size P (bytes)
  int64_t size;           // bytes per shard (chunk C)
  ShardRef in[kMaxK];
  ShardRef out[kMaxR];
};

// Host helper: fill one cell for coefficient c.
void make_cell(uint8_t c, CoefCell &cell);

// Launchers (return hipError_t of the launch).  grid_blocks <= 0 picks a default.
hipError_t launch_bytewise(const ApplyArgs &a, hipStream_t stream, int grid_blocks = 0);
hipError_t launch_bitsliced(const ApplyArgs &a, hipStream_t stream, int grid_blocks = 0);

// Variant selection knobs for experiments: 0 = default
void set_kernel_variant(int bytewise_variant, int bitsliced_variant);

}  // namespace lsec
