// ec_jit.h -- run-time compiled XOR networks for wide GF(2^8) matrix codes (ec_jit.cpp).
// Internal to liblstore_ec.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "ec_kernels.h"

namespace lsec {
namespace jit {

constexpr int kMaxRows = 8;   // output rows one network computes
constexpr int kMaxCols = 32;  // input columns (registers: 8 slices per input per lane)

// whether an R x K bytewise matrix is served by a network (wide codes only; LSEC_JIT=0: never)
bool wants_xornet(int R, int K);
// whether an R x K GF(2^w) matrix (w = 16 / 32, word layout) is served by a network
bool wants_gfw_net(int R, int K, int w);
// HIP source of the network for the row-major R x K matrix (exposed for tests and tools)
std::string xornet_source(const uint8_t *mat, int R, int K);
// HIP source of the bit-sliced network for an R x K GF(2^w) matrix, w = 16 / 32
std::string gfw_source(const uint32_t *mat, int R, int K, int w);
// bytes of a shard one block of an R-row w = 16 / 32 network covers per tile; it serves whole
// tiles only
int gfw_tile(int w, int R);
// whether the R-row network at w takes the wave-pair slice split (4 rows at w = 32; ec_jit.cpp)
bool gfw_rowsplit(int w, int R);
// bytes of a shard one 256-lane block of the network covers per tile
int xornet_tile(int K, int R);
// LSEC_JIT_VARIANT (code shape knobs for A/B runs; 0 = default)
int jit_variant();
// Associate a device coefficient image with its matrix and start compiling that matrix's
// network in the background (once per matrix per process).  unbind before the image is freed.
void bind(const void *image, const uint8_t *mat, int R, int K);
void bind_w(const void *image, const uint32_t *mat, int R, int K, int w);  // w = 16 / 32
void bind_entry(const void *image, const uint32_t *mat, int R, int K, int w);
void bind_key(const void *image, const std::vector<uint32_t> &key, const uint32_t *mat, size_t n, int R, int K, int w,
              int D, int S);
// whether an R-output bitmatrix code over K inputs at w is served by a packet network
bool wants_pktnet(int R, int K, int w);
// HIP source of the packet network for bitmatrix row masks [(r*w + l)*K + j] (w <= 32), D dwords
// per lane (exposed for tests and tools)
std::string pktnet_source(const uint32_t *masks, int R, int K, int w, int D, int S = 1);
// bind a bitmatrix image (ungrouped row masks, K <= 32) to its packet network; the lane width
// follows the packet size
void bind_pkt(const void *image, const uint32_t *masks, int R, int K, int w, int packet);
// the same for an R x K GF(2^w) coefficient matrix in Cauchy's packet layout (w = 8 / 16 / 32)
void bind_pkt_field(const void *image, const uint32_t *coef, int R, int K, int w, int packet);
// out[r] packets = the bitmatrix rows' XORs of the input packets, every stripe; the shard bases
// and strides must be aligned to the lane width (pkt_aligned)
hipError_t launch_pkt(hipFunction_t fn, int R, int K, const ShardRef *in, const ShardRef *out, int nstripes, int64_t size,
                      int packet, int w, hipStream_t st);
// lane width (dwords, 0: none) and output groups of the packet network for R outputs at w
void pkt_shape(int R, int w, int packet, int *D, int *S);
bool pkt_aligned(const ShardRef *in, int K, const ShardRef *out, int R, int w, int packet);
void unbind(const void *image);
// Block until the image's network is compiled (or failed, or timeout): 1 ready, 0 otherwise
// (also 0 when the image has no network).
int wait(const void *image, int timeout_ms);
// The compiled network for `image` on the current device, or nullptr (not bound / not ready).
hipFunction_t ready(const void *image, int R, int K);
// out[r] = sum_j A[r][j] in[j] for every stripe (same shard addressing as ApplyArgs); at
// w = 16 / 32 over the first size / gfw_tile(w, R) whole tiles of every shard only.
hipError_t launch(hipFunction_t fn, int R, int K, const ShardRef *in, const ShardRef *out, int nstripes, int64_t size,
                  hipStream_t st, int w = 8);

}  // namespace jit
}  // namespace lsec
