// ec_kernels.hip -- host-side launch policy for the gfx950 erasure kernels
// (device code: ec_kernels_impl.h, instantiated per R in ec_kernels_inst.hip).
#include <cstdlib>
#include <type_traits>

#include "ec_kernels_impl.h"

namespace lsec {

namespace {

int g_bw_variant = 0, g_bs_variant = 0;

int default_grid(uint64_t ntiles) {
  // One tile per block: on this streaming pattern a full grid beat every grid-stride
  // size from 2 to 16 blocks per CU by 5-7% (tools/kprobe.hip).  LSEC_GRID_CAP overrides.
  static const uint64_t cap = [] {
    const char *s = getenv("LSEC_GRID_CAP");
    return s ? std::max<uint64_t>(1, strtoull(s, nullptr, 10)) : (1ull << 31) - 1;
  }();
  return static_cast<int>(std::min<uint64_t>(std::max<uint64_t>(ntiles, 1), cap));
}

template <typename F>
hipError_t by_r(int R, F f) {
  switch (R) {
    case 1: return f(std::integral_constant<int, 1>());
    case 2: return f(std::integral_constant<int, 2>());
    case 3: return f(std::integral_constant<int, 3>());
    case 4: return f(std::integral_constant<int, 4>());
    case 5: return f(std::integral_constant<int, 5>());
    case 6: return f(std::integral_constant<int, 6>());
    case 7: return f(std::integral_constant<int, 7>());
    case 8: return f(std::integral_constant<int, 8>());
    default: return hipErrorInvalidValue;
  }
}

// (IT, MINW) shape for a K x R bytewise launch.  variant 0 = automatic policy, measured
// (tools/kbench.py): two 4 KiB steps per lane while all K*IT loads of a lane fit the register
// file at >= 2 waves/SIMD; the widest shapes (K*R >= 100, e.g. RS(20+6)) drop to one step.
int bytewise_shape(int K, int R) {
  if (g_bw_variant > 0) return g_bw_variant - 1;
  return K * R >= 100 ? 1 : 0;
}

}  // namespace

void set_kernel_variant(int bw, int bs) {
  g_bw_variant = bw;
  g_bs_variant = bs;
}

hipError_t launch_bytewise(const ApplyArgs &a, hipStream_t st, int grid_blocks) {
  if (a.K < 1 || a.K > kMaxK || a.R < 1 || a.R > 8 || a.size % 8 != 0) return hipErrorInvalidValue;
  if (a.nstripes <= 0 || a.size == 0) return hipSuccess;
  const int shape = bytewise_shape(a.K, a.R);
  const int it = (shape == 1 || shape == 3) ? 1 : 2;
  const uint64_t tile = static_cast<uint64_t>(kBlock) * 16 * it;
  const uint64_t ntiles = ((a.size + tile - 1) / tile) * static_cast<uint64_t>(a.nstripes);
  if (ntiles >= (1ull << 31)) return hipErrorInvalidValue;
  const int grid = grid_blocks > 0 ? grid_blocks : default_grid(ntiles);
  return by_r(a.R, [&](auto r) { return dispatch_bytewise<decltype(r)::value>(a, st, grid, shape); });
}

hipError_t launch_bitsliced(const ApplyArgs &a, hipStream_t st, int grid_blocks) {
  if (a.K < 1 || a.K > kMaxK || a.R < 1 || a.R > 8 || a.packet <= 0 || a.packet % 4 != 0 ||
      a.size % (8LL * a.packet) != 0)
    return hipErrorInvalidValue;
  if (a.nstripes <= 0 || a.size == 0) return hipSuccess;
  int dw = (g_bs_variant == 2 || g_bs_variant == 4) ? g_bs_variant : 1;
  while (dw > 1 && a.packet % (4 * dw) != 0) dw >>= 1;
  const uint64_t col_bytes = a.size / 8;
  const uint64_t tile = kBlock * 4ull * dw;
  const uint64_t ntiles = ((col_bytes + tile - 1) / tile) * static_cast<uint64_t>(a.nstripes);
  if (ntiles >= (1ull << 31)) return hipErrorInvalidValue;
  const int grid = grid_blocks > 0 ? grid_blocks : default_grid(ntiles);
  return by_r(a.R, [&](auto r) { return dispatch_bitsliced<decltype(r)::value>(a, st, grid, dw); });
}

}  // namespace lsec
