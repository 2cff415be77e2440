// ec_host.h -- host-side helpers shared inside liblstore_ec.so (not part of the C ABI).
#pragma once

#include <cstddef>
#include <vector>

namespace lsec {

// Record a printf-style message for lsec_last_error() (thread-local) and return -1.
int set_error(const char *fmt, ...) __attribute__((format(printf, 1, 2)));

struct HostCopy {
  char *dst;
  const char *src;
  size_t bytes;
};

// memcpy every job, spread over the engine's host copy pool (the caller thread works too)
void parallel_copy(std::vector<HostCopy> &jobs);

// One piece of a scattered host <-> device transfer: `bytes` at device address `dev` and host
// address `host` (pageable; nullptr on the H2D side means zeros).
struct DevPiece {
  char *dev;
  char *host;
  size_t bytes;
};

// Many small pageable transfers as a few large DMAs: pieces are packed into (H2D) or unpacked
// from (D2H) a per-device pinned ring of two 32 MiB buffers by the host copy pool, one buffer
// being packed while the other is on the wire.  Pieces whose device ranges continue each
// other share a DMA, so list them in device-address order.  Both enqueue on `st`:
//   h2d_pieces returns once every byte has left host memory (the device copy completes in
//              stream order, before any later work on st)
//   d2h_pieces waits for st's earlier work and returns once every byte has landed
// 0 / -1 (hipError recorded for lsec_last_error()).
int h2d_pieces(const std::vector<DevPiece> &pieces, void *st);
int d2h_pieces(const std::vector<DevPiece> &pieces, void *st);

}  // namespace lsec
