// ec_host.h -- host-side helpers shared inside liblstore_ec.so (not part of the C ABI).
#pragma once

#include <cstddef>
#include <vector>

namespace lsec {

struct HostCopy {
  char *dst;
  const char *src;
  size_t bytes;
};

// memcpy every job, spread over the engine's host copy pool (the caller thread works too)
void parallel_copy(std::vector<HostCopy> &jobs);

}  // namespace lsec
