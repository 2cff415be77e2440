// ec_hiperr.h -- runtime calls that must not touch the caller's pending HIP error.
#pragma once
#include <hip/hip_runtime.h>

#include <functional>

namespace lsec {

// HIP keeps one last-error slot per thread, and a call runs on the caller's thread, whose slot may
// hold an error of the caller's own that the caller has not read yet.  Runtime calls that can fail
// (by design: hipHostGetFlags on a registered range, an address-range query, a registration the
// runtime refuses; or an allocation that fails) go through quiet(): inline when the caller's slot
// is clear (the engine then clears the error it caused itself), and on the engine's one helper
// thread (a slot of its own; it takes the caller's current device first) when the caller has an
// error pending, so that the caller's error stays where the caller left it.  A caller that leaves
// an error unread pays a thread hand-off (a few microseconds) per such call until it reads it.
// Defined in ec_pinning.cpp.
hipError_t quiet(const std::function<hipError_t()> &f);

}  // namespace lsec
