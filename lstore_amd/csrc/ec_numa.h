// ec_numa.h -- host NUMA placement of a device's engine threads (per GPU "its own
// host thread, its own streams, device buffers, and pinned NUMA-local staging").  Internal to
// liblstore_ec.
//
// LStore is one process per node with one process-wide gop pool (lio_config.c:87, :1110-1132),
// so the engine places its own per-device threads: a device's dispatcher thread, the threads
// that run its stripe range of a split host batch, and the copy pool that packs its staging run
// on the CPUs of the device's NUMA node (PCI bus id -> sysfs numa_node -> the node's cpulist),
// and the page-locked staging they allocate is allocated by those threads for that device.
#pragma once

#include <string>
#include <vector>

namespace lsec {
namespace numa {

struct Placement {
  int node = -1;          // -1: unknown (no sysfs entry, a single-node host, or LSEC_NUMA=0)
  std::vector<int> cpus;  // the node's CPUs this process may use; empty: do not bind
};

// "0-3,8,10-11" -> {0,1,2,3,8,10,11}; malformed pieces are skipped
std::vector<int> parse_cpulist(const std::string &s);

// Placement of the PCI function `bus` ("0000:c1:00.0", any case) under the sysfs tree `root`
// (normally "/sys"): <root>/bus/pci/devices/<bus>/numa_node, then
// <root>/devices/system/node/node<N>/cpulist, intersected with `allowed` (empty: no filter).
Placement for_bus(const std::string &root, const std::string &bus, const std::vector<int> &allowed);

// Placement of HIP device `dev` (cached per device; the process's CPU affinity at library load
// is the filter; LSEC_SYSFS_ROOT overrides "/sys", LSEC_NUMA=0 turns placement off).
const Placement &of_device(int dev);

// Pin the calling thread to dev's node CPUs (no-op when the placement is unknown).  true if pinned.
bool bind_this_thread(int dev);

}  // namespace numa
}  // namespace lsec
