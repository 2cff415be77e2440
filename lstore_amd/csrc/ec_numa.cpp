// ec_numa.cpp -- device -> host NUMA node -> CPUs, and thread pinning (see ec_numa.h).
#include "ec_numa.h"

#include "ec_hiperr.h"

#include <hip/hip_runtime.h>
#include <pthread.h>
#include <sched.h>

#include <algorithm>
#include <cctype>
#include <cstdlib>
#include <fstream>
#include <map>
#include <memory>
#include <mutex>
#include <sstream>

namespace lsec {
namespace numa {

namespace {

std::vector<int> affinity_now() {
  std::vector<int> v;
  cpu_set_t set;
  CPU_ZERO(&set);
  if (sched_getaffinity(0, sizeof(set), &set) != 0) return v;
  for (int c = 0; c < CPU_SETSIZE; ++c)
    if (CPU_ISSET(c, &set)) v.push_back(c);
  return v;
}

// the CPUs the process was allowed when the library was loaded: placements are filtered by it,
// not by the (possibly already pinned) affinity of whichever thread asks first
const std::vector<int> g_allowed = affinity_now();

bool read_line(const std::string &path, std::string &out) {
  std::ifstream f(path);
  if (!f) return false;
  std::getline(f, out);
  return true;
}

}  // namespace

std::vector<int> parse_cpulist(const std::string &s) {
  std::vector<int> v;
  std::stringstream ss(s);
  std::string piece;
  while (std::getline(ss, piece, ',')) {
    piece.erase(std::remove_if(piece.begin(), piece.end(), [](unsigned char ch) { return std::isspace(ch); }), piece.end());
    if (piece.empty()) continue;
    char *end = nullptr;
    const long a = strtol(piece.c_str(), &end, 10);
    if (end == piece.c_str() || a < 0) continue;
    long b = a;
    if (*end == '-') {
      const char *q = end + 1;
      b = strtol(q, &end, 10);
      if (end == q || b < a) continue;
    }
    if (*end != '\0' || b >= CPU_SETSIZE) continue;
    for (long c = a; c <= b; ++c) v.push_back(static_cast<int>(c));
  }
  std::sort(v.begin(), v.end());
  v.erase(std::unique(v.begin(), v.end()), v.end());
  return v;
}

Placement for_bus(const std::string &root, const std::string &bus, const std::vector<int> &allowed) {
  Placement pl;
  std::string id = bus;
  std::transform(id.begin(), id.end(), id.begin(), [](unsigned char ch) { return std::tolower(ch); });
  std::string line;
  if (id.empty() || !read_line(root + "/bus/pci/devices/" + id + "/numa_node", line)) return pl;
  char *end = nullptr;
  const long node = strtol(line.c_str(), &end, 10);
  if (end == line.c_str() || node < 0) return pl;  // -1: the firmware reports no affinity
  if (!read_line(root + "/devices/system/node/node" + std::to_string(node) + "/cpulist", line)) return pl;
  pl.node = static_cast<int>(node);
  for (int c : parse_cpulist(line))
    if (allowed.empty() || std::binary_search(allowed.begin(), allowed.end(), c)) pl.cpus.push_back(c);
  return pl;
}

const Placement &of_device(int dev) {
  static std::mutex mu;
  static auto *cache = new std::map<int, std::unique_ptr<Placement>>();  // leaked: used until exit
  std::lock_guard<std::mutex> lk(mu);
  std::unique_ptr<Placement> &p = (*cache)[dev];
  if (!p) {
    p.reset(new Placement());
    const char *off = getenv("LSEC_NUMA");
    char bus[64] = {0};
    if (!(off && *off == '0') && quiet([&] { return hipDeviceGetPCIBusId(bus, sizeof(bus), dev); }) == hipSuccess) {
      const char *root = getenv("LSEC_SYSFS_ROOT");
      *p = for_bus(root ? root : "/sys", bus, g_allowed);
    }
  }
  return *p;
}

bool bind_this_thread(int dev) {
  const Placement &pl = of_device(dev);
  if (pl.cpus.empty()) return false;
  cpu_set_t set;
  CPU_ZERO(&set);
  for (int c : pl.cpus) CPU_SET(c, &set);
  return pthread_setaffinity_np(pthread_self(), sizeof(set), &set) == 0;
}

}  // namespace numa
}  // namespace lsec
