// Development probe: what bounds packing a 1 MiB RS(6+3) stripe's 6 MiB of survivors into a
// zero-copy slot (the own-slot route's pack phase, 166 us at one thread and no faster on the copy
// pool, profiles/r03_v20_slot_phases.txt)?  Copies 6 MiB from a cold pageable source (a 2 GiB
// working set walked in order) into destinations of each memory kind, with 1, 2, 4 and 8 threads,
// non-temporal and plain stores; threads bound to the GPU's NUMA node or to the other one.
// Prints one JSON line per case: median microseconds per 6 MiB and GB/s.
// Build: hipcc -O2 -o build/pack_probe tools/probes/pack_probe.cpp -lpthread
#include <hip/hip_runtime.h>
#include <immintrin.h>
#include <pthread.h>
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <thread>
#include <vector>

static void nt_copy(char *dst, const char *src, size_t n) {
  for (; n >= 64; n -= 64, dst += 64, src += 64) {
    const __m128i a = _mm_loadu_si128(reinterpret_cast<const __m128i *>(src));
    const __m128i b = _mm_loadu_si128(reinterpret_cast<const __m128i *>(src + 16));
    const __m128i c = _mm_loadu_si128(reinterpret_cast<const __m128i *>(src + 32));
    const __m128i d = _mm_loadu_si128(reinterpret_cast<const __m128i *>(src + 48));
    _mm_stream_si128(reinterpret_cast<__m128i *>(dst), a);
    _mm_stream_si128(reinterpret_cast<__m128i *>(dst + 16), b);
    _mm_stream_si128(reinterpret_cast<__m128i *>(dst + 32), c);
    _mm_stream_si128(reinterpret_cast<__m128i *>(dst + 48), d);
  }
  if (n) std::memcpy(dst, src, n);
}

static std::vector<int> parse_cpulist(const std::string &s) {
  std::vector<int> v;
  size_t i = 0;
  while (i < s.size()) {
    size_t j = s.find(',', i);
    if (j == std::string::npos) j = s.size();
    const std::string t = s.substr(i, j - i);
    const size_t dash = t.find('-');
    if (!t.empty()) {
      const int a = atoi(t.c_str()), b = dash == std::string::npos ? a : atoi(t.c_str() + dash + 1);
      for (int c = a; c <= b; ++c) v.push_back(c);
    }
    i = j + 1;
  }
  return v;
}

static std::vector<int> allowed_on_node(int node) {
  std::ifstream f("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist");
  std::string s;
  std::getline(f, s);
  cpu_set_t set;
  sched_getaffinity(0, sizeof(set), &set);
  std::vector<int> out;
  for (int c : parse_cpulist(s))
    if (CPU_ISSET(c, &set)) out.push_back(c);
  return out;
}

static int gpu_node() {
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, sizeof(bus), 0) != hipSuccess) return -1;
  for (char *p = bus; *p; ++p) *p = static_cast<char>(tolower(*p));
  std::ifstream f(std::string("/sys/bus/pci/devices/") + bus + "/numa_node");
  int n = -1;
  f >> n;
  return n;
}

int main() {
  const size_t kBytes = 6u << 20, kSet = 2048u << 20;
  char *src = static_cast<char *>(aligned_alloc(4096, kSet));
  std::memset(src, 3, kSet);
  const int gnode = gpu_node();
  const int other = gnode == 0 ? 1 : 0;
  struct Dst {
    const char *name;
    char *p;
  };
  std::vector<Dst> dsts;
  char *h = nullptr;
  if (hipHostMalloc(reinterpret_cast<void **>(&h), kBytes, hipHostMallocCoherent) == hipSuccess) dsts.push_back({"hostmalloc_coherent", h});
  h = nullptr;
  if (hipHostMalloc(reinterpret_cast<void **>(&h), kBytes, hipHostMallocNonCoherent) == hipSuccess) dsts.push_back({"hostmalloc_noncoherent", h});
  h = nullptr;
  if (hipHostMalloc(reinterpret_cast<void **>(&h), kBytes, hipHostMallocDefault) == hipSuccess) dsts.push_back({"hostmalloc_default", h});
  h = nullptr;
  if (hipHostMalloc(reinterpret_cast<void **>(&h), kBytes, hipHostMallocCoherent | hipHostMallocNumaUser) == hipSuccess)
    dsts.push_back({"hostmalloc_coherent_numauser", h});
  char *plain = static_cast<char *>(aligned_alloc(4096, kBytes));
  std::memset(plain, 0, kBytes);
  dsts.push_back({"malloc", plain});
  for (const Dst &d : dsts) std::memset(d.p, 1, kBytes);
  size_t at = 0;
  for (int node : {gnode, other}) {
    const std::vector<int> cpus = allowed_on_node(node);
    if (cpus.empty()) continue;
    for (const Dst &d : dsts)
      for (int nt : {1, 0})
        for (int threads : {1, 2, 4, 8}) {
          if (threads > static_cast<int>(cpus.size())) continue;
          std::vector<double> us;
          for (int rep = 0; rep < 30; ++rep) {
            if (at + kBytes > kSet) at = 0;
            const char *s = src + at;
            at += kBytes;
            std::atomic<int> ready{0};
            std::atomic<bool> go{false};
            std::vector<std::thread> th;
            std::vector<double> t_end(threads);
            const size_t per = kBytes / threads;
            for (int t = 0; t < threads; ++t)
              th.emplace_back([&, t] {
                cpu_set_t set;
                CPU_ZERO(&set);
                CPU_SET(cpus[t % cpus.size()], &set);
                pthread_setaffinity_np(pthread_self(), sizeof(set), &set);
                ready.fetch_add(1);
                while (!go.load()) {
                }
                if (nt) nt_copy(d.p + t * per, s + t * per, per);
                else std::memcpy(d.p + t * per, s + t * per, per);
                _mm_sfence();
              });
            while (ready.load() < threads) {
            }
            const auto t0 = std::chrono::steady_clock::now();
            go.store(true);
            for (auto &x : th) x.join();
            us.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
          }
          std::sort(us.begin(), us.end());
          const double m = us[us.size() / 2];
          printf("{\"dst\": \"%s\", \"threads_node\": %d, \"gpu_node\": %d, \"threads\": %d, \"nt\": %d, \"us\": %.1f, \"gbps\": %.1f}\n",
                 d.name, node, gnode, threads, nt, m, kBytes / m / 1e3);
          fflush(stdout);
        }
  }
  return 0;
}
