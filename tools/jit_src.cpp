// Print the XOR-network source ec_jit.cpp generates for a matrix read from stdin
// ("R K W" then R*K coefficients; W = 8, 16 or 32), so it can be compiled offline (hipcc -c,
// resource usage).
#include <cstdio>
#include <vector>

#include "../lstore_amd/csrc/ec_jit.h"

int main() {
  int R = 0, K = 0, W = 0;
  if (scanf("%d %d %d", &R, &K, &W) != 3 || R < 1 || K < 1 || (W != 8 && W != 16 && W != 32)) return 2;
  std::vector<uint32_t> m(static_cast<size_t>(R) * K);
  for (auto &c : m) {
    unsigned long v = 0;
    if (scanf("%lu", &v) != 1) return 2;
    c = static_cast<uint32_t>(v);
  }
  if (W == 8) {
    std::vector<uint8_t> m8(m.begin(), m.end());
    fputs(lsec::jit::xornet_source(m8.data(), R, K).c_str(), stdout);
  } else {
    fputs(lsec::jit::gfw_source(m.data(), R, K, W).c_str(), stdout);
  }
  return 0;
}
