// Print the XOR-network source ec_jit.cpp generates for a matrix read from stdin
// ("R K" then R*K coefficients), so it can be compiled offline (hipcc -c, resource usage).
#include <cstdio>
#include <vector>

#include "../lstore_amd/csrc/ec_jit.h"

int main() {
  int R = 0, K = 0;
  if (scanf("%d %d", &R, &K) != 2 || R < 1 || K < 1) return 2;
  std::vector<uint8_t> m(static_cast<size_t>(R) * K);
  for (auto &c : m) {
    int v = 0;
    if (scanf("%d", &v) != 1) return 2;
    c = static_cast<uint8_t>(v);
  }
  fputs(lsec::jit::xornet_source(m.data(), R, K).c_str(), stdout);
  return 0;
}
