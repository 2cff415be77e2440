// ec_jitc.cpp -- lsec_jitc, the engine's network compiler, run as a child process per compile.
//
// The engine (ec_jit.cpp) generates the HIP source of a per-matrix network and hands it to this
// program instead of calling hipRTC in its own process: hipRTC's compiler keeps global state that
// a process's exit destroys, so an in-process compile still running at exit corrupted the heap
// (round 4), and waiting for it held the exit of a storage daemon for as long as the compile took
// (up to 30 s for the widest w = 32 networks).  A child can be killed at any moment instead, and
// the engine's process never loads the compiler at all.
//
// Protocol: the source arrives on stdin (to EOF).  stdout gets one record:
//   "LSJC" | status (1 byte: 0 = compiled, 1 = failed) | length (8 bytes, little-endian) | bytes
// where the bytes are the gfx950 code object, or the compiler's log when the compile failed.
// argv[1], when present, is the parent's pid: the child dies with the thread that started it
// (PR_SET_PDEATHSIG), and leaves at once if that parent is already gone.
#include <hip/hiprtc.h>
#include <signal.h>
#include <sys/prctl.h>
#include <unistd.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

namespace {

bool write_all(const void *p, size_t n) {
  const char *c = static_cast<const char *>(p);
  while (n > 0) {
    const ssize_t w = write(1, c, n);
    if (w <= 0) return false;
    c += w;
    n -= static_cast<size_t>(w);
  }
  return true;
}

int reply(uint8_t status, const char *data, size_t n) {
  char head[13] = {'L', 'S', 'J', 'C', static_cast<char>(status)};
  for (int i = 0; i < 8; ++i) head[5 + i] = static_cast<char>((static_cast<uint64_t>(n) >> (8 * i)) & 0xFF);
  return write_all(head, sizeof(head)) && write_all(data, n) ? 0 : 2;
}

}  // namespace

int main(int argc, char **argv) {
  prctl(PR_SET_PDEATHSIG, SIGKILL);
  if (argc > 1 && getppid() != static_cast<pid_t>(atol(argv[1]))) return 3;  // the parent is gone
  std::string src;
  char buf[1 << 16];
  for (;;) {
    const ssize_t r = read(0, buf, sizeof(buf));
    if (r < 0) return reply(1, "lsec_jitc: cannot read the source", 33);
    if (r == 0) break;
    src.append(buf, static_cast<size_t>(r));
  }
  hiprtcProgram prog = nullptr;
  if (hiprtcCreateProgram(&prog, src.c_str(), "lsec_xornet.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS)
    return reply(1, "hiprtcCreateProgram failed", 26);
  const char *opts[] = {"--offload-arch=gfx950", "-O3"};
  if (hiprtcCompileProgram(prog, 2, opts) != HIPRTC_SUCCESS) {
    size_t n = 0;
    hiprtcGetProgramLogSize(prog, &n);
    std::string log(n, '\0');
    if (n) hiprtcGetProgramLog(prog, &log[0]);
    log = "hiprtc compile failed: " + log.substr(0, 400);
    return reply(1, log.data(), log.size());
  }
  size_t n = 0;
  hiprtcGetCodeSize(prog, &n);
  std::vector<char> code(n);
  hiprtcGetCode(prog, code.data());
  hiprtcDestroyProgram(&prog);
  return reply(0, code.data(), code.size());
}
