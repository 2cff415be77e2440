"""CPU tests of the network compile queue (ec_jit.cpp): hipRTC compiles on the host, so no GPU is
needed.  A process that binds several networks and exits while compiles are queued and running
must exit cleanly: the exit drain starts no queued compile and waits for the running ones (a
thread per network, compiling while hipRTC's global state was destroyed at exit, corrupted the
heap: "free(): corrupted unsorted chunks" after a GPU test run)."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

SCRIPT = """
import ctypes, sys
sys.path.insert(0, {root!r})
from lstore_amd import erasure as E
lib = E.lib()
lib.lsec_test_jit_queue.argtypes = [ctypes.c_int, ctypes.c_int]
lib.lsec_test_jit_queue.restype = ctypes.c_int
print(lib.lsec_test_jit_queue({n}, {wait_ms}))
"""


def run(n, wait_ms):
    return subprocess.run([sys.executable, "-c", SCRIPT.format(root=ROOT, n=n, wait_ms=wait_ms)],
                          capture_output=True, text=True, timeout=300)


def test_compiles_complete_and_exit_is_clean(built):
    r = run(3, 120000)
    assert r.returncode == 0, r.stderr[-2000:]
    assert int(r.stdout.strip().splitlines()[-1]) >= 1  # the waited-for network compiled on the host
    assert "corrupted" not in r.stderr and "Aborted" not in r.stderr


def test_exit_with_compiles_queued_and_running(built):
    r = run(12, 0)  # returns at once: two compiles running, ten queued at exit
    assert r.returncode == 0, r.stderr[-2000:]
    assert "corrupted" not in r.stderr and "Aborted" not in r.stderr
