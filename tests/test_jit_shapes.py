"""CPU tests of the network generators (ec_jit.cpp): every generator shape -- w = 8 XOR networks,
w = 16 / 32 bit-sliced networks in the one-wave form and the wave-pair split, and the packet
networks of bitmatrix and Cauchy codes -- generated for pseudo-random matrices and compiled for
gfx950 by hipRTC on the host (lsec_test_jit_compile; no GPU).  The GPU tests run the networks of
real plans against the reference; these keep a generator change that breaks the emitted source
from reaching them, also under the A/B knobs of LSEC_JIT_VARIANT."""
import ctypes
import os
import subprocess
import sys

import pytest

from lstore_amd import erasure as E

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# (shape, R, K, w, packet): shape 0 = w = 8 network, 1 = w = 16 / 32 network, 2 = bitmatrix packet
# network, 3 = Cauchy packet network
SHAPES = [
    (0, 6, 20, 8, 0),     # RS(20+6): capped common pairs, 16 B lanes
    (0, 8, 12, 8, 0),     # 8 rows over 12 inputs: 8 B lanes
    (0, 8, 32, 8, 0),     # the widest
    (1, 3, 6, 32, 0),     # one wave
    (1, 4, 10, 32, 0),    # wave-pair split
    (1, 6, 10, 32, 0),    # split, 12 KiB LDS slots
    (1, 4, 10, 16, 0),    # one wave
    (1, 6, 20, 16, 0),    # split at w = 16
    (2, 2, 6, 7, 32),     # liberation-like, 16 B lanes
    (2, 2, 16, 16, 32),   # 8 B lanes by the register cap
    (2, 2, 8, 8, 40),     # 8 B lanes by the packet
    (3, 4, 10, 32, 64),   # Cauchy w = 32, 4 B lanes
    (3, 4, 10, 16, 32),   # Cauchy w = 16
]


def _lib():
    lib = E.lib()
    lib.lsec_test_jit_compile.argtypes = [ctypes.c_int] * 5 + [ctypes.c_uint]
    lib.lsec_test_jit_compile.restype = ctypes.c_int
    return lib


@pytest.mark.parametrize("shape,R,K,w,packet", SHAPES)
def test_generated_network_compiles(built, shape, R, K, w, packet):
    assert _lib().lsec_test_jit_compile(shape, R, K, w, packet, 7) == 0, E.last_error()


def test_bad_arguments_are_errors(built):
    assert _lib().lsec_test_jit_compile(9, 4, 10, 32, 0, 1) == -1
    assert "bad arguments" in E.last_error()


KNOB_SCRIPT = """
import ctypes, sys
sys.path.insert(0, {root!r})
from lstore_amd import erasure as E
lib = E.lib()
lib.lsec_test_jit_compile.argtypes = [ctypes.c_int] * 5 + [ctypes.c_uint]
bad = [s for s in {shapes!r} if lib.lsec_test_jit_compile(*s, 3) != 0]
print(bad, E.last_error() if bad else "")
sys.exit(1 if bad else 0)
"""


@pytest.mark.parametrize("variant,pick", [
    (0x80000, lambda s: s[0] == 1 and s[3] == 32),    # w = 32 split off: the one-wave form at 4+ rows
    (0x380000, lambda s: s[0] == 1 and s[1] >= 4),    # split: no prefetch, tree folds
    (0x1000000, lambda s: s[0] == 1 and s[3] == 16),  # w = 16 split off
    (0x2000000, lambda s: s[0] >= 2),                 # packet networks in 2 output groups
    (0x9, lambda s: s[0] == 0),                       # w = 8: uncapped pairs (bit 0), no pairs (bit 3)
    (0x28, lambda s: s[0] == 0),                      # w = 8: 2-dword lanes, no pairs
])
def test_knob_shapes_compile(built, variant, pick):
    shapes = [s for s in SHAPES if pick(s)]
    r = subprocess.run([sys.executable, "-c", KNOB_SCRIPT.format(root=ROOT, shapes=shapes)], capture_output=True,
                       text=True, timeout=600, env=dict(os.environ, LSEC_JIT_VARIANT=str(variant)))
    assert r.returncode == 0, (r.stdout[-1500:], r.stderr[-1500:])
