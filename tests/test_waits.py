"""CPU tests of the completion waits behind the per-stripe calls (ec_waits.cpp FlagWaits:
bounded spinning, lock-free futex parking, poller threads): host threads stand in for the GPU
and write the flags (lsec_selftest_waits), so no GPU is needed.  Waiters wait on 1..16 flags
set in random order after 0-300 us, as a call's server parts complete."""
import ctypes

import pytest

from lstore_amd import erasure as E


def _lib():
    lib = E.lib()
    lib.lsec_selftest_waits.argtypes = [ctypes.c_int, ctypes.c_int]
    lib.lsec_selftest_waits.restype = ctypes.c_int
    return lib


@pytest.mark.parametrize("threads,iters", [(1, 300), (8, 200), (64, 60), (300, 10)])
def test_waits_end_exactly_when_all_flags_are_set(built, threads, iters):
    lib = _lib()
    assert lib.lsec_selftest_waits(threads, iters) == 0, E.last_error()


def test_waits_reject_bad_arguments(built):
    lib = _lib()
    assert lib.lsec_selftest_waits(0, 1) == -1
    assert "bad arguments" in E.last_error()
