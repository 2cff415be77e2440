"""CPU test of the in-place stall guard (ec_engine.h note_inplace_drain / inplace_suspended): DMA from
host pages pinned in place stalled ~25 ms a call under unmap churn (profiles/r06_v2_free_after_churn.jsonl);
three stalls -- a drain over 5 ms at under 1 GB/s -- within 64 pinned calls suspend pinning in place, and
ordinary drains, slow but large ones, or stalls spread over more than one window do not.  No GPU is
needed: the hook drives the guard's bookkeeping directly."""
import ctypes

from lstore_amd import erasure as E

MIB = 1 << 20


def _lib():
    lib = E.lib()
    lib.lsec_test_inplace_guard.argtypes = [ctypes.c_int, ctypes.c_ulonglong, ctypes.c_double]
    lib.lsec_test_inplace_guard.restype = ctypes.c_int
    return lib


def test_three_stalls_in_a_window_suspend_pinning(built):
    lib = _lib()
    lib.lsec_test_inplace_guard(0, 0, 0.0)
    try:
        assert lib.lsec_test_inplace_guard(2, 0, 0.0) == 0
        for _ in range(2):
            lib.lsec_test_inplace_guard(1, 7 * MIB, 25.0)  # 7 MiB in 25 ms: 0.29 GB/s, a stall
        assert lib.lsec_test_inplace_guard(2, 0, 0.0) == 0
        lib.lsec_test_inplace_guard(1, 7 * MIB, 0.17)      # a normal call in between
        lib.lsec_test_inplace_guard(1, 7 * MIB, 30.0)      # the third stall
        assert lib.lsec_test_inplace_guard(2, 0, 0.0) == 1
    finally:
        lib.lsec_test_inplace_guard(0, 0, 0.0)
    assert lib.lsec_test_inplace_guard(2, 0, 0.0) == 0


def test_slow_large_or_spread_out_drains_do_not_suspend(built):
    lib = _lib()
    lib.lsec_test_inplace_guard(0, 0, 0.0)
    try:
        for _ in range(10):
            lib.lsec_test_inplace_guard(1, 7 * MIB, 0.2)      # ordinary per-stripe calls
            lib.lsec_test_inplace_guard(1, 1 << 30, 25.0)     # 1 GiB in 25 ms: 43 GB/s, not a stall
            lib.lsec_test_inplace_guard(1, 7 * MIB, 4.0)      # slow, but under 5 ms
        assert lib.lsec_test_inplace_guard(2, 0, 0.0) == 0
        # two stalls, a full window of normal calls, then two more: never three in one window
        for _ in range(2):
            lib.lsec_test_inplace_guard(1, 7 * MIB, 25.0)
        for _ in range(70):
            lib.lsec_test_inplace_guard(1, 7 * MIB, 0.2)
        for _ in range(2):
            lib.lsec_test_inplace_guard(1, 7 * MIB, 25.0)
        assert lib.lsec_test_inplace_guard(2, 0, 0.0) == 0
    finally:
        lib.lsec_test_inplace_guard(0, 0, 0.0)
