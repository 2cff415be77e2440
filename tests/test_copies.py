"""CPU tests of the host copies behind packing and unpacking (ec_hostcopy.cpp stream_copy: 16-byte
non-temporal stores after a byte-wise head, memcpy tail; and the copy pool that spreads pieces
over its workers): random source / destination offsets and lengths against memcpy, with the
bytes around every destination checked untouched (lsec_selftest_copies), so no GPU is needed."""
import ctypes

from lstore_amd import erasure as E


def _lib():
    lib = E.lib()
    lib.lsec_selftest_copies.argtypes = [ctypes.c_int, ctypes.c_uint]
    lib.lsec_selftest_copies.restype = ctypes.c_int
    return lib


def test_streamed_and_pooled_copies_equal_memcpy(built):
    lib = _lib()
    for seed in (1, 2, 3):
        assert lib.lsec_selftest_copies(400, seed) == 0, E.last_error()


def test_copy_selftest_rejects_bad_arguments(built):
    assert _lib().lsec_selftest_copies(0, 1) == -1
    assert "bad arguments" in E.last_error()
