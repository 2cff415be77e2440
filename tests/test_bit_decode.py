"""CPU tests of the bitmatrix decode planner (gf8.cpp make_bit_decode), which the liberation
family's decodes use: it solves for the lost data bits only, so its rows must equal those of an
inversion of the whole (k*w)-square survivor bitmatrix -- the way jerasure_invert_bitmatrix
decodes (vendor/jerasure/src/jerasure.c:1049-1104, called from
jerasure_generate_decoding_schedule :823-951) -- for every pattern of one and two lost devices
(lsec_selftest_bit_decode).  No GPU is needed; the GPU tests decode through these rows."""
import ctypes

import pytest

import lstore_amd as L
from lstore_amd import erasure as E


def _lib():
    lib = E.lib()
    lib.lsec_selftest_bit_decode.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int]
    lib.lsec_selftest_bit_decode.restype = ctypes.c_int
    return lib


@pytest.mark.parametrize("method,k,w", [(L.LIBERATION, 3, 3), (L.LIBERATION, 7, 7), (L.LIBERATION, 5, 7),
                                        (L.LIBERATION, 11, 11), (L.BLAUM_ROTH, 4, 4), (L.BLAUM_ROTH, 10, 10),
                                        (L.LIBER8TION, 8, 8), (L.LIBER8TION, 3, 8), (L.LIBERATION, 17, 17)])
def test_lost_bits_planner_equals_dense_inversion(built, method, k, w):
    n = _lib().lsec_selftest_bit_decode(method, k, w)
    assert n == (k + 2) * (k + 3) // 2, E.last_error()


def test_bit_decode_selftest_rejects_unknown_codes(built):
    assert _lib().lsec_selftest_bit_decode(L.LIBERATION, 8, 7) == -1  # liberation needs k <= w
    assert "no" in E.last_error()
