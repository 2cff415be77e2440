"""oracle -- TEST INFRASTRUCTURE ONLY.

ctypes front-ends for
  * ``libec_oracle.so``           our CPU restatement of erasure_tools.c + Jerasure (ec_oracle.c)
  * ``_ref/libjerasure_ref.so``   the real reference (vendor/jerasure + raid4.c) compiled from
                                  /root/reference by oracle/Makefile

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
package, and only as the checker / baseline -- never as the thing measured or shipped.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "libec_oracle.so")
REF_SO = os.path.join(HERE, "_ref", "libjerasure_ref.so")

# method ids: src/lio/erasure_tools.h:37-45
REED_SOL_VAN, REED_SOL_R6_OP, CAUCHY_ORIG, CAUCHY_GOOD, BLAUM_ROTH, LIBERATION, LIBER8TION, RAID4 = range(8)
BITMATRIX_METHODS = (CAUCHY_ORIG, CAUCHY_GOOD, BLAUM_ROTH, LIBERATION, LIBER8TION)

_ora = None
_ref = None


def build(force: bool = False) -> None:
    """Compile the restatement (and the reference, when /root/reference exists)."""
    if force or not os.path.exists(ORACLE_SO) or (
        os.path.isdir("/root/reference") and not os.path.exists(REF_SO)
    ):
        subprocess.run(["make", "-s", "-C", HERE], check=True)


def _ptrs(arrs):
    return (C.c_char_p * len(arrs))(*[a.ctypes.data_as(C.c_char_p) for a in arrs])


def _iarr(vals):
    return (C.c_int * len(vals))(*vals)


def oracle():
    global _ora
    if _ora is None:
        if not os.path.exists(ORACLE_SO):
            build()
        lib = C.CDLL(ORACLE_SO)
        lib.eco_generate_plan.argtypes = [C.c_longlong, C.c_int, C.c_int, C.c_int, C.c_int, C.c_int,
                                          C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int),
                                          C.POINTER(C.c_longlong), C.POINTER(C.c_int)]
        lib.eco_adler32.restype = C.c_uint
        lib.eco_adler32.argtypes = [C.c_uint, C.c_void_p, C.c_longlong]
        lib.eco_init()
        _ora = lib
    return _ora


def ref_available() -> bool:
    return os.path.exists(REF_SO)


def ref():
    global _ref
    if _ref is None:
        if not os.path.exists(REF_SO):
            raise FileNotFoundError(f"{REF_SO} not built (needs /root/reference; run make -C oracle ref)")
        lib = C.CDLL(REF_SO)
        lib.ref_plan_new.restype = C.c_void_p
        lib.ref_plan_new.argtypes = [C.c_int] * 5
        for f in ("ref_plan_free",):
            getattr(lib, f).argtypes = [C.c_void_p]
        for f in ("ref_plan_matrix", "ref_plan_bitmatrix", "ref_plan_schedule"):
            getattr(lib, f).argtypes = [C.c_void_p, C.c_void_p]
        lib.ref_plan_encode.argtypes = [C.c_void_p, C.c_void_p, C.c_int]
        lib.ref_plan_decode.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_void_p]
        lib.ref_plan_encode_many.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int]
        lib.ref_plan_decode_many.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_void_p]
        lib.ref_segment_write.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_longlong,
                                          C.c_void_p]
        lib.ref_segment_write.restype = None
        lib.ref_segment_write_iov.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int,
                                              C.c_longlong, C.c_void_p]
        lib.ref_segment_write_iov.restype = None
        lib.ref_segment_inspect.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p,
                                            C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
        lib.ref_segment_inspect.restype = None
        lib.ref_segment_read.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_longlong, C.c_int,
                                         C.c_int, C.c_void_p, C.c_void_p]
        _ref = lib
    return _ref


# ----------------------------------------------------------------------------- restatement
def generate_plan(file_size, method, k, m, w=-1, plow=-1, phigh=-1):
    """eco_generate_plan -> dict(w, packet_size, strip_size, base_unit) or None."""
    lib = oracle()
    wo, po, bo = C.c_int(), C.c_int(), C.c_int()
    so = C.c_longlong()
    rc = lib.eco_generate_plan(file_size, method, k, m, w, plow, phigh, C.byref(wo), C.byref(po),
                               C.byref(so), C.byref(bo))
    if rc != 0:
        return None
    return dict(w=wo.value, packet_size=po.value, strip_size=so.value, base_unit=bo.value)


def coding_matrix(method, k, m, w=8):
    out = (C.c_int * (k * m))()
    if oracle().eco_coding_matrix(method, k, m, w, out) != 0:
        return None
    return np.array(out[:], dtype=np.int32).reshape(m, k)


def bitmatrix(matrix, w=8):
    m, k = matrix.shape
    out = (C.c_int * (k * m * w * w))()
    mat = np.ascontiguousarray(matrix, dtype=np.int32)
    oracle().eco_matrix_to_bitmatrix(k, m, w, mat.ctypes.data_as(C.c_void_p), out)
    return np.array(out[:], dtype=np.int32).reshape(m * w, k * w)


def encode(method, data, m, packet=0, w=8):
    """data: uint8 [k, C] -> parity uint8 [m, C] (restatement)."""
    k, size = data.shape
    data = np.ascontiguousarray(data)
    par = np.zeros((m, size), dtype=np.uint8)
    mat = coding_matrix(method, k, m, w)
    d = _ptrs([data[j] for j in range(k)])
    p = _ptrs([par[i] for i in range(m)])
    lib = oracle()
    if method in BITMATRIX_METHODS:
        bm = np.ascontiguousarray(bitmatrix(mat, w))
        rc = lib.eco_bitmatrix_encode(k, m, w, bm.ctypes.data_as(C.c_void_p), d, p, size, packet)
        if rc:
            raise ValueError("bitmatrix encode: size must be a multiple of w*packet")
    else:
        mat = np.ascontiguousarray(mat)
        lib.eco_matrix_encode(k, m, w, mat.ctypes.data_as(C.c_void_p), d, p, size)
    return par


def decode(method, shards, k, erasures, packet=0, w=8):
    """shards: uint8 [k+m, C], erased rows are overwritten in place. Returns rc."""
    km, size = shards.shape
    m = km - k
    mat = coding_matrix(method, k, m, w)
    ptrs = _ptrs([shards[i] for i in range(km)])
    er = _iarr(list(erasures) + [-1])
    lib = oracle()
    if method in BITMATRIX_METHODS:
        bm = np.ascontiguousarray(bitmatrix(mat, w))
        return lib.eco_bitmatrix_decode(k, m, w, bm.ctypes.data_as(C.c_void_p), er, ptrs, size, packet)
    mat = np.ascontiguousarray(mat)
    return lib.eco_matrix_decode(k, m, w, mat.ctypes.data_as(C.c_void_p), er, ptrs, size)


def adler32(buf, adler=1):
    buf = np.ascontiguousarray(buf)
    return oracle().eco_adler32(adler, buf.ctypes.data, buf.nbytes)


# ----------------------------------------------------------------------------- reference
class RefPlan:
    """The real reference (jerasure + erasure_tools dispatch) for one (method,k,m,w,packet)."""

    def __init__(self, method, k, m, w=8, packet=0):
        self.lib = ref()
        self.method, self.k, self.m, self.w, self.packet = method, k, m, w, packet
        self.h = self.lib.ref_plan_new(method, k, m, w, packet)
        if not self.h:
            raise ValueError("ref_plan_new failed")

    def close(self):
        if self.h:
            self.lib.ref_plan_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def matrix(self):
        buf = (C.c_int * (2 * self.k * max(self.m, 2)))()
        n = self.lib.ref_plan_matrix(self.h, buf)
        if n < 0:
            return None
        rows = 2 if self.method == REED_SOL_R6_OP else self.m
        return np.array(buf[:n], dtype=np.int32).reshape(rows, self.k)

    def bitmatrix(self):
        n = self.k * self.m * self.w * self.w
        buf = (C.c_int * n)()
        if self.lib.ref_plan_bitmatrix(self.h, buf) < 0:
            return None
        return np.array(buf[:], dtype=np.int32).reshape(self.m * self.w, self.k * self.w)

    def schedule(self):
        n = self.lib.ref_plan_schedule(self.h, None)
        if n < 0:
            return None
        buf = (C.c_int * (5 * n))()
        self.lib.ref_plan_schedule(self.h, buf)
        return np.array(buf[:], dtype=np.int32).reshape(n, 5)

    def encode(self, data):
        k, size = data.shape
        sh = np.zeros((k + self.m, size), dtype=np.uint8)
        sh[:k] = data
        self.lib.ref_plan_encode(self.h, _ptrs([sh[i] for i in range(k + self.m)]), size)
        return sh[k:].copy()

    def decode(self, shards, erasures):
        km, size = shards.shape
        return self.lib.ref_plan_decode(self.h, _ptrs([shards[i] for i in range(km)]), size,
                                        _iarr(list(erasures) + [-1]))

    def segment_write(self, data, nstripes, chunk, n_shift=1, first_stripe=0, out=None):
        """segjerase_write_func + LUN placement restated over the real jerasure (config c1).
        data: uint8 [nstripes, k, C]; returns uint8 [k+m, nstripes*(C+4)] device images (into
        `out` when given)."""
        n = self.k + self.m
        dev = out if out is not None else np.zeros((n, nstripes * (chunk + 4)), dtype=np.uint8)
        ptrs = _ptrs([dev[i] for i in range(n)])
        data = np.ascontiguousarray(data)
        self.lib.ref_segment_write(self.h, data.ctypes.data, nstripes, chunk, n_shift, first_stripe, ptrs)
        return dev

    def segment_write_iov(self, pieces, nstripes, chunk, n_shift=1, first_stripe=0):
        """segjerase_write_func's scatter-list / straddle / error-page handling restated over the
        real jerasure.  pieces: uint8 arrays, or ints for error pages of that many bytes."""
        n = self.k + self.m
        dev = np.zeros((n, nstripes * (chunk + 4)), dtype=np.uint8)
        keep = [np.ascontiguousarray(pc, dtype=np.uint8) for pc in pieces if not isinstance(pc, (int, np.integer))]
        bases, it = [], iter(keep)
        for pc in pieces:
            bases.append(0 if isinstance(pc, (int, np.integer)) else next(it).ctypes.data)
        lens = np.array([int(pc) if isinstance(pc, (int, np.integer)) else np.asarray(pc).size for pc in pieces],
                        dtype=np.int64)
        base_arr = (C.c_void_p * max(1, len(pieces)))(*bases)
        self.lib.ref_segment_write_iov(self.h, base_arr, lens.ctypes.data, len(pieces), nstripes, chunk, n_shift,
                                       first_stripe, _ptrs([dev[i] for i in range(n)]))
        return dev

    def segment_inspect(self, buf, nstripes, chunk, magic_cksum=1, do_fix=0, brute=None):
        """segjerase_inspect_full_func's per-stripe loop restated over the real jerasure (buf is
        modified in place as the reference's buffer is).  Returns (status, badmap, rewrite,
        counters[bad, unrecoverable, silent, empty], brute state)."""
        n = self.k + self.m
        status = np.zeros(nstripes, np.int32)
        badmap = np.zeros((nstripes, n), np.uint8)
        rewrite = np.zeros((nstripes, n), np.uint8)
        counters = np.zeros(4, np.int64)
        brute = np.zeros(1 + n, np.int32) if brute is None else brute
        self.lib.ref_segment_inspect(self.h, buf.ctypes.data, nstripes, chunk, magic_cksum, do_fix, status.ctypes.data,
                                     badmap.ctypes.data, rewrite.ctypes.data, counters.ctypes.data, brute.ctypes.data)
        return status, badmap, rewrite, counters, brute

    def segment_read(self, dev, nstripes, chunk, n_shift=1, first_stripe=0, paranoid=0, magic_cksum=1):
        """segjerase_read_func's verification restated: (data [N,k,C], status, n_unrecoverable)."""
        n = self.k + self.m
        ptrs = _ptrs([dev[i] for i in range(n)])
        data = np.zeros((nstripes, self.k, chunk), np.uint8)
        status = np.zeros(nstripes, np.int32)
        bad = self.lib.ref_segment_read(self.h, ptrs, nstripes, chunk, n_shift, first_stripe, paranoid, magic_cksum,
                                        data.ctypes.data, status.ctypes.data)
        return data, status, bad

    def encode_many(self, ptr_array, nstripes, size, nthreads):
        return self.lib.ref_plan_encode_many(self.h, ptr_array, nstripes, size, nthreads)

    def decode_many(self, ptr_array, nstripes, size, nthreads, erasures):
        return self.lib.ref_plan_decode_many(self.h, ptr_array, nstripes, size, nthreads,
                                             _iarr(list(erasures) + [-1]))
