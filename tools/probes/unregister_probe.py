#!/usr/bin/env python3
"""Development probe: does the caller's own hipHostUnregister of an arena it registered still
succeed after the engine has served calls over that arena?  (The round-5 stale-error test saw it
fail once the engine had run encode/decode calls on a caller-registered arena.)  Prints one JSON
line per case: arena kind (numpy heap view / fresh mmap), chunk size, what the engine did between
register and unregister, and the unregister's return code.

python tools/probes/unregister_probe.py
"""
import ctypes
import json
import mmap
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import lstore_amd as L  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")


def arena(kind, n):
    if kind == "mmap":
        m = mmap.mmap(-1, n)
        a = np.frombuffer(m, np.uint8)
        return a, m
    a = np.zeros(n + 4096, np.uint8)
    off = (-a.ctypes.data) % 4096
    return a[off:off + n], a


def case(kind, C, action, pageable_first):
    if pageable_first:  # an engine call that pins a pageable arena in place (1 MiB: own pipeline)
        p1 = L.Plan.for_chunk(L.CAUCHY_GOOD, 6, 3, 1 << 20)
        d1 = np.random.default_rng(1).integers(0, 256, (9, 1 << 20), dtype=np.uint8)
        p1.encode_block([d1[j] for j in range(9)])
        p1.close()
        del d1
    n = 9 * C
    a, keep = arena(kind, n)
    ptr = a.ctypes.data
    rc_reg = hip.hipHostRegister(ctypes.c_void_p(ptr), ctypes.c_size_t(n), 0)
    p = L.Plan.for_chunk(L.CAUCHY_GOOD, 6, 3, C)
    d = a.reshape(9, C)
    d[:6] = np.random.default_rng(2).integers(0, 256, (6, C), dtype=np.uint8)
    if action in ("encode", "both"):
        p.encode_block([d[j] for j in range(9)])
    if action in ("decode", "both"):
        d[0] = 0
        p.decode_block([d[j] for j in range(9)], [0])
    rc_unreg = hip.hipHostUnregister(ctypes.c_void_p(ptr))
    err_after = hip.hipGetLastError()
    p.close()
    print(json.dumps({"arena": kind, "chunk": C, "engine": action, "pageable_call_before": pageable_first,
                      "ptr_mod_4k": ptr % 4096, "register_rc": rc_reg, "unregister_rc": rc_unreg,
                      "last_error_after": err_after}), flush=True)
    del keep


def ranges():
    """what the runtime reports as the extent of a page-locked range (interior pointer)"""
    for kind in ("numpy", "mmap", "hostmalloc"):
        n = 9 << 20
        if kind == "hostmalloc":
            hp = ctypes.c_void_p()
            assert hip.hipHostMalloc(ctypes.byref(hp), ctypes.c_size_t(n), 0) == 0
            ptr, keep = hp.value, None
        else:
            a, keep = arena(kind, n)
            ptr = a.ctypes.data
            assert hip.hipHostRegister(ctypes.c_void_p(ptr), ctypes.c_size_t(n), 0) == 0
        q = ptr + n // 2 + 4096 + 16
        base, size = ctypes.c_void_p(), ctypes.c_size_t()
        rc = hip.hipMemGetAddressRange(ctypes.byref(base), ctypes.byref(size), ctypes.c_void_p(q))
        start, rsize = ctypes.c_void_p(), ctypes.c_size_t()
        rc_s = hip.hipPointerGetAttribute(ctypes.byref(start), 11, ctypes.c_void_p(q))  # HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR
        rc_z = hip.hipPointerGetAttribute(ctypes.byref(rsize), 12, ctypes.c_void_p(q))  # HIP_POINTER_ATTRIBUTE_RANGE_SIZE
        hip.hipGetLastError()
        print(json.dumps({"arena": kind, "registered": n, "range_rc": rc, "range_base_minus_start": (base.value or 0) - ptr,
                          "range_size": size.value, "attr_start_rc": rc_s, "attr_start_minus_start": (start.value or 0) - ptr,
                          "attr_size_rc": rc_z, "attr_size": rsize.value}), flush=True)
        if kind == "hostmalloc":
            hip.hipHostFree(ctypes.c_void_p(ptr))
        else:
            hip.hipHostUnregister(ctypes.c_void_p(ptr))
        del keep


ranges()
for pageable_first in (False, True):
    for kind in ("numpy", "mmap"):
        for C in (65536, 1 << 20):
            for action in ("none", "encode", "decode", "both"):
                case(kind, C, action, pageable_first)
