#!/usr/bin/env python3
"""How fast is pinning pageable memory in place (hipHostRegister) compared with copying it
into already-pinned staging?  (development probe)"""
import ctypes as C
import time

import numpy as np

hip = C.CDLL("libamdhip64.so")
hip.hipHostRegister.argtypes = [C.c_void_p, C.c_size_t, C.c_uint]
hip.hipHostUnregister.argtypes = [C.c_void_p]
hip.hipHostMalloc.argtypes = [C.POINTER(C.c_void_p), C.c_size_t, C.c_uint]
hip.hipSetDevice(0)
for mib in (64, 256, 1024):
    n = mib << 20
    buf = np.ones(n, np.uint8)  # touched
    t0 = time.perf_counter()
    rc = hip.hipHostRegister(buf.ctypes.data, n, 0)
    t1 = time.perf_counter()
    rc2 = hip.hipHostUnregister(buf.ctypes.data)
    t2 = time.perf_counter()
    p = C.c_void_p()
    hip.hipHostMalloc(C.byref(p), n, 0)
    dst = np.ctypeslib.as_array((C.c_uint8 * n).from_address(p.value))
    t3 = time.perf_counter()
    np.copyto(dst, buf)
    t4 = time.perf_counter()
    print(f"{mib} MiB: register {n / (t1 - t0) / 1e9:.1f} GB/s (rc {rc}), unregister {n / (t2 - t1) / 1e9:.1f} GB/s (rc {rc2}), "
          f"1-thread memcpy into pinned {n / (t4 - t3) / 1e9:.1f} GB/s", flush=True)
