#!/usr/bin/env python3
"""Development probe: can a kernel move host bytes faster than the DMA engines when the
host runs are small?  (evidence for the small-chunk host path)

Pageable numpy memory is pinned in place (hipHostRegister, mapped) and its device alias
(hipHostGetDevicePointer) is handed to lsec_hbm_copy_dev, so the kernel itself reads or
writes host memory over PCIe.  Compared with hipMemcpyAsync of the same registered bytes cut
into runs of 256 KiB .. 64 MiB (one DMA per run, as the staging pipeline issues them).
Every transfer is checked byte-exactly after it is timed.
"""
import ctypes as C
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

from lstore_amd import erasure as E  # noqa: E402

hip = C.CDLL("libamdhip64.so")
hip.hipHostRegister.argtypes = [C.c_void_p, C.c_size_t, C.c_uint]
hip.hipHostUnregister.argtypes = [C.c_void_p]
hip.hipHostGetDevicePointer.argtypes = [C.POINTER(C.c_void_p), C.c_void_p, C.c_uint]
hip.hipMemcpyAsync.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
H2D, D2H = 1, 2
MAPPED = 2  # hipHostRegisterMapped


def timed(fn, stream, reps=3):
    fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        stream.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best


def main():
    lib = E.lib()
    dev = torch.device("cuda:0")
    torch.cuda.set_device(0)
    st = torch.cuda.current_stream()
    sh = st.cuda_stream
    n = 1 << 30
    host = np.random.default_rng(5).integers(0, 256, n, dtype=np.uint8)
    back = np.zeros(n, dtype=np.uint8)
    assert host.ctypes.data % 16 == 0 and back.ctypes.data % 16 == 0
    for b in (host, back):
        rc = hip.hipHostRegister(b.ctypes.data, n, MAPPED)
        assert rc == 0, f"hipHostRegister rc {rc}"
    dh, db = C.c_void_p(), C.c_void_p()
    assert hip.hipHostGetDevicePointer(C.byref(dh), host.ctypes.data, 0) == 0
    assert hip.hipHostGetDevicePointer(C.byref(db), back.ctypes.data, 0) == 0
    d = torch.empty(n, dtype=torch.uint8, device=dev)
    try:
        def kcopy(dst, src):
            if lib.lsec_hbm_copy_dev(dst, src, n, sh):
                raise RuntimeError(E.last_error())

        t = timed(lambda: kcopy(d.data_ptr(), dh.value), st)
        ok = bool(np.array_equal(d.cpu().numpy(), host))
        print(f"kernel reads host (H2D)   {n / t / 1e9:6.1f} GB/s  exact={ok}", flush=True)
        t = timed(lambda: kcopy(db.value, d.data_ptr()), st)
        ok = bool(np.array_equal(back, host))
        print(f"kernel writes host (D2H)  {n / t / 1e9:6.1f} GB/s  exact={ok}", flush=True)
        for run in (256 << 10, 1 << 20, 4 << 20, 16 << 20, 64 << 20):
            def dma(kind):
                for o in range(0, n, run):
                    if kind == H2D:
                        hip.hipMemcpyAsync(d.data_ptr() + o, host.ctypes.data + o, run, H2D, sh)
                    else:
                        hip.hipMemcpyAsync(back.ctypes.data + o, d.data_ptr() + o, run, D2H, sh)
            back[:] = 0
            th, td = timed(lambda: dma(H2D), st), timed(lambda: dma(D2H), st)
            ok = bool(np.array_equal(back, host))
            print(f"DMA runs of {run >> 10:6d} KiB   H2D {n / th / 1e9:6.1f} GB/s   D2H {n / td / 1e9:6.1f} GB/s  "
                  f"exact={ok}", flush=True)
    finally:
        torch.cuda.synchronize()
        for b in (host, back):
            hip.hipHostUnregister(b.ctypes.data)


if __name__ == "__main__":
    main()
