#!/usr/bin/env python3
"""Stress of host calls: fresh or reused buffers every iteration (pageable, or caller page-locked
with --pinned), encode and multi-erasure decode through et_*_stripes, every byte checked against
the oracle restatement; --churn recycles host virtual ranges and physical pages between calls,
--small-mix puts stripe-server calls in between.  Prints one JSON line with the mismatch counts.
(It found that GPU kernels reading and writing per-call registrations of pageable memory return
stale bytes under churn, while DMA over the same registrations stays exact: DESIGN.md §1.)

python tools/reg_stress.py [--iters 40] [--reuse] [--k 20 --m 6 --chunk 65536 --stripes 3]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import lstore_amd as L  # noqa: E402
import oracle as O  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=40)
    ap.add_argument("--reuse", action="store_true")
    ap.add_argument("--k", type=int, default=20)
    ap.add_argument("--m", type=int, default=6)
    ap.add_argument("--chunk", type=int, default=65536)
    ap.add_argument("--stripes", type=int, default=3)
    ap.add_argument("--w", type=int, default=8)
    ap.add_argument("--fresh-plan", action="store_true", help="a new plan (new device images) every iteration")
    ap.add_argument("--dev-first", action="store_true", help="a device-resident encode before the host calls")
    ap.add_argument("--offset", type=int, default=-1,
                    help="stripes start this many bytes past a page boundary (-1: wherever numpy puts them)")
    ap.add_argument("--method", default="reed_sol_van")
    ap.add_argument("--small-mix", action="store_true",
                    help="a 16 KiB per-stripe Cauchy(6+3) encode (stripe server) before every large call")
    ap.add_argument("--churn", action="store_true",
                    help="allocate, touch and free other host arrays (64 KiB-8 MiB) between calls, so "
                         "virtual ranges and physical pages are recycled")
    ap.add_argument("--seconds", type=float, default=0, help="run until this much time has passed (iters ignored)")
    ap.add_argument("--caller-registered", action="store_true",
                    help="the stripes in pageable memory the caller hipHostRegister's for the iteration and "
                         "unregisters after it (registrations recycled, as an allocator that pins and unpins its arenas)")
    ap.add_argument("--pinned", action="store_true",
                    help="the stripes in caller page-locked memory: a fresh hipHostMalloc each iteration, the "
                         "previous one hipHostFree'd (page-locked virtual ranges recycled)")
    a = ap.parse_args()
    if a.dev_first:
        import torch
        torch.zeros(1, device="cuda")  # torch's HIP runtime first, as in the tests and bench.py
    k, m, C, n = a.k, a.m, a.chunk, a.stripes
    meth = getattr(L, a.method.upper())
    rng = np.random.default_rng(1)
    bad_enc = bad_dec = 0
    first = None
    lost = list(range(m))
    if a.w != 8:
        lost = [0, 3, 5, 9][:m]

    def new_plan():
        if a.method == "reed_sol_van":
            p = L.Plan.new(meth, C, k, m, a.w, 8, 8)
            assert p.form_encoding_matrix() == 0 and p.form_decoding_matrix() == 0
        else:
            p = L.Plan.for_chunk(meth, k, m, C, a.w)
        p.prepare_encode()
        p.prepare_decode(lost)
        return p

    p = new_plan()
    small = L.Plan.for_chunk(L.CAUCHY_GOOD, 6, 3, 16384) if a.small_mix else None
    pool = []
    bad_small = 0
    import time
    t_end = time.time() + a.seconds if a.seconds > 0 else None
    it = -1
    if True:
        buf = None
        while True:
            it += 1
            if (t_end is None and it >= a.iters) or (t_end is not None and time.time() > t_end):
                break
            if a.churn:
                for _ in range(int(rng.integers(1, 4))):
                    if pool and (len(pool) > 8 or rng.random() < 0.5):
                        pool.pop(int(rng.integers(0, len(pool))))
                    else:
                        x = np.empty(int(rng.integers(1 << 16, 8 << 20)), np.uint8)
                        x[::4096] = 1
                        pool.append(x)
            if small is not None:
                sd = rng.integers(0, 256, (9, 16384), dtype=np.uint8)
                sd[6:] = 0
                small.encode_block([sd[i] for i in range(9)])
                if not np.array_equal(sd[6:], O.encode(L.CAUCHY_GOOD, sd[:6], 3, small.packet_size)):
                    bad_small += 1
            if a.fresh_plan and it:
                p.close()
                p = new_plan()
            if a.dev_first:
                import torch
                d = torch.from_numpy(rng.integers(0, 256, (n, k, C), dtype=np.uint8)).cuda()
                par = torch.empty((n, m, C), dtype=torch.uint8, device="cuda")
                p.encode_dev(d, par)
                torch.cuda.synchronize()
            if a.pinned and (buf is None or not a.reuse):
                import ctypes
                hip = ctypes.CDLL("libamdhip64.so")
                nb = n * (k + m) * C
                ptr = ctypes.c_void_p()
                assert hip.hipHostMalloc(ctypes.byref(ptr), ctypes.c_size_t(nb), ctypes.c_uint(0)) == 0
                if buf is not None:
                    old = buf
                    buf = None
                    hip.hipHostFree(ctypes.c_void_p(old.ctypes.data))
                    del old
                buf = np.ctypeslib.as_array((ctypes.c_uint8 * nb).from_address(ptr.value)).reshape(n, k + m, C)
            elif a.caller_registered:
                import ctypes
                hip = ctypes.CDLL("libamdhip64.so")
                if buf is not None:
                    hip.hipHostUnregister(ctypes.c_void_p(reg_base))
                raw = np.empty(n * (k + m) * C + 8192, np.uint8)
                at = (-raw.ctypes.data) % 4096
                buf = raw[at:at + n * (k + m) * C].reshape(n, k + m, C)
                reg_base = buf.ctypes.data
                assert hip.hipHostRegister(ctypes.c_void_p(reg_base), ctypes.c_size_t(buf.nbytes), ctypes.c_uint(0)) == 0
            elif buf is None or not a.reuse:
                if a.offset < 0:
                    buf = np.empty((n, k + m, C), np.uint8)
                else:  # a page-aligned allocation, viewed a.offset bytes in
                    raw = np.empty(n * (k + m) * C + a.offset + 8192, np.uint8)
                    at = (-raw.ctypes.data) % 4096 + a.offset
                    buf = raw[at:at + n * (k + m) * C].reshape(n, k + m, C)
            buf[:, :k] = rng.integers(0, 256, (n, k, C), dtype=np.uint8)
            buf[:, k:] = 0x5A
            want = np.stack([O.encode(meth, buf[s, :k], m, p.packet_size, a.w) for s in range(n)])
            if small is not None:
                small.encode_block([sd[i] for i in range(9)])
            p.encode_stripes(buf)
            if not np.array_equal(buf[:, k:], want):
                bad_enc += 1
                buf[:, k:] = want
            full = buf.copy()
            buf[:, lost] = 0x33
            if small is not None:
                small.encode_block([sd[i] for i in range(9)])
            p.decode_stripes(buf, lost)
            if not np.array_equal(buf, full):
                bad_dec += 1
                if first is None:
                    d = np.argwhere(buf != full)
                    first = {"iter": it, "n_bytes": int(len(d)), "first": d[0].tolist(), "last": d[-1].tolist()}
    p.close()
    if small is not None:
        small.close()
    print(json.dumps({"k": k, "m": m, "w": a.w, "chunk": C, "stripes": n, "iters": it, "reuse": a.reuse,
                      "small_mix": a.small_mix, "churn": a.churn, "pinned": a.pinned, "caller_registered": a.caller_registered, "bad_small": bad_small, "server": os.environ.get("LSEC_SERVER", ""),
                      "fresh_plan": a.fresh_plan, "dev_first": a.dev_first, "offset": a.offset, "method": a.method, "bad_encode": bad_enc, "bad_decode": bad_dec,
                      "first_bad": first}), flush=True)


if __name__ == "__main__":
    main()
