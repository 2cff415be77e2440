#!/usr/bin/env python3
"""Stress of host calls served in place (registered zero-copy route): fresh or reused pageable
buffers every iteration, encode and multi-erasure decode through et_*_stripes, every byte checked
against the oracle restatement.  Prints one JSON line with the mismatch count.

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
    if True:
        buf = None
        for it in range(a.iters):
            if a.fresh_plan and it:
                p.close()
                p = new_plan()
            if a.dev_first:
                import torch
                d = torch.from_numpy(rng.integers(0, 256, (n, k, C), dtype=np.uint8)).cuda()
                par = torch.empty((n, m, C), dtype=torch.uint8, device="cuda")
                p.encode_dev(d, par)
                torch.cuda.synchronize()
            if buf is None or not a.reuse:
                if a.offset < 0:
                    buf = np.empty((n, k + m, C), np.uint8)
                else:  # a page-aligned allocation, viewed a.offset bytes in
                    raw = np.empty(n * (k + m) * C + a.offset + 8192, np.uint8)
                    at = (-raw.ctypes.data) % 4096 + a.offset
                    buf = raw[at:at + n * (k + m) * C].reshape(n, k + m, C)
            buf[:, :k] = rng.integers(0, 256, (n, k, C), dtype=np.uint8)
            buf[:, k:] = 0x5A
            want = np.stack([O.encode(meth, buf[s, :k], m, p.packet_size, a.w) for s in range(n)])
            p.encode_stripes(buf)
            if not np.array_equal(buf[:, k:], want):
                bad_enc += 1
                buf[:, k:] = want
            full = buf.copy()
            buf[:, lost] = 0x33
            p.decode_stripes(buf, lost)
            if not np.array_equal(buf, full):
                bad_dec += 1
                if first is None:
                    d = np.argwhere(buf != full)
                    first = {"iter": it, "n_bytes": int(len(d)), "first": d[0].tolist(), "last": d[-1].tolist()}
    p.close()
    print(json.dumps({"k": k, "m": m, "w": a.w, "chunk": C, "stripes": n, "iters": a.iters, "reuse": a.reuse,
                      "fresh_plan": a.fresh_plan, "dev_first": a.dev_first, "reg_zc": os.environ.get("LSEC_REG_ZC", ""),
                      "reg_flags": os.environ.get("LSEC_REG_FLAGS", ""), "offset": a.offset, "method": a.method, "bad_encode": bad_enc, "bad_decode": bad_dec,
                      "first_bad": first}), flush=True)


if __name__ == "__main__":
    main()
