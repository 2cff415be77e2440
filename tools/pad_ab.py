#!/usr/bin/env python3
"""Shard-padding A/B in one process (development tool): the same RS / Cauchy encode + decode
over [N][k][C + pad] layouts, timing rounds interleaved so box drift hits both sides.

python tools/pad_ab.py [--config rs63] [--pads 0,256,4096] [--rounds 6]
HBM GB/s = algorithmic bytes (k+m)*C*N (encode), (k+1)*C*N (decode) / launch time.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import lstore_amd as L  # noqa: E402

CONFIGS = {"rs63": (L.REED_SOL_VAN, 6, 3, 1 << 20, 4096), "cg104": (L.CAUCHY_GOOD, 10, 4, 4 << 20, 614)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="rs63")
    ap.add_argument("--pads", default="0,256,4096")
    ap.add_argument("--rounds", type=int, default=6)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--stripes", type=int, default=0, help="override the config's stripe count")
    a = ap.parse_args()
    meth, k, m, C, N = CONFIGS[a.config]
    N = a.stripes or N
    pads = [int(x) for x in a.pads.split(",")]
    dev = torch.device("cuda:0")
    plan = L.Plan.for_chunk(meth, k, m, C)
    bufs = {}
    base = torch.randint(0, 256, (N, k, C), dtype=torch.uint8, device=dev)
    for pad in pads:
        d = torch.empty((N, k, C + pad), dtype=torch.uint8, device=dev)[:, :, :C]
        d.copy_(base)
        p = torch.empty((N, m, C + pad), dtype=torch.uint8, device=dev)[:, :, :C]
        o = torch.empty((N, 1, C + pad), dtype=torch.uint8, device=dev)[:, :, :C]
        bufs[len(bufs)] = (d, p, o)
    st = torch.cuda.current_stream()
    del base
    res = {i: ([], []) for i in range(len(pads))}
    for _ in range(a.rounds):
        for i, pad in enumerate(pads):
            d, p, o = bufs[i]
            plan.encode_dev(d, p)
            ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            ev[0].record(st)
            for _ in range(a.reps):
                plan.encode_dev(d, p)
            ev[1].record(st)
            for _ in range(a.reps):
                plan.decode_dev(d, p, [0], out=o)
            ev[2].record(st)
            torch.cuda.synchronize()
            res[i][0].append(ev[0].elapsed_time(ev[1]) / a.reps)
            res[i][1].append(ev[1].elapsed_time(ev[2]) / a.reps)
            assert torch.equal(o[:, 0], d[:, 0])
    ref = bufs[0][1]
    for i in range(1, len(pads)):
        assert torch.equal(bufs[i][1], ref), "parity differs between layouts"
    for i, pad in enumerate(pads):
        te = sorted(res[i][0])[a.rounds // 2]
        td = sorted(res[i][1])[a.rounds // 2]
        eb, db = (k + m) * C * N, (k + 1) * C * N
        print(f"{a.config} pad={pad:6d}  encode {te:.3f} ms {eb / te / 1e6:7.1f} GB/s ({eb / te / 8e9:5.1%})  "
              f"decode {td:.3f} ms {db / td / 1e6:7.1f} GB/s ({db / td / 8e9:5.1%})", flush=True)


if __name__ == "__main__":
    main()
