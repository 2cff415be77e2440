#!/usr/bin/env python3
"""Shard-pad A/B in ONE allocation (development tool for the C = 8 MiB encode dip).

python tools/pad_ab.py --configs rs84c8,cg164c8 --pads 0,262144,1048576 [--rounds 5] [--data-gib 16]

Per configuration one data and one parity allocation sized for the largest pad; every pad is a view
of the same allocations (shard row j of stripe s at (s*k + j) * (C + pad)), so every pad draws the
same physical pages (placement moves whole allocations by up to 8 %, DESIGN.md §2, which swamps a
per-allocation A/B).  Rounds interleave the pads; prints the median encode / decode launch time per
pad (HIP events on the launch stream) and checks every pad's parity against pad 0's.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

import torch  # noqa: E402

import lstore_amd as L  # noqa: E402
from kbench import CONFIGS  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="rs84c8,cg164c8,cg206c8,rs84")
    ap.add_argument("--pads", default="0,262144,1048576")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--data-gib", type=float, default=16.0)
    ap.add_argument("--pad-on", default="both", choices=("both", "data", "parity"),
                    help="pad only the data rows (the reads) or only the parity rows (the writes)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    pads = [int(x) for x in a.pads.split(",")]
    big = max(pads)
    stream = torch.cuda.current_stream()
    for name in a.configs.split(","):
        meth, k, m, C = CONFIGS[name][:4]
        N = max(8, int(a.data_gib * 2**30 / (k * C)))
        plan = L.Plan.for_chunk(meth, k, m, C)
        plan.prepare_encode()
        plan.prepare_decode([0])
        fd = torch.randint(0, 256, (N * k * (C + big),), dtype=torch.uint8, device=dev)
        fp = torch.empty((N * m * (C + big),), dtype=torch.uint8, device=dev)
        out = torch.empty((N, 1, C), dtype=torch.uint8, device=dev)
        views = {}
        for pad in pads:
            pd = pad if a.pad_on in ("both", "data") else 0
            pp = pad if a.pad_on in ("both", "parity") else 0
            d = fd[: N * k * (C + pd)].view(N, k, C + pd)[:, :, :C]
            p = fp[: N * m * (C + pp)].view(N, m, C + pp)[:, :, :C]
            views[pad] = (d, p)
        # the same data bytes under every pad: copy pad 0's chunks into each padded view
        d0 = views[pads[0]][0].clone()
        times = {pad: ([], []) for pad in pads}
        ref = None
        for _ in range(a.rounds):
            for pad in pads:
                d, p = views[pad]
                d.copy_(d0)
                plan.encode_dev(d, p)
                e0, e1, e2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
                e0.record(stream)
                for _ in range(a.reps):
                    plan.encode_dev(d, p)
                e1.record(stream)
                for _ in range(a.reps):
                    plan.decode_dev(d, p, [0], out=out)
                e2.record(stream)
                torch.cuda.synchronize()
                times[pad][0].append(e0.elapsed_time(e1) / a.reps)
                times[pad][1].append(e1.elapsed_time(e2) / a.reps)
                if ref is None:
                    ref = p.clone()
                assert torch.equal(p, ref), f"{name}: pad {pad} changed the parity"
                assert torch.equal(out[:, 0], d[:, 0]), f"{name}: pad {pad} decode mismatch"
        eb, db = (k + m) * C * N, (k + 1) * C * N
        for pad in pads:
            te = sorted(times[pad][0])[len(times[pad][0]) // 2]
            td = sorted(times[pad][1])[len(times[pad][1]) // 2]
            print(f"{name:8s} N={N:5d} pad={pad:8d} ({a.pad_on})  encode {te:7.3f} ms ({eb / te / 8e9:5.1%})   "
                  f"decode {td:7.3f} ms ({db / td / 8e9:5.1%})", flush=True)
        del fd, fp, out, views, d0, ref
        torch.cuda.empty_cache()
        plan.close()


if __name__ == "__main__":
    main()
