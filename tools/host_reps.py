#!/usr/bin/env python3
"""Host-path calls repeated over the SAME buffer: et_encode_stripes /
et_decode_stripes of a ~1 GiB batch, N times each, per-call wall time and the link fraction of each
direction.  The c5 sweep's host encodes vary 2x from one call to the next over one buffer; this
shows whether a call's rate depends on how recently its pages were moved.  Pageable (numpy) and
page-locked (torch pin_memory = hipHostMalloc) buffers.

python tools/host_reps.py --method reed_sol_van --k 20 --m 6 --chunk 4194304 [--reps 8]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import lstore_amd as L  # noqa: E402
from lstore_amd import erasure as E  # noqa: E402

LINK_GBPS = 57.5  # one direction alone; 48.6 each way with both busy (profiles/r05_v3_duplex_probe.jsonl)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--method", default="reed_sol_van")
    ap.add_argument("--k", type=int, default=20)
    ap.add_argument("--m", type=int, default=6)
    ap.add_argument("--chunk", type=int, default=4 << 20)
    ap.add_argument("--gib", type=float, default=1.0)
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--pinned", action="store_true")
    a = ap.parse_args()
    k, m, C = a.k, a.m, a.chunk
    n = max(2, int(a.gib * 2**30 / (k * C)))
    plan = L.Plan.for_chunk(E.JE_METHOD_NAMES.index(a.method), k, m, C)
    plan.prepare_encode()
    plan.prepare_decode([0])
    if a.pinned:
        import torch
        buf = torch.empty((n, k + m, C), dtype=torch.uint8, pin_memory=True).numpy()
    else:
        buf = np.empty((n, k + m, C), dtype=np.uint8)
    buf[:] = np.random.default_rng(1).integers(0, 256, (1, k + m, C), dtype=np.uint8)
    plan.encode_stripes(buf[:1])
    for op in ("encode", "decode"):
        for i in range(a.reps):
            t0 = time.perf_counter()
            if op == "encode":
                plan.encode_stripes(buf)
            else:
                plan.decode_stripes(buf, [0])
            t = time.perf_counter() - t0
            inb, outb = k * C * n, (m if op == "encode" else 1) * C * n
            print(json.dumps({"op": op, "rep": i, "pinned": a.pinned, "config": f"{a.method}({k}+{m}) {C} B x {n}",
                              "ms": round(t * 1e3, 2), "user_gibps": round(k * C * n / t / 2**30, 2),
                              "h2d_link_frac": round(inb / t / 1e9 / LINK_GBPS, 3),
                              "d2h_link_frac": round(outb / t / 1e9 / LINK_GBPS, 3)}), flush=True)


if __name__ == "__main__":
    main()
