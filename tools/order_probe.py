#!/usr/bin/env python3
"""Tile-order / shard-layout A/B probe (development tool).

For each configuration, times the encode and single-erasure decode kernels over device-resident
stripes for every (shard pad, tile order) pair, interleaved round by round so box drift hits all
pairs alike; checks parity against the first pair.  Tile orders (ApplyArgs::order, tile_at):
G | rot << 8 -- G stripes column-major per group, rot = per-stripe column rotation.

python tools/order_probe.py --configs rs63,rs104_8m --pads 0,1024 --orders 0,2,4,8 [--rounds 5]
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import lstore_amd as L  # noqa: E402
from lstore_amd import erasure as E  # noqa: E402

CONFIGS = {
    "rs63": (L.REED_SOL_VAN, 6, 3, 1 << 20),
    "cg63": (L.CAUCHY_GOOD, 6, 3, 1 << 20),
    "rs104": (L.REED_SOL_VAN, 10, 4, 1 << 20),
    "rs104_4m": (L.REED_SOL_VAN, 10, 4, 4 << 20),
    "rs104_8m": (L.REED_SOL_VAN, 10, 4, 8 << 20),
    "rs124_8m": (L.REED_SOL_VAN, 12, 4, 8 << 20),
    "cg104_4m": (L.CAUCHY_GOOD, 10, 4, 4 << 20),
    "cg104_8m": (L.CAUCHY_GOOD, 10, 4, 8 << 20),
    "cg164_8m": (L.CAUCHY_GOOD, 16, 4, 8 << 20),
    "cg124_8m": (L.CAUCHY_GOOD, 12, 4, 8 << 20),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="rs63")
    ap.add_argument("--pads", default="0,1024", help="shard pads: P (all shards) or D:P (data rows : parity rows)")
    ap.add_argument("--orders", default="0")
    ap.add_argument("--data-gib", type=float, default=24.0)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    lib = E.lib()
    lib.lsec_set_tile_order.argtypes = [ctypes.c_int]
    lib.lsec_set_tile_order.restype = None
    dev = torch.device("cuda:0")
    stream = torch.cuda.current_stream()
    pads = [x for x in a.pads.split(",")]
    orders = [int(x) for x in a.orders.split(",")]
    out = []
    for name in a.configs.split(","):
        meth, k, m, C = CONFIGS[name]
        N = max(8, int(a.data_gib * 2**30 / (k * C)))
        plan = L.Plan.for_chunk(meth, k, m, C)
        bufs = {}
        for pad in pads:
            dp, pp = (int(x) for x in (pad.split(":") if ":" in pad else (pad, pad)))
            g = torch.Generator(device=dev).manual_seed(7)
            data = torch.randint(0, 256, (N, k, C + dp), dtype=torch.uint8, device=dev, generator=g)[:, :, :C]
            par = torch.empty((N, m, C + pp), dtype=torch.uint8, device=dev)[:, :, :C]
            rb = torch.empty((N, 1, C + pp), dtype=torch.uint8, device=dev)[:, :, :C]
            bufs[pad] = (data, par, rb)
        plan.prepare_decode([0])
        lib.lsec_set_tile_order(0)
        ref = {}
        res = {(p, o): ([], []) for p in pads for o in orders}
        for _ in range(a.rounds):
            for pad in pads:
                data, par, rb = bufs[pad]
                for o in orders:
                    lib.lsec_set_tile_order(o)
                    plan.encode_dev(data, par)
                    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
                    ev[0].record(stream)
                    for _ in range(a.reps):
                        plan.encode_dev(data, par)
                    ev[1].record(stream)
                    for _ in range(a.reps):
                        plan.decode_dev(data, par, [0], out=rb)
                    ev[2].record(stream)
                    torch.cuda.synchronize()
                    res[(pad, o)][0].append(ev[0].elapsed_time(ev[1]) / a.reps)
                    res[(pad, o)][1].append(ev[1].elapsed_time(ev[2]) / a.reps)
                    sample = par[:: max(1, N // 7)].cpu()
                    ref.setdefault(pad, sample)
                    assert torch.equal(sample, ref[pad]), f"{name} pad {pad} order {o}: parity differs"
                    assert torch.equal(rb[:: max(1, N // 7), 0].cpu(), data[:: max(1, N // 7), 0].cpu())
        lib.lsec_set_tile_order(-1)
        for (pad, o), (te, td) in res.items():
            te, td = sorted(te)[len(te) // 2], sorted(td)[len(td) // 2]
            ef, df = (k + m) * C * N / te / 8e9, (k + 1) * C * N / td / 8e9
            rec = {"config": name, "k": k, "m": m, "chunk": C, "stripes": N, "pad": pad, "order": o,
                   "encode_ms": round(te, 4), "decode_ms": round(td, 4), "encode_frac": round(ef, 4),
                   "decode_frac": round(df, 4)}
            out.append(rec)
            print(json.dumps(rec), flush=True)
        del bufs
        plan.close()
        torch.cuda.empty_cache()
    if a.json:
        with open(a.json, "w") as f:
            for r in out:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
