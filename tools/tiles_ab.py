#!/usr/bin/env python3
"""Work-sharing tiles A/B (lsec_set_tile_sharing): the headline RS(6+3) 1 MiB encode and
single-erasure decode over the SAME fresh allocation, static XCD eighths, all tiles shared and a
static prefix with a shared tail timed alternately, over several fresh allocations; parity and
rebuilt shards compared between the modes.

python tools/tiles_ab.py [--trials 4] [--rounds 4] [--reps 5] [--method reed_sol_van --k 6 --m 3 --chunk 1048576]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import lstore_amd as L  # noqa: E402
from lstore_amd import erasure as E  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=4)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--method", default="reed_sol_van")
    ap.add_argument("--k", type=int, default=6)
    ap.add_argument("--m", type=int, default=3)
    ap.add_argument("--chunk", type=int, default=1 << 20)
    ap.add_argument("--data-gib", type=float, default=24.0)
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    k, m, C = a.k, a.m, a.chunk
    N = int(a.data_gib * 2**30 / (k * C))
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream()
    plan = L.Plan.for_chunk(E.JE_METHOD_NAMES.index(a.method), k, m, C)
    plan.prepare_encode()
    plan.prepare_decode([0])
    out = []
    for trial in range(a.trials):
        torch.cuda.empty_cache()
        spacer = torch.empty(((trial * 37) % 11 + 1) << 28, dtype=torch.uint8, device=dev)
        d = torch.randint(0, 256, (N, k, C), dtype=torch.uint8, device=dev)
        p = torch.empty((N, m, C), dtype=torch.uint8, device=dev)
        r = torch.empty((N, 1, C), dtype=torch.uint8, device=dev)
        del spacer
        times = {"static": ([], []), "shared": ([], []), "tail": ([], [])}
        ref = None
        same = True
        for rnd in range(a.rounds):
            for mode in ("static", "shared", "tail"):
                E.set_tile_sharing({"static": E.TILES_STATIC, "shared": E.TILES_SHARED, "tail": E.TILES_TAIL}[mode])
                plan.encode_dev(d, p)
                plan.decode_dev(d, p, [0], out=r)
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
                ev[0].record(st)
                for _ in range(a.reps):
                    plan.encode_dev(d, p)
                ev[1].record(st)
                for _ in range(a.reps):
                    plan.decode_dev(d, p, [0], out=r)
                ev[2].record(st)
                torch.cuda.synchronize()
                times[mode][0].append(ev[0].elapsed_time(ev[1]) / a.reps)
                times[mode][1].append(ev[1].elapsed_time(ev[2]) / a.reps)
                # parity of sampled stripes identical across modes and rounds; every rebuilt shard
                # equal to the lost one
                sample = p[:: max(1, N // 61)].clone()
                if ref is None:
                    ref = sample
                same &= bool(torch.equal(sample, ref)) and bool(torch.equal(r[:, 0], d[:, 0]))
                del sample
        rec = {"trial": trial, "method": a.method, "k": k, "m": m, "chunk": C, "stripes": N, "identical": same}
        for mode, (te, td) in times.items():
            te_m, td_m = sorted(te)[len(te) // 2], sorted(td)[len(td) // 2]
            rec[mode] = {"encode_ms": round(te_m, 4), "decode_ms": round(td_m, 4),
                         "encode_frac": round((k + m) * C * N / (te_m / 1e3) / 8e12, 4),
                         "decode_frac": round((k + 1) * C * N / (td_m / 1e3) / 8e12, 4)}
        for mode in ("shared", "tail"):
            rec[mode]["encode_gain"] = round(rec["static"]["encode_ms"] / rec[mode]["encode_ms"], 4)
            rec[mode]["decode_gain"] = round(rec["static"]["decode_ms"] / rec[mode]["decode_ms"], 4)
        out.append(rec)
        print(json.dumps(rec), flush=True)
        del d, p, r
    E.set_tile_sharing(E.TILES_TAIL)
    if a.json:
        with open(a.json, "w") as f:
            for rec in out:
                f.write(json.dumps(rec) + "\n")


if __name__ == "__main__":
    main()
