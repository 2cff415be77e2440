#!/usr/bin/env python3
"""When does each XCD finish the headline kernels?  

tools/probes/xcd_balance.hip showed, on the encode's memory shape with XOR arithmetic, the odd XCDs
(blocks b with b % 8 odd) ending ~6 % later than the even ones.  This runs the engine's own
RS(6+3) 1 MiB encode and single-erasure decode (4096 stripes, one tile per workgroup, static XCD
eighths) with the measurement hook lsec_test_set_stamps: every workgroup writes its end time
(s_memrealtime, 100 MHz) and the per-XCD last end is reported relative to the first workgroup's
end.  Several fresh allocations; tile sharing off and on.

python tools/xcd_stamps.py [--trials 3]
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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=3)
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    k, m, C, N = 6, 3, 1 << 20, 4096
    dev = torch.device("cuda:0")
    st = torch.cuda.current_stream()
    lib = E.lib()
    lib.lsec_test_set_stamps.argtypes = [ctypes.c_void_p, ctypes.c_uint]
    lib.lsec_test_set_stamps.restype = None
    plan = L.Plan.for_chunk(L.REED_SOL_VAN, k, m, C)
    plan.prepare_decode([0])
    nst = 1 << 22
    stamps = torch.zeros(nst, dtype=torch.int64, device=dev)
    out = []
    for trial in range(a.trials):
        torch.cuda.empty_cache()
        spacer = torch.empty(((trial * 37) % 11 + 1) << 28, dtype=torch.uint8, device=dev)
        d = torch.randint(0, 256, (N, k, C), dtype=torch.uint8, device=dev)
        p = torch.empty((N, m, C), dtype=torch.uint8, device=dev)
        r = torch.empty((N, 1, C), dtype=torch.uint8, device=dev)
        del spacer
        for mode in ("static", "shared", "tail"):
            E.set_tile_sharing({"static": E.TILES_STATIC, "shared": E.TILES_SHARED, "tail": E.TILES_TAIL}[mode])
            for op in ("encode", "decode"):
                run = (lambda: plan.encode_dev(d, p)) if op == "encode" else (lambda: plan.decode_dev(d, p, [0], out=r))
                run()
                run()
                stamps.zero_()
                lib.lsec_test_set_stamps(ctypes.c_void_p(stamps.data_ptr()), nst)
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
                ev[0].record(st)
                run()
                ev[1].record(st)
                torch.cuda.synchronize()
                lib.lsec_test_set_stamps(None, 0)
                ms = ev[0].elapsed_time(ev[1])
                s = stamps.cpu()
                nz = torch.nonzero(s).flatten()
                v = s[nz]
                first = int(v.min())
                xcd = (nz % 8)
                last = [round((int(v[xcd == x].max()) - first) / 100.0, 1) for x in range(8)]
                rec = {"trial": trial, "op": op, "tiles": mode, "ms": round(ms, 4),
                       "workgroups": int(nz.numel()), "xcd_last_end_us": last,
                       "spread_us": round(max(last) - min(last), 1),
                       "odd_minus_even_us": round(sum(last[1::2]) / 4 - sum(last[0::2]) / 4, 1)}
                out.append(rec)
                print(json.dumps(rec), flush=True)
        E.set_tile_sharing(E.TILES_TAIL)
        del d, p, r
    if a.json:
        with open(a.json, "w") as f:
            for rec in out:
                f.write(json.dumps(rec) + "\n")


if __name__ == "__main__":
    main()
