#!/usr/bin/env python3
"""Development probe: host-path call time by call pattern (round 5, c5 host lows).  One ~1 GiB
pageable batch; `--pattern` is a string of E (et_encode_stripes) and D (et_decode_stripes, shard 0
erased), run in order; `--dev-first` runs the sweep's device-resident phase (8 GiB of torch
tensors, freed with empty_cache) before the host calls, as tools/sweep.py does.  One JSON line per
call.  Set LSEC_TRACE=1 for the engine's per-call phase line.

python tools/probes/host_pattern.py --km 8+3 --chunk 524288 --pattern EEEDDDEDEDED [--dev-first]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import lstore_amd as L  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--km", default="8+3")
    ap.add_argument("--chunk", type=int, default=512 << 10)
    ap.add_argument("--pattern", default="EEEDDDEDEDED")
    ap.add_argument("--dev-first", action="store_true")
    ap.add_argument("--tag", default="")
    ap.add_argument("--keep-cache", action="store_true", help="free the device phase's tensors to torch's cache only")
    ap.add_argument("--sleep", type=float, default=0.0, help="seconds to wait after the device phase")
    a = ap.parse_args()
    k, m = (int(x) for x in a.km.split("+"))
    C = a.chunk
    p = L.Plan.for_chunk(L.REED_SOL_VAN, k, m, C)
    p.prepare_encode()
    p.prepare_decode([0])
    if a.dev_first:
        N = int(8 * 2**30 / (k * C))
        d = torch.randint(0, 256, (N, k, C), dtype=torch.uint8, device="cuda")
        par = torch.empty((N, m, C), dtype=torch.uint8, device="cuda")
        p.encode_dev(d, par)
        torch.cuda.synchronize()
        del d, par
        if not a.keep_cache:
            torch.cuda.empty_cache()
        time.sleep(a.sleep)
    n = max(2, (1 << 30) // (k * C))
    buf = np.empty((n, k + m, C), dtype=np.uint8)
    buf[:] = np.random.default_rng(1).integers(0, 256, (1, k + m, C), dtype=np.uint8)
    p.encode_stripes(buf[:1])
    for i, op in enumerate(a.pattern):
        t0 = time.perf_counter()
        if op == "E":
            p.encode_stripes(buf)
        else:
            p.decode_stripes(buf, [0])
        t = time.perf_counter() - t0
        print(json.dumps({"tag": a.tag, "km": a.km, "chunk": C, "dev_first": a.dev_first, "keep_cache": a.keep_cache, "sleep": a.sleep, "i": i, "op": op,
                          "ms": round(t * 1e3, 2), "user_gibps": round(k * C * n / t / 2**30, 2)}), flush=True)


if __name__ == "__main__":
    main()
