#!/usr/bin/env python3
"""Host-path A/B of the in-place pinning threshold (development probe): et_encode_stripes /
et_decode_stripes of pageable (N, k+m, C) host stripes, ~--gib GiB of user data, with
a knob (default LSEC_PIN_MIN_RUN_KB; also LSEC_KERNEL_COPY) alternating between the given values
call by call (the engine reads both per call), median of --reps per setting.  A decode of one
lost chunk makes a k-chunk input run and a 1-chunk output run per stripe, so its average run is
(k+1)*C/2 and packed under round 1's 4 MiB threshold where the encode's (k+m)*C/2 pinned."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--codes", default="6+3,10+4")
    ap.add_argument("--chunks", default="262144,524288,1048576,2097152")
    ap.add_argument("--settings", default="4096,1024,0", help="values of --env ('-' = unset)")
    ap.add_argument("--env", default="LSEC_PIN_MIN_RUN_KB", help="knob the engine reads per call")
    ap.add_argument("--gib", type=float, default=1.5)
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    import lstore_amd as L

    settings = a.settings.split(",")
    for code in a.codes.split(","):
        k, m = (int(x) for x in code.split("+"))
        for C in [int(x) for x in a.chunks.split(",")]:
            n = max(2, int(a.gib * 2**30 / (k * C)))
            buf = np.empty((n, k + m, C), dtype=np.uint8)
            buf[:] = np.random.default_rng(C).integers(0, 256, (1, k + m, C), dtype=np.uint8)
            gib = k * C * n / 2**30
            t = {s: {"enc": [], "dec": []} for s in settings}
            with L.Plan.for_chunk(L.REED_SOL_VAN, k, m, C) as p:
                p.encode_stripes(buf[:16])
                p.decode_stripes(buf[:16], [0])
                for _ in range(a.reps):
                    for s in settings:
                        if s == "-":
                            os.environ.pop(a.env, None)
                        else:
                            os.environ[a.env] = s
                        t0 = time.perf_counter()
                        p.encode_stripes(buf)
                        t1 = time.perf_counter()
                        p.decode_stripes(buf, [0])
                        t2 = time.perf_counter()
                        t[s]["enc"].append(t1 - t0)
                        t[s]["dec"].append(t2 - t1)
            row = {"k": k, "m": m, "chunk": C, "stripes": n}
            for s in settings:
                med = {x: sorted(v)[len(v) // 2] for x, v in t[s].items()}
                row[f"{a.env}={s}"] = {"encode_gibps": round(gib / med["enc"], 2), "decode_gibps": round(gib / med["dec"], 2)}
            print(json.dumps(row), flush=True)
            del buf


if __name__ == "__main__":
    main()
