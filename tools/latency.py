#!/usr/bin/env python3
"""Per-call cost of the unmodified LStore call pattern: plan->encode_block / decode_block once per
stripe (segment/jerasure.c:1847, :245) with host buffers, from T concurrent threads on one plan
(the gop pool, lio_config.c:87), versus the batched et_encode_stripes on the same stripes.
Reports per-call latency and aggregate user-data GiB/s.  (development / measurement tool)
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--chunks", default="16384,65536,1048576")
    ap.add_argument("--threads", default="1,8,32")
    ap.add_argument("--calls", type=int, default=64)
    a = ap.parse_args()
    import lstore_amd as L

    k, m = 6, 3
    for C in (int(x) for x in a.chunks.split(",")):
        with L.Plan.for_chunk(L.CAUCHY_GOOD, k, m, C) as p:
            for T in (int(x) for x in a.threads.split(",")):
                bufs = [np.random.default_rng(t).integers(0, 256, (k + m, C), dtype=np.uint8) for t in range(T)]
                for b in bufs:  # warm staging / images
                    p.encode_block([b[i] for i in range(k + m)])
                lat = [[] for _ in range(T)]

                def worker(t):
                    b = bufs[t]
                    ptrs = [b[i] for i in range(k + m)]
                    for _ in range(a.calls):
                        t0 = time.perf_counter()
                        p.encode_block(ptrs)
                        lat[t].append(time.perf_counter() - t0)

                th = [threading.Thread(target=worker, args=(t,)) for t in range(T)]
                t0 = time.perf_counter()
                for x in th:
                    x.start()
                for x in th:
                    x.join()
                wall = time.perf_counter() - t0
                allv = sorted(v for l in lat for v in l)
                n = T * a.calls
                st = np.zeros((n, k + m, C), np.uint8)
                p.encode_stripes(st[:2])
                t1 = time.perf_counter()
                p.encode_stripes(st)
                tb = time.perf_counter() - t1
                print(json.dumps({"chunk": C, "threads": T, "calls": n,
                                  "per_call_us_p50": round(allv[len(allv) // 2] * 1e6, 1),
                                  "per_call_us_p99": round(allv[int(len(allv) * 0.99)] * 1e6, 1),
                                  "fnptr_gibps": round(n * k * C / wall / 2**30, 3),
                                  "batched_gibps": round(n * k * C / tb / 2**30, 3)}), flush=True)


if __name__ == "__main__":
    main()
