#!/usr/bin/env python3
"""Host-path rate vs chunk size (development probe): et_encode_stripes / et_decode_stripes over
~1 GiB of user data in one (N, k+m, C) host array, median of --reps calls, for pageable and
page-locked callers.  Run once per LSEC_NO_HOST_REGISTER / LSEC_KERNEL_COPY setting
(tools/gpu_host_chunk_ab.sh, tools/gpu_kcopy_ab.sh; kcopy = small runs moved by kernel)."""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--k", type=int, default=6)
    ap.add_argument("--m", type=int, default=3)
    ap.add_argument("--chunks", default="262144,524288,1048576,4194304")
    ap.add_argument("--gib", type=float, default=1.0)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch

    import lstore_amd as L

    mode = ("packed" if os.environ.get("LSEC_NO_HOST_REGISTER") else
            "kcopy" if os.environ.get("LSEC_KERNEL_COPY") == "1" else "inplace")
    k, m = a.k, a.m
    for C in [int(x) for x in a.chunks.split(",")]:
        n = max(2, int(a.gib * 2**30 / (k * C)))
        with L.Plan.for_chunk(L.REED_SOL_VAN, k, m, C) as p:
            for kind in ("pageable", "pinned"):
                if kind == "pinned":
                    buf = torch.empty((n, k + m, C), dtype=torch.uint8, pin_memory=True).numpy()
                else:
                    buf = np.empty((n, k + m, C), dtype=np.uint8)
                buf[:] = np.random.default_rng(C).integers(0, 256, (1, k + m, C), dtype=np.uint8)
                p.encode_stripes(buf[:1])
                te, td = [], []
                for _ in range(a.reps):
                    t0 = time.perf_counter()
                    p.encode_stripes(buf)
                    te.append(time.perf_counter() - t0)
                    t0 = time.perf_counter()
                    p.decode_stripes(buf, [0])
                    td.append(time.perf_counter() - t0)
                gib = k * C * n / 2**30
                print(f"{mode:7s} {kind:8s} C={C:8d} n={n:5d} encode {gib / sorted(te)[a.reps // 2]:6.1f} GiB/s "
                      f"decode {gib / sorted(td)[a.reps // 2]:6.1f} GiB/s", flush=True)
                del buf


if __name__ == "__main__":
    main()
