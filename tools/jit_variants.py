#!/usr/bin/env python3
"""Compile the XOR networks of a matrix code offline for every LSEC_JIT_VARIANT given and print
the kernel resource usage (VGPRs, spills, occupancy) and the VALU instruction count of the
tile loop.  Needs build/jit_src (tools/jit_src.cpp)."""
import argparse
import os
import re
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--km", default="20+6")
    ap.add_argument("--method", default="reed_sol_van")
    ap.add_argument("--variants", default="0,1,2,3,0x41,0x40")
    ap.add_argument("--w", type=int, default=8)
    a = ap.parse_args()
    import oracle as O
    from lstore_amd import erasure as E
    k, m = (int(x) for x in a.km.split("+"))
    M = np.array(O.coding_matrix(E.JE_METHOD_NAMES.index(a.method), k, m, a.w), dtype=np.int64).reshape(m, k)
    M &= (1 << a.w) - 1
    if a.w == 32:
        M = M[:8]  # a network takes at most 8 rows (the encode binds all m rows)
    inp = f"{M.shape[0]} {k} {a.w} " + " ".join(map(str, M.flatten()))
    os.makedirs(os.path.join(ROOT, "build", "jit"), exist_ok=True)
    for v in a.variants.split(","):
        v = int(v, 0)
        env = dict(os.environ, LSEC_JIT_VARIANT=str(v))
        src = subprocess.run([os.path.join(ROOT, "build", "jit_src")], input=inp, capture_output=True, text=True,
                             env=env, check=True).stdout
        base = os.path.join(ROOT, "build", "jit", f"{a.method}_{k}_{m}_w{a.w}_v{v:#x}")
        open(base + ".hip", "w").write(src)
        r = subprocess.run(["hipcc", "-c", "--offload-arch=gfx950", "-O3", "--cuda-device-only", "-S", "-include", "hip/hip_runtime.h",
                            "-Rpass-analysis=kernel-resource-usage", "-o", base + ".s", base + ".hip"],
                           capture_output=True, text=True)
        if r.returncode:
            print(f"{v:#x} compile failed:\n{r.stderr[:1500]}")
            continue
        res = {}
        for key in ("VGPRs", "AGPRs", "SGPRs Spill", "VGPRs Spill", "Occupancy"):
            mm = re.search(key + r"[^:]*: (\d+)", r.stderr)
            res[key] = int(mm.group(1)) if mm else None
        asm = open(base + ".s").read()
        valu = len(re.findall(r"^\s+v_", asm, re.M))
        print(f"variant {v:#x}: {res}, v_ instructions {valu}")


if __name__ == "__main__":
    main()
