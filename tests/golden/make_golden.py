#!/usr/bin/env python3
"""Generate the committed golden fixtures from the REAL reference.

Runs in the build container only (needs /root/reference): it loads
oracle/_ref/libjerasure_ref.so -- vendor/jerasure + src/lio/raid4.c compiled from the
unmodified reference sources by oracle/Makefile, driven through the plan-service
dispatch restated in oracle/ref_harness.c -- and records what the reference computes:

  plans.json         coding matrix, bitmatrix (rows as hex), smart-schedule length and
                     SHA-256 per (method, k, m, w)
  vectors.json       per-case parity CRC32 / first 16 bytes, decode return codes
  parity_small.npz   full parity bytes for the small cases (numpy, no pickle)

Inputs are the deterministic patterns of tests/patterns.py, so only outputs are stored.
Usage:  python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import sys
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(HERE))

import oracle as O  # noqa: E402
from patterns import affine, stripe  # noqa: E402

NAMES = ["reed_sol_van", "reed_sol_r6_op", "cauchy_orig", "cauchy_good", "blaum_roth",
         "liberation", "liber8tion", "raid4"]
SWEEP_KM = [(4, 2), (6, 3), (8, 3), (8, 4), (10, 4), (12, 4), (16, 4), (20, 6)]


def plan_entries():
    out = []
    for k, m in SWEEP_KM:
        for meth in (O.REED_SOL_VAN, O.CAUCHY_ORIG, O.CAUCHY_GOOD):
            out.append((meth, k, m, 8))
    out += [(O.REED_SOL_R6_OP, 6, 2, 8), (O.REED_SOL_R6_OP, 10, 2, 8),
            (O.CAUCHY_GOOD, 2, 2, 8), (O.CAUCHY_GOOD, 32, 2, 8), (O.CAUCHY_GOOD, 3, 5, 8),
            (O.REED_SOL_VAN, 3, 5, 8), (O.REED_SOL_VAN, 32, 8, 8),
            (O.LIBERATION, 6, 2, 7), (O.BLAUM_ROTH, 6, 2, 6), (O.LIBER8TION, 6, 2, 8),
            # wide stripes (k + m = 128, 256 at w = 8) and word sizes past 32 (k > 31 liberation)
            (O.REED_SOL_VAN, 100, 28, 8), (O.CAUCHY_GOOD, 100, 28, 8), (O.REED_SOL_VAN, 200, 56, 8),
            (O.LIBERATION, 37, 2, 37), (O.BLAUM_ROTH, 36, 2, 36)]
    # wide fields (erasure_tools.c:806-811 accepts w = 16 / 32 for the matrix methods)
    for w in (16, 32):
        out += [(O.REED_SOL_VAN, 6, 3, w), (O.REED_SOL_VAN, 10, 4, w), (O.REED_SOL_R6_OP, 6, 2, w),
                (O.CAUCHY_ORIG, 6, 3, w), (O.CAUCHY_GOOD, 6, 3, w), (O.CAUCHY_GOOD, 10, 4, w),
                (O.CAUCHY_GOOD, 4, 2, w)]
    return out


def bits_hex(row):
    s = "".join(str(int(b)) for b in row)
    s += "0" * (-len(s) % 4)
    return "%0*x" % (len(s) // 4, int(s, 2))


def make_plans():
    plans = []
    for meth, k, m, w in plan_entries():
        rp = O.RefPlan(meth, k, m, w, 8)
        mat, bm, sch = rp.matrix(), rp.bitmatrix(), rp.schedule()
        e = dict(method=meth, name=NAMES[meth], k=k, m=m, w=w,
                 matrix=None if mat is None else mat.tolist(),
                 bitmatrix_hex=None if bm is None else [bits_hex(r) for r in bm],
                 bitmatrix_ones=None if bm is None else int(bm.sum()),
                 schedule_ops=None if sch is None else int(len(sch)),
                 schedule_sha256=None if sch is None else hashlib.sha256(
                     np.ascontiguousarray(sch, dtype="<i4").tobytes()).hexdigest())
        if sch is not None and len(sch) <= 400:
            e["schedule"] = sch.tolist()
        plans.append(e)
        rp.close()
    return plans


def cases():
    c = []
    # (method, k, m, w, C, P, pattern)
    for pat in ("affine", "splitmix"):
        c += [(O.REED_SOL_VAN, 6, 3, 8, 1024, 0, pat), (O.CAUCHY_GOOD, 6, 3, 8, 1024, 16, pat),
              (O.CAUCHY_GOOD, 10, 4, 8, 4096, 64, pat), (O.REED_SOL_VAN, 10, 4, 8, 4096, 0, pat),
              (O.CAUCHY_ORIG, 6, 3, 8, 1024, 16, pat), (O.REED_SOL_R6_OP, 6, 2, 8, 1024, 0, pat),
              (O.RAID4, 6, 1, 8, 1024, 0, pat)]
    for k, m in SWEEP_KM:
        c += [(O.REED_SOL_VAN, k, m, 8, 4096, 0, "splitmix"), (O.CAUCHY_GOOD, k, m, 8, 4096, 64, "splitmix"),
              (O.CAUCHY_ORIG, k, m, 8, 2048, 32, "splitmix")]
    # BASELINE geometries (CRC only): c1 64 KiB (P=1024), c2/c3 1 MiB, c4 4 MiB (P=4096), c5 256 KiB
    c += [(O.REED_SOL_VAN, 6, 3, 8, 65536, 0, "splitmix"), (O.CAUCHY_GOOD, 6, 3, 8, 65536, 1024, "splitmix"),
          (O.REED_SOL_VAN, 6, 3, 8, 1 << 20, 0, "splitmix"), (O.CAUCHY_GOOD, 6, 3, 8, 1 << 20, 4096, "splitmix"),
          (O.CAUCHY_GOOD, 10, 4, 8, 4 << 20, 4096, "splitmix"), (O.REED_SOL_VAN, 10, 4, 8, 4 << 20, 0, "splitmix"),
          (O.REED_SOL_VAN, 20, 6, 8, 256 << 10, 0, "splitmix"), (O.CAUCHY_GOOD, 20, 6, 8, 256 << 10, 4096, "splitmix"),
          (O.CAUCHY_GOOD, 16, 4, 8, 256 << 10, 4096, "splitmix"), (O.CAUCHY_GOOD, 4, 2, 8, 256 << 10, 4096, "splitmix"),
          (O.CAUCHY_GOOD, 6, 3, 8, 196608, 3072, "splitmix"), (O.CAUCHY_GOOD, 6, 3, 8, 16384, 256, "splitmix")]
    # bitmatrix families (not on the configs; fixtures for the next row)
    c += [(O.LIBERATION, 6, 2, 7, 7 * 64 * 4, 64, "splitmix"), (O.BLAUM_ROTH, 6, 2, 6, 6 * 64 * 4, 64, "splitmix"),
          (O.LIBER8TION, 6, 2, 8, 8 * 64 * 4, 64, "splitmix")]
    # wide stripes: k + m = 128 and 256 at w = 8 (more inputs than one kernel launch takes), and
    # liberation / blaum_roth past w = 32 (k > 31: w = 37, 67; blaum_roth w + 1 = 37 prime)
    c += [(O.REED_SOL_VAN, 100, 28, 8, 4096, 0, "splitmix"), (O.CAUCHY_GOOD, 100, 28, 8, 4096, 64, "splitmix"),
          (O.REED_SOL_VAN, 200, 56, 8, 2048, 0, "splitmix"), (O.CAUCHY_ORIG, 120, 8, 8, 2048, 32, "splitmix"),
          (O.LIBERATION, 37, 2, 37, 37 * 32 * 2, 32, "splitmix"), (O.LIBERATION, 33, 2, 37, 37 * 64, 64, "affine"),
          (O.LIBERATION, 67, 2, 67, 67 * 32, 32, "splitmix"), (O.BLAUM_ROTH, 36, 2, 36, 36 * 32 * 2, 32, "splitmix")]
    # wide fields: little-endian uint16 / uint32 elements (matrix codes), w*P super-packets (Cauchy)
    for w in (16, 32):
        for pat in ("affine", "splitmix"):
            c += [(O.REED_SOL_VAN, 6, 3, w, 1024, 0, pat), (O.CAUCHY_GOOD, 6, 3, w, 1024, 1024 // w, pat)]
        c += [(O.REED_SOL_VAN, 10, 4, w, 4096, 0, "splitmix"), (O.REED_SOL_R6_OP, 6, 2, w, 1024, 0, "splitmix"),
              (O.CAUCHY_ORIG, 6, 3, w, 2048, 2048 // w, "splitmix"), (O.CAUCHY_GOOD, 10, 4, w, 4096, 64, "splitmix"),
              (O.REED_SOL_VAN, 6, 3, w, 65536, 0, "splitmix")]
    return c


def erasure_sets(k, m):
    s = [[0], [k - 1], [k]]
    if m >= 2:
        s += [[k + 1], [0, k + 1], [1, k - 2]]
    if m >= 3:
        s += [[0, 3, k + 2], list(range(k, k + m)), [2, k]]
    s.append(list(range(m + 1)))  # one too many -> rc -1
    return s


def main():
    plans = make_plans()
    vectors, small = [], {}
    for idx, (meth, k, m, w, size, P, pat) in enumerate(cases()):
        data = affine(k, size) if pat == "affine" else stripe(k, size, 0)
        rp = O.RefPlan(meth, k, m, w, P)
        par = rp.encode(data)
        full = np.vstack([data, par])
        dec = []
        if size <= (4 << 20):  # every geometry up to c4's 4 MiB chunks
            for er in erasure_sets(k, m):
                sh = full.copy()
                for e in er:
                    sh[e] = 0
                rc = rp.decode(sh, er)
                ok = bool((sh == full).all())
                if meth == O.RAID4 and rc == 0 and all(e >= k for e in er):
                    ok = None  # raid4_decode returns early on parity loss (raid4.c:52)
                ent = dict(erasures=er, rc=int(rc), recovered=ok)
                if rc == 0:  # CRC32 of what the reference rebuilt, erased shards in ascending order
                    ent["rebuilt_crc32"] = ["%08x" % zlib.crc32(sh[e].tobytes()) for e in sorted(set(er))]
                dec.append(ent)
        rp.close()
        key = None
        if size * m <= 12 * 1024:
            key = "case%03d" % idx
            small[key] = par
        vectors.append(dict(method=meth, name=NAMES[meth], k=k, m=m, w=w, size=size, packet=P,
                            pattern=pat, parity_crc32=["%08x" % zlib.crc32(par[i].tobytes()) for i in range(m)],
                            parity_head=[par[i][:16].tobytes().hex() for i in range(m)],
                            full=key, decode=dec))
        print(f"case {idx}: {NAMES[meth]} {k}+{m} C={size} P={P} {pat}", flush=True)
    with open(os.path.join(HERE, "plans.json"), "w") as f:
        json.dump(dict(source="oracle/_ref/libjerasure_ref.so (vendor/jerasure 1.2A + src/lio/raid4.c)",
                       plans=plans), f, indent=0)
    with open(os.path.join(HERE, "vectors.json"), "w") as f:
        json.dump(dict(source="oracle/_ref/libjerasure_ref.so", generator="tests/golden/make_golden.py",
                       vectors=vectors), f, indent=0)
    np.savez_compressed(os.path.join(HERE, "parity_small.npz"), **small)


if __name__ == "__main__":
    main()
