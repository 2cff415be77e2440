#!/usr/bin/env python3
"""BASELINE config c1: RS(6+3) encode of 1000 x 64 KiB stripes through the segment write path,
and the segment read / inspection paths over the images it wrote.

The reference's c1 runs src/lio over vendor/jerasure into loopback IBP depots.  IBP
(APR/ZMQ/leveldb) cannot be built offline, so the depots are files:
  reference  oracle/_ref ref_segment_write: segjerase_write_func's per-stripe loop restated
             over the real jerasure encode_block + zlib adler32 magic + LUN placement
  engine     lsec_segment_write: one call, parity + magic on the GPU
Both produce k+m device images; they must be byte-identical.  Rates are user-data GiB/s,
with and without writing the images to depot files (--depot-dir, default /tmp).

Then, over the same images, reference harness vs engine:
  read        segjerase_read_func's verification (lsec_segment_read): clean, paranoid (every
              stripe verified), and degraded (device 0's magic stale in every stripe: quorum,
              rebuild of one chunk per stripe, verification)
  inspect     segjerase_inspect_full_func (lsec_segment_inspect) over the LUN records with
              one silently corrupted byte in every 25th stripe (brute-force search)
Outputs (user data, stripe status, bad-device maps) must be identical.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def write_depots(dev, dirname, tag):
    t0 = time.perf_counter()
    for i in range(dev.shape[0]):
        with open(os.path.join(dirname, f"{tag}_depot{i}.bin"), "wb") as f:
            f.write(dev[i].tobytes())
            f.flush()
            os.fsync(f.fileno())
    return time.perf_counter() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--stripes", type=int, default=1000)
    ap.add_argument("--chunk", type=int, default=64 << 10)
    ap.add_argument("--k", type=int, default=6)
    ap.add_argument("--m", type=int, default=3)
    ap.add_argument("--method", default="reed_sol_van")
    ap.add_argument("--n-shift", type=int, default=1)
    ap.add_argument("--depot-dir", default="/tmp")
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()

    import lstore_amd as L
    import oracle as O
    from lstore_amd import erasure as E

    meth = E.JE_METHOD_NAMES.index(a.method)
    k, m, C, N = a.k, a.m, a.chunk, a.stripes
    rng = np.random.default_rng(0x4C53544F5245)
    data = rng.integers(0, 256, (N, k, C), dtype=np.uint8)
    gib = k * C * N / 2**30

    plan = L.Plan.for_chunk(meth, k, m, C)
    rp = O.RefPlan(meth, k, m, 8, plan.packet_size)

    # the depots' buffers: allocated and touched once, reused by every rep (an image allocation
    # per call would time the kernel's zeroing of fresh pages, for the reference and engine alike)
    n = k + m
    ref = np.zeros((n, N * (C + 4)), np.uint8)
    ours = np.zeros((n, N * (C + 4)), np.uint8)
    ref.fill(1)
    ours.fill(1)
    par = np.ones((N, m, C), np.uint8)
    mag = np.ones((N, 4), np.uint8)
    flat = np.ascontiguousarray(data.reshape(-1))
    plan.segment_write(data[:2], a.n_shift, 0)  # warm staging / device images
    plan.segment_encode_iov([flat[:2 * k * C]], 2, C)
    t_ref, t_eng, t_iov = [], [], []
    for _ in range(a.reps):
        t0 = time.perf_counter()
        rp.segment_write(data, N, C, a.n_shift, 0, out=ref)
        t_ref.append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        plan.segment_write(data, a.n_shift, 0, out=ours)
        t_eng.append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        iovs, _, _, keep = plan.segment_encode_iov([flat], N, C, parity=par, magic=mag)
        t_iov.append(time.perf_counter() - t0)
    # the iovec stream, placed by the LUN rule, must give the same images
    stream = np.concatenate([np.frombuffer((ctypes.c_uint8 * int(ln)).from_address(int(b)), np.uint8)
                             for b, ln in iovs])
    rec = stream.reshape(N, n, C + 4)
    placed = np.empty_like(ours)
    for d in range(n):
        rows = placed[d].reshape(N, C + 4)
        for s_ in range(N):
            rows[s_] = rec[s_, (d + s_ * a.n_shift) % n]
    iov_identical = bool(np.array_equal(placed, ref))
    identical = bool(np.array_equal(ref, ours))
    t_io_ref = write_depots(ref, a.depot_dir, "c1ref")
    t_io_eng = write_depots(ours, a.depot_dir, "c1eng")
    for tag in ("c1ref", "c1eng"):
        for i in range(k + m):
            os.remove(os.path.join(a.depot_dir, f"{tag}_depot{i}.bin"))
    tr, te, ti = min(t_ref), min(t_eng), min(t_iov)
    paths = verify_paths(plan, rp, ours, N, C, k, m, a.n_shift, a.reps) if identical else {}
    print(json.dumps({
        "config": "c1", "workload": f"{a.method}({k}+{m}) segment write, {N} stripes x C={C} B, n_shift={a.n_shift}",
        "images_identical": identical,
        "reference_cpu_gibps": round(gib / tr, 3), "reference_cores": 1,
        "engine_gibps": round(gib / te, 3),
        "engine_iov_gibps": round(gib / ti, 3), "iov_stream_identical": iov_identical,
        "reference_with_depot_files_gibps": round(gib / (tr + t_io_ref), 3),
        "engine_with_depot_files_gibps": round(gib / (te + t_io_eng), 3),
        "depot_dir": a.depot_dir,
        "note": "reference = segjerase_write_func loop over real jerasure + zlib (oracle/_ref), into depot "
                "images; engine = lsec_segment_write into the same images (GPU parity + magic, host memory in/out, "
                "PCIe included); engine_iov = lsec_segment_encode_iov, the reference's own hand-off (parity + magic "
                "on the GPU, iovecs into the user data, no image copies); images preallocated for all three",
        "read_inspect": paths,
    }), flush=True)
    if not identical or not iov_identical or not all(v.get("identical") for v in paths.values()):
        sys.exit(1)


def timed(fn, reps):
    best, out = None, None
    for _ in range(reps):
        t0 = time.perf_counter()
        out = fn()
        t = time.perf_counter() - t0
        best = t if best is None else min(best, t)
    return best, out


def verify_paths(plan, rp, img, N, C, k, m, n_shift, reps):
    """Read (clean / paranoid / degraded) and inspection: reference harness vs engine."""
    n, lc = k + m, C + 4
    gib = k * C * N / 2**30
    res = {}
    degraded = img.copy()
    degraded[0].reshape(N, lc)[:, 0] ^= 0x11          # device 0: stale magic in every stripe
    for name, im, par in (("read_clean", img, 0), ("read_paranoid", img, 1), ("read_degraded", degraded, 0)):
        tr, (rout, rst, rbad) = timed(lambda: rp.segment_read(im, N, C, n_shift, 0, par, 1), reps)
        te, (out, st, bad) = timed(lambda: plan.segment_read(im, N, C, n_shift, 0, paranoid=bool(par)), reps)
        res[name] = {"identical": bool(np.array_equal(out, rout) and np.array_equal(st, rst) and bad == rbad),
                     "reference_cpu_gibps": round(gib / tr, 3), "engine_gibps": round(gib / te, 3),
                     "stripes_recovered": int((st == 1).sum())}
    # LUN records [N][n][C+4] (device d holds logical chunk (d + s*n_shift) % n of stripe s)
    rec = np.empty((N, n, lc), np.uint8)
    for d in range(n):
        rows = img[d].reshape(N, lc)
        for s in range(N):
            rec[s, (d + s * n_shift) % n] = rows[s]
    rng = np.random.default_rng(25)
    for s in range(0, N, 25):                         # silent corruption: one byte of one chunk
        rec[s, int(rng.integers(0, n)), 4 + int(rng.integers(0, C))] ^= 0x5A
    tr, (rst, rbm, _, rcnt, _) = timed(lambda: rp.segment_inspect(rec.copy(), N, C, 1, 0), reps)
    te, (st, bm, _, state) = timed(lambda: plan.segment_inspect(rec.copy(), C), reps)
    res["inspect"] = {"identical": bool(np.array_equal(st, rst) and np.array_equal(bm, rbm) and
                                        state.bad_stripes == rcnt[0] and state.silent_errors == rcnt[2]),
                      "reference_cpu_gibps": round(gib / tr, 3), "engine_gibps": round(gib / te, 3),
                      "stripes_repaired": int((st == 3).sum())}
    return res


if __name__ == "__main__":
    main()
