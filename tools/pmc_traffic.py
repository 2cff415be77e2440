#!/usr/bin/env python3
"""Measure HBM traffic of the bench kernels with rocprofv3 PMC counters (development tool).

Two separate passes (MI355X_MICROARCH.md §rocprofv3 PMC slots: FETCH_SIZE and WRITE_SIZE do not
fit one pass), each with --kernel-trace only, over a short bench.py run.  Corrections per
MI355X_MICROARCH.md §HBM: FETCH_SIZE/WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE reports half
the bytes of a wide (16 B/lane) coalesced streaming read, so it is doubled.  The bitsliced
kernel reads 4 B/lane; its FETCH factor is calibrated separately, here we
report raw and corrected values side by side.

Writes profiles/<tag>_pmc_traffic.json.  This process never touches the GPU itself; it only
launches rocprofv3 (with python bench.py after --) as a child.
"""
import csv
import glob
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def run_pass(counter, outdir, bench_args):
    os.makedirs(outdir, exist_ok=True)
    cmd = ["rocprofv3", "--pmc", counter, "--kernel-trace", "--output-format", "csv", "-d", outdir, "-o", "pmc",
           "--", sys.executable, os.path.join(ROOT, "bench.py")] + bench_args
    env = dict(os.environ, TMPDIR="/tmp")
    subprocess.run(cmd, check=True, cwd="/tmp", env=env, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL,
                   timeout=600)
    files = glob.glob(os.path.join(outdir, "**", "*counter_collection.csv"), recursive=True)
    per_kernel = {}
    for f in files:
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row.get("Counter_Name") != counter:
                    continue
                name = row["Kernel_Name"]
                per_kernel.setdefault(name, []).append(float(row["Counter_Value"]))
    return per_kernel


def annotate(res, extra):
    """Geometry of the bench run and, per kernel, algorithmic bytes and traffic per stripe
    (bench.py reads traffic_per_stripe back for its roofline.traffic field)."""
    def arg(name, default):
        return int(extra[extra.index(name) + 1]) if name in extra else default
    k, m, C, N = arg("--k", 6), arg("--m", 3), arg("--chunk", 1 << 20), arg("--stripes", 4096)
    res.update({"bench_stripes": N, "chunk": C, "k": k, "m": m, "pad": arg("--pad", 0)})
    for name, v in res["kernels"].items():
        if "k_hbm_copy" in name:  # bench.py's ceiling probe: (k+m)*C*N/2 bytes read and written
            v["algorithmic"] = (k + m) * C * N
        else:
            R = int(name.split("<")[1].split(",")[0])  # output rows: m (encode) or erased shards (decode)
            v["algorithmic"] = (k + R) * C * N
        v["traffic_over_algorithmic"] = round(v["traffic"] / v["algorithmic"], 4)
        v["traffic_per_stripe"] = v["traffic"] / N


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
    extra = sys.argv[2:]
    bench_args = ["--steps", "2", "--warmup", "1", "--no-cpu", "--no-host-path", "--no-layout-ab", "--no-copy-ref"] + extra
    out = os.path.join(ROOT, "gpurun_out", f"pmc_{tag}")
    fetch = run_pass("FETCH_SIZE", os.path.join(out, "fetch"), bench_args)
    write = run_pass("WRITE_SIZE", os.path.join(out, "write"), bench_args)
    res = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), bench.py " + " ".join(bench_args),
           "units": "bytes per launch; FETCH_SIZE/WRITE_SIZE KiB*1024; fetch_corrected = 2*FETCH (gfx950 16B/lane)",
           "kernels": {}}
    for name in sorted(set(fetch) | set(write)):
        if "lsec" not in name:
            continue
        f = sorted(fetch.get(name, [0]))[len(fetch.get(name, [0])) // 2] * 1024
        w = sorted(write.get(name, [0]))[len(write.get(name, [0])) // 2] * 1024
        res["kernels"][name] = {"fetch_raw": f, "fetch_corrected": 2 * f, "write": w,
                                "traffic": 2 * f + w, "dispatches": len(fetch.get(name, []))}
    annotate(res, extra)
    path = os.path.join(ROOT, "gpurun_out", f"{tag}_pmc_traffic.json")
    with open(path, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
