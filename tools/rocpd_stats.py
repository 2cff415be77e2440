#!/usr/bin/env python3
"""Kernel-trace summary per (kernel, grid) from rocprofv3 output: the rocpd database (the
default output on ROCm 7.2) or the --output-format csv kernel trace.

python tools/rocpd_stats.py gpurun_out/prof_x/run_results.db [out.csv] [--all]
python tools/rocpd_stats.py gpurun_out/prof_x/run_kernel_trace.csv [out.csv] [--all]
python tools/rocpd_stats.py gpurun_out/prof_x/run_results.db out.csv --first=33

--first=N splits each (kernel, grid) group by launch order into its first N launches and the
rest (column Phase: "first<N>" / "rest").  For a default bench.py run N = 33 separates the
padded-layout launches (3 warm-up + 20 steps + 10 HIP-event reps) from the unpadded
re-timing (1 + 10), so the "first" row compares directly with roofline.avg_launch_ms.

Writes Name,GridX,Calls,AverageNs,MinNs,MaxNs,VGPRs,SGPRs per (kernel, grid) -- the same
columns as the profiles/*_kernel_stats.csv summaries -- for the engine's kernels (lsec::)
unless --all is given.  Per grid, because one kernel name is launched at several batch sizes.
"""
import csv
import sqlite3
import sys


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    every = "--all" in sys.argv
    if args[0].endswith(".csv"):
        groups = {}
        for r in csv.DictReader(open(args[0])):
            key = (r["Kernel_Name"], int(r["Grid_Size_X"]))
            d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            g = groups.setdefault(key, [[], 0, 0])
            g[0].append(d)
            g[1] = max(g[1], int(r["VGPR_Count"]) + int(r["Accum_VGPR_Count"]))
            g[2] = max(g[2], int(r["SGPR_Count"]))
        rows = [(n, gx, len(v), sum(v) / len(v), min(v), max(v), vg, sg) for (n, gx), (v, vg, sg) in groups.items()]
        rows.sort(key=lambda r: -r[2] * r[3])
    else:
        db = sqlite3.connect(args[0])
        rows = db.execute(
            "select name, grid_x, count(*), avg(duration), min(duration), max(duration), "
            "max(vgpr_count + accum_vgpr_count), max(sgpr_count) from kernels group by name, grid_x "
            "order by sum(duration) desc").fetchall()
    first = next((int(a.split("=", 1)[1]) for a in sys.argv[1:] if a.startswith("--first=")), 0)
    if first:
        per = {}
        if args[0].endswith(".csv"):
            recs = sorted(csv.DictReader(open(args[0])), key=lambda r: int(r["Start_Timestamp"]))
            launches = ((r["Kernel_Name"], int(r["Grid_Size_X"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                         int(r["VGPR_Count"]) + int(r["Accum_VGPR_Count"]), int(r["SGPR_Count"])) for r in recs)
        else:
            launches = db.execute("select name, grid_x, duration, vgpr_count + accum_vgpr_count, sgpr_count "
                                  "from kernels order by start")
        for name, gx, d, vg, sg in launches:
            per.setdefault((name, gx), []).append((d, vg, sg))
        rows = []
        for (name, gx), v in per.items():
            for tag, part in (("first%d" % first, v[:first]), ("rest", v[first:])):
                if part:
                    ds = [x[0] for x in part]
                    rows.append((name, gx, len(ds), sum(ds) / len(ds), min(ds), max(ds), part[0][1], part[0][2], tag))
        rows.sort(key=lambda r: -r[2] * r[3])
    out = open(args[1], "w", newline="") if len(args) > 1 else sys.stdout
    w = csv.writer(out, quoting=csv.QUOTE_MINIMAL)
    w.writerow(["Name", "GridX", "Calls", "AverageNs", "MinNs", "MaxNs", "VGPRs", "SGPRs"] + (["Phase"] if first else []))
    for r in rows:
        if every or "lsec::" in r[0]:
            w.writerow([r[0], r[1], r[2], round(r[3], 1), r[4], r[5], r[6], r[7]] + list(r[8:]))


if __name__ == "__main__":
    main()
