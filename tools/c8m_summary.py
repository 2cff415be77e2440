#!/usr/bin/env python3
"""Summarise tools/gpu_cauchy8m.sh: per config, the encode kernel's HIP-event rate (bench json)
and its counters per launch (rocprofv3 --pmc csv), normalised per MiB of algorithmic traffic."""
import collections
import csv
import glob
import json
import os
import sys

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/c8m"
for tag in ("k20m6c4", "k20m6c8", "k10m4c4", "k10m4c8"):
    b = json.load(open(os.path.join(root, f"bench_{tag}.json")))
    rf = b["roofline"]
    algo = rf["algorithmic_bytes_per_launch"]
    row = {"config": tag, "encode_frac": rf["frac"], "decode_frac": rf.get("decode_frac"),
           "launch_ms": rf["avg_launch_ms"], "algo_MiB": round(algo / 2**20)}
    for grp in ("utcl", "tcc"):
        f = os.path.join(root, f"{grp}_{tag}", "p_counter_collection.csv")
        agg = collections.defaultdict(float)
        disp = collections.defaultdict(set)
        for r in csv.DictReader(open(f)):
            if "bitsliced<" not in r["Kernel_Name"] or r["Kernel_Name"].count("<1,") :
                continue
            if int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0) < 10**6:
                continue  # the bench's parity/warm-up launches on a few stripes
            agg[r["Counter_Name"]] += float(r["Counter_Value"])
            disp[r["Counter_Name"]].add(r["Dispatch_Id"])
        for c, v in agg.items():
            n = len(disp[c])
            row[c] = round(v / n / (algo / 2**20), 3)  # per launch, per MiB of traffic
    hit, miss = row.get("TCC_HIT_sum", 0), row.get("TCC_MISS_sum", 0)
    if hit + miss:
        row["TCC_hit_rate"] = round(hit / (hit + miss), 4)
    th, tm = row.get("TCP_UTCL1_TRANSLATION_HIT_sum", 0), row.get("TCP_UTCL1_TRANSLATION_MISS_sum", 0)
    if th + tm:
        row["UTCL1_miss_rate"] = round(tm / (th + tm), 5)
    print(json.dumps(row))
