#!/usr/bin/env python3
"""Summarise tools/pmc_sq.sh: the encode (and decode) kernels' SQ counters at C = 4 vs 8 MiB.

python tools/pmc_sq_summary.py gpurun_out/sq > profiles/<name>.json

Per configuration and kernel (median over its launches): launch time, waves, wave lifetime
(SQ_WAVE_CYCLES / SQ_WAVES), the share of wave time spent waiting for an instruction's inputs
(SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES) and for anything (SQ_WAIT_ANY / SQ_WAVE_CYCLES), vector-memory
instructions per wave, and the average number of vector-memory instructions in flight
(SQ_INST_LEVEL_VMEM / SQ_BUSY_CYCLES: Little's law over the SQs' busy time).  Also the tile ->
(stripe, column) mapping of the bytewise / bit-sliced kernels at each size: tiles per stripe and
how many stripes one XCD's resident workgroups span at once.
"""
import csv
import glob
import json
import os
import statistics
import sys
from collections import defaultdict

TILE = 256 * 32  # bytes of a shard one workgroup tile covers (2 x 16 B per lane)


def load(d):
    rows = defaultdict(lambda: defaultdict(list))  # kernel -> counter -> [values]
    dur = defaultdict(list)
    info = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            seen = set()
            for r in csv.DictReader(fh):
                name = r["Kernel_Name"]
                if "k_gf8" not in name:
                    continue
                rows[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
                key = (name, r["Dispatch_Id"])
                if key not in seen:
                    seen.add(key)
                    dur[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
                    info[name] = {"vgpr": int(r["VGPR_Count"]), "grid": int(r["Grid_Size"]),
                                  "workgroup": int(r["Workgroup_Size"])}
    return rows, dur, info


def load_all(dirs):
    rows = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    info = {}
    for d in dirs:
        r, du, inf = load(d)
        for k, ctr in r.items():
            for c, v in ctr.items():
                rows[k][c].extend(v)
        for k, v in du.items():
            dur[k].extend(v)
        info.update(inf)
    return rows, dur, info


def summarise(rows, dur, info):
    out = {}
    for name, ctr in rows.items():
        m = {c: statistics.median(v) for c, v in ctr.items()}
        waves = m.get("SQ_WAVES", 0) or 1
        wave_cycles = m.get("SQ_WAVE_CYCLES", 0) or 1
        busy = m.get("SQ_BUSY_CYCLES", 0) or 1
        vgpr = info[name]["vgpr"]
        out[name] = {
            "launches": len(dur[name]), "ms_median": round(statistics.median(dur[name]), 4),
            "vgprs": vgpr, "waves_per_simd_by_vgprs": min(8, 512 // max(8, vgpr)),
            "counters": {c: m[c] for c in sorted(m)},
            "wave_lifetime_cycles": round(wave_cycles / waves, 1),
            "wait_inst_any_share": round(m.get("SQ_WAIT_INST_ANY", 0) / wave_cycles, 4),
            "wait_any_share": round(m.get("SQ_WAIT_ANY", 0) / wave_cycles, 4),
            "vmem_rd_per_wave": round(m.get("SQ_INSTS_VMEM_RD", 0) / waves, 2),
            "vmem_wr_per_wave": round(m.get("SQ_INSTS_VMEM_WR", 0) / waves, 2),
            "vmem_in_flight_avg": round(m.get("SQ_INST_LEVEL_VMEM", 0) / busy, 2),
        }
        if m.get("TCP_TCC_READ_REQ_sum"):
            out[name]["l1_to_l2_read_latency_cycles"] = round(m["TCP_TCC_READ_REQ_LATENCY_sum"] / m["TCP_TCC_READ_REQ_sum"], 1)
    return out


def mapping(chunk, stripes, waves_per_simd):
    tps = chunk // TILE
    resident_per_xcd = 32 * 4 * waves_per_simd // 4  # 32 CUs x 4 SIMDs x waves, 4 waves per 256-lane workgroup
    return {"tiles_per_stripe": tps, "tiles_per_xcd": stripes * tps // 8,
            "resident_workgroups_per_xcd": resident_per_xcd,
            "stripes_spanned_by_one_xcd_at_once": round(resident_per_xcd / tps, 3)}


def main():
    base = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/sq"
    res = {"what": "SQ counters, encode and decode kernels at C = 4 vs 8 MiB, same bytes per launch (tools/pmc_sq.sh)",
           "cases": {}}
    tags = sorted({os.path.basename(d).rsplit("_", 1)[0] if os.path.basename(d).rsplit("_", 1)[-1] in ("sq", "tcp1", "tcp2")
                   else os.path.basename(d) for d in glob.glob(os.path.join(base, "*")) if os.path.isdir(d)})
    for tag in tags:
        rows, dur, info = load_all([d for d in glob.glob(os.path.join(base, tag + "*")) if os.path.isdir(d)])
        s = summarise(rows, dur, info)
        chunk = (8 if tag.endswith("c8") else 4) << 20
        stripes = {"reed_sol_van_k10m4c4": 204, "reed_sol_van_k10m4c8": 102, "cauchy_good_k12m4c4": 170,
                   "cauchy_good_k12m4c8": 85}.get(tag, 0)
        for name, v in s.items():
            v["mapping"] = mapping(chunk, stripes, v["waves_per_simd_by_vgprs"])
        res["cases"][tag] = s
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
