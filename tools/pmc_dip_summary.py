#!/usr/bin/env python3
"""Summarise tools/pmc_dip.sh: per configuration, the encode kernel's (the longest engine kernel of
the run: the bench's encode moves more bytes than its decode) counters,
median over launches, with the derived ratios of tools/pmc_sq_summary.py.

python tools/pmc_dip_summary.py gpurun_out/dip_<tag> > profiles/<name>.json
"""
import csv
import glob
import json
import os
import re
import statistics
import sys
from collections import defaultdict


def main(d):
    out = {}
    for sub in sorted(glob.glob(os.path.join(d, "*_*"))):
        if not os.path.isdir(sub):
            continue
        cfg, pas = os.path.basename(sub).rsplit("_", 1)
        vals = defaultdict(lambda: defaultdict(list))
        dur = defaultdict(list)
        meta = {}
        for f in glob.glob(os.path.join(sub, "**", "*counter_collection.csv"), recursive=True):
            with open(f) as fh:
                seen = set()
                for r in csv.DictReader(fh):
                    name = r["Kernel_Name"]
                    if "lsec" not in name or "hbm_" in name or "probe" in name:
                        continue
                    vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
                    key = (name, r["Dispatch_Id"])
                    if key not in seen:
                        seen.add(key)
                        dur[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
                        meta[name] = {"grid": int(r["Grid_Size"]), "vgpr": int(r.get("VGPR_Count", 0) or 0),
                                      "lds": int(r.get("LDS_Block_Size", 0) or 0)}
        if not dur:
            continue
        # the encode: the longest kernel (the decode is not in this run; magic/probes excluded above)
        enc = max(dur, key=lambda n: statistics.median(dur[n]))
        rec = out.setdefault(cfg, {"kernel": re.sub(r"\(.*", "", enc)[:120], **meta[enc],
                                   "launch_ms": round(statistics.median(dur[enc]), 4)})
        med = {c: statistics.median(v) for c, v in vals[enc].items()}
        rec.update({c: round(v, 1) for c, v in med.items()})
        if "SQ_WAVES" in med and med["SQ_WAVES"]:
            rec["wave_cycles_per_wave"] = round(med["SQ_WAVE_CYCLES"] / med["SQ_WAVES"], 1)
            rec["vmem_per_wave"] = round((med["SQ_INSTS_VMEM_RD"] + med["SQ_INSTS_VMEM_WR"]) / med["SQ_WAVES"], 2)
            rec["vmem_in_flight"] = round(med["SQ_INST_LEVEL_VMEM"] / med["SQ_BUSY_CYCLES"], 2)
        if "TCP_TCC_READ_REQ_sum" in med and med["TCP_TCC_READ_REQ_sum"]:
            rec["l1_l2_read_latency"] = round(med["TCP_TCC_READ_REQ_LATENCY_sum"] / med["TCP_TCC_READ_REQ_sum"], 1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
