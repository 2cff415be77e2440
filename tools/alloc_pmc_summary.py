#!/usr/bin/env python3
"""Summarise tools/gpu_alloc_modes.sh: per counter pass, join each encode / decode launch's
counters (rocprofv3 --pmc, dispatch order) to the probe's trials, and set the low-rate trials
against the high-rate ones.

python tools/alloc_pmc_summary.py gpurun_out/alloc [--json out.json]

A trial made exactly `reps` encodes (k_gf8_bytewise<3,...>) then `reps` decodes
(k_gf8_bytewise<1,...>); launch i of a kind belongs to trial i // reps.  Launch time is the
counter record's own (End - Start).  For each pass: per trial the median launch time and the median
of each counter, then the Pearson correlation of every counter with the launch time over the
trials, and the ratio of the counter's mean over the slowest third of trials to that over the
fastest third.  Counters that are per-launch constants (bytes) read 1.0; a placement mechanism
shows as a counter that moves with the time.
"""
import argparse
import csv
import glob
import json
import os
import statistics as st
from collections import defaultdict

ENC, DEC = "k_gf8_bytewise<3,", "k_gf8_bytewise<1,"


def load_pass(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        return None
    launches = {ENC: {}, DEC: {}}  # kind -> dispatch id -> {"t": ms, counter: value}
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                name = r["Kernel_Name"]
                kind = ENC if ENC in name else DEC if DEC in name else None
                if kind is None:
                    continue
                rec = launches[kind].setdefault(int(r["Dispatch_Id"]), {})
                rec["t"] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
                rec[r["Counter_Name"]] = rec.get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    return {kind: [v for _, v in sorted(m.items())] for kind, m in launches.items()}


def pearson(x, y):
    if len(x) < 3:
        return None
    mx, my = st.mean(x), st.mean(y)
    sx = sum((a - mx) ** 2 for a in x) ** 0.5
    sy = sum((b - my) ** 2 for b in y) ** 0.5
    return None if sx == 0 or sy == 0 else round(sum((a - mx) * (b - my) for a, b in zip(x, y)) / (sx * sy), 3)


def summarise(launches, reps):
    out = {}
    for kind, label in ((ENC, "encode"), (DEC, "decode")):
        ls = launches[kind]
        trials = defaultdict(list)
        for i, rec in enumerate(ls):
            trials[i // reps].append(rec)
        rows = []
        for t, recs in sorted(trials.items()):
            recs = recs[1:] if label == "encode" and len(recs) > 2 else recs  # first encode: cold parity pages
            keys = sorted({k for r in recs for k in r if k != "t"})
            rows.append({"trial": t, "ms": round(st.median(r["t"] for r in recs), 4),
                         **{k: st.median(r[k] for r in recs if k in r) for k in keys}})
        if not rows:
            continue
        ms = [r["ms"] for r in rows]
        order = sorted(range(len(rows)), key=lambda i: ms[i])
        third = max(1, len(rows) // 3)
        fast, slow = order[:third], order[-third:]
        keys = sorted(k for k in rows[0] if k not in ("trial", "ms"))
        corr = {}
        for k in keys:
            v = [r.get(k, 0.0) for r in rows]
            mf, msl = st.mean(v[i] for i in fast), st.mean(v[i] for i in slow)
            corr[k] = {"r_with_time": pearson(v, ms), "slow_over_fast": round(msl / mf, 4) if mf else None,
                       "fast_mean": mf, "slow_mean": msl}
        out[label] = {"trials": rows, "ms_fast_mean": round(st.mean(ms[i] for i in fast), 4),
                      "ms_slow_mean": round(st.mean(ms[i] for i in slow), 4), "counters": corr}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--json", default="")
    a = ap.parse_args()
    res = {}
    for d in sorted(glob.glob(os.path.join(a.dir, "*"))):
        if not os.path.isdir(d):
            continue
        ls = load_pass(d)
        if not ls:
            continue
        res[os.path.basename(d)] = summarise(ls, a.reps)
    for name, r in res.items():
        for label, s in r.items():
            print(f"== {name} {label}: fast third {s['ms_fast_mean']} ms, slow third {s['ms_slow_mean']} ms "
                  f"({len(s['trials'])} trials)")
            for k, c in sorted(s["counters"].items(), key=lambda kv: -abs(kv[1]["r_with_time"] or 0)):
                print(f"   {k:44s} r={c['r_with_time']!s:>7}  slow/fast={c['slow_over_fast']}")
    if a.json:
        with open(a.json, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
