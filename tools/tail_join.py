#!/usr/bin/env python3
"""Join a one-thread tools/fnptr_bench.c run's per-call latencies (FNPTR_LAT_OUT) with the engine's
per-call phases (LSEC_TRACE=1 on stderr) and say what the slowest calls spend their time on.

    tools/tail_join.py <trace.txt> <lat.txt> [--match "6 in / 1 out"] [--tail 0.01]

At one thread every call is one route-4 host call, so the last N trace lines of the matching shape
are the N timed calls, in order (the warm-up calls come first).  Prints one JSON line per group
(the slowest `tail` fraction, the rest): latency, each phase's mean (entry / exit: the fn-pointer
call's time before run_host began and after it ended; call: the whole call as the engine saw it), how
many calls paid a registration miss (register > 50 us), and the part of the caller's latency outside
every traced phase (the call's own entry and return, and the trace print itself).
"""
import argparse
import json
import re
import sys

PHASE = re.compile(r"pin ([\d.]+) ms \(query ([\d.]+), register ([\d.]+)\), submit ([\d.]+) ms, drain ([\d.]+) ms, "
                   r"unpin ([\d.]+) ms(?:, entry ([\d.]+) ms, exit ([\d.]+) ms, call ([\d.]+) ms)?")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("lat")
    ap.add_argument("--match", default="6 in / 1 out")
    ap.add_argument("--tail", type=float, default=0.01)
    ap.add_argument("--miss-us", type=float, default=50.0)
    a = ap.parse_args()
    phases = []
    with open(a.trace) as f:
        for line in f:
            if "[lsec trace] host call" in line and a.match in line:
                m = PHASE.search(line)
                if m:
                    phases.append([float(x) * 1e3 if x is not None else 0.0 for x in m.groups()])  # us
    lats = []
    with open(a.lat) as f:
        for line in f:
            t, us = line.split()
            if t == "0":
                lats.append(float(us))
    if len(phases) < len(lats):
        sys.exit(f"{len(phases)} traced calls for {len(lats)} timed ones: not a one-route run")
    rows = list(zip(lats, phases[len(phases) - len(lats):]))
    rows.sort(key=lambda r: r[0])
    cut = max(1, int(round(len(rows) * a.tail)))
    names = ("pin", "query", "register", "submit", "drain", "unpin", "entry", "exit", "call")
    lat_sorted = [r[0] for r in rows]

    def pct(p):
        return round(lat_sorted[min(len(lat_sorted) - 1, int(len(lat_sorted) * p))], 1)

    print(json.dumps({"calls": len(rows), "traced_lines": len(phases), "p50_us": pct(0.5), "p99_us": pct(0.99),
                      "p999_us": pct(0.999), "max_us": round(lat_sorted[-1], 1),
                      "register_miss_frac_all": round(sum(r[1][2] > a.miss_us for r in rows) / len(rows), 4)}))
    for label, grp in (("slowest %g" % a.tail, rows[-cut:]), ("rest", rows[:-cut])):
        n = len(grp)
        mean = [sum(r[1][i] for r in grp) / n for i in range(len(names))]
        outside = sum(r[0] - (r[1][0] + r[1][3] + r[1][4] + r[1][5] + r[1][6] + r[1][7]) for r in grp) / n
        print(json.dumps({"group": label, "calls": n, "latency_mean_us": round(sum(r[0] for r in grp) / n, 1),
                          **{f"{nm}_mean_us": round(v, 1) for nm, v in zip(names, mean)},
                          "outside_phases_mean_us": round(outside, 1),
                          "register_miss_frac": round(sum(r[1][2] > a.miss_us for r in grp) / n, 4),
                          "drain_max_us": round(max(r[1][4] for r in grp), 1)}))


if __name__ == "__main__":
    main()
