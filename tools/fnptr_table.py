#!/usr/bin/env python3
"""Tabulate tools/fnptr_bench.c JSON lines (gpurun_out/fnptr_*.jsonl): per (op, method, chunk,
threads) the reference, the engine's default small-call path, the dispatcher path and the
page-locked-caller case, GiB/s of user data and p50 / p99 latency per call."""
import json
import sys
from collections import defaultdict


def main():
    g = defaultdict(dict)
    for path in sys.argv[1:]:
        for line in open(path):
            r = json.loads(line)
            key = (r["op"], r["method"], r["chunk"], r["threads"])
            kind = "ref" if r["impl"] == "reference" else ("pin" if r["pinned"] else
                                                          ("disp" if r["small_path"] == "dispatch" else "eng"))
            g[key][kind] = r
    cols = [("ref", "reference"), ("eng", "engine"), ("disp", "dispatcher"), ("pin", "engine, page-locked")]
    print("| op | method | C | threads | " + " | ".join(f"{n} GiB/s (p50 / p99 us)" for _, n in cols) + " |")
    print("|---" * (4 + len(cols)) + "|")
    for key in sorted(g):
        d = g[key]
        cells = []
        for k, _ in cols:
            r = d.get(k)
            cells.append(f"{r['gibps']:.1f} ({r['per_call_us_p50']:.0f} / {r['per_call_us_p99']:.0f})" if r else "-")
        print(f"| {key[0]} | {key[1]} | {key[2] >> 10} KiB | {key[3]} | " + " | ".join(cells) + " |")


if __name__ == "__main__":
    main()
