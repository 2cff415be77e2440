#!/usr/bin/env python3
"""Tabulate tools/fnptr_bench.c JSON lines (gpurun_out/fnptr_*.jsonl, e.g. from
tools/gpu_fnptr_fair.sh): per (op, method, chunk, threads) the reference (oracle/_ref, the real
Jerasure) and the engine (pageable or page-locked buffers, and any environment the run set), GiB/s
of user data with p50 / p99 latency per call.  Several lines of one kind are averaged
(gpu_fnptr_fair.sh times the reference twice per case).

python tools/fnptr_table.py gpurun_out/fnptr_fair_<tag>.jsonl [...]
"""
import json
import sys
from collections import defaultdict


def cell(rs):
    mean = lambda f: sum(r[f] for r in rs) / len(rs)  # noqa: E731
    return f"{mean('gibps'):.1f} ({mean('per_call_us_p50'):.0f} / {mean('per_call_us_p99'):.0f})", mean("gibps")


def main():
    ref = defaultdict(list)
    eng = defaultdict(list)
    for path in sys.argv[1:]:
        for line in open(path):
            r = json.loads(line)
            key = (r["op"], r["method"], r["chunk"], r["threads"])
            fa = r.get("free_after", 0)  # the harness's buffer lifetime: compared like with like
            if r["impl"] == "reference":
                ref[key + (fa,)].append(r)
            else:
                env = r.get("env", "").strip()
                eng[key + (("page-locked " if r["pinned"] else "") + env, fa)].append(r)
    print("| op | method | C | threads | engine run | reference GiB/s (p50 / p99 us) | engine GiB/s (p50 / p99 us) | engine / reference |")
    print("|---|---|---|---|---|---|---|---|")
    for key in sorted(eng, key=lambda k: (k[0], k[1], k[2], k[3], k[4])):
        rk = key[:4] + (key[5],)
        rc, rv = cell(ref[rk]) if ref.get(rk) else ("-", None)
        ec, ev = cell(eng[key])
        ratio = f"{ev / rv:.2f}" if rv else "-"
        print(f"| {key[0]} | {key[1]} | {key[2] >> 10} KiB | {key[3]} | {key[4] or 'default'} | {rc} | {ec} | {ratio} |")


if __name__ == "__main__":
    main()
