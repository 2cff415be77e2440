#!/bin/bash
# GPU box, round 6: the munmap stall (tools/probes/munmap_evict_probe.cpp; the two-thread fresh-mmap
# per-stripe calls traced), the one-thread tail with entry / exit phases, and the C = 1 vs 8 MiB
# encode counters (tools/pmc_dip.sh).  Each step has its own limit.
#   gpurun --timeout 1200 -- bash tools/gpu_r06c.sh <tag> [evict churn2 tail dip]
set -o pipefail
tag=${1:-r06c}
shift
steps=${*:-evict churn2 tail dip}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for s in $steps; do
  case $s in
    evict)
      timeout -k 10 120 build/munmap_evict_probe > gpurun_out/munmap_evict_${tag}.jsonl || { echo "evict probe failed"; exit 1; }
      cat gpurun_out/munmap_evict_${tag}.jsonl ;;
    churn2)
      LSEC_TRACE=1 FNPTR_FREE_AFTER=2 FNPTR_LAT_OUT=gpurun_out/churn2_lat_${tag}.txt timeout -k 10 60 build/fnptr_bench 1048576 2 1 cauchy_good decode \
        > gpurun_out/churn2_${tag}.json 2> gpurun_out/churn2_trace_${tag}.txt || { echo "churn2 failed"; exit 1; }
      cat gpurun_out/churn2_${tag}.json
      python - "$tag" <<'PY'
import re, sys, statistics
tag = sys.argv[1]
rx = re.compile(r"pin ([\d.]+) ms \(query ([\d.]+), register ([\d.]+)\), submit ([\d.]+) ms, drain ([\d.]+) ms, unpin ([\d.]+) ms, entry ([\d.]+) ms, exit ([\d.]+) ms, call ([\d.]+) ms")
rows = [[float(x) for x in m.groups()] for m in (rx.search(l) for l in open(f"gpurun_out/churn2_trace_{tag}.txt")) if m]
names = ("pin", "query", "register", "submit", "drain", "unpin", "entry", "exit", "call")
print("churn2 traced calls", len(rows))
for i, n in enumerate(names):
    v = sorted(r[i] for r in rows)
    print(f"  {n:9s} median {v[len(v)//2]:.4f} ms  p90 {v[int(len(v)*0.9)]:.4f}  max {v[-1]:.4f}")
PY
      ;;
    tail)
      timeout -k 10 200 bash tools/gpu_fnptr_tail.sh ${tag} || { echo "tail failed"; exit 1; } ;;
    dip)
      timeout -k 10 900 bash tools/pmc_dip.sh ${tag} tcp sq > gpurun_out/dip_${tag}.log 2>&1 || { echo "dip failed"; tail -5 gpurun_out/dip_${tag}.log; exit 1; }
      python tools/pmc_dip_summary.py gpurun_out/dip_${tag} > gpurun_out/dip_summary_${tag}.json && cat gpurun_out/dip_summary_${tag}.json ;;
  esac
done
