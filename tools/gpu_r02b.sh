#!/bin/bash
# Round 2 re-measure after the kernel fix: smoke, headline bench under rocprofv3 (kernel trace +
# stats), a plain bench run (in-run PMC traffic), PMC passes, then the c5 sweep.
#   gpurun --timeout 1200 -- bash tools/gpu_r02b.sh <tag>
set -o pipefail
tag=${1:-run}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "gpurun_out/smoke_${tag}.txt" 2>&1 || { echo "smoke failed"; exit 1; }
echo "smoke ok"
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OLDPWD/gpurun_out/prof_${tag}" -o run -- \
    python "$OLDPWD/bench.py" --json-out "$OLDPWD/gpurun_out/bench_${tag}_rocprof.json") > "gpurun_out/bench_${tag}_rocprof.log" 2>&1 \
    || { echo "bench under rocprof failed"; tail -20 "gpurun_out/bench_${tag}_rocprof.log"; exit 1; }
echo "bench (rocprof) ok"
timeout -k 10 600 python bench.py --json-out "gpurun_out/bench_${tag}.json" > "gpurun_out/bench_${tag}.log" 2>&1 || { echo "bench failed"; exit 1; }
echo "bench ok"
timeout -k 10 600 python tools/pmc_traffic.py "${tag}" > "gpurun_out/pmc_${tag}.log" 2>&1 || { echo "pmc failed"; exit 1; }
echo "pmc ok"
timeout -k 10 600 python -u tools/sweep.py --methods reed_sol_van,cauchy_good --out "gpurun_out/sweep_c5_${tag}.jsonl" > "gpurun_out/sweep_${tag}.log" 2>&1 || { echo "sweep failed"; exit 1; }
echo "sweep ok"
