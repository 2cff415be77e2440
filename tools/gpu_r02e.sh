#!/bin/bash
# GPU box, round 2 closing measurements of the current build: headline bench under rocprofv3
# (kernel trace + stats), a plain bench run (in-run PMC traffic), and config c1 (segment write /
# read / inspect, engine vs the reference plumbing).
set -o pipefail
tag=${1:-run}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OLDPWD/gpurun_out/prof_${tag}" -o run -- \
    python "$OLDPWD/bench.py" --json-out "$OLDPWD/gpurun_out/bench_${tag}_rocprof.json") > "gpurun_out/bench_${tag}_rocprof.log" 2>&1 \
    || { echo "bench under rocprof failed"; tail -20 "gpurun_out/bench_${tag}_rocprof.log"; exit 1; }
echo "bench (rocprof) ok"
timeout -k 10 600 python bench.py --json-out "gpurun_out/bench_${tag}.json" > "gpurun_out/bench_${tag}.log" 2>&1 || { echo "bench failed"; tail -20 "gpurun_out/bench_${tag}.log"; exit 1; }
echo "bench ok"
timeout -k 10 400 python -u tools/c1_depot.py > "gpurun_out/c1_${tag}.log" 2>&1 || { echo "c1 failed"; tail -20 "gpurun_out/c1_${tag}.log"; exit 1; }
echo "c1 ok"
