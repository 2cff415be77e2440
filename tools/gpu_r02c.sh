#!/bin/bash
# GPU box, round 2 validation of the tree: GPU tests, smoke, the headline bench under rocprofv3
# (kernel trace + stats), then a plain bench run (in-run PMC traffic).  Every GPU step has its
# own time limit; the first failure ends the script.
#   gpurun --timeout 1200 -- bash tools/gpu_r02c.sh <tag> [skip-tests]
set -o pipefail
tag=${1:-run}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
      > "gpurun_out/pytest_gpu_${tag}.txt" 2>&1 || { echo "gpu tests failed"; tail -30 "gpurun_out/pytest_gpu_${tag}.txt"; exit 1; }
  echo "gpu tests ok: $(tail -1 gpurun_out/pytest_gpu_${tag}.txt)"
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "gpurun_out/smoke_${tag}.txt" 2>&1 || { echo "smoke failed"; exit 1; }
  echo "smoke ok"
fi
(cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OLDPWD/gpurun_out/prof_${tag}" -o run -- \
    python "$OLDPWD/bench.py" --json-out "$OLDPWD/gpurun_out/bench_${tag}_rocprof.json") > "gpurun_out/bench_${tag}_rocprof.log" 2>&1 \
    || { echo "bench under rocprof failed"; tail -20 "gpurun_out/bench_${tag}_rocprof.log"; exit 1; }
echo "bench (rocprof) ok"
timeout -k 10 600 python bench.py --json-out "gpurun_out/bench_${tag}.json" > "gpurun_out/bench_${tag}.log" 2>&1 || { echo "bench failed"; tail -20 "gpurun_out/bench_${tag}.log"; exit 1; }
echo "bench ok"
