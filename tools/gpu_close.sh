#!/bin/bash
# GPU box, closing measurements of a build: GPU tests, smoke, the headline bench under rocprofv3
# (kernel trace + stats; tools/rocpd_stats.py splits it), a plain bench run (in-run PMC
# traffic) and config c1 (segment write / read / inspect vs the reference plumbing).
#   gpurun --timeout 1200 -- bash tools/gpu_close.sh <tag> [steps...]   (steps: tests smoke prof bench c1)
set -o pipefail
tag=${1:-run}
shift
steps=${*:-tests smoke prof bench c1}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for s in $steps; do
  case $s in
    tests)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
        > "gpurun_out/pytest_gpu_${tag}.txt" 2>&1 || { echo "tests failed"; tail -30 "gpurun_out/pytest_gpu_${tag}.txt"; exit 1; }
      tail -1 "gpurun_out/pytest_gpu_${tag}.txt" ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "gpurun_out/smoke_${tag}.txt" 2>&1 \
        || { echo "smoke failed"; tail -20 "gpurun_out/smoke_${tag}.txt"; exit 1; }
      echo "smoke ok" ;;
    prof)
      (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OLDPWD/gpurun_out/prof_${tag}" -o run -- \
          python "$OLDPWD/bench.py" --json-out "$OLDPWD/gpurun_out/bench_${tag}_rocprof.json") > "gpurun_out/bench_${tag}_rocprof.log" 2>&1 \
          || { echo "bench under rocprof failed"; tail -20 "gpurun_out/bench_${tag}_rocprof.log"; exit 1; }
      echo "bench (rocprof) ok" ;;
    bench)
      timeout -k 10 600 python bench.py --json-out "gpurun_out/bench_${tag}.json" > "gpurun_out/bench_${tag}.log" 2>&1 \
        || { echo "bench failed"; tail -20 "gpurun_out/bench_${tag}.log"; exit 1; }
      echo "bench ok" ;;
    c1)
      timeout -k 10 400 python -u tools/c1_depot.py > "gpurun_out/c1_${tag}.log" 2>&1 \
        || { echo "c1 failed"; tail -20 "gpurun_out/c1_${tag}.log"; exit 1; }
      echo "c1 ok" ;;
  esac
done
