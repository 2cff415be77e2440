#!/bin/bash
# GPU-box run of one build: the GPU tests, the 1-GPU headline, a 2-rank self-launched rehearsal
# (both ranks on the box's one GPU, control plane over gloo: per-rank + aggregate host path) and
# the c4 strong split over 2 ranks.  Every step has its own time limit; the first failure ends it.
#   gpurun --timeout 1200 -- bash tools/gpu_round.sh <tag> [steps...]   (steps: tests bench ranks c4)
set -o pipefail
tag=${1:-run}
shift
steps=${*:-tests bench ranks c4}
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for s in $steps; do
  case $s in
    tests)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread \
        > "gpurun_out/pytest_gpu_${tag}.txt" 2>&1 || { echo "tests failed"; tail -30 "gpurun_out/pytest_gpu_${tag}.txt"; exit 1; }
      tail -2 "gpurun_out/pytest_gpu_${tag}.txt" ;;
    bench)
      timeout -k 10 420 python bench.py --json-out "gpurun_out/bench_${tag}.json" > "gpurun_out/bench_${tag}.log" 2>&1 \
        || { echo "bench failed"; tail -20 "gpurun_out/bench_${tag}.log"; exit 1; }
      echo "bench ok" ;;
    ranks)
      timeout -k 10 300 python bench.py --gpus 2 --share-gpus --steps 10 --json-out "gpurun_out/bench2_${tag}.json" \
        > "gpurun_out/bench2_${tag}.log" 2>&1 || { echo "2-rank bench failed"; tail -20 "gpurun_out/bench2_${tag}.log"; exit 1; }
      echo "2-rank ok" ;;
    c4)
      timeout -k 10 300 python bench.py --method cauchy_good --k 10 --m 4 --chunk 4194304 --total-stripes 2048 --gpus 2 --share-gpus \
        --steps 10 --json-out "gpurun_out/c4_2rank_${tag}.json" > "gpurun_out/c4_2rank_${tag}.log" 2>&1 \
        || { echo "c4 2-rank failed"; tail -20 "gpurun_out/c4_2rank_${tag}.log"; exit 1; }
      echo "c4 2-rank ok" ;;
  esac
done
