set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -x > gpurun_out/pytest_gpu17.log 2>&1 && echo "pytest ok" && \
timeout -k 10 900 python tools/kbench.py --configs rs63,rs84,rs104,rs124,rs164,rs206 --variants "0,0" --rounds 3 --magic > gpurun_out/kbench17.log 2>&1 && echo "kbench ok" && \
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof17 -o run -- python bench.py > gpurun_out/bench17.log 2>&1 && echo "bench ok"
