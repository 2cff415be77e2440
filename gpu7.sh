set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu7.log 2>&1 && echo "pytest ok" && \
timeout -k 10 300 python tools/c1_depot.py > gpurun_out/c1.log 2>&1 && echo "c1 ok"
