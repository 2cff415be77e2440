set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu10.log 2>&1 && echo "pytest ok" && \
timeout -k 10 900 python tools/kbench.py --configs rs63,rs104,rs164,rs206 --variants "0,0;1,0;2,0;3,0;4,0" --rounds 3 > gpurun_out/kbench4.log 2>&1 && echo "kbench ok"
