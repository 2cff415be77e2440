set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu11.log 2>&1 && echo "pytest ok" && \
timeout -k 10 300 python tools/latency.py > gpurun_out/latency.log 2>&1 && echo "latency ok" && \
timeout -k 10 300 python bench.py > gpurun_out/bench11.log 2>&1 && echo "bench ok" && \
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof11" -o run --output-format csv -- python "$GRAFT_REPO_ROOT/bench.py" --steps 10 --warmup 2 --no-cpu --no-host-path > "$GRAFT_REPO_ROOT/gpurun_out/prof11.log" 2>&1 && echo "prof ok"
