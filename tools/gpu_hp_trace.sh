set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
LSEC_TRACE=1 timeout -k 10 300 python tools/sweep.py --km 8+4,6+3,16+4 --chunks 262144,524288,4194304 --methods reed_sol_van --dev-gib 1 --out gpurun_out/hp_trace.jsonl > gpurun_out/hp_trace.log 2>&1
