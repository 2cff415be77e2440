set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 500 python tools/pmc_traffic.py r01_rs63 > gpurun_out/pmc_rs63.log 2>&1 && echo "pmc rs ok" && \
timeout -k 10 500 python tools/pmc_traffic.py r01_cg104 --method cauchy_good --k 10 --m 4 --chunk 4194304 --stripes 614 > gpurun_out/pmc_cg104.log 2>&1 && echo "pmc cg ok" && \
LSEC_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 1 --stripes 512 --no-cpu > gpurun_out/bench_2rank.log 2>&1 && echo "2rank ok"
