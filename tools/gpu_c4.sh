set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python bench.py --method cauchy_good --k 10 --m 4 --chunk 4194304 --stripes 614 --no-host-path --cpu-seconds 8 > gpurun_out/c4.log 2>&1 && echo c4-ok && \
timeout -k 10 300 python bench.py --method cauchy_good --k 10 --m 4 --chunk 4194304 --total-stripes 2048 --no-host-path --no-cpu --steps 5 > gpurun_out/c4_strong.log 2>&1 && echo c4s-ok && \
LSEC_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --stripes 1024 --steps 5 --warmup 2 > gpurun_out/r2.log 2>&1 && echo r2-ok
