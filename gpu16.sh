set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python tools/kbench.py --configs rs63,rs84,rs104,rs164,rs206,cg104 --variants "0,0;5,0;6,0;7,0;8,0" --rounds 3 > gpurun_out/kbench16.log 2>&1 && echo "kbench ok" && \
timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/bench16a.log 2>&1 && echo "bench a ok" && \
LSEC_COPY_THREADS=16 timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/bench16b.log 2>&1 && echo "bench b ok"
