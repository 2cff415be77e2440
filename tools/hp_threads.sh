cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for t in 4 8 12 16; do
  LSEC_COPY_THREADS=$t timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu --stripes 1024 > gpurun_out/hp_$t.log 2>&1 || exit 1
done
echo done
