# Cauchy-good encode at C = 4 / 8 MiB, unpadded vs 1 KiB shard-row pad, alternating runs.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/c8m
for rep in 1 2; do
for cfg in "20 6 4194304 102" "20 6 8388608 51" "10 4 4194304 204" "10 4 8388608 102"; do
  set -- $cfg
  for pad in 0 1024; do
    tag="k$1m$2c$(( $3 >> 20 ))p${pad}r$rep"
    timeout -k 10 120 python bench.py --method cauchy_good --k $1 --m $2 --chunk $3 --stripes $4 --pad $pad --steps 5 --warmup 1 \
      --no-cpu --no-host-path --no-layout-ab --no-copy-ref --json-out gpurun_out/c8m/pad_$tag.json > gpurun_out/c8m/pad_$tag.log 2>&1 || exit 1
    python -c "import json;d=json.load(open('gpurun_out/c8m/pad_$tag.json'));print('$tag', d['roofline']['frac'], d['roofline']['decode_frac'])"
  done
done
done
