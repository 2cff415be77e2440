set -o pipefail
O=gpurun_out/tiles_c; mkdir -p $O
LSEC_TRACE=1 timeout -k 10 300 python tools/tiles_ab.py --trials 2 --json $O/ab_default.jsonl > $O/ab_default.log 2>&1 || exit 1
LSEC_TILES_WGS=8 timeout -k 10 300 python tools/tiles_ab.py --trials 2 --json $O/ab_wgs8.jsonl > $O/ab_wgs8.log 2>&1 || exit 1
LSEC_TILES_WGS=16 timeout -k 10 300 python tools/tiles_ab.py --trials 2 --json $O/ab_wgs16.jsonl > $O/ab_wgs16.log 2>&1 || exit 1
echo ok ab
bash tools/gpu_c5_lows.sh r5a
