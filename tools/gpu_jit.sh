# Round 2: VALU mix of RS(20+6) with and without the compiled XOR network, then the c5 sweep.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
B="python bench.py --k 20 --m 6 --chunk 262144 --stripes 4915 --steps 2 --warmup 1 --no-cpu --no-host-path"
LSEC_JIT=0 timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmc_jit0 -o mix -- $B > gpurun_out/pmc_jit0.log 2>&1 && echo ok-jit0 && \
LSEC_JIT=1 timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmc_jit1 -o mix -- $B > gpurun_out/pmc_jit1.log 2>&1 && echo ok-jit1 && \
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/stats_jit1 -o st -- $B > gpurun_out/stats_jit1.log 2>&1 && echo ok-stats && \
timeout -k 10 600 python -u tools/sweep.py --methods reed_sol_van,cauchy_good --out gpurun_out/sweep_c5.jsonl > gpurun_out/sweep_c5.log 2>&1 && echo ok-sweep
