set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
C="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmc_mix206 -o mix -- python bench.py --k 20 --m 6 --chunk 262144 --stripes 4915 --steps 2 --warmup 1 --no-cpu --no-host-path > gpurun_out/pmc_mix206.log 2>&1 && echo ok206 && \
timeout -s KILL 120 rocprofv3 --pmc $C --kernel-trace --output-format csv -d gpurun_out/pmc_mix63 -o mix -- python bench.py --steps 2 --warmup 1 --no-cpu --no-host-path > gpurun_out/pmc_mix63.log 2>&1 && echo ok63
