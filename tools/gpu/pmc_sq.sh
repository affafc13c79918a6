set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
export ZKP_SERIAL=1
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/pmc_sq -o run -- python3 bench.py --steps 2 --warmup 1 --cpu-baseline none --no-kernels > gpurun_out/pmc_sq.log 2>&1
