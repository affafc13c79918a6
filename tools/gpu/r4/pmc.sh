# round 4: PMC passes (one counter group per run, kernel trace off) of one short bench command for
# the per-launch VALU instructions per mixed addition and HBM bytes (tools/prof/pmc_launch.py)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4/pmc
B="python3 bench.py --steps 4 --warmup 1 --cpu-baseline none --batch 0 --no-kernels --no-bool0-line"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INSTS_SALU --output-format csv -d gpurun_out/r4/pmc/sq -o run -- $B > gpurun_out/r4/pmc/sq.json 2> gpurun_out/r4/pmc/sq.err
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r4/pmc/fetch -o run -- $B > gpurun_out/r4/pmc/fetch.json 2> gpurun_out/r4/pmc/fetch.err
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r4/pmc/write -o run -- $B > gpurun_out/r4/pmc/write.json 2> gpurun_out/r4/pmc/write.err
