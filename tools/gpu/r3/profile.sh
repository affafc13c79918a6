# round 3 profiles of HEAD: concurrent + serial kernel traces of the headline loop (rocprofv3
# --kernel-trace --stats), FETCH/WRITE/SQ counter passes (one pass each), summaries made on the box
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
B="python3 bench.py --steps 4 --warmup 1 --cpu-baseline none --no-kernels --batch 0"
W=/tmp/zkp_prof
rm -rf $W && mkdir -p $W
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $W/conc -o run -- $B > gpurun_out/prof/conc.log 2>&1
ZKP_SERIAL=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $W/ser -o run -- $B > gpurun_out/prof/ser.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $W/fetch -o run -- $B > gpurun_out/prof/fetch.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $W/write -o run -- $B > gpurun_out/prof/write.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $W/sq -o run -- $B > gpurun_out/prof/sq.log 2>&1
cp $W/conc/run_kernel_stats.csv gpurun_out/prof/conc_kernel_stats.csv
cp $W/ser/run_kernel_stats.csv gpurun_out/prof/ser_kernel_stats.csv
cd tools/prof
python3 timeline.py $W/conc/run_kernel_trace.csv 2 > ../../gpurun_out/prof/timeline.txt
python3 breakdown.py $W/ser/run_kernel_stats.csv > ../../gpurun_out/prof/serial_breakdown.txt
python3 pmc_accumulate.py $W/fetch/run_counter_collection.csv $W/write/run_counter_collection.csv $W/sq/run_counter_collection.csv ../../gpurun_out/prof/pmc_accumulate.json > /dev/null
python3 pmc_by_kernel.py 'k_\w+(<[^>(]*>)?' $W/fetch/run_counter_collection.csv $W/write/run_counter_collection.csv $W/sq/run_counter_collection.csv > ../../gpurun_out/prof/pmc_by_kernel.txt
rm -rf $W
