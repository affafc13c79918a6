# round 4, second call: accumulation variants (microbenchmark), NTT tile variants, the raw-T Y3
# operand A/B in the proof, the witness-window sweep
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
timeout -k 10 300 tools/ubench/acc_bench 19 208 5 > gpurun_out/r4/acc_bench_2.txt 2>&1
timeout -k 10 400 python tools/probe/ntt_ab.py 2 tools/gpu/r4/libs/lib_ntt_base.so tools/gpu/r4/libs/lib_ntt_A.so tools/gpu/r4/libs/lib_ntt_B.so tools/gpu/r4/libs/lib_ntt_C.so > gpurun_out/r4/ntt_tiles.txt 2>&1
bash tools/gpu/r4/abx.sh tools/gpu/r4/libs/lib_prev.so 2 rawt
timeout -k 10 600 python tools/probe/wsweep.py --bools 0,70,90 --cs 17,18,19,20 --steps 8 --reps 2 > gpurun_out/r4/wsweep.txt 2> gpurun_out/r4/wsweep.err
