# A/B of the stream scheduling knob ZKP_SCHED (1: witness accumulations wait for the
# quotient, 2: for the H plan too, 3: as 2 for the G1 MSMs only, G2 runs from the start)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for g in 3 0 3 0; do
  ZKP_SCHED=$g timeout -k 10 200 python bench.py --steps 8 --warmup 2 --cpu-baseline none --no-kernels >> gpurun_out/b_g${g}.log 2>&1
done
ZKP_SCHED=3 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_conc_g3 -o run -- python3 bench.py --steps 4 --warmup 1 --cpu-baseline none --no-kernels > gpurun_out/pc.log 2>&1
