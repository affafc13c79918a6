# G2-only gates: ZKP_SCHED=4 (G2 waits for the quotient), 5 (and for the H plan) vs free-running 0
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for g in 4 5 0 4 5 0; do
  ZKP_SCHED=$g timeout -k 10 200 python bench.py --steps 10 --warmup 2 --cpu-baseline none --no-kernels >> gpurun_out/bs_$g.log 2>&1
done
