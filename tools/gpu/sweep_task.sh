# entries per accumulate task (MsmParams::S) for the witness / H plans
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for sw in 32 64 48 24; do for sh in 32 64; do
  ZKP_TASK_W=$sw ZKP_TASK_H=$sh timeout -k 10 200 python bench.py --steps 8 --warmup 2 --cpu-baseline none --no-kernels > gpurun_out/b_s${sw}_${sh}.log 2>&1
done; done
