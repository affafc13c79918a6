set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 ./tools/ubench/int_mul_rate > gpurun_out/ubench.txt 2>&1
timeout -k 10 900 bash tools/gpu/experiments/r2_dsort.sh
