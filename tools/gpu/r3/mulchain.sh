# round 3: FIPS-29 multiply shape microbenchmark (tools/ubench/mul_chain.hip, built in-tree beforehand)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 ./tools/ubench/mul_chain > gpurun_out/mul_chain.txt 2>&1
