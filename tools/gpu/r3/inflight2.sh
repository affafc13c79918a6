# round 3: two staged proofs in flight per GPU (one prover, ZKP_INFLIGHT=2, two host threads) with
# the chained/paired kernels, vs one at a time
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/inflight2.txt
timeout -k 10 300 python tools/probe/staged_inflight.py 16 2 >> gpurun_out/inflight2.txt 2>&1
timeout -k 10 300 python tools/probe/staged_inflight.py 18 3 >> gpurun_out/inflight2.txt 2>&1
