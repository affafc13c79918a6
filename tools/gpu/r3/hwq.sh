# round 3: two proofs in flight per GPU vs the number of HIP hardware queues per process
# (GPU_MAX_HW_QUEUES, HIP's default 4: the 8 streams of two pipelines then share 4 queues).
# One prover, ZKP_INFLIGHT=2, concurrent staged callers (tools/probe/staged_inflight.py).
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/hwq.txt
for q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python tools/probe/staged_inflight.py 16 2 >> gpurun_out/hwq.txt 2>&1
done
GPU_MAX_HW_QUEUES=8 timeout -k 10 300 python tools/probe/staged_inflight.py 18 3 >> gpurun_out/hwq.txt 2>&1
