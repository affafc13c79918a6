# round 4: NTT issue rate at 2^20 and 2^23: a PMC pass and a kernel trace of
# the same ntt_run command per size, joined by tools/prof/ntt_issue.py
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
for k in 20 23; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES --output-format csv -d gpurun_out/r4/nttpmc$k -o run -- python3 tools/probe/ntt_run.py $k 20 > gpurun_out/r4/nttpmc$k.log 2>&1
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4/ntttr$k -o run -- python3 tools/probe/ntt_run.py $k 20 > gpurun_out/r4/ntttr$k.log 2>&1
done
python3 tools/prof/ntt_issue.py gpurun_out/r4 > gpurun_out/r4/ntt_issue.json
