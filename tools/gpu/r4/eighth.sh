# round 4, eighth call: which MSM sum goes wrong for the all-large witness (tools/probe/transfer_diag.py)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
timeout -k 10 600 python -u tools/probe/transfer_diag.py > gpurun_out/r4/transfer_diag.txt 2> gpurun_out/r4/transfer_diag.err
