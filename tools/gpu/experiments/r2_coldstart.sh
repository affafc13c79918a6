set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python3 -u tools/bench_coldstart.py gpurun_out/coldstart.json > gpurun_out/coldstart.log 2>&1
