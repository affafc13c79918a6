# round 4, fourth call: host-encode threads 16 vs 8 (latency A/B),
# then phase-2 setup at the Venmo shape
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
bash tools/gpu/r4/abx.sh tools/gpu/r4/libs/lib_nc16.so 2 nc16
timeout -k 10 700 python -u tools/bench_setup.py --cpu-check --out gpurun_out/r4/bench_setup_venmo.json > gpurun_out/r4/bench_setup.log 2>&1
