# persistent job threads + per-call tree knobs: prove/kernel GPU tests (incl. new knob variants), proof A/B
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "prove or golden or msm or batch or node" > gpurun_out/jobs_tests.log 2>&1
bash tools/gpu/ab.sh 3
python tools/gpu/ab_summary.py > gpurun_out/ab_summary.txt
