# C = A o B formed in the first NTT pass of C's coset extension: quotient/proof/split GPU tests, proof A/B
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "ntt or quotient or golden or prove or split or fullsize" > gpurun_out/cprod_tests.log 2>&1
bash tools/gpu/ab.sh 3
python tools/gpu/ab_summary.py > gpurun_out/ab_summary.txt
