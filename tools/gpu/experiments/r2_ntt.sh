# NTT change check: NTT / quotient / golden-proof GPU tests, then an A/B bench against
# abtest/libzkp_amd_base.so (alternating, 2 rounds each).
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "ntt or quotient or prove or golden or smoke" > gpurun_out/ntt_tests.log 2>&1
bash tools/gpu/ab.sh 2
python tools/gpu/ab_summary.py > gpurun_out/ab_summary.txt
