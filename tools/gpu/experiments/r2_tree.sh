# LDS-tree subset sums + dense kernel-level MSM: MSM / proof GPU tests, 2^20 MSM A/B, proof A/B
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "msm or golden or prove or split or setup" > gpurun_out/tree_tests.log 2>&1
timeout -k 10 300 python tools/probe/msm_ab.py 2 abtest/libzkp_amd_base.so zk-p2p-onramp_amd/lib/libzkp_amd.so > gpurun_out/tree_msm_ab.txt 2>&1
bash tools/gpu/ab.sh 2
python tools/gpu/ab_summary.py > gpurun_out/ab_summary.txt
