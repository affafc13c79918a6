# round 5: with the H-plan task size 48 as default: proof parity, then the witness-plan task size
# (task_w 24 / 40 / 48 vs 32) alternated 3 rounds on the short staged bench
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5/task3
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_prove.py tests/test_gpu_configs.py tests/test_gpu_witness_transfer.py -x -v --timeout 200 --timeout-method thread > $O/gt.log 2>&1
echo gt done
bash tools/gpu/r5/ab.sh 3 task3 "base:-" "tw24:ZKP_MSM=task_w=24" "tw40:ZKP_MSM=task_w=40" "tw48:ZKP_MSM=task_w=48"
echo ab done
