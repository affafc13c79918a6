# round 5: the tests the deferred second witness configuration touches; the 8-logical-device
# rehearsal; H window bits 20 vs 22 alternated (3 rounds); the default bench (two-in-flight side line)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_witness_transfer.py tests/test_gpu_verify.py tests/test_gpu_prove.py tests/test_gpu_configs.py -x -v --timeout 200 --timeout-method thread > $O/gt_fourth.log 2>&1
echo tests done
timeout -k 10 900 python3 bench.py --gpus 8 --rehearsal --no-kernels --cpu-baseline none --no-bool0-line > $O/rehearsal8.json 2> $O/rehearsal8.err
echo rehearsal done
bash tools/gpu/r5/ab.sh 3 h22 "h20:-" "h22:ZKP_MSM=h=22"
echo ab done
timeout -k 10 500 python bench.py > $O/bench_b.json 2> $O/bench_b.err
echo bench done
