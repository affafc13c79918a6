# round 4: bucket folding fused into the segment reduction (no bucket array): MSM / proof parity
# tests, then an alternating A/B against the previous library
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_prove.py tests/test_gpu_split.py tests/test_gpu_configs.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4/fusedseg_tests.txt 2>&1
bash tools/gpu/r4/abx.sh tools/gpu/r4/libs/lib_head.so 3 fseg
