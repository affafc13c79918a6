# correctness of the dense plan's sort at c = 17..22, then per-c timing of the 2^20 MSM (dense)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread -k "dense_window_bits" > gpurun_out/hsc_tests.log 2>&1
rm -f gpurun_out/hsc_time.txt
for c in 17 18 19 20 21 22; do echo "c=$c $(ZKP_MSM_C=$c timeout -k 10 120 python3 tools/probe/msm_run.py 20 | tail -1)" >> gpurun_out/hsc_time.txt; done
