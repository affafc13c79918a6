# Shoup NTT stage products: NTT/quotient/proof/split GPU tests, NTT A/B, proof A/B, proof-boundary timeline
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "ntt or quotient or golden or prove or split" > gpurun_out/shoup_tests.log 2>&1
timeout -k 10 300 python tools/probe/ntt_ab.py 2 abtest/libzkp_amd_base.so zk-p2p-onramp_amd/lib/libzkp_amd.so > gpurun_out/shoup_ntt_ab.txt 2>&1
bash tools/gpu/ab.sh 2
python tools/gpu/ab_summary.py > gpurun_out/ab_summary.txt
W=/tmp/zkp_prof; rm -rf $W && mkdir -p $W
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $W/conc -o run -- python3 bench.py --steps 4 --warmup 1 --cpu-baseline none --no-kernels --batch 0 > gpurun_out/prof/conc2.log 2>&1
(cd tools/prof && python3 timeline.py $W/conc/run_kernel_trace.csv 2 > ../../gpurun_out/prof/timeline2.txt)
rm -rf $W
