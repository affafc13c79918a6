# round 4, fifth call: NTT occupancy policy (2 workgroups per CU when the last round of 3 is mostly
# empty) A/B + tests, NTT kernel traces at 2^20 / 2^23, the host-witness latency probe, the bench
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "ntt or quotient" > gpurun_out/r4/gt_ntt_occ.log 2>&1
timeout -k 10 400 python tools/probe/ntt_ab.py 2 tools/gpu/r4/libs/lib_ntt_occ0.so zk-p2p-onramp_amd/lib/libzkp_amd.so > gpurun_out/r4/ntt_occ_ab.txt 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4/ntt20 -o run -- python3 tools/probe/ntt_run.py 20 > gpurun_out/r4/ntt20.log 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4/ntt23 -o run -- python3 tools/probe/ntt_run.py 23 > gpurun_out/r4/ntt23.log 2>&1
timeout -k 10 300 python tools/probe/latency_probe.py > gpurun_out/r4/latency_probe.txt 2> gpurun_out/r4/latency_probe.err
timeout -k 10 400 python bench.py > gpurun_out/r4/bench_fifth.json 2> gpurun_out/r4/bench_fifth.err
