# round 4, twelfth call: non-temporal bit-walk encoder vs the branch-free one: the encoder alone on
# the box's CPU, the transfer tests, and the latency probe alternating (3 rounds)
# (historical: wtns_pack_test_old_bin was the encoder test of the revision before c4fbc20, built
# here with `git show c4fbc20^:zk-p2p-onramp_amd/csrc/wtns_pack.hpp` in place; it is no longer tracked)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
for t in 8 16; do
  timeout -k 10 120 tools/hosttest/wtns_pack_test_old_bin 6400000 $t > gpurun_out/r4/enc_old_$t.txt 2>&1
  timeout -k 10 120 tools/hosttest/wtns_pack_test_bin 6400000 $t > gpurun_out/r4/enc_new_$t.txt 2>&1
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_witness_transfer.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r4/gt_ntenc.log 2>&1
for i in 1 2 3; do
  ZKP_LIB_PATH=$PWD/tools/gpu/r4/libs/lib_oldenc.so timeout -k 10 300 python tools/probe/latency_probe.py > gpurun_out/r4/lat_oldenc_$i.txt 2> gpurun_out/r4/lat_oldenc_$i.err
  timeout -k 10 300 python tools/probe/latency_probe.py > gpurun_out/r4/lat_ntenc_$i.txt 2> gpurun_out/r4/lat_ntenc_$i.err
done
