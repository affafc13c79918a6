# round 5: the witness encoder's lane classification with AVX-512 + BMI2 (8 signals per step) on the GPU
# box's host.  (1) the host round trip (AVX-512 encoding == portable encoding) and the transfer / proof
# tests; (2) host_capacity probe, previous encoder (base) vs new: 1 group x 16 threads and 8 groups x 2
# threads, both mixes, alternated 2 rounds; (3) host-witness latency probe, base vs new, 3 rounds
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5/avx
mkdir -p $O
g++ -O2 -std=c++17 -pthread tools/hosttest/wtns_pack_test.cpp -o $O/wpt && timeout -k 10 120 $O/wpt 6400000 16 > $O/wpt.txt 2>&1
grep -m1 roundtrip $O/wpt.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_witness_transfer.py tests/test_gpu_prove.py -x -v --timeout 200 --timeout-method thread > $O/gt.log 2>&1
echo gt done
for i in 1 2; do
  for v in base new; do
    if [ $v = base ]; then B=tools/gpu/r5/libs/host_capacity_base; else B=tools/hosttest/host_capacity_bin; fi
    for pct in 70 0; do
      timeout -k 10 60 $B 6400562 1 16 4 $pct 2 >> $O/hc_$v.txt 2>&1
      timeout -k 10 60 $B 6400562 8 2 4 $pct 2 >> $O/hc_$v.txt 2>&1
    done
  done
done
echo hc done
for i in 1 2 3; do
  ZKP_LIB_PATH=$PWD/tools/gpu/r5/libs/base.so timeout -k 10 300 python3 tools/probe/latency_probe.py > $O/lat_base_$i.txt 2> $O/lat_base_$i.err
  timeout -k 10 300 python3 tools/probe/latency_probe.py > $O/lat_new_$i.txt 2> $O/lat_new_$i.err
  echo "round $i base $(grep host_witness $O/lat_base_$i.txt) new $(grep host_witness $O/lat_new_$i.txt)"
done
