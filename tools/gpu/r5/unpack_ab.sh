# round 5: the witness expansion per chunk, right behind each chunk's copy on its copy queue, instead of
# one expansion after the last copy.  (1) transfer / proof tests on the new library; (2) the host-witness
# latency probe, previous library (base) vs new, alternated 3 rounds; (3) one default bench line
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5/unpack
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_witness_transfer.py tests/test_gpu_prove.py tests/test_gpu_verify.py -x -v --timeout 200 --timeout-method thread > $O/gt.log 2>&1
echo gt done
for i in 1 2 3; do
  ZKP_LIB_PATH=$PWD/tools/gpu/r5/libs/base.so timeout -k 10 300 python3 tools/probe/latency_probe.py > $O/lat_base_$i.txt 2> $O/lat_base_$i.err
  timeout -k 10 300 python3 tools/probe/latency_probe.py > $O/lat_new_$i.txt 2> $O/lat_new_$i.err
  echo "round $i base $(grep host_witness $O/lat_base_$i.txt) new $(grep host_witness $O/lat_new_$i.txt)"
done
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err
echo bench done
