# round 5: host-witness latency A/B (round-4 library, this library with lazy upload slots, the same with
# the slots allocated at load), alternated; the transfer tests on this library; the 8-logical-device
# rehearsal (8 pipelines' worth of host threads on GPU 0; a pipeline keeps one witness configuration
# when HBM runs out)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5
L=$PWD/tools/gpu/r5/libs
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_witness_transfer.py tests/test_gpu_verify.py -x -v --timeout 200 --timeout-method thread > $O/gt_transfer2.log 2>&1
echo tests done
for i in 1 2; do
  for v in base cur2 eager; do
    ZKP_LIB_PATH=$L/$v.so timeout -k 10 300 python3 tools/probe/latency_probe.py > $O/lat2_${v}_$i.txt 2> $O/lat2_${v}_$i.err
  done
done
echo latency done
timeout -k 10 900 python3 bench.py --gpus 8 --rehearsal --no-kernels --cpu-baseline none --no-bool0-line > $O/rehearsal8.json 2> $O/rehearsal8.err
echo rehearsal done
