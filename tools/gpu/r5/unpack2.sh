# round 5: per-chunk witness expansion again, now only for a lone upload (no proof computing in the
# process) and on a stream of its own joined to each chunk's copy by an event (copy queues never wait).
# (1) transfer / proof / verify tests; (2) host-witness latency probe, base vs new, alternated 3 rounds;
# (3) 256-proof batches, base vs new, alternated 2 rounds
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5/unpack2
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_witness_transfer.py tests/test_gpu_prove.py tests/test_gpu_verify.py -x -v --timeout 200 --timeout-method thread > $O/gt.log 2>&1
echo gt done
for i in 1 2 3; do
  ZKP_LIB_PATH=$PWD/tools/gpu/r5/libs/base.so timeout -k 10 300 python3 tools/probe/latency_probe.py > $O/lat_base_$i.txt 2> $O/lat_base_$i.err
  timeout -k 10 300 python3 tools/probe/latency_probe.py > $O/lat_new_$i.txt 2> $O/lat_new_$i.err
  echo "round $i base $(grep host_witness $O/lat_base_$i.txt) new $(grep host_witness $O/lat_new_$i.txt)"
done
for i in 1 2; do
  for v in base new; do
    if [ $v = base ]; then L="ZKP_LIB_PATH=$PWD/tools/gpu/r5/libs/base.so"; else L="ZKP_X=1"; fi
    env $L timeout -k 10 400 python3 bench.py --steps 20 --warmup 3 --cpu-baseline none --batch 256 --no-kernels --no-bool0-line > $O/${v}_$i.json 2> $O/${v}_$i.err
    echo "$v round $i $(tail -1 $O/${v}_$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); b=d["batch_pcie_inclusive"]; print(d["value"], d["latency_ms"], d["witness_upload"]["ms"], b["proofs_per_s"], b["vs_staged_headline"], b["verified"])')"
  done
done
