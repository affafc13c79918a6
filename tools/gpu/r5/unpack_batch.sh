# round 5: does the per-chunk witness expansion (98 small kernels on the copy queues) slow the batch,
# where they land inside the other pipeline's proof?  256-proof batches, previous library (base) vs
# new, alternated 2 rounds
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5/unpackb
mkdir -p $O
for i in 1 2; do
  for v in base new; do
    if [ $v = base ]; then L="ZKP_LIB_PATH=$PWD/tools/gpu/r5/libs/base.so"; else L="ZKP_X=1"; fi
    env $L timeout -k 10 400 python3 bench.py --steps 20 --warmup 3 --cpu-baseline none --batch 256 --no-kernels --no-bool0-line > $O/${v}_$i.json 2> $O/${v}_$i.err
    echo "$v round $i $(tail -1 $O/${v}_$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); b=d["batch_pcie_inclusive"]; print(d["value"], d["latency_ms"], d["witness_upload"]["ms"], b["proofs_per_s"], b["vs_staged_headline"], b["verified"])')"
  done
done
