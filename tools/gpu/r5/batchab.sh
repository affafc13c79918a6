# round 5: the batch line (256 host witnesses, zkp_prove_batch, verify-before-return on) with encode
# threads shared out among concurrent uploads (this library) vs a fixed 16 per upload (t16.so),
# alternated 3 rounds; then the second witness configuration at c = 20 vs c = 22 on an all-uniform witness
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5
mkdir -p $O
for i in 1 2 3; do
  for v in cur t16; do
    if [ $v = t16 ]; then export ZKP_LIB_PATH=$PWD/tools/gpu/r5/libs/t16.so; else unset ZKP_LIB_PATH; fi
    timeout -k 10 400 python bench.py --steps 20 --warmup 3 --cpu-baseline none --no-kernels --no-bool0-line > $O/batchab_${v}_$i.json 2> $O/batchab_${v}_$i.err
    echo "batch $v $i $(tail -1 $O/batchab_${v}_$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); b=d["batch_pcie_inclusive"]; print(d["value"], b["proofs_per_s"], b["vs_staged_headline"], b["verified"], d["latency_ms"])')"
  done
done
unset ZKP_LIB_PATH
echo batch ab done
bash tools/gpu/r5/w2ab.sh
echo w2 done
