# round 5: is the batch line's ~5 % deficit the batch path or the load's duration?  Under rocprofv3 a
# 64-proof batch ran at 1.004 of the 20-step staged rate.  Staged loops of 20 and 256 steps, each
# followed by batches of 64 and 256 proofs, alternated 2 rounds.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5/sus
mkdir -p $O
for i in 1 2; do
  for cfg in "20 64" "256 256"; do
    set -- $cfg
    timeout -k 10 400 python3 bench.py --steps $1 --warmup 3 --cpu-baseline none --batch $2 --no-kernels --no-bool0-line > $O/s$1_b$2_$i.json 2> $O/s$1_b$2_$i.err
    echo "steps $1 batch $2 round $i $(tail -1 $O/s$1_b$2_$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); b=d["batch_pcie_inclusive"]; print(d["value"], d["ms_per_step"], d["roofline"]["frac"], b["proofs_per_s"], b["vs_staged_headline"], b["verified"])')"
  done
done
