# round 5: a 64-proof batch runs at ~1.007 of the staged rate, a 256-proof batch at ~0.977 (sustain.sh),
# while a 256-step staged loop keeps the 20-step rate.  (1) the 256-proof batch under rocprofv3
# --kernel-trace (tools/prof/batch_gaps.py: GPU busy and the H launch's time per tenth of the batch);
# (2) 256-proof batches with one pipeline per device (ZKP_INFLIGHT=1) vs two, alternated 2 rounds
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5/b256
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 3 --cpu-baseline none --batch 256 --no-kernels --no-bool0-line > $O/bench_prof.json 2> $O/bench_prof.err
python3 tools/prof/batch_gaps.py $O/prof/run_kernel_trace.csv $O/prof/run_marker_api_trace.csv $O/batch_gaps.json > /dev/null
echo trace done
for i in 1 2; do
  for inf in 1 2; do
    ZKP_INFLIGHT=$inf timeout -k 10 400 python3 bench.py --steps 20 --warmup 3 --cpu-baseline none --batch 256 --no-kernels --no-bool0-line > $O/inf${inf}_$i.json 2> $O/inf${inf}_$i.err
    echo "inflight $inf round $i $(tail -1 $O/inf${inf}_$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); b=d["batch_pcie_inclusive"]; print(d["value"], b["proofs_per_s"], b["vs_staged_headline"], b["verified"], b["pipelines_per_device"])')"
  done
done
