# round 5: the bench freezes Python's GC before its timed regions (a full collection walked the
# harness's heap for 215-260 ms inside a 256-proof batch): batches of 64 and 256 after the fix, 2 rounds,
# and the 256-proof batch under rocprofv3 --kernel-trace --marker-trace (tools/prof/batch_gaps.py)
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5/gc
mkdir -p $O
for i in 1 2; do
  for b in 64 256; do
    timeout -k 10 400 python3 bench.py --steps 20 --warmup 3 --cpu-baseline none --batch $b --no-kernels --no-bool0-line > $O/b${b}_$i.json 2> $O/b${b}_$i.err
    echo "batch $b round $i $(tail -1 $O/b${b}_$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); b=d["batch_pcie_inclusive"]; print(d["value"], b["proofs_per_s"], b["vs_staged_headline"], b["verified"])')"
  done
done
timeout -k 10 400 rocprofv3 --kernel-trace --marker-trace --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 3 --cpu-baseline none --batch 256 --no-kernels --no-bool0-line > $O/bench_prof.json 2> $O/bench_prof.err
python3 tools/prof/batch_gaps.py $O/prof/run_kernel_trace.csv $O/prof/run_marker_api_trace.csv $O/batch_gaps.json > /dev/null
echo trace done
