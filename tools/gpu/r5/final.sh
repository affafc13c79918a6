# round 5, final library: the whole GPU suite, smoke(), the default bench line, the same bench under
# rocprofv3 --kernel-trace --marker-trace --stats with the per-launch split, and the batch with
# verify-before-return off vs the default (on), alternated 2 rounds
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5f
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gt_final.log 2>&1
echo suite done
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
echo smoke done
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err
echo bench done
timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 3 --cpu-baseline none --batch 0 --no-kernels --no-bool0-line > $O/bench_prof.json 2> $O/bench_prof.err
python3 tools/prof/launch_split.py $O/prof/run_kernel_trace.csv $O/prof/run_marker_api_trace.csv $O/bench_prof.json $O/launch_split.json > /dev/null
echo trace done
for i in 1 2; do
  for v in 0 2; do
    ZKP_VERIFY=$v timeout -k 10 400 python bench.py --steps 20 --warmup 3 --cpu-baseline none --no-kernels --no-bool0-line > $O/verifyab_${v}_$i.json 2> $O/verifyab_${v}_$i.err
    echo "verify $v $i $(tail -1 $O/verifyab_${v}_$i.json | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); b=d["batch_pcie_inclusive"]; print(d["value"], b["proofs_per_s"], b["vs_staged_headline"], b["verified"])')"
  done
done
