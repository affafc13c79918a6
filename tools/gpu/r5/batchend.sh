# round 5: a 256-proof batch's GPU work ends ~215 ms before zkp_prove_batch returns (64 proofs: ~4 ms).
# The same bench under rocprofv3 --kernel-trace --hip-trace --marker-trace: the HIP calls of that tail
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5/bend
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --hip-trace --marker-trace --output-format csv -d $O/prof -o run -- python3 bench.py --steps 4 --warmup 2 --cpu-baseline none --batch 256 --no-kernels --no-bool0-line > $O/bench_prof.json 2> $O/bench_prof.err
echo trace done
