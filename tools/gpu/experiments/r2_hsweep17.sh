# H-plan window bits 17 (top window 16 bits: no deep low buckets) against the default 20
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/hsweep.txt
run() { tag="$*"; env "$@" timeout -k 10 300 python bench.py --steps 16 --warmup 3 --cpu-baseline none --batch 0 --no-kernels > gpurun_out/b_hs.log 2>&1; echo "$tag $(tail -1 gpurun_out/b_hs.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"]["msm"])')" >> gpurun_out/hsweep.txt; }
for i in 1 2; do
  run ZKP_NONE=0
  run ZKP_WINDOW_BITS_H=17
  run ZKP_WINDOW_BITS_H=16
done
