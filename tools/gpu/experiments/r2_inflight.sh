# ZKP_INFLIGHT A/B on the batch line: k pipelines per device sharing the base tables
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
ZKP_INFLIGHT=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_prove.py -x -q --timeout 120 --timeout-method thread -k "batch" > gpurun_out/inflight_tests.log 2>&1
for i in 1 2; do
  for k in 1 2; do
    ZKP_INFLIGHT=$k timeout -k 10 300 python bench.py --steps 8 --warmup 2 --cpu-baseline none --batch 192 > gpurun_out/inflight_${k}_$i.log 2>&1
  done
done
python - <<'PY' > gpurun_out/inflight_summary.txt
import json, glob
for f in sorted(glob.glob("gpurun_out/inflight_[12]_*.log")):
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line); b = d.get("batch_pcie_inclusive") or {}
            print(f, "headline", d["value"], "batch", b.get("proofs_per_s"))
PY
