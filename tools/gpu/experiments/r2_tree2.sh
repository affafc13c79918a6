# subset-sum trees: proof A/B (HEAD base vs tree with chain-first above 512 WGs vs ZKP_SUBSET_TREE=0), MSM 2^20
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rm -f gpurun_out/tree2.txt
run() { tag=$1; shift; env "$@" timeout -k 10 300 python bench.py --steps 16 --warmup 3 --cpu-baseline none --batch 0 --no-kernels > gpurun_out/b_tree.log 2>&1; echo "$tag $(tail -1 gpurun_out/b_tree.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["roofline"]["frac"])')" >> gpurun_out/tree2.txt; }
for i in 1 2; do
  run base ZKP_LIB_PATH=$PWD/abtest/libzkp_amd_base.so
  run tree512 ZKP_TREE_FIRST_MAX=512
  run notree ZKP_SUBSET_TREE=0
  run tree0 ZKP_TREE_FIRST_MAX=0
done
timeout -k 10 300 python tools/probe/msm_ab.py 1 abtest/libzkp_amd_base.so zk-p2p-onramp_amd/lib/libzkp_amd.so >> gpurun_out/tree2.txt 2>&1
