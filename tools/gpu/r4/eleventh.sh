# round 4, eleventh call: batch line (256 host witnesses, two pipelines) with 16 encode threads always
# (in-tree) vs a quarter of them beside a proof in flight (lib_adapt), alternating, 3 rounds
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-baseline none --no-kernels --no-bool0-line > gpurun_out/r4/ab_bt_base_$i.json 2> gpurun_out/r4/ab_bt_base_$i.err
  ZKP_LIB_PATH=$PWD/tools/gpu/r4/libs/lib_adapt.so timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-baseline none --no-kernels --no-bool0-line > gpurun_out/r4/ab_bt_new_$i.json 2> gpurun_out/r4/ab_bt_new_$i.err
done
