# configs[4] S24 split into 8 slices on one GPU (emulation): the slices' H plans are 2^21 domains
# (dense window bits 18 before the top-window fix, 17 after); new library, then the base library
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 1000 python bench.py --mode split --parts 8 --steps 2 --warmup 1 > gpurun_out/split8_new.log 2>&1
ZKP_LIB_PATH=$PWD/abtest/libzkp_amd_base.so timeout -k 10 1000 python bench.py --mode split --parts 8 --steps 2 --warmup 1 > gpurun_out/split8_base.log 2>&1
