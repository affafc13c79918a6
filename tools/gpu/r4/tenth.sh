# round 4, tenth call: the witness encoder alone on the box's CPU (16 threads, Venmo size)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
for t in 4 8 16; do timeout -k 10 120 tools/hosttest/wtns_pack_test_bin 6400000 $t > gpurun_out/r4/encode_$t.txt 2>&1; done
nproc >> gpurun_out/r4/encode_16.txt
