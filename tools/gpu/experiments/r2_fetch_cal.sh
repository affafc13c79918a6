# FETCH_SIZE / WRITE_SIZE calibration on the accumulate's 64-B gather (and the coalesced case).
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 60 ./tools/ubench/gather_fetch > gpurun_out/gather_fetch.txt 2>&1
timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/cal_fetch -o run -- ./tools/ubench/gather_fetch > gpurun_out/cal_fetch.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/cal_write -o run -- ./tools/ubench/gather_fetch > gpurun_out/cal_write.log 2>&1
timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d gpurun_out/cal_rdreq -o run -- ./tools/ubench/gather_fetch > gpurun_out/cal_rdreq.log 2>&1
