# round 5: the inter-pass twiddles and the coset key as Shoup products from 72-B table entries (plain
# limbs + quotient limbs) instead of Montgomery products of packed table values.  (1) NTT / quotient /
# proof parity; (2) coset-extension times, previous library (base) vs new, alternated 3 rounds;
# (3) one SQ + GRBM PMC pass per size on the new library; (4) the short staged bench alternated, 3 rounds
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5/shouptw
L=$PWD/tools/gpu/r5/libs
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_prove.py -x -v --timeout 200 --timeout-method thread > $O/gt.log 2>&1
echo gt done
timeout -k 10 600 python3 tools/probe/ntt_ab.py 3 $L/base.so zk-p2p-onramp_amd/lib/libzkp_amd.so > $O/ntt_ab.txt 2>&1
echo ntt ab done
SQ="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
for k in 20 23; do
  timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d $O/ntt${k} -o run -- python3 tools/probe/ntt_run.py $k 20 > $O/ntt${k}.log 2>&1
done
echo ntt pmc done
bash tools/gpu/r5/ab.sh 3 shouptw "base:ZKP_LIB_PATH=tools/gpu/r5/libs/base.so" "shouptw:-"
echo ab done
