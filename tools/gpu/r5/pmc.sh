# round 5, first GPU call.  (1) parity of the round-5 NTT unit + addressing (cur.so) and of the new
# MSM sort splits; (2) the v_mad peak sweep; (3) NTT A/B: r4 library (base), lazy unit (lazy), lazy unit
# + scalar tile addressing (cur): timing alternated and one SQ PMC pass each at 2^23 / 2^20;
# (4) VERDICT r4 item 1, where the H launch's cycles go: one rocprofv3 --pmc pass per counter group of
# one short bench command (the counter collection serialises kernels, so every launch runs alone):
# wave-cycle split (WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES), VALU issue,
# GRBM_GUI_ACTIVE for the effective clock; the same on an all-uniform witness; FETCH/WRITE; L2/TLB.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5/pmc
L=$PWD/tools/gpu/r5/libs
mkdir -p $O
ZKP_LIB_PATH=$L/cur.so timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_prove.py -x -v --timeout 120 --timeout-method thread -k "ntt or quotient or prove_bit_exact or params" > $O/gt_ntt.log 2>&1
echo gt done
timeout -k 10 120 tools/ubench/int_mul_rate > $O/ubench.txt 2>&1
for r in 1 2 3; do
  for v in base lazy cur; do
    ZKP_LIB_PATH=$L/$v.so timeout -k 10 120 python3 tools/probe/ntt_run.py 23 20 >> $O/ntt_ab_$v.txt 2>&1
    ZKP_LIB_PATH=$L/$v.so timeout -k 10 120 python3 tools/probe/ntt_run.py 20 20 >> $O/ntt_ab20_$v.txt 2>&1
  done
done
echo ntt ab done
SQ="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
for v in base cur; do
  for k in 20 23; do
    ZKP_LIB_PATH=$L/$v.so timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d $O/ntt${k}_$v -o run -- python3 tools/probe/ntt_run.py $k 20 > $O/ntt${k}_$v.log 2>&1
  done
done
echo ntt pmc done
B="python3 bench.py --steps 4 --warmup 1 --cpu-baseline none --batch 0 --no-kernels --no-bool0-line"
timeout -s KILL 300 rocprofv3 --pmc $SQ --output-format csv -d $O/sq -o run -- $B > $O/sq.json 2> $O/sq.err
echo sq done
timeout -s KILL 300 rocprofv3 --pmc $SQ --output-format csv -d $O/sq_u -o run -- $B --bool-pct 0 > $O/sq_u.json 2> $O/sq_u.err
echo sq_u done
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $B > $O/fetch.json 2> $O/fetch.err
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum --output-format csv -d $O/write -o run -- $B > $O/write.json 2> $O/write.err
echo tcc done
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_VMEM --output-format csv -d $O/sq2 -o run -- $B > $O/sq2.json 2> $O/sq2.err
echo sq2 done
timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum --output-format csv -d $O/tcp -o run -- $B > $O/tcp.json 2> $O/tcp.err
echo tcp done
