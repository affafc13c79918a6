# round 5, VERDICT r4 item 1: where the H launch's cycles go. One rocprofv3 --pmc pass per counter
# group of one short bench command (the counter collection serialises kernels, so every launch runs
# alone): wave-cycle split (WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY ~ WAVE_CYCLES), VALU issue,
# GRBM_GUI_ACTIVE for the effective clock; the same SQ pass on an all-uniform witness (witness
# launches of the H launch's size, other bucket count); L2/TLB passes; FETCH/WRITE for traffic;
# the NTT's SQ pass at 2^20 and 2^23.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r5/pmc
mkdir -p $O
B="python3 bench.py --steps 4 --warmup 1 --cpu-baseline none --batch 0 --no-kernels --no-bool0-line"
SQ="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
timeout -s KILL 300 rocprofv3 --pmc $SQ --output-format csv -d $O/sq -o run -- $B > $O/sq.json 2> $O/sq.err
echo sq done
timeout -s KILL 300 rocprofv3 --pmc $SQ --output-format csv -d $O/sq_u -o run -- $B --bool-pct 0 > $O/sq_u.json 2> $O/sq_u.err
echo sq_u done
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $B > $O/fetch.json 2> $O/fetch.err
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum --output-format csv -d $O/write -o run -- $B > $O/write.json 2> $O/write.err
echo tcc done
for k in 20 23; do
  timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d $O/ntt$k -o run -- python3 tools/probe/ntt_run.py $k 20 > $O/ntt$k.log 2>&1
done
echo ntt done
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_VMEM --output-format csv -d $O/sq2 -o run -- $B > $O/sq2.json 2> $O/sq2.err
echo sq2 done
timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum --output-format csv -d $O/tcp -o run -- $B > $O/tcp.json 2> $O/tcp.err
echo tcp done
