# rocprofv3 --pmc passes over the short bench command, one pass per counter set (the collection serialises
# dispatches: every launch runs alone).  Sets: sq (wave-cycle split, tools/prof/pmc_stall.py), valu (counted
# VALU busy: SQ_ACTIVE_INST_VALU2, int32/int64, tools/prof/valu_counted.py), fetch, write (HBM bytes,
# tools/prof/pmc_launch5.py), tcp (L1 TLB), ntt (the NTT probe at 2^23 and 2^20 with the sq and valu sets)
#   bash tools/gpu/pmc.sh <tag> sq valu fetch write tcp ntt  ->  $O/<set>/run_counter_collection.csv
source "$(dirname "$0")/common.sh"
SQ="SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
VALU="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
for s in "$@"; do
  case $s in
    sq) C=$SQ ;;
    valu) C=$VALU ;;
    fetch) C="FETCH_SIZE" ;;
    write) C="WRITE_SIZE TCC_HIT_sum" ;;
    tcp) C="TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" ;;
    ntt)
      for k in 23 20; do
        timeout -s KILL 120 rocprofv3 --pmc $SQ --output-format csv -d $O/ntt${k}_sq -o run -- python3 tools/probe/ntt_run.py $k 20 > $O/ntt${k}_sq.log 2>&1
        timeout -s KILL 120 rocprofv3 --pmc $VALU --output-format csv -d $O/ntt${k}_valu -o run -- python3 tools/probe/ntt_run.py $k 20 > $O/ntt${k}_valu.log 2>&1
      done
      echo ntt done
      continue ;;
    *) echo "unknown set $s"; exit 2 ;;
  esac
  timeout -s KILL 300 rocprofv3 --pmc $C --output-format csv -d $O/$s -o run -- $SHORT > $O/$s.json 2> $O/$s.err
  echo $s done
done
