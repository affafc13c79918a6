# round 6, VERDICT r5 item 4: per-opcode VALU cycles (tools/ubench/valu_rates.hip) and a counted dual-issue /
# int32-int64 split of the real kernels: one rocprofv3 --pmc pass over the opcode ubench (known mixes), the
# short bench command (accumulate launches; split per launch kind by tools/prof/valu_weighted.py) and the
# NTT probe at 2^23 / 2^20.
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
O=gpurun_out/r6/valu
mkdir -p $O
for w in 2 4 8; do timeout -k 10 120 ./tools/ubench/valu_rates $w > $O/valu_rates_wg$w.txt 2>&1; done
echo rates done
PMC="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAVES SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $PMC --output-format csv -d $O/ub -o run -- ./tools/ubench/valu_rates 4 > $O/ub.txt 2>&1
echo ub pmc done
B="python3 bench.py --steps 4 --warmup 1 --cpu-baseline none --batch 0 --no-kernels --no-bool0-line --sustain-s 0"
timeout -s KILL 300 rocprofv3 --pmc $PMC --output-format csv -d $O/acc -o run -- $B > $O/acc.json 2> $O/acc.err
echo acc pmc done
for k in 23 20; do
  timeout -s KILL 120 rocprofv3 --pmc $PMC --output-format csv -d $O/ntt$k -o run -- python3 tools/probe/ntt_run.py $k 20 > $O/ntt$k.log 2>&1
done
echo ntt pmc done
