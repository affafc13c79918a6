# the microbenchmarks (built on the CPU beforehand: tools/ubench/README.md): v_mad peak sweep, per-opcode
# VALU cycles (2, 4, 8 workgroups per CU), the accumulation variants and the batch-affine prototype
#   bash tools/gpu/ubench.sh <tag> [which...]   (default: int_mul_rate valu_rates acc_bench affine_bench)
source "$(dirname "$0")/common.sh"
W=${*:-int_mul_rate valu_rates acc_bench affine_bench}
for u in $W; do
  case $u in
    valu_rates) for w in 2 4 8; do timeout -k 10 120 tools/ubench/valu_rates $w > $O/valu_rates_wg$w.txt 2>&1; done ;;
    affine_bench) timeout -k 10 300 tools/ubench/affine_bench 5 64,128,256,512 > $O/affine_bench.txt 2>&1 ;;
    *) timeout -k 10 300 tools/ubench/$u > $O/$u.txt 2>&1 ;;
  esac
  echo $u done
done
