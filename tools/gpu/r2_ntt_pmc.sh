# LDS bank-conflict / VALU counters of the NTT kernels (one 2^23 coset-extension bench), per library
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ntt_pmc
for lib in "$@"; do
  tag=$(basename $lib .so)
  ZKP_LIB_PATH=$PWD/$lib timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d gpurun_out/ntt_pmc/$tag -o pmc --output-format csv -- python3 tools/probe/ntt_run.py 23 > gpurun_out/ntt_pmc/$tag.log 2>&1
done
