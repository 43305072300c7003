#!/bin/bash
# SQ counters of the MFMA-reduction squaring probe (variant 1) against the VALU squaring
# (variant 0): one rocprofv3 --pmc pass per variant (tools/probe/sqchain_mfma.py).
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/sqpmc
mkdir -p $OUT
CTR="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE"
for v in 0 1; do
  SQ_LIB=${SQ_LIB:-libsqchain_bw12.so} SQ_VARIANTS=$v timeout -s KILL 90 rocprofv3 --pmc $CTR -d $OUT/v$v -o pmc --output-format csv -- python3 $R/tools/probe/sqchain_mfma.py 98304 32 > $OUT/v$v.log 2>&1
  echo "variant $v done"
done
