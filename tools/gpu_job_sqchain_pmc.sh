#!/bin/bash
# SQ counters of the MFMA-reduction squaring probe (variant 1) against the VALU squaring
# (variant 0): one rocprofv3 --pmc pass per (variant, counter set) (tools/probe/sqchain_mfma.py).
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/sqpmc2
mkdir -p $OUT
SETS=(
 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_WAIT_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES"
 "SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_INT32 SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_MFMA SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU"
)
for v in 0 1; do
  for i in 0 1; do
    SQ_LIB=${SQ_LIB:-libsqchain_bw12.so} SQ_VARIANTS=$v timeout -s KILL 90 rocprofv3 --pmc ${SETS[$i]} -d $OUT/v${v}s$i -o pmc --output-format csv -- python3 $R/tools/probe/sqchain_mfma.py 98304 32 > $OUT/v${v}s$i.log 2>&1
    echo "variant $v set $i done"
  done
done
