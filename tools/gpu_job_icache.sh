#!/bin/bash
# Instruction-cache counters (SQC_ICACHE_*) of the encrypt kernel and of the squaring probe
# (variant 0 = the engine's VALU squaring, 1 = MFMA reduction); one --pmc pass per pair.
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/icache
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
i=0
for SET in "SQC_ICACHE_HITS SQC_ICACHE_MISSES" "SQC_ICACHE_REQ SQC_TC_INST_REQ"; do
  timeout -s KILL 90 rocprofv3 --pmc $SET --output-format csv -d $OUT/enc$i -o pmc -- python3 $R/bench.py --n 262144 --steps 1 --warmup 0 --no-extras --no-cpu-baseline > $OUT/enc$i.log 2>&1 || { echo "enc pass $i failed"; tail -5 $OUT/enc$i.log; exit 1; }
  for v in 0 1; do
    SQ_LIB=libsqchain_E4.so SQ_VARIANTS=$v timeout -s KILL 90 rocprofv3 --pmc $SET --output-format csv -d $OUT/sq${v}_$i -o pmc -- python3 $R/tools/probe/sqchain_mfma.py 98304 32 > $OUT/sq${v}_$i.log 2>&1 || { echo "sq $v pass $i failed"; tail -5 $OUT/sq${v}_$i.log; exit 1; }
  done
  i=$((i+1))
done
echo icache_ok
