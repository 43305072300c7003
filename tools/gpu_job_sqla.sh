#!/bin/bash
# MFMA-reduction squaring probe: table-read lookahead sweep (tools/probe/sqchain_mfma.hip
# built with -DSQ_LOOKAHEAD=L as libsqchain_L<L>.so); variant 0 = VALU squaring, 1 = MFMA.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
for L in ${LS:-0 2 3 4 6}; do
  SQ_LIB=libsqchain_L$L.so timeout -k 10 120 python3 $R/tools/probe/sqchain_mfma.py ${NE:-196608} 32 > $R/gpurun_out/sqla_L$L.json 2>&1 || { echo "L=$L failed"; cat $R/gpurun_out/sqla_L$L.json | tail -5; exit 1; }
  echo "L=$L $(cat $R/gpurun_out/sqla_L$L.json)"
done
