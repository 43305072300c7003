#!/bin/bash
# BASELINE config 5 at N=1: one 100M-element 2048-bit encrypt (spans of ~2M elements,
# ~4.5 min).  The single bench step prints nothing until it ends, so a heartbeat file under
# gpurun_out/ shows the run is alive; it stops with the step.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
( while sleep 30; do date +%T >> $R/gpurun_out/config5_heartbeat.txt; done ) &
HB=$!
timeout -k 10 ${CFG5_TIMEOUT:-700} python -u $R/bench.py --total ${CFG5_TOTAL:-100000000} --steps 1 --warmup 0 \
  --no-extras --no-cpu-baseline > $R/gpurun_out/config5_n1.txt 2>&1
rc=$?
kill $HB
tail -2 $R/gpurun_out/config5_n1.txt
exit $rc
