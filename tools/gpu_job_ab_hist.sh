# same-box A/B of the SecureBoost iupdate leg (tools/bench_legs/hist_leg.py):
# tools/gpu_job_ab_hist.sh TAG VARIANT...  (fate_amd/lib/ab/lib_<V>.so; "main" = the shipped build)
# the fold tests run once per variant first
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
T=$1; shift
for V in "$@"; do
  L=$R/fate_amd/lib/ab/lib_$V.so; [ "$V" = main ] && L=$R/fate_amd/lib/libfatephe.so
  FPHE_LIB_PATH=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_fold.py -q --timeout 240 --timeout-method thread > gpurun_out/${T}_${V}_tests.txt 2>&1 || { echo tests_failed $V; tail -30 gpurun_out/${T}_${V}_tests.txt; exit 1; }
  echo "$V tests: $(tail -1 gpurun_out/${T}_${V}_tests.txt)"
done
for rep in 1 2; do
  for V in "$@"; do
    L=$R/fate_amd/lib/ab/lib_$V.so; [ "$V" = main ] && L=$R/fate_amd/lib/libfatephe.so
    FPHE_LIB_PATH=$L timeout -k 10 300 python -u tools/bench_legs/hist_leg.py ${HIST_ARGS:-} > gpurun_out/${T}_${V}_$rep.txt 2>&1 || { echo leg_failed $V; tail -30 gpurun_out/${T}_${V}_$rep.txt; exit 1; }
    echo "$V $rep $(tail -1 gpurun_out/${T}_${V}_$rep.txt)"
  done
done
echo all_ok
