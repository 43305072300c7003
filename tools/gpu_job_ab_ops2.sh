# same-box A/B of the op legs (tools/bench_legs/ab_ops_leg.py): tools/gpu_job_ab_ops2.sh TAG VARIANT...
# (fate_amd/lib/ab/lib_<V>.so; "main" = fate_amd/lib/libfatephe.so), two alternating rounds
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
T=$1; shift
for rep in 1 2; do
  for V in "$@"; do
    L=$R/fate_amd/lib/ab/lib_$V.so; [ "$V" = main ] && L=$R/fate_amd/lib/libfatephe.so
    FPHE_LIB_PATH=$L timeout -k 10 300 python -u tools/bench_legs/ab_ops_leg.py > gpurun_out/${T}_${V}_$rep.txt 2>&1 || { echo leg_failed $V; tail -30 gpurun_out/${T}_${V}_$rep.txt; exit 1; }
    echo "$V $rep $(tail -1 gpurun_out/${T}_${V}_$rep.txt)"
  done
done
echo all_ok
