# general-product rows unrolled by 2 (FPHE_ROW_UNROLL): same-box A/B of the op legs and the
# histogram leg, lib_u1.so vs lib_u2.so, alternating (tag $1)
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-unroll}
cd $R && mkdir -p gpurun_out
bash tools/gpu_job_ab_ops2.sh $T u1 u2 || exit 1
for rep in 1 2; do
  for V in u1 u2; do
    FPHE_LIB_PATH=$R/fate_amd/lib/ab/lib_$V.so timeout -k 10 180 python3 tools/bench_legs/hist_leg.py > gpurun_out/${T}_hist_${V}_$rep.txt 2>&1 || { echo hist_failed; exit 1; }
    echo "hist $V $rep $(tail -1 gpurun_out/${T}_hist_${V}_$rep.txt)"
  done
done
echo all_ok
