# vector-op kernels (k_mul27, k_sqmul27, k_align27, k_align_rows27) at 2 waves/SIMD instead of 3:
# same-box A/B of the op legs and the histogram leg (tag $1)
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-misc}
cd $R && mkdir -p gpurun_out
bash tools/gpu_job_ab_ops2.sh $T main3 misc2 || exit 1
for rep in 1 2; do
  for V in main3 misc2; do
    FPHE_LIB_PATH=$R/fate_amd/lib/ab/lib_$V.so timeout -k 10 180 python3 tools/bench_legs/hist_leg.py > gpurun_out/${T}_hist_${V}_$rep.txt 2>&1 || { echo hist_failed; exit 1; }
    echo "hist $V $rep $(tail -1 gpurun_out/${T}_hist_${V}_$rep.txt)"
  done
done
echo all_ok
