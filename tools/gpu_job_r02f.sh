# full GPU suite on the shipped build, then same-box A/B of the vector-op legs at 2 vs 3
# waves/SIMD (tools/gpu_job_ab_ops.sh; lib/ab/lib_occ3.so = -DFPHE_MISC_OCC=3)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
T=${1:-r02f}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.txt 2>&1 || { echo tests_failed; tail -40 gpurun_out/${T}_tests.txt; exit 1; }
tail -1 gpurun_out/${T}_tests.txt
bash tools/gpu_job_ab_ops.sh ${T}_ab main occ3 || exit 1
