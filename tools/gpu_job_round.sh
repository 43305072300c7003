# round-end evidence in one call (tag in $1): full GPU test suite, the default bench line
# (with the CPU baseline), then rocprofv3 kernel-trace stats and FETCH/WRITE PMC passes
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-round}
cd $R
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.txt 2>&1 || { echo tests_failed; tail -40 gpurun_out/${T}_tests.txt; exit 1; }
tail -2 gpurun_out/${T}_tests.txt
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench.txt 2>&1 || { echo bench_failed; tail -30 gpurun_out/${T}_bench.txt; exit 1; }
tail -1 gpurun_out/${T}_bench.txt > gpurun_out/${T}_bench.json
bash tools/gpu_job_prof.sh $T || exit 1
echo all_ok
