# fold tests, then the SecureBoost leg under rocprofv3 kernel trace (per-kernel time of iupdate)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-fold}
timeout -k 10 600 python -u -m pytest tests/test_gpu_fold.py tests/test_gpu_ops.py -v --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.txt 2>&1
rc=$?
tail -6 gpurun_out/${T}_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests aborted rc=$rc"; exit 1; fi
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run -- python3 -u tools/bench_legs/hist_leg.py > gpurun_out/${T}_hist.txt 2>&1 || { echo hist_failed; tail -20 gpurun_out/${T}_hist.txt; exit 1; }
grep rep gpurun_out/${T}_hist.txt
find gpurun_out/${T}_prof -name "*kernel_stats.csv" | head -3
echo tests_rc=$rc
