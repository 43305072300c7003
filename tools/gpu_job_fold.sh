# the device-grouped fold: its tests, the other fold users, then the SecureBoost leg timed
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-fold}
timeout -k 10 600 python -u -m pytest tests/test_gpu_fold.py tests/test_gpu_ops.py tests/test_gpu_rccl.py tests/test_gpu_protocol.py -v --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.txt 2>&1
rc=$?
tail -12 gpurun_out/${T}_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests aborted rc=$rc"; exit 1; fi
timeout -k 10 300 python -u tools/bench_legs/hist_leg.py > gpurun_out/${T}_hist.txt 2>&1 || { echo hist_failed; tail -20 gpurun_out/${T}_hist.txt; exit 1; }
cat gpurun_out/${T}_hist.txt
echo tests_rc=$rc
