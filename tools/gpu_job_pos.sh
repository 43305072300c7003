# fphe_positions_terms: fold / ops / config-4 tests, then the histogram leg's timeline
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-pos}
set -o pipefail
timeout -k 10 900 python -u -m pytest tests/test_gpu_fold.py tests/test_gpu_ops.py tests/test_gpu_config4_gmp.py tests/test_gpu_protocol.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.txt 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/${T}_tests.txt | tail -2; grep -E "^FAILED|^ERROR" gpurun_out/${T}_tests.txt | head
[ $rc -eq 0 ] || exit 1
TL_LAST=200 bash tools/gpu_job.sh ${T} timeline
