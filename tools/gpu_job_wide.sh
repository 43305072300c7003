cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
set -o pipefail

mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_golden_ops.py tests/test_gpu_config4_gmp.py tests/test_gpu_edges.py -k "squeeze or other_key_sizes or config4" -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r05f_tests.txt 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/r05f_tests.txt | tail -2; grep -E "^FAILED|^ERROR" gpurun_out/r05f_tests.txt | head
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python -u tools/bench_legs/squeeze_leg.py > gpurun_out/r05f_squeeze_leg.txt 2>&1 || { tail -20 gpurun_out/r05f_squeeze_leg.txt; exit 1; }
grep '^{' gpurun_out/r05f_squeeze_leg.txt
