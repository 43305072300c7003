# ct x pt with masked batch inversion: parity tests (neg/sub/mul), then the bench's mul leg
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_parity.py tests/test_gpu_edges.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/mulinv_tests.txt 2>&1 || { echo tests_failed; tail -40 gpurun_out/mulinv_tests.txt; exit 1; }
timeout -k 10 200 python -u tools/bench_legs/mul_leg.py > gpurun_out/mul_leg_batch.txt 2>&1 || { echo leg_failed; tail -20 gpurun_out/mul_leg_batch.txt; exit 1; }
FPHE_NEG_BATCH_MIN=1000000000000 timeout -k 10 200 python -u tools/bench_legs/mul_leg.py > gpurun_out/mul_leg_single.txt 2>&1 || { echo leg2_failed; tail -20 gpurun_out/mul_leg_single.txt; exit 1; }
tail -3 gpurun_out/mulinv_tests.txt; cat gpurun_out/mul_leg_*.txt
echo all_ok
