# neg / sub: parity tests, then batch-inversion vs per-element-inverse timing (2048 and 1024 bits)
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_ops.py -m gpu -x -v --timeout 200 --timeout-method thread -k "neg or sub" > gpurun_out/neg_tests.txt 2>&1 || { echo tests_failed; tail -40 gpurun_out/neg_tests.txt; exit 1; }
timeout -k 10 200 python -u tools/bench_legs/neg_leg.py > gpurun_out/neg_leg_batch.txt 2>&1 || { echo leg_failed; tail -20 gpurun_out/neg_leg_batch.txt; exit 1; }
FPHE_NEG_BATCH_MIN=1000000000000 timeout -k 10 200 python -u tools/bench_legs/neg_leg.py > gpurun_out/neg_leg_single.txt 2>&1 || { echo leg2_failed; tail -20 gpurun_out/neg_leg_single.txt; exit 1; }
timeout -k 10 200 python -u tools/bench_legs/neg_leg.py 1048576 1024 > gpurun_out/neg_leg_batch1024.txt 2>&1 || { echo leg3_failed; exit 1; }
FPHE_NEG_BATCH_MIN=1000000000000 timeout -k 10 200 python -u tools/bench_legs/neg_leg.py 1048576 1024 > gpurun_out/neg_leg_single1024.txt 2>&1 || { echo leg4_failed; exit 1; }
tail -3 gpurun_out/neg_tests.txt; cat gpurun_out/neg_leg_*.txt
echo all_ok
