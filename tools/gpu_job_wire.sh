# wire format: GPU tests, then a 2^20-element 2048-bit encode/decode timing
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_wire.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/wire_tests.txt 2>&1 || { echo tests_failed; tail -40 gpurun_out/wire_tests.txt; exit 1; }
tail -2 gpurun_out/wire_tests.txt
timeout -k 10 300 python -u tools/bench_legs/wire_leg.py > gpurun_out/wire_leg.txt 2>&1 || { echo leg_failed; tail -20 gpurun_out/wire_leg.txt; exit 1; }
cat gpurun_out/wire_leg.txt
echo all_ok
