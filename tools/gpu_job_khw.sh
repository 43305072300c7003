# Key-holder latency kernel: parity/edge/config tests, then the latency leg (wide vs throughput)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-khw}
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_gpu_configs.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.txt 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/${T}_tests.txt | tail -2; grep -E "^FAILED|^ERROR" gpurun_out/${T}_tests.txt | head
[ $rc -eq 0 ] || exit 1
timeout -k 10 400 python -u tools/bench_legs/latency_leg.py > gpurun_out/${T}_latency_leg.txt 2>&1 || { tail -20 gpurun_out/${T}_latency_leg.txt; exit 1; }
cat gpurun_out/${T}_latency_leg.txt
