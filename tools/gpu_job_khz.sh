# Key-holder direct (z_p, z_q) draw: parity/edge/config tests, then the key-holder rate with
# the direct draw (default) and with FPHE_KH_DIRECT_Z=0 (r drawn, two-step modexp)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:-khz}
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_gpu_configs.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.txt 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/${T}_tests.txt | tail -2; grep -E "^FAILED|^ERROR" gpurun_out/${T}_tests.txt | head
[ $rc -eq 0 ] || exit 1
timeout -k 10 180 python -u tools/bench_legs/kh_leg.py > gpurun_out/${T}_kh_direct.txt 2>&1 || { tail -20 gpurun_out/${T}_kh_direct.txt; exit 1; }
FPHE_KH_DIRECT_Z=0 timeout -k 10 180 python -u tools/bench_legs/kh_leg.py > gpurun_out/${T}_kh_twostep.txt 2>&1 || { tail -20 gpurun_out/${T}_kh_twostep.txt; exit 1; }
tail -1 gpurun_out/${T}_kh_direct.txt; tail -1 gpurun_out/${T}_kh_twostep.txt
