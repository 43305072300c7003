# encrypt-path iteration: parity tests, then the headline encrypt leg only (tag in $1)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
T=${1:-enc}
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.txt 2>&1 || { echo tests_failed; tail -30 gpurun_out/${T}_tests.txt; exit 1; }
timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/${T}_bench.txt 2>&1 || { echo bench_failed; tail -30 gpurun_out/${T}_bench.txt; exit 1; }
tail -1 gpurun_out/${T}_bench.txt
echo all_ok
