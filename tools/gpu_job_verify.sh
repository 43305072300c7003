set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/verify_tests.txt 2>&1 || { echo tests_failed; exit 1; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/verify_smoke.txt 2>&1 || { echo smoke_failed; exit 1; }
timeout -k 10 400 python bench.py --steps 2 --warmup 1 > gpurun_out/verify_bench.txt 2>&1 || { echo bench_failed; exit 1; }
echo all_ok
