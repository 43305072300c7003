set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/r01c_tests.txt 2>&1 || { echo tests_failed; exit 1; }
timeout -k 10 400 python bench.py > gpurun_out/r01c_bench.txt 2>&1 || { echo bench_failed; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r01c_trace -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/r01c_trace_bench.txt 2>&1 || { echo trace_failed; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/r01c_pmc_fetch -o run -- python3 $R/bench.py --n 131072 --steps 1 --warmup 0 --no-extras --no-cpu-baseline > $R/gpurun_out/r01c_pmc_fetch.txt 2>&1 || { echo pmc1_failed; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/r01c_pmc_write -o run -- python3 $R/bench.py --n 131072 --steps 1 --warmup 0 --no-extras --no-cpu-baseline > $R/gpurun_out/r01c_pmc_write.txt 2>&1 || { echo pmc2_failed; exit 1; }
echo all_ok
