# rocprofv3 kernel-trace stats over bench.py, then FETCH_SIZE / WRITE_SIZE passes (tag in $1)
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-prof}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_trace -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline > $R/gpurun_out/${T}_trace_bench.txt 2>&1 || { echo trace_failed; tail -20 $R/gpurun_out/${T}_trace_bench.txt; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/${T}_pmc_fetch -o run -- python3 $R/bench.py --n 131072 --steps 1 --warmup 0 --no-extras --no-cpu-baseline > $R/gpurun_out/${T}_pmc_fetch.txt 2>&1 || { echo pmc1_failed; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/${T}_pmc_write -o run -- python3 $R/bench.py --n 131072 --steps 1 --warmup 0 --no-extras --no-cpu-baseline > $R/gpurun_out/${T}_pmc_write.txt 2>&1 || { echo pmc2_failed; exit 1; }
echo all_ok
