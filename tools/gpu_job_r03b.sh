# round-3 check in one call (tag in $1): the GPU test suite (all tests, no -x), smoke, the
# default bench line (with the CPU baseline), then FETCH/WRITE PMC passes over the
# decrypt / ct-add leg
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-r03b}
cd $R
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.txt 2>&1
rc=$?
tail -15 gpurun_out/${T}_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests aborted rc=$rc"; exit 1; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { echo smoke_failed; tail -20 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench.txt 2>&1 || { echo bench_failed; tail -30 gpurun_out/${T}_bench.txt; exit 1; }
tail -1 gpurun_out/${T}_bench.txt > gpurun_out/${T}_bench.json
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/${T}_fetch -o run -- python3 $R/tools/bench_legs/ops_pmc_leg.py > $R/gpurun_out/${T}_fetch.txt 2>&1 || { echo fetch_failed; tail -20 $R/gpurun_out/${T}_fetch.txt; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/${T}_write -o run -- python3 $R/tools/bench_legs/ops_pmc_leg.py > $R/gpurun_out/${T}_write.txt 2>&1 || { echo write_failed; tail -20 $R/gpurun_out/${T}_write.txt; exit 1; }
cd $R && python tools/pmc_ops_summary.py gpurun_out/$T gpurun_out/${T}_pmc_ops.json && grep -A3 '"ct_add"' gpurun_out/${T}_pmc_ops.json; grep hbm_bytes_per_elem gpurun_out/${T}_pmc_ops.json
echo tests_rc=$rc
