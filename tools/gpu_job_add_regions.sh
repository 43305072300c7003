# ct-add XCD runs: parity tests of the ops that run k_add27, same-box A/B of the op legs
# (new build vs lib_head.so with the round-2 global gap sort), FETCH/WRITE PMC passes over the
# ct-add/decrypt leg on the new build (tag $1)
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-addreg}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_fold.py tests/test_gpu_edges.py tests/test_gpu_parity.py tests/test_gpu_golden_ops.py -k "add or fold or chain or literal or iupdate or sub or neg or cumsum or order" > gpurun_out/${T}_tests.txt 2>&1 || { echo tests_failed; tail -40 gpurun_out/${T}_tests.txt; exit 1; }
tail -3 gpurun_out/${T}_tests.txt
for rep in 1 2; do
  timeout -k 10 300 python -u tools/bench_legs/ab_ops_leg.py > gpurun_out/${T}_new_$rep.txt 2>&1 || { echo leg_failed; tail -30 gpurun_out/${T}_new_$rep.txt; exit 1; }
  echo "new $rep $(tail -1 gpurun_out/${T}_new_$rep.txt)"
  FPHE_ADD_REGION_SORT=0 FPHE_LIB_PATH=$R/fate_amd/lib/ab/lib_head.so timeout -k 10 300 python -u tools/bench_legs/ab_ops_leg.py > gpurun_out/${T}_head_$rep.txt 2>&1 || { echo leg_failed; tail -30 gpurun_out/${T}_head_$rep.txt; exit 1; }
  echo "head $rep $(tail -1 gpurun_out/${T}_head_$rep.txt)"
done
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/${T}_fetch -o run -- python3 $R/tools/bench_legs/ops_pmc_leg.py > $R/gpurun_out/${T}_fetch.txt 2>&1 || { echo fetch_failed; tail -20 $R/gpurun_out/${T}_fetch.txt; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/${T}_write -o run -- python3 $R/tools/bench_legs/ops_pmc_leg.py > $R/gpurun_out/${T}_write.txt 2>&1 || { echo write_failed; tail -20 $R/gpurun_out/${T}_write.txt; exit 1; }
cd $R && python tools/pmc_ops_summary.py gpurun_out/$T gpurun_out/${T}_pmc_ops.json && cat gpurun_out/${T}_pmc_ops.json
echo all_ok
