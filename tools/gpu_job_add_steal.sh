# k_add27 run stealing: ct-add parity tests, then a same-box A/B of the op legs against
# lib_nosteal.so (the XCD runs without stealing), alternating (tag $1)
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-steal}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_edges.py tests/test_gpu_parity.py -k "add or chain or literal or order or neg or sub" > gpurun_out/${T}_tests.txt 2>&1 || { echo tests_failed; tail -40 gpurun_out/${T}_tests.txt; exit 1; }
tail -2 gpurun_out/${T}_tests.txt
for rep in 1 2 3; do
  timeout -k 10 300 python -u tools/bench_legs/ab_ops_leg.py > gpurun_out/${T}_new_$rep.txt 2>&1 || { echo leg_failed; tail -30 gpurun_out/${T}_new_$rep.txt; exit 1; }
  echo "steal $rep $(tail -1 gpurun_out/${T}_new_$rep.txt)"
  FPHE_LIB_PATH=$R/fate_amd/lib/ab/lib_nosteal.so timeout -k 10 300 python -u tools/bench_legs/ab_ops_leg.py > gpurun_out/${T}_old_$rep.txt 2>&1 || { echo leg_failed; tail -30 gpurun_out/${T}_old_$rep.txt; exit 1; }
  echo "nosteal $rep $(tail -1 gpurun_out/${T}_old_$rep.txt)"
done
timeout -k 10 180 python3 tools/bench_legs/hist_leg.py > gpurun_out/${T}_hist.txt 2>&1 || { echo hist_failed; tail -20 gpurun_out/${T}_hist.txt; exit 1; }
cat gpurun_out/${T}_hist.txt
echo all_ok
