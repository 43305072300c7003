# fold tests + the synthetic fold leg under a kernel trace; tag $1
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-fold}
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fold.py tests/test_gpu_ops.py tests/test_gpu_rccl.py -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.txt 2>&1
rc=$?
tail -4 gpurun_out/${T}_tests.txt
if [ $rc -ne 0 ]; then echo "tests rc=$rc"; exit 1; fi
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_kt -o run -- python3 $R/tools/bench_legs/fold_leg.py 1048576 4 3 > $R/gpurun_out/${T}_kt.txt 2>&1 || { echo kt_failed; tail -20 $R/gpurun_out/${T}_kt.txt; exit 1; }
grep rep $R/gpurun_out/${T}_kt.txt
timeout -k 10 180 python3 $R/tools/bench_legs/fold_leg.py 1048576 4 3
echo all_ok
