# fold tests + the bench-shape histogram leg (real encryptions, tools/bench_legs/hist_leg.py)
# under a kernel trace, with the last iupdate's timeline; tag $1
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-fold4}
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_fold.py tests/test_gpu_ops.py -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.txt 2>&1
rc=$?
tail -4 gpurun_out/${T}_tests.txt
if [ $rc -ne 0 ]; then echo "tests rc=$rc"; exit 1; fi
timeout -k 10 180 python3 tools/bench_legs/hist_leg.py > gpurun_out/${T}_hist.txt 2>&1 || { echo hist_failed; tail -20 gpurun_out/${T}_hist.txt; exit 1; }
cat gpurun_out/${T}_hist.txt
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_kt -o run -- python3 $R/tools/bench_legs/hist_leg.py > $R/gpurun_out/${T}_kt.txt 2>&1 || { echo kt_failed; tail -20 $R/gpurun_out/${T}_kt.txt; exit 1; }
cd $R && python tools/rocpd_timeline.py $(ls gpurun_out/${T}_kt/*.db | head -1) 45
echo all_ok
