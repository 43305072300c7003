set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python tools/bench_legs/hist_leg.py > gpurun_out/hist_leg.txt 2>&1 || { echo hist_failed; tail gpurun_out/hist_leg.txt; exit 1; }
cat gpurun_out/hist_leg.txt | grep rep
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/hist_trace -o run -- python3 $R/tools/bench_legs/hist_leg.py > $R/gpurun_out/hist_trace.txt 2>&1 || { echo trace_failed; exit 1; }
echo all_ok
