# same-box comparison: the throughput probe's general-product fold loop (256 products per
# wave, random operands) against k_segfold27 on the bench's histogram shape (tag $1)
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-segprobe}
cd $R && mkdir -p gpurun_out
timeout -k 10 120 tools/probe/mulsq_probe 256 1 > gpurun_out/${T}_probe.txt 2>&1 || { echo probe_failed; exit 1; }
cat gpurun_out/${T}_probe.txt
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 180 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_kt -o run -- python3 $R/tools/bench_legs/fold_host_time.py > $R/gpurun_out/${T}_kt.txt 2>&1 || { echo kt_failed; tail -20 $R/gpurun_out/${T}_kt.txt; exit 1; }
grep -E "segfold|fold27|align_rows|tiles_to_rows" $R/gpurun_out/${T}_kt/run_kernel_stats.csv | cut -c1-60,200-400
echo all_ok
