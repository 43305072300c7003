set -o pipefail
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 200 python3 -u $R/tools/bench_legs/neg_leg.py > $R/gpurun_out/r02z5_neg_leg.txt 2>&1 || exit 1
tail -1 $R/gpurun_out/r02z5_neg_leg.txt
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/r02z5_prof -o mul -- python3 -u $R/tools/bench_legs/mul_leg.py > $R/gpurun_out/r02z5_mul_leg.txt 2>&1 || exit 1
tail -2 $R/gpurun_out/r02z5_mul_leg.txt
find $R/gpurun_out/r02z5_prof -name "*kernel_stats.csv" | head -1 | xargs -I{} sh -c 'cut -d, -f1-4 {} | head -12'
