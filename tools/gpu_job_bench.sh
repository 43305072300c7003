# the default bench line alone (tag $1)
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-bench}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u bench.py > gpurun_out/${T}_bench.txt 2>&1 || { echo bench_failed; tail -30 gpurun_out/${T}_bench.txt; exit 1; }
tail -1 gpurun_out/${T}_bench.txt > gpurun_out/${T}_bench.json
echo all_ok
