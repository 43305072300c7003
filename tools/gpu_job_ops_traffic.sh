# FETCH_SIZE and WRITE_SIZE passes (separate runs) over the decrypt / ct-add leg (tag in $1)
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-opstraffic}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/${T}_fetch -o run -- python3 $R/tools/bench_legs/ops_pmc_leg.py > $R/gpurun_out/${T}_fetch.txt 2>&1 || { echo fetch_failed; tail -20 $R/gpurun_out/${T}_fetch.txt; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/${T}_write -o run -- python3 $R/tools/bench_legs/ops_pmc_leg.py > $R/gpurun_out/${T}_write.txt 2>&1 || { echo write_failed; tail -20 $R/gpurun_out/${T}_write.txt; exit 1; }
echo all_ok
