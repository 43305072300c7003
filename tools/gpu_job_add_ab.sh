# ct-add variants (FPHE_ADD_KEEPY / FPHE_ADD_OCC): same-box A/B of the op legs, then FETCH_SIZE /
# WRITE_SIZE passes over the ct-add leg for variant $2 (tag $1)
set -o pipefail
R=$GRAFT_REPO_ROOT
T=$1; V=$2; shift 2
cd $R && mkdir -p gpurun_out
bash tools/gpu_job_ab_ops2.sh $T "$@" || exit 1
export FPHE_LIB_PATH=$R/fate_amd/lib/ab/lib_$V.so
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/${T}_fetch -o run -- python3 $R/tools/bench_legs/ops_pmc_leg.py > $R/gpurun_out/${T}_fetch.txt 2>&1 || { echo fetch_failed; tail -20 $R/gpurun_out/${T}_fetch.txt; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/${T}_write -o run -- python3 $R/tools/bench_legs/ops_pmc_leg.py > $R/gpurun_out/${T}_write.txt 2>&1 || { echo write_failed; tail -20 $R/gpurun_out/${T}_write.txt; exit 1; }
cd $R && python tools/pmc_ops_summary.py gpurun_out/$T gpurun_out/${T}_pmc_ops.json && cat gpurun_out/${T}_pmc_ops.json
echo all_ok
