# SQ counter passes over the fold kernels (tools/bench_legs/fold_leg.py), one --pmc pass each; tag $1
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-foldpmc}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $R/gpurun_out/${T}_sq -o run -- python3 $R/tools/bench_legs/fold_leg.py 1048576 4 2 > $R/gpurun_out/${T}_sq.txt 2>&1 || { echo pmc_sq_failed; tail -20 $R/gpurun_out/${T}_sq.txt; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH --output-format csv -d $R/gpurun_out/${T}_sq2 -o run -- python3 $R/tools/bench_legs/fold_leg.py 1048576 4 2 > $R/gpurun_out/${T}_sq2.txt 2>&1 || { echo pmc_sq2_failed; tail -20 $R/gpurun_out/${T}_sq2.txt; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_kt -o run -- python3 $R/tools/bench_legs/fold_leg.py 1048576 4 3 > $R/gpurun_out/${T}_kt.txt 2>&1 || { echo kt_failed; tail -20 $R/gpurun_out/${T}_kt.txt; exit 1; }
cat $R/gpurun_out/${T}_kt.txt | grep rep
echo all_ok
