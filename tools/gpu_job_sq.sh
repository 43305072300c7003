# SQ issue/wait counters + GRBM clocks for the encrypt kernel (one --pmc pass; tag in $1)
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-sq}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc ${PMC:-SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT} --output-format csv -d $R/gpurun_out/${T}_pmc -o run -- python3 $R/bench.py --n 262144 --steps 1 --warmup 0 --no-extras --no-cpu-baseline > $R/gpurun_out/${T}_pmc.txt 2>&1 || { echo pmc_failed; tail -20 $R/gpurun_out/${T}_pmc.txt; exit 1; }
echo all_ok
