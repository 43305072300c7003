# GPU tests of the ops touched (ct-add, folds), then SQ counter passes over the iupdate leg
# (k_segfold27 and the grouping) and over the throughput probe's fold loop, for comparison (tag $1)
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-segpmc}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_fold.py tests/test_gpu_edges.py -k "add or fold or chain or literal or iupdate" > gpurun_out/${T}_tests.txt 2>&1 || { echo tests_failed; tail -40 gpurun_out/${T}_tests.txt; exit 1; }
tail -3 gpurun_out/${T}_tests.txt
timeout -k 10 120 tools/probe/mulsq_probe 300 1 > gpurun_out/${T}_probe_rnd.txt 2>&1 || { echo probe_failed; exit 1; }
cat gpurun_out/${T}_probe_rnd.txt
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM"
P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_VALU"
for p in 1 2; do
  eval C=\$P$p
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $R/gpurun_out/${T}_h$p -o run -- python3 $R/tools/bench_legs/hist_leg.py > $R/gpurun_out/${T}_h$p.txt 2>&1 || { echo pmc_h${p}_failed; tail -20 $R/gpurun_out/${T}_h$p.txt; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $R/gpurun_out/${T}_p$p -o run -- $R/tools/probe/mulsq_probe 100 > $R/gpurun_out/${T}_p$p.txt 2>&1 || { echo pmc_p${p}_failed; tail -20 $R/gpurun_out/${T}_p$p.txt; exit 1; }
done
echo all_ok
