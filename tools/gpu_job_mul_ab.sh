# ct x pt: parity tests of the ops that run k_mul27, a same-box A/B of the mul leg against
# variant library $2 (alternating), then two SQ counter passes over the mul leg (tag $1)
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-mulab}; V=${2:-mul0}
cd $R && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_ops.py tests/test_gpu_golden_ops.py tests/test_gpu_protocol.py tests/test_gpu_parity.py tests/test_gpu_edges.py -k "mul or matmul or chain or span or squeeze" > gpurun_out/${T}_tests.txt 2>&1 || { echo tests_failed; tail -40 gpurun_out/${T}_tests.txt; exit 1; }
tail -3 gpurun_out/${T}_tests.txt
for i in 1 2; do
  timeout -k 10 200 python -u tools/bench_legs/mul_leg.py > gpurun_out/${T}_new$i.txt 2>&1 || { echo leg_failed; tail -20 gpurun_out/${T}_new$i.txt; exit 1; }
  FPHE_LIB_PATH=$R/fate_amd/lib/ab/lib_$V.so timeout -k 10 200 python -u tools/bench_legs/mul_leg.py > gpurun_out/${T}_old$i.txt 2>&1 || { echo leg_old_failed; tail -20 gpurun_out/${T}_old$i.txt; exit 1; }
done
for f in gpurun_out/${T}_new*.txt gpurun_out/${T}_old*.txt; do echo $f; grep rep $f; done
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM"
P2="SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_VALU"
for p in 1 2; do
  eval C=\$P$p
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $R/gpurun_out/${T}_m$p -o run -- python3 $R/tools/bench_legs/mul_leg.py 262144 > $R/gpurun_out/${T}_m$p.txt 2>&1 || { echo pmc_m${p}_failed; tail -20 $R/gpurun_out/${T}_m$p.txt; exit 1; }
done
echo all_ok
