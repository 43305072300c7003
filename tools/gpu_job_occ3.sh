# Round-2 opening call (tag in $1): the GPU suite and a bench line on the shipped library,
# then the 3-wave vector-op build (tools/build_ab.sh occ3 -DFPHE_MISC_OCC=3) through the
# parity/ops tests with kernels serialised, so a fault names its kernel and test.  The
# variant runs last: a fault ends the call.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
T=${1:-occ3}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.txt 2>&1 || { echo tests_failed; tail -30 gpurun_out/${T}_tests.txt; exit 1; }
tail -1 gpurun_out/${T}_tests.txt
timeout -k 10 400 python -u bench.py --steps 2 --warmup 1 > gpurun_out/${T}_bench.txt 2>&1 || { echo bench_failed; tail -30 gpurun_out/${T}_bench.txt; exit 1; }
tail -1 gpurun_out/${T}_bench.txt
FPHE_LIB_PATH=$R/fate_amd/lib/ab/lib_occ3.so AMD_SERIALIZE_KERNEL=3 AMD_LOG_LEVEL=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ops.py tests/test_gpu_edges.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_variant_tests.txt 2>&1 || { echo variant_failed; tail -40 gpurun_out/${T}_variant_tests.txt; exit 1; }
tail -1 gpurun_out/${T}_variant_tests.txt
echo all_ok
