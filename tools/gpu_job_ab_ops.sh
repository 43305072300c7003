# same-box A/B of the vector-op legs (ct-add, ct x pt, histograms, Hetero-LR): tools/gpu_job_ab_ops.sh TAG VARIANT...
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
T=$1; shift
for V in "$@"; do
  L=$R/fate_amd/lib/ab/lib_$V.so; [ "$V" = main ] && L=$R/fate_amd/lib/libfatephe.so
  FPHE_LIB_PATH=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ops.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_${V}_tests.txt 2>&1 || { echo tests_failed $V; tail -30 gpurun_out/${T}_${V}_tests.txt; exit 1; }
done
for rep in 1 2; do
  for V in "$@"; do
    L=$R/fate_amd/lib/ab/lib_$V.so; [ "$V" = main ] && L=$R/fate_amd/lib/libfatephe.so
    FPHE_LIB_PATH=$L timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_${V}_b$rep.txt 2>&1 || { echo bench_failed $V; tail -30 gpurun_out/${T}_${V}_b$rep.txt; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'add', d['ct_add_per_s'], 'mul', d['ct_mul_per_s'], 'hist', d['histogram_scatter_adds_per_s'], 'hlr_rmatmul_s', d['hetero_lr_gradient']['host_rmatmul_s'], 'sq_s', d['histogram_packed']['squeeze_s'])" gpurun_out/${T}_${V}_b$rep.txt $V
  done
done
echo all_ok
