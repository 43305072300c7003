# same-box A/B of the pow_half27 users (decrypt, key-holder encrypt): tools/gpu_job_ab_dec.sh TAG VARIANT...
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
T=$1; shift
for V in "$@"; do
  L=$R/fate_amd/lib/ab/lib_$V.so; [ "$V" = main ] && L=$R/fate_amd/lib/libfatephe.so
  FPHE_LIB_PATH=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_${V}_tests.txt 2>&1 || { echo tests_failed $V; tail -30 gpurun_out/${T}_${V}_tests.txt; exit 1; }
done
for rep in 1 2; do
  for V in "$@"; do
    L=$R/fate_amd/lib/ab/lib_$V.so; [ "$V" = main ] && L=$R/fate_amd/lib/libfatephe.so
    FPHE_LIB_PATH=$L timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_${V}_b$rep.txt 2>&1 || { echo bench_failed $V; tail -30 gpurun_out/${T}_${V}_b$rep.txt; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'enc', d['value'], 'dec', d['decrypt_per_s'], 'crt_enc', d['encrypt_keyholder_crt_per_s'])" gpurun_out/${T}_${V}_b$rep.txt $V
  done
done
echo all_ok
