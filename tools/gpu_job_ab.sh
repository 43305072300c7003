# Same-box A/B of library variants: tools/gpu_job_ab.sh TAG [--no-tests] VARIANT...
# (fate_amd/lib/ab/lib_<V>.so; "main" = fate_amd/lib/libfatephe.so).  Each variant: the parity
# tests (unless --no-tests: a variant from before an ABI change), then two alternating
# encrypt-only bench runs (or, with LEG=script.py, runs of tools/bench_legs/script.py with the
# arguments in LEGARGS; TESTFILES replaces the parity tests run per variant).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
T=$1; shift
TESTS=1
if [ "$1" = "--no-tests" ]; then TESTS=0; shift; fi
lib_of() { if [ "$1" = main ]; then echo $R/fate_amd/lib/libfatephe.so; else echo $R/fate_amd/lib/ab/lib_$1.so; fi; }
if [ $TESTS = 1 ]; then
  for V in "$@"; do
    FPHE_LIB_PATH=$(lib_of $V) timeout -k 10 300 python -u -m pytest ${TESTFILES:-tests/test_gpu_parity.py} -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_${V}_tests.txt 2>&1 || { echo tests_failed $V; tail -30 gpurun_out/${T}_${V}_tests.txt; exit 1; }
  done
fi
for rep in 1 2; do
  for V in "$@"; do
    if [ -n "$LEG" ]; then  # LEG=script.py: a tools/bench_legs script printing one JSON line
      FPHE_LIB_PATH=$(lib_of $V) timeout -k 10 300 python tools/bench_legs/$LEG $LEGARGS > gpurun_out/${T}_${V}_b$rep.txt 2>&1 || { echo leg_failed $V; tail -30 gpurun_out/${T}_${V}_b$rep.txt; exit 1; }
      echo "$V $(tail -1 gpurun_out/${T}_${V}_b$rep.txt)"
      continue
    fi
    FPHE_LIB_PATH=$(lib_of $V) timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-extras > gpurun_out/${T}_${V}_b$rep.txt 2>&1 || { echo bench_failed $V; tail -30 gpurun_out/${T}_${V}_b$rep.txt; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['value'], d['roofline']['frac'], d['roofline']['kernel_ms'])" gpurun_out/${T}_${V}_b$rep.txt $V
  done
done
echo all_ok
