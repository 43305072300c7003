# Parameterised GPU job (replaces the round-1..3 one-off gpu_job_*.sh scripts).
#   tools/gpu_job.sh TAG MODE [pytest-args...]
# MODE: tests   the GPU test suite (no -x: every failure listed), args select tests
#       round   tests + smoke + the default bench line
#       bench   the default bench line only
#       prof    rocprofv3 kernel trace + stats of a short bench run
# Every GPU step runs under its own time limit; the script stops at the first abort.
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:?tag}
M=${2:-round}
shift 2 || true
cd $R
mkdir -p gpurun_out
run_tests() {
  timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread "$@" > gpurun_out/${T}_tests.txt 2>&1
  local rc=$?
  grep -E "passed|failed|error" gpurun_out/${T}_tests.txt | tail -3
  grep -E "^FAILED|^ERROR" gpurun_out/${T}_tests.txt | head -40
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests aborted rc=$rc"; exit 1; fi
  echo tests_rc=$rc
}
run_bench() {
  timeout -k 10 900 python -u bench.py "$@" > gpurun_out/${T}_bench.txt 2>&1 || { echo bench_failed; tail -30 gpurun_out/${T}_bench.txt; exit 1; }
  tail -1 gpurun_out/${T}_bench.txt > gpurun_out/${T}_bench.json
  python -c "import json;d=json.load(open('gpurun_out/${T}_bench.json'));print(d['value'], d['roofline']['frac'], {k: d.get(k) for k in ('decrypt_per_s','ct_add_per_s','ct_mul_per_s','histogram_iupdate_s')})"
}
case $M in
  tests) run_tests "$@" ;;
  round)
    run_tests "$@"
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { echo smoke_failed; tail -20 gpurun_out/${T}_smoke.log; exit 1; }
    tail -1 gpurun_out/${T}_smoke.log
    run_bench ;;
  bench) run_bench "$@" ;;
  prof)
    cd /tmp && export TMPDIR=/tmp && cd $R
    timeout -k 10 900 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run -- python3 -u bench.py "$@" > gpurun_out/${T}_prof_bench.txt 2>&1 || { echo prof_failed; tail -30 gpurun_out/${T}_prof_bench.txt; exit 1; }
    tail -1 gpurun_out/${T}_prof_bench.txt > gpurun_out/${T}_prof_bench.json
    find gpurun_out/${T}_prof -name "*kernel_stats.csv" | head -3 ;;
  *) echo "unknown mode $M"; exit 2 ;;
esac
