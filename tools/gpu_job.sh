# Parameterised GPU job (replaces rounds 1-3's fifty one-off tools/gpu_job_*.sh scripts;
# same-box A/B of library variants stays in tools/gpu_job_ab.sh).
#   bash tools/gpu_job.sh TAG MODE [args...]
# MODE  tests     the GPU test suite (no -x: every failure listed); args: test files / -k filters
#                 in place of the whole tests/ directory
#       round     tests + smoke + the default bench line (args go to bench.py)
#       bench     the default bench line only (args go to bench.py)
#       prof      rocprofv3 --kernel-trace --stats of a short bench run
#       profhead  the same of the headline leg alone (its stats average = the per-step kernel time)
#       pmc       FETCH_SIZE / WRITE_SIZE passes (one counter per run): the encrypt kernel over
#                 bench.py --n 131072, the op kernels over tools/bench_legs/ops_pmc_leg.py,
#                 summarised into gpurun_out/TAG_pmc_encrypt27.json / TAG_pmc_ops.json
#       sq        SQ / GRBM counter passes over tools/bench_legs/ops_pmc_leg.py (or the leg
#                 script named by args, e.g. k1024_leg.py), tabled into gpurun_out/TAG_sq.txt,
#                 with each dispatch's shader clock in gpurun_out/TAG_clock.txt
#       evidence  round, then prof, then pmc (the end-of-round record for profiles/)
#       final     prof, pmc, then the 2-rank gloo rehearsal of the N > 1 bench line on the one GPU
#                 (after `round`: the rest of the end-of-round record)
#       gloo2     the 2-rank gloo rehearsal alone (config 5 at 1M per rank)
#       sqenc     SQ counter passes over the headline encrypt kernel alone
#       leg       python tools/bench_legs/ARGS (one bench leg script)
#       timeline  rocprofv3 kernel trace of tools/bench_legs/hist_leg.py ARGS (PHASES=0), last
#                 TL_LAST (90) dispatches as a timeline
# Every GPU step runs under its own time limit and the script stops at the first failure.
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:?tag}
M=${2:-round}
shift 2 || true
cd $R
mkdir -p gpurun_out

run_tests() {
  local sel=("$@")
  [ ${#sel[@]} -eq 0 ] && sel=(tests)
  timeout -k 10 1200 python -u -m pytest "${sel[@]}" -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.txt 2>&1
  local rc=$?
  grep -E "passed|failed|error" gpurun_out/${T}_tests.txt | tail -3
  grep -E "^FAILED|^ERROR" gpurun_out/${T}_tests.txt | head -40
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests aborted rc=$rc"; exit 1; fi
  echo tests_rc=$rc
}
run_smoke() {
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { echo smoke_failed; tail -20 gpurun_out/${T}_smoke.log; exit 1; }
  tail -1 gpurun_out/${T}_smoke.log
}
run_bench() {
  timeout -k 10 1000 python -u bench.py "$@" > gpurun_out/${T}_bench.txt 2>&1 || { echo bench_failed; tail -30 gpurun_out/${T}_bench.txt; exit 1; }
  tail -1 gpurun_out/${T}_bench.txt > gpurun_out/${T}_bench.json
  python tools/bench_summary.py gpurun_out/${T}_bench.json
}
run_prof() {
  (cd /tmp && export TMPDIR=/tmp && timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_trace -o run -- python3 $R/bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@" > $R/gpurun_out/${T}_trace_bench.txt 2>&1) || { echo trace_failed; tail -20 gpurun_out/${T}_trace_bench.txt; exit 1; }
  grep '^{"metric"' gpurun_out/${T}_trace_bench.txt | tail -1 > gpurun_out/${T}_trace_bench.json
  echo prof_ok
}
pmc_pass() {  # pmc_pass NAME COUNTER CMD...
  local name=$1 counter=$2
  shift 2
  (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 300 rocprofv3 --pmc $counter --output-format csv -d $R/gpurun_out/${T}_${name} -o run -- "$@" > $R/gpurun_out/${T}_${name}.txt 2>&1) || { echo pmc_${name}_failed; tail -20 gpurun_out/${T}_${name}.txt; exit 1; }
}
run_pmc() {
  pmc_pass pmc_fetch FETCH_SIZE python3 $R/bench.py --n 131072 --steps 1 --warmup 0 --no-extras --no-cpu-baseline --config5-per-rank 0
  pmc_pass pmc_write WRITE_SIZE python3 $R/bench.py --n 131072 --steps 1 --warmup 0 --no-extras --no-cpu-baseline --config5-per-rank 0
  python tools/pmc_summary.py gpurun_out/$T gpurun_out/${T}_pmc_encrypt27.json > /dev/null || exit 1
  pmc_pass fetch FETCH_SIZE python3 $R/tools/bench_legs/ops_pmc_leg.py
  pmc_pass write WRITE_SIZE python3 $R/tools/bench_legs/ops_pmc_leg.py
  python tools/pmc_ops_summary.py gpurun_out/$T gpurun_out/${T}_pmc_ops.json || exit 1
  grep hbm_bytes_per_elem gpurun_out/${T}_pmc_encrypt27.json
}
run_sq() {
  local leg=${1:-ops_pmc_leg.py}
  [ $# -gt 0 ] && shift
  pmc_pass sq "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT" python3 $R/tools/bench_legs/$leg "$@"
  pmc_pass sq2 "SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH" python3 $R/tools/bench_legs/$leg "$@"
  python tools/pmc_sq_compare.py gpurun_out/${T}_sq gpurun_out/${T}_sq2 > gpurun_out/${T}_sq.txt || exit 1
  python tools/pmc_clock.py gpurun_out/${T}_sq > gpurun_out/${T}_clock.txt || exit 1  # GRBM_GUI_ACTIVE per dispatch
  echo sq_ok
}

run_gloo2() {  # the N > 1 bench line rehearsed with two gloo ranks sharing the one GPU
  FPHE_DIST_BACKEND=gloo timeout -k 10 600 python -u bench.py --gpus 2 --steps 1 --warmup 1 --config4-samples 400000 --config5-per-rank 1000000 > gpurun_out/${T}_gloo2.txt 2>&1 || { echo gloo_failed; tail -20 gpurun_out/${T}_gloo2.txt; exit 1; }
  grep '^{"metric"' gpurun_out/${T}_gloo2.txt | tail -1 > gpurun_out/${T}_gloo2.json
  python -c "import json; d=json.load(open('gpurun_out/${T}_gloo2.json')); print(d['n_gpus'], d['value'], d.get('per_rank'), d.get('allgather'), d.get('histogram_multi_gpu'), d.get('config5'))"
}

case $M in
  tests) run_tests "$@" ;;
  round) run_tests; run_smoke; run_bench "$@" ;;
  bench) run_bench "$@" ;;
  prof) run_prof "$@" ;;
  profhead)  # kernel trace of the headline alone: every k_encrypt27<128,6> launch is a 2^20 step,
             # so the stats' average duration is the bench's per-step kernel time
    (cd /tmp && export TMPDIR=/tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/${T}_head -o run -- python3 $R/bench.py --steps 5 --warmup 2 --no-extras --no-cpu-baseline --config5-per-rank 0 > $R/gpurun_out/${T}_head_bench.txt 2>&1) || { echo trace_failed; tail -20 gpurun_out/${T}_head_bench.txt; exit 1; }
    grep '^{"metric"' gpurun_out/${T}_head_bench.txt | tail -1 > gpurun_out/${T}_head_bench.json
    python3 -c "
import csv, json
b = json.load(open('gpurun_out/${T}_head_bench.json'))
for r in csv.DictReader(open('gpurun_out/${T}_head/run_kernel_stats.csv')):
    if 'k_encrypt27<128, 6>' in r['Name'] or 'k_draw_r' in r['Name'] or 'k_mont_const27<128>' in r['Name']:
        print(r['Name'].split('(')[0][-40:], r['Calls'], round(float(r['AverageNs']) / 1e6, 3), 'ms avg')
print('bench HIP-event kernel_ms per step', b['roofline']['kernel_ms_per_step'], 'mean', b['roofline']['kernel_ms'])
" ;;
  pmc) run_pmc ;;
  sq) run_sq "$@" ;;
  sqhist)  # SQ / GRBM counters over tools/bench_legs/hist_leg.py ARGS (PHASES=0)
    export PHASES=0
    pmc_pass sqh "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT" python3 $R/tools/bench_legs/hist_leg.py "$@"
    python3 - gpurun_out/${T}_sqh <<'PYEOF'
import csv, glob, sys, collections
agg = collections.defaultdict(dict)
for f in glob.glob(sys.argv[1] + "/**/run_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "segfold" in r["Kernel_Name"] or "align_rows" in r["Kernel_Name"]:
            k = (r["Kernel_Name"].split("(")[0][-40:], int(r["Dispatch_Id"]))
            agg[k][r["Counter_Name"]] = agg[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
for k, v in sorted(agg.items(), key=lambda kv: kv[0][1]):
    print(k, {c: round(x) for c, x in sorted(v.items())})
PYEOF
    ;;
  evidence) run_tests; run_smoke; run_bench "$@"; run_prof; run_pmc ;;
  final) run_prof; run_pmc; run_gloo2 ;;
  gloo2) run_gloo2 ;;
  sqenc)  # SQ counters of the headline encrypt (k_encrypt27<128,6>): wait shares, VMEM/LDS mix
    ENC="python3 $R/bench.py --n 131072 --steps 1 --warmup 0 --no-extras --no-cpu-baseline --config5-per-rank 0"
    pmc_pass sqe1 "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT" $ENC
    pmc_pass sqe2 "SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_WAVES" $ENC
    python tools/pmc_sq_compare.py gpurun_out/${T}_sqe1 gpurun_out/${T}_sqe2 --match k_encrypt27 > gpurun_out/${T}_sqenc.txt || exit 1
    pmc_pass sqe3 "SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES" $ENC
    python tools/pmc_sq_compare.py gpurun_out/${T}_sqe3 --match k_encrypt27 >> gpurun_out/${T}_sqenc.txt || exit 1
    cat gpurun_out/${T}_sqenc.txt ;;
  timeline)  # kernel timeline of the last ~90 dispatches of a histogram leg: args go to hist_leg.py
    (cd /tmp && export TMPDIR=/tmp PHASES=0 && timeout -k 10 600 rocprofv3 --kernel-trace --output-format rocpd -d $R/gpurun_out/${T}_kt -o run -- python3 $R/tools/bench_legs/hist_leg.py "$@" > $R/gpurun_out/${T}_kt.txt 2>&1) || { echo timeline_failed; tail -20 gpurun_out/${T}_kt.txt; exit 1; }
    python tools/rocpd_timeline.py $(ls gpurun_out/${T}_kt/*.db gpurun_out/${T}_kt/*/*.db 2>/dev/null | head -1) ${TL_LAST:-90} > gpurun_out/${T}_timeline.txt
    rm -rf gpurun_out/${T}_kt  # the trace database: tens of MB, the timeline holds what is read
    grep -E "total_s|burst" gpurun_out/${T}_kt.txt | tail -3; grep -E "segfold|align_rows|k_gr_plan|span" gpurun_out/${T}_timeline.txt ;;
  leg)
    L=$1; shift
    timeout -k 10 900 python -u tools/bench_legs/$L "$@" > gpurun_out/${T}_leg.txt 2>&1 || { echo leg_failed; tail -30 gpurun_out/${T}_leg.txt; exit 1; }
    tail -5 gpurun_out/${T}_leg.txt ;;
  *) echo "unknown mode $M"; exit 2 ;;
esac
echo all_ok
