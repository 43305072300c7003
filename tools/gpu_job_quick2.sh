# GPU suite, the Hetero-LR ct-add leg, a short bench line (tag in $1)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
T=${1:-quick2}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.txt 2>&1 || { echo tests_failed; tail -40 gpurun_out/${T}_tests.txt; exit 1; }
tail -1 gpurun_out/${T}_tests.txt
timeout -k 10 300 python -u tools/bench_legs/add_leg.py > gpurun_out/${T}_add_leg.txt 2>&1 || { echo addleg_failed; tail -20 gpurun_out/${T}_add_leg.txt; exit 1; }
cat gpurun_out/${T}_add_leg.txt
timeout -k 10 400 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_bench.txt 2>&1 || { echo bench_failed; tail -30 gpurun_out/${T}_bench.txt; exit 1; }
tail -1 gpurun_out/${T}_bench.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ('value','ct_add_per_s','ct_mul_per_s','decrypt_per_s','histogram_scatter_adds_per_s')}, d['roofline']['frac'])"
echo all_ok
