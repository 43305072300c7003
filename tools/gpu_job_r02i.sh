# GPU suite; bench line (roofline blocks for encrypt / decrypt / ct-add); `bench.py --gpus 2`
# rehearsed with two gloo ranks sharing the box's GPU (must print n_gpus 2) (tag in $1)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
T=${1:-r02i}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.txt 2>&1 || { echo tests_failed; tail -40 gpurun_out/${T}_tests.txt; exit 1; }
tail -1 gpurun_out/${T}_tests.txt
timeout -k 10 400 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_bench.txt 2>&1 || { echo bench_failed; tail -30 gpurun_out/${T}_bench.txt; exit 1; }
tail -1 gpurun_out/${T}_bench.txt | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']['frac'], d['ct_add_per_s'], json.dumps(d['rooflines']))"
FPHE_DIST_BACKEND=gloo timeout -k 10 400 python -u bench.py --gpus 2 --steps 1 --warmup 1 --n 65536 --no-extras > gpurun_out/${T}_dist2.txt 2>&1 || { echo dist2_failed; tail -30 gpurun_out/${T}_dist2.txt; exit 1; }
tail -1 gpurun_out/${T}_dist2.txt
echo all_ok
