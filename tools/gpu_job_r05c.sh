set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/gpu_job.sh r05c prof > gpurun_out/r05c_prof_job.txt 2>&1; rc=$?
echo "prof job rc=$rc"
tail -3 gpurun_out/r05c_prof_job.txt
[ $rc -eq 0 ] || exit 1
FPHE_DIST_BACKEND=gloo timeout -k 10 600 python -u bench.py --gpus 2 --steps 1 --warmup 1 --config4-samples 400000 > gpurun_out/r05c_gloo2.txt 2>&1; rc=$?
echo "gloo rehearsal rc=$rc"
grep '^{"metric"' gpurun_out/r05c_gloo2.txt | tail -1 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['n_gpus'], d.get('per_rank'), d.get('allgather'), d.get('gather_to_rank0'), d.get('histogram_multi_gpu'))"
