# End-of-round record after `tools/gpu_job.sh TAG round`: kernel trace + PMC passes of the same
# build, then the 2-rank gloo rehearsal of the N > 1 bench path on the one GPU
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
T=${1:?tag}
bash tools/gpu_job.sh $T prof > gpurun_out/${T}_prof_job.txt 2>&1 || { tail -5 gpurun_out/${T}_prof_job.txt; exit 1; }
tail -2 gpurun_out/${T}_prof_job.txt
bash tools/gpu_job.sh $T pmc > gpurun_out/${T}_pmc_job.txt 2>&1 || { tail -5 gpurun_out/${T}_pmc_job.txt; exit 1; }
tail -2 gpurun_out/${T}_pmc_job.txt
FPHE_DIST_BACKEND=gloo timeout -k 10 600 python -u bench.py --gpus 2 --steps 1 --warmup 1 --config4-samples 400000 > gpurun_out/${T}_gloo2.txt 2>&1; rc=$?
echo "gloo rehearsal rc=$rc"
[ $rc -eq 0 ] || { tail -20 gpurun_out/${T}_gloo2.txt; exit 1; }
grep '^{"metric"' gpurun_out/${T}_gloo2.txt | tail -1 > gpurun_out/${T}_gloo2.json
python -c "import json; d=json.load(open('gpurun_out/${T}_gloo2.json')); print(d['n_gpus'], d['value'], d.get('per_rank'), d.get('allgather'), d.get('histogram_multi_gpu'))"
