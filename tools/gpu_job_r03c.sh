# round-3 evidence in one call (tag in $1): GPU suite + smoke + bench + ops PMC
# (tools/gpu_job_r03b.sh), then the rocprofv3 kernel-trace stats of bench.py and the encrypt
# FETCH/WRITE PMC passes (tools/gpu_job_prof.sh)
T=${1:-r03c}
bash $GRAFT_REPO_ROOT/tools/gpu_job_r03b.sh $T || exit 1
bash $GRAFT_REPO_ROOT/tools/gpu_job_prof.sh $T || exit 1
echo all_ok
