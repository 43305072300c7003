# BASELINE config 4 at full size on the round-3 build, the bench-shape histogram leg, and the
# 2-rank gloo rehearsal of bench.py's N>1 path (tag $1)
set -o pipefail
R=$GRAFT_REPO_ROOT
T=${1:-r03d}
cd $R && mkdir -p gpurun_out
timeout -k 10 180 python3 -u tools/bench_legs/hist_leg.py > gpurun_out/${T}_hist.txt 2>&1 || { echo hist_failed; tail -20 gpurun_out/${T}_hist.txt; exit 1; }
cat gpurun_out/${T}_hist.txt
timeout -k 10 400 python3 -u tools/bench_legs/secureboost_full.py > gpurun_out/${T}_secureboost_full.txt 2>&1 || { echo sb_failed; tail -20 gpurun_out/${T}_secureboost_full.txt; exit 1; }
tail -1 gpurun_out/${T}_secureboost_full.txt
bash tools/gpu_job_dist2.sh || exit 1
cp gpurun_out/dist2.txt gpurun_out/${T}_dist2.txt
echo all_ok
