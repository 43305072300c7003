# Rehearse bench.py's N>1 path (all-gather leg, cross-rank histogram fold) with 2 ranks on
# ONE GPU over gloo (RCCL refuses two ranks on one device).  Rates are not meaningful (the
# ranks share the GPU); the check is that every leg runs and every allclose holds.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
FPHE_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 1 --warmup 1 --elements 65536 \
  > gpurun_out/dist2.txt 2>&1 || { echo dist2_failed; tail -20 gpurun_out/dist2.txt; exit 1; }
grep '^{"metric"' gpurun_out/dist2.txt
