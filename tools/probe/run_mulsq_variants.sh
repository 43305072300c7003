# Runs tools/probe/mulsq_<variant> binaries (built with -D switches, e.g. -DPROBE_TPI=2) in turn:
#   bash tools/probe/run_mulsq_variants.sh t2_base t2_c64 ...
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
OUT=${OUT:-gpurun_out/mulsq_variants.txt}
for v in "$@"; do
  echo "== $v" >> $OUT
  it=400; case $v in t2*) it=800;; esac
  timeout -k 10 120 tools/probe/mulsq_$v $it 1 >> $OUT 2>&1 || exit 1
done
grep -E "==|^sq|^mul " $OUT
