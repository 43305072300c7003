set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/calib_fetch -o run -- $R/tools/probe/fetch_calib_probe > $R/gpurun_out/calib_fetch.txt 2>&1 || { echo f1; exit 1; }
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/calib_write -o run -- $R/tools/probe/fetch_calib_probe > $R/gpurun_out/calib_write.txt 2>&1 || { echo f2; exit 1; }
echo ok
