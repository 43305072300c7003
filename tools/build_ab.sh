# build variant libraries for same-box A/B runs: tools/build_ab.sh NAME "-DFLAG=.. ..."
set -e
cd "$(dirname "$0")/../fate_amd"
mkdir -p lib/ab
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -Wall -Wno-unused-result $2 -o lib/ab/lib_$1.so csrc/fate_phe.hip
