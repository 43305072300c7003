# GPU suite, a short bench line with the headline, decrypt/ct-add rooflines and 1024-bit legs (tag in $1)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
T=${1:-quick3}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.txt 2>&1 || { echo tests_failed; tail -40 gpurun_out/${T}_tests.txt; exit 1; }
tail -1 gpurun_out/${T}_tests.txt
timeout -k 10 500 python -u bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_bench.txt 2>&1 || { echo bench_failed; tail -30 gpurun_out/${T}_bench.txt; exit 1; }
tail -1 gpurun_out/${T}_bench.txt > gpurun_out/${T}_bench.json
python - gpurun_out/${T}_bench.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print("value", d["value"], "frac", d["roofline"]["frac"])
print("decrypt", d["decrypt_per_s"], d["rooflines"]["decrypt"]["frac"], d["rooflines"]["decrypt"]["kernel_ms"])
print("ct_add", d["ct_add_per_s"], d["rooflines"]["ct_add"]["frac"], d["rooflines"]["ct_add"]["kernel_ms"])
print("keyholder", d["encrypt_keyholder_crt_per_s"], d["encrypt_keyholder_crt_roofline_frac"])
print("key_1024", d["key_1024"])
print("mul", d["ct_mul_per_s"], d["rooflines"]["ct_mul"]["frac"], d["rooflines"]["ct_mul"]["kernel_ms"])
print("hist", d["histogram_scatter_adds_per_s"], "hlr", d["hetero_lr_gradient"])
PY
echo all_ok
