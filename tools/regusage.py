"""Print per-kernel VGPR/AGPR/scratch/occupancy of libfatephe's device code (hipcc remarks)."""
import re
import subprocess
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "fate_amd/csrc/fate_phe.hip"
flt = sys.argv[2] if len(sys.argv) > 2 else ""
out = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-c",
                      "--cuda-device-only", "-Rpass-analysis=kernel-resource-usage", src, "-o", "/dev/null"],
                     capture_output=True, text=True).stderr
cur = None
rows = []
for line in out.splitlines():
    m = re.search(r"remark:\s+(.*?)\s*\[-Rpass", line)
    if not m:
        continue
    t = m.group(1)
    if t.startswith("Function Name:"):
        cur = {"name": t.split(":", 1)[1].strip()}
        rows.append(cur)
    elif cur is not None and ":" in t:
        k, v = t.split(":", 1)
        cur[k.strip()] = v.strip()
for r in rows:
    n = re.sub(r"^_ZN12_GLOBAL__N_1\d+", "", r["name"])
    n = re.sub(r"EEEv.*|Ev.*", "", n)
    if flt in n:
        print(f"{n:40s} vgpr={r.get('VGPRs','?'):>4} agpr={r.get('AGPRs','?'):>4} "
              f"scratch={r.get('ScratchSize [bytes/lane]','?'):>4} occ={r.get('Occupancy [waves/SIMD]','?')}")
