"""CPU guard over the SHIPPED device code: the listing and resource remarks
the build keeps next to libfatephe.so (fate_amd/Makefile: hipcc -save-temps of the same
compile, so the listing is the code that was assembled into the library).

1. No waterfall loops in any kernel (tools/wfcheck.py).  A buffer access through a per-lane
   descriptor becomes a readfirstlane loop, and at the 168-VGPR budget the register
   allocator once placed a spill reload inside such a loop: the round-1 3-wave fault
   (DESIGN.md §3).  The kernels never pick a descriptor per lane, so any loop is a regression.
2. No fused-row clobber reads (tools/wfcheck.py).
3. Register budgets: every Montgomery-engine kernel keeps the occupancy it is built for
   (3 waves/SIMD = <= 168 VGPRs for the modexp and vector-op kernels, 2 for the fold and
   the ct-add, which holds both operands across its squarings), and
   no kernel uses dynamic stack.
"""
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "fate_amd", "lib", "libfatephe.so")
LISTING = os.path.join(ROOT, "fate_amd", "build", "fate_phe-gfx950.s")
REMARKS = os.path.join(ROOT, "fate_amd", "build", "kernel_resources.txt")

# kernel name fragment -> the least occupancy (waves/SIMD) it must keep
OCCUPANCY = {
    "k_encrypt27": 3, "k_pow_half27": 3, "k_add27": 2, "k_mul27": 3, "k_sqmul27": 3, "k_align27": 3,
    "k_fold27": 2, "k_segfold27": 2, "k_align_rows27": 3, "k_encrypt_crt27": 2, "k_inv_lift27": 2, "k_binv_pre27": 2, "k_binv_post27": 2,
    "k_inv_n27": 1,
}


def _fresh() -> bool:
    return all(os.path.exists(p) for p in (LIB, LISTING, REMARKS)) and \
        os.path.getmtime(LISTING) >= os.path.getmtime(LIB) - 5


@pytest.fixture(scope="module")
def artefacts():
    if not _fresh():  # built by another recipe (or not at all): rebuild with the by-products
        if os.path.exists(LIB):
            os.utime(os.path.join(ROOT, "fate_amd", "csrc", "fate_phe.hip"))
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "fate_amd")], check=True)
    assert _fresh()
    return LISTING, REMARKS


def kernel_resources(path):
    rows, cur = [], None
    for line in open(path):
        # "remark: FILE:L:C: TEXT [-Rpass...]" (the -save-temps build) or "FILE:L:C: remark: TEXT [...]"
        m = re.search(r"remark:\s+(?:[^ ]+:\d+:\d+:\s+)?(.*?)\s*\[-Rpass", line)
        if not m:
            continue
        t = m.group(1)
        if t.startswith("Function Name:"):
            cur = {"name": t.split(":", 1)[1].strip()}
            rows.append(cur)
        elif cur is not None and ":" in t:
            k, v = t.split(":", 1)
            cur[k.strip()] = v.strip()
    return rows


def test_no_waterfall_loops_or_clobber_reads(artefacts):
    listing, _ = artefacts
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "wfcheck.py"), listing], capture_output=True,
                       text=True, timeout=600)
    lines = [ln for ln in r.stdout.splitlines() if "waterfall_loops=" in ln]
    assert len(lines) >= 40, r.stdout[-2000:] + r.stderr[-2000:]  # every kernel was parsed
    bad = [ln for ln in lines if not ln.startswith("ok")]
    assert r.returncode == 0 and not bad, "\n".join(bad) + r.stdout[-3000:]


def test_register_budgets(artefacts):
    _, remarks = artefacts
    rows = kernel_resources(remarks)
    assert len(rows) >= 40
    seen = set()
    for r in rows:
        name = r["name"]
        assert r.get("Dynamic Stack") == "False", name
        for frag, occ in OCCUPANCY.items():
            if frag + "I" in name:  # template kernels: the fragment then "ILi..."
                seen.add(frag)
                got = int(r["Occupancy [waves/SIMD]"])
                assert got >= occ, f"{name}: occupancy {got} < {occ} (VGPRs {r.get('VGPRs')})"
    assert seen == set(OCCUPANCY), set(OCCUPANCY) - seen
