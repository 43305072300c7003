"""HBM traffic of the decrypt, ct-add, ct x pt and iupdate kernels from FETCH_SIZE / WRITE_SIZE
passes over tools/bench_legs/ops_pmc_leg.py (tools/gpu_job.sh pmc): decrypt of 2^18 elements
(k_pow_half27<128, 6, false, false> + k_decrypt_crt<128>), the Hetero-LR-shaped ct-add of 2^20
(k_add27<128>), ct x pt of 2^18 (classify, batch inverse, k_mul27), the histogram fold's copy
and balanced level over 8.4M terms, 2048-bit key.  The counters are scaled per kernel by the
calibration probe's factors for that kernel's access pattern (CAL below).  bench.py reports the result as the
`traffic` of rooflines.decrypt / ct_add / ct_mul / iupdate.

    python tools/pmc_ops_summary.py gpurun_out/TAG profiles/r02/TAG_pmc_ops.json
"""
import collections
import csv
import json
import sys

KERNELS = {"decrypt": (["k_pow_half27<128, 6, false, false>", "k_decrypt_crt<128>"], 1 << 18,
                       "algorithmic: read 512 B C (+ sign/exp), write 4-256 B plaintext"),
           "ct_add": (["k_add27<128>"], 1 << 20, "algorithmic: two 517-B operands read, one written (+4-B order)"),
           "ct_mul": (["k_mul_prep<128>", "k_binv_pre27<128>", "k_inv_n27<128>", "k_inv_lift27<128>",
                       "k_binv_post27<128>", "k_mul27<128, 4>"], 1 << 18,
                      "algorithmic: one 517-B operand and a 13-B plaintext read, 517 B written"),
           "iupdate": (["k_tiles_to_rows<128>", "k_segfold27<128, true>"], 8 << 20,
                       "per term: the source row copy (element-major, once per source element) and the "
                       "balanced fold level, which gathers one 512-B row per term (algorithmic: 517 B per term)")}


# Per-kernel counter calibration (bytes moved per counted byte), measured with
# tools/probe/fetch_calib.hip on a known byte count in each kernel's own access pattern
# (profiles/r04/r04n_fetch_calib.txt).  Default: one dword per lane over whole 256-B rows (the
# window tables, ColIO rows) and 16-B-per-lane row loads -- FETCH_SIZE counts half the bytes,
# WRITE_SIZE all of them.  k_add27: a wave holds 16 elements x 4 lanes, so each dword load or
# store touches four 64-B segments 8 KiB apart (FETCH_SIZE counts 0.746 of the bytes,
# WRITE_SIZE 1.122).
CAL_DEFAULT = (2.0, 1.0)
CAL = {"k_add27<128>": (2097120 / 1563423.375, 2097120 / 2353716.1875)}


def per_kernel(path, counter):
    agg = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            agg[(r["Kernel_Name"], r["Dispatch_Id"])] += float(r["Counter_Value"])
    return agg


def main(prefix, out):
    f = per_kernel(f"{prefix}_fetch/run_counter_collection.csv", "FETCH_SIZE")
    w = per_kernel(f"{prefix}_write/run_counter_collection.csv", "WRITE_SIZE")
    res = {"source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes) over tools/bench_legs/ops_pmc_leg.py",
           "calibration": {"default": {"fetch_bytes_per_counted_byte": CAL_DEFAULT[0],
                                       "write_bytes_per_counted_byte": CAL_DEFAULT[1]},
                           **{k: {"fetch_bytes_per_counted_byte": round(v[0], 4),
                                  "write_bytes_per_counted_byte": round(v[1], 4)} for k, v in CAL.items()},
                           "source": "tools/probe/fetch_calib.hip, profiles/r04/r04n_fetch_calib.txt"}}
    for name, (kerns, elems, note) in KERNELS.items():
        rd = wr = 0.0
        detail = {}
        for k in kerns:
            # the first dispatch of the kernel in the leg's order (the iupdate's final add is a
            # second k_add27 dispatch, after the ct-add leg's)
            fk = [v for (kn, d), v in sorted(f.items(), key=lambda kv: int(kv[0][1])) if k in kn][:1]
            wk = [v for (kn, d), v in sorted(w.items(), key=lambda kv: int(kv[0][1])) if k in kn][:1]
            if len(fk) != 1 or len(wk) != 1:
                raise SystemExit(f"expected a {k} dispatch in each pass, found {len(fk)}/{len(wk)}")
            detail[k] = {"FETCH_SIZE_KiB": fk[0], "WRITE_SIZE_KiB": wk[0]}
            cf, cw = CAL.get(k, CAL_DEFAULT)
            rd += fk[0] * 1024 * cf
            wr += wk[0] * 1024 * cw
        res[name] = {"kernels": detail, "elements": elems, "hbm_read_bytes_per_elem": round(rd / elems, 1),
                     "hbm_write_bytes_per_elem": round(wr / elems, 1),
                     "hbm_bytes_per_elem": round((rd + wr) / elems, 1), "note": note}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v.get("hbm_bytes_per_elem") for k, v in res.items() if isinstance(v, dict) and "elements" in v}))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
