"""Turn the FETCH_SIZE / WRITE_SIZE rocprofv3 passes (tools/gpu_job.sh pmc) into the per-element
HBM traffic json that bench.py reports as roofline.traffic.

    python tools/pmc_summary.py gpurun_out/r01d profiles/r01d_pmc_encrypt27.json [elements]

Calibration (tools/probe/fetch_calib.hip, profiles/r01c_calib_*): with one dword per lane over
256-B rows FETCH_SIZE counts half the bytes read and WRITE_SIZE all bytes written."""
import collections
import csv
import json
import sys


def total(path: str, counter: str, kernel: str) -> float:
    agg = collections.defaultdict(float)
    for r in csv.DictReader(open(path)):
        if kernel in r["Kernel_Name"] and r["Counter_Name"] == counter:
            agg[r["Dispatch_Id"]] += float(r["Counter_Value"])
    if len(agg) != 1:
        raise SystemExit(f"expected one {kernel} dispatch in {path}, found {len(agg)}")
    return next(iter(agg.values()))


def main(prefix: str, out: str, elements: int = 131072, kernel: str = "k_encrypt27<128, 6>") -> None:
    fk = total(f"{prefix}_pmc_fetch/run_counter_collection.csv", "FETCH_SIZE", kernel)
    wk = total(f"{prefix}_pmc_write/run_counter_collection.csv", "WRITE_SIZE", kernel)
    rd = fk * 1024 * 2.0 / elements
    wr = wk * 1024 * 1.0 / elements
    d = {
        "kernel": "k_encrypt27<128,6>",
        "workload": f"bench.py --n {elements} --steps 1 --warmup 0 (2048-bit key)",
        "elements": elements,
        "FETCH_SIZE_KiB": fk,
        "WRITE_SIZE_KiB": wk,
        "calibration": {"probe": "tools/probe/fetch_calib.hip (buffer_load/store_dword per lane, 256-B rows, 2 GiB)",
                        "fetch_bytes_per_counted_byte": 2.0, "write_bytes_per_counted_byte": 1.0},
        "hbm_read_bytes_per_elem": round(rd, 1),
        "hbm_write_bytes_per_elem": round(wr, 1),
        "note": "dominated by the per-wave sliding-window table in global scratch (33 entries x 592 B per element "
                "written, one 592-B entry read per window product); algorithmic traffic is 526 B/element",
        "hbm_bytes_per_elem": round(rd + wr, 1),
    }
    with open(out, "w") as f:
        json.dump(d, f, indent=1)
    print(json.dumps(d, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], *(int(a) for a in sys.argv[3:4]))
