"""Effective shader clock per dispatch from a rocprofv3 --pmc pass that holds GRBM_GUI_ACTIVE
(tools/gpu_job.sh sq): the counter is summed over the 8 XCDs, so GRBM_GUI_ACTIVE / 8 over the
dispatch's duration is the mean GFX clock the kernel ran at.  The roofline peaks price
the VALU at 2.4 GHz (MI355X_MICROARCH.md); a kernel's fraction at its own clock is
frac x 2.4 / clock.
    python tools/pmc_clock.py gpurun_out/TAG_sq [more dirs] [--min-ms 1]"""
import csv
import sys

XCDS = 8
PEAK_GHZ = 2.4


def main(argv):
    min_ms, dirs = 1.0, list(argv)
    if "--min-ms" in dirs:
        i = dirs.index("--min-ms")
        min_ms = float(dirs[i + 1])
        del dirs[i:i + 2]
    print(f"{'dispatch':>8}  {'ms':>10}  {'GHz':>6}  {'x 2.4 GHz':>9}  kernel")
    for d in dirs:
        for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
            if r["Counter_Name"] != "GRBM_GUI_ACTIVE":
                continue
            dt = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            if dt < min_ms * 1e6:
                continue
            ghz = float(r["Counter_Value"]) / XCDS / dt
            name = r["Kernel_Name"]
            for pre in ("void ", "(anonymous namespace)::", "k28::"):
                name = name.replace(pre, "")
            name = name.split("((")[0].split("(")[0]
            print(f"{r['Dispatch_Id']:>8}  {dt / 1e6:10.3f}  {ghz:6.3f}  {ghz / PEAK_GHZ:9.3f}  {name}")


if __name__ == "__main__":
    main(sys.argv[1:])
