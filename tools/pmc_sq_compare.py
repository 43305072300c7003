"""Per-kernel SQ counter table from rocprofv3 --pmc csv passes (tools/gpu_job.sh sq):
    python tools/pmc_sq_compare.py gpurun_out/TAG_h1 gpurun_out/TAG_h2 ... [--match k_segfold27 k_probe]
prints, per kernel name fragment, the counters summed over its dispatches and the derived
rates (VALU instructions per wave-cycle, wait fractions)."""
import collections
import csv
import sys


def load(d):
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(f"{d}/run_counter_collection.csv")):
        agg[r["Kernel_Name"]][r["Counter_Name"]] += float(r["Counter_Value"])
    return agg


def main(argv):
    dirs = [a for a in argv if not a.startswith("--")]
    match = argv[argv.index("--match") + 1:] if "--match" in argv else []
    if match:
        dirs = [a for a in argv[:argv.index("--match")]]
    rows = collections.defaultdict(dict)
    for d in dirs:
        for k, cs in load(d).items():
            if match and not any(m in k for m in match):
                continue
            rows[k].update(cs)
    for k, cs in sorted(rows.items()):
        print(k[:110])
        wc = cs.get("SQ_WAVE_CYCLES", 0)
        for c, v in sorted(cs.items()):
            extra = f"  ({v / wc:.3f} of wave cycles)" if wc and c.startswith(("SQ_WAIT", "SQ_ACTIVE")) else ""
            print(f"   {c:24s} {v:16.0f}{extra}")
        if wc and cs.get("SQ_INSTS_VALU"):
            print(f"   VALU insts per wave-cycle x4 (issue share per SIMD, 4-cycle wave64 op): "
                  f"{4 * cs['SQ_INSTS_VALU'] / wc:.3f}")


if __name__ == "__main__":
    main(sys.argv[1:])
