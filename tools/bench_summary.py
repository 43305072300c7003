"""One-screen summary of a bench.py JSON line (tools/gpu_job.sh prints it after each run).

    python tools/bench_summary.py gpurun_out/TAG_bench.json
"""
import json
import sys


def main(path: str) -> None:
    d = json.loads(open(path).read().strip().splitlines()[-1])
    r = d["roofline"]
    print(f"encrypt {d['value']:.0f}/s frac {r['frac']} kernel {r['kernel_ms']} ms; "
          f"hbm counter {r['hbm'].get('hbm_counter_GBps')} GB/s")
    for k, v in (d.get("rooflines") or {}).items():
        print(f"  {k:8s} frac {v.get('frac')} {v.get('kernel_ms')} ms issue {(v.get('issue') or {}).get('frac')} "
              f"hbm counter {v['hbm'].get('hbm_counter_GBps')} GB/s x{v['hbm'].get('counter_over_algorithmic')}")
    keys = ("decrypt_per_s", "ct_add_per_s", "ct_mul_per_s", "histogram_iupdate_s", "e2e_host_encrypts_per_s")
    print("  " + ", ".join(f"{k}={d.get(k)}" for k in keys))
    he = d.get("histogram_edge_values")
    if he:
        print(f"  edge-value histogram {he}")
    c4 = d.get("histogram_config4")
    if c4:
        print("  config4 " + json.dumps({k: v for k, v in c4.items() if not isinstance(v, dict)}))
    cb = d.get("cpu_baseline")
    if cb:
        print(f"  cpu {cb.get('value')} encrypts/s on {cb.get('cores')} cores; gpu/cpu {cb.get('gpu_over_cpu')}")


if __name__ == "__main__":
    main(sys.argv[1])
