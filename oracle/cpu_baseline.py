"""CPU baseline for bench.py -- TEST INFRASTRUCTURE ONLY (cpu_baseline.kind = "port").

Times the libgmp restatement of the reference's per-element call sequence
(oracle/gmp_ref.c: encrypt = crates/paillier/src/lib.rs:104-121, decrypt = :163-176,
ct-add = :35-37) the way FATE runs it: one worker PROCESS per core, each a serial
element loop (the reference's Rust call is single-threaded, and FATE parallelises by a
process pool of os.cpu_count() workers, arch/computing/backends/standalone/
_standalone.py:470-478 and _csession.py:41-42).

Run as its own process (bench.py starts it as a child after its GPU work, so the forked
workers never share a GPU-initialised parent):

    python -m oracle.cpu_baseline --p HEX --q HEX [--procs P] [--seconds S]

prints one JSON object: per op the aggregate rate, the per-core rate, the sample size.
"""
from __future__ import annotations

import argparse
import json
import multiprocessing as mp
import os
import platform
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
if os.path.dirname(HERE) not in sys.path:
    sys.path.insert(0, os.path.dirname(HERE))

OPS = ("encrypt", "decrypt", "add", "add_gap")


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def usable_cores() -> int:
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        return os.cpu_count() or 1


def _worker(args):
    p, q, op, count, seed = args
    from oracle import gmp_ref
    key = gmp_ref.GmpKey(p * q, p, q)
    return key.bench(op, count, 1, seed)


def measure(p: int, q: int, procs: int, seconds: float, ops=OPS) -> dict:
    """Per op: calibrate the single-core rate on a short serial run, then give each of
    `procs` worker processes about `seconds` of elements; rate = total / wall time."""
    from oracle import gmp_ref
    key = gmp_ref.GmpKey(p * q, p, q)
    out = {}
    ctx = mp.get_context("fork")
    with ctx.Pool(procs) as pool:
        pool.map(_worker, [(p, q, "add", 10, i) for i in range(procs)])  # start + load the library
        for op in ops:
            n1 = {"encrypt": 20, "decrypt": 60, "add": 20000, "add_gap": 4000}[op]
            t1 = key.bench(op, n1, 1, 99)
            per_core = n1 / t1
            per_proc = max(8, int(per_core * seconds))
            t0 = time.perf_counter()
            pool.map(_worker, [(p, q, op, per_proc, 1000 + i) for i in range(procs)])
            wall = time.perf_counter() - t0
            out[op] = {"per_s": round(per_proc * procs / wall, 2), "per_core_per_s": round(per_core, 2),
                       "elements": per_proc * procs, "wall_s": round(wall, 3)}
    return out


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--p", required=True)
    ap.add_argument("--q", required=True)
    ap.add_argument("--procs", type=int, default=0, help="worker processes (default: usable cores, at most 16)")
    ap.add_argument("--seconds", type=float, default=3.0, help="CPU seconds per worker per op")
    a = ap.parse_args()
    p, q = int(a.p, 16), int(a.q, 16)
    procs = a.procs or min(16, usable_cores())
    res = measure(p, q, procs, a.seconds)
    print(json.dumps({"procs": procs, "usable_cores": usable_cores(), "machine_cores": os.cpu_count(),
                      "cpu_model": cpu_model(), "key_bits": (p * q).bit_length(), "ops": res}))


if __name__ == "__main__":
    main()
