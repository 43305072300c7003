"""CPU baseline for bench.py -- TEST INFRASTRUCTURE ONLY (cpu_baseline.kind = "port").

Times the libgmp restatement of the reference's per-element call sequence
(oracle/gmp_ref.c: encrypt = crates/paillier/src/lib.rs:104-121, decrypt = :163-176,
ct-add = :35-37, ct x pt = fixedpoint_paillier/src/lib.rs:334-349, the iupdate scatter-add =
:724-735) the way FATE runs it: one worker PROCESS per core, each a serial
element loop (the reference's Rust call is single-threaded, and FATE parallelises by a
process pool of os.cpu_count() workers, arch/computing/backends/standalone/
_standalone.py:470-478 and _csession.py:41-42).

What is measured, and what is projected (all in one JSON line):
  * the single-process rate of every op (one core, otherwise idle);
  * the rate of `procs` worker processes (default: the CPU share this process may use: the
    cgroup quota when one is set, else the affinity mask, capped by --max-procs);
  * for encrypt, the SMT uplift: two processes pinned to the two hardware threads of one
    core against one process alone on that core;
  * the host's topology (/proc/cpuinfo: sockets, physical cores, threads) and, from the
    above, a projection of the whole host's encrypt rate: physical cores x the per-process
    rate of the multi-process run x the SMT uplift (linear in cores, so it ignores the
    all-core clock drop -- an over-estimate of the CPU, i.e. conservative for a GPU/CPU ratio).

Run as its own process (bench.py starts it as a child after its GPU work, so the forked
workers never share a GPU-initialised parent):

    python -m oracle.cpu_baseline --p HEX --q HEX [--procs P] [--max-procs M] [--seconds S]
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

OPS = ("encrypt", "decrypt", "add", "add_gap", "mul", "iupdate")
# elements of the short serial calibration run per op
CALIB = {"encrypt": 20, "decrypt": 60, "add": 20000, "add_gap": 4000, "mul": 200, "iupdate": 10000}


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def topology() -> dict:
    """Sockets, physical cores and hardware threads of the host (/proc/cpuinfo)."""
    cores, sockets, threads = set(), set(), 0
    phys = core = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                k, _, v = line.partition(":")
                k = k.strip()
                if k == "processor":
                    threads += 1
                elif k == "physical id":
                    phys = v.strip()
                    sockets.add(phys)
                elif k == "core id":
                    core = v.strip()
                    cores.add((phys, core))
    except OSError:
        pass
    n_cores = len(cores) or threads
    return {"sockets": len(sockets) or 1, "physical_cores": n_cores, "hw_threads": threads,
            "threads_per_core": round(threads / n_cores, 2) if n_cores else None}


def usable_cores() -> int:
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        return os.cpu_count() or 1


def cgroup_quota():
    """CPUs granted by the cgroup CPU controller (cgroup v2 cpu.max or v1 cfs quota), with the
    raw file contents; None when no quota is set (or readable)."""
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            raw = open(path).read().strip()
        except OSError:
            continue
        q, _, per = raw.partition(" ")
        if q != "max" and per:
            return float(q) / float(per), f"{path}: {raw}"
        return None, f"{path}: {raw}"
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        raw = f"cfs_quota_us={q} cfs_period_us={per}"
        return (q / per, raw) if q > 0 else (None, raw)
    except OSError:
        return None, "no cgroup cpu controller file readable"


def siblings(cpu: int):
    try:
        txt = open(f"/sys/devices/system/cpu/cpu{cpu}/topology/thread_siblings_list").read().strip()
    except OSError:
        return [cpu]
    out = []
    for part in txt.split(","):
        a, _, b = part.partition("-")
        out += list(range(int(a), int(b or a) + 1))
    return out


def _worker(args):
    p, q, op, count, seed, pin = args
    if pin is not None:
        os.sched_setaffinity(0, {pin})
    from oracle import gmp_ref
    key = gmp_ref.GmpKey(p * q, p, q)
    return key.bench(op, count, 1, seed)


def measure(p: int, q: int, procs: int, seconds: float, ops=OPS) -> dict:
    """Per op: the single-process rate from a short serial run, then `procs` worker processes
    with about `seconds` of elements each; rate = total / wall time."""
    from oracle import gmp_ref
    key = gmp_ref.GmpKey(p * q, p, q)
    out = {}
    ctx = mp.get_context("fork")
    with ctx.Pool(procs) as pool:
        pool.map(_worker, [(p, q, "add", 10, i, None) for i in range(procs)])  # start + load the library
        for op in ops:
            n1 = CALIB[op]
            t1 = key.bench(op, n1, 1, 99)
            per_core = n1 / t1
            per_proc = max(8, int(per_core * seconds))
            t0 = time.perf_counter()
            pool.map(_worker, [(p, q, op, per_proc, 1000 + i, None) for i in range(procs)])
            wall = time.perf_counter() - t0
            out[op] = {"per_s": round(per_proc * procs / wall, 2), "per_core_per_s": round(per_core, 2),
                       "single_process_per_s": round(per_core, 2), "per_process_per_s": round(per_proc / wall, 2),
                       "elements": per_proc * procs, "wall_s": round(wall, 3)}
    return out


def smt_uplift(p: int, q: int, seconds: float):
    """Encrypt rate of two processes on the two hardware threads of one core over one process
    alone on it (None without an SMT sibling inside our affinity mask)."""
    allowed = sorted(os.sched_getaffinity(0))
    pair = None
    for c in allowed:
        sib = [s for s in siblings(c) if s != c and s in allowed]
        if sib:
            pair = (c, sib[0])
            break
    if pair is None:
        return None
    from oracle import gmp_ref
    per_core = CALIB["encrypt"] / gmp_ref.GmpKey(p * q, p, q).bench("encrypt", CALIB["encrypt"], 1, 99)
    n = max(8, int(per_core * seconds))
    ctx = mp.get_context("fork")
    with ctx.Pool(2) as pool:
        t0 = time.perf_counter()
        pool.map(_worker, [(p, q, "encrypt", n, 7, pair[0])])
        one = n / (time.perf_counter() - t0)
        t0 = time.perf_counter()
        pool.map(_worker, [(p, q, "encrypt", n, 7 + i, pair[i]) for i in range(2)])
        two = 2 * n / (time.perf_counter() - t0)
    return {"cpus": list(pair), "one_thread_per_s": round(one, 2), "two_threads_per_s": round(two, 2),
            "uplift": round(two / one, 3)}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--p", required=True)
    ap.add_argument("--q", required=True)
    ap.add_argument("--procs", type=int, default=0,
                    help="worker processes (default: the CPU share -- cgroup quota, else affinity -- "
                         "capped by --max-procs)")
    ap.add_argument("--max-procs", type=int, default=0, help="cap on the default worker count (0: none)")
    ap.add_argument("--seconds", type=float, default=3.0, help="CPU seconds per worker per op")
    ap.add_argument("--no-smt", action="store_true")
    a = ap.parse_args()
    p, q = int(a.p, 16), int(a.q, 16)
    quota, quota_raw = cgroup_quota()
    share = usable_cores() if quota is None else max(1, min(usable_cores(), int(quota)))
    procs = a.procs or (min(share, a.max_procs) if a.max_procs else share)
    res = measure(p, q, procs, a.seconds)
    topo = topology()
    smt = None if a.no_smt else smt_uplift(p, q, min(a.seconds, 3.0))
    enc = res["encrypt"]
    uplift = smt["uplift"] if smt else 1.0
    proj = topo["physical_cores"] * enc["per_process_per_s"] * (uplift if (topo["threads_per_core"] or 1) > 1 else 1.0)
    print(json.dumps({"procs": procs, "usable_cores": usable_cores(), "machine_cores": os.cpu_count(),
                      "cgroup_quota_cpus": quota, "cgroup_cpu_max": quota_raw, "cpu_share": share,
                      "cpu_model": cpu_model(), "topology": topo, "smt": smt,
                      "host_projection": {"encrypt_per_s": round(proj, 1),
                                          "formula": "physical_cores x per-process encrypt rate of the "
                                                     "multi-process run x SMT uplift"},
                      "key_bits": (p * q).bit_length(), "ops": res}))


if __name__ == "__main__":
    main()
