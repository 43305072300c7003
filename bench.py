#!/usr/bin/env python3
"""bench.py -- Paillier-2048 encrypt throughput, device-resident (BASELINE.json metric).

Workload (BASELINE.json configs[1]): 2048-bit key, float32 tensor of 2^20 elements per GPU
(x = randn*4, seed 20241218+rank, first 8 entries [0,-0,1e-30,-1e-30,3.4e38,-3.4e38,1,-1]),
already resident in HBM.  One step = fixed-point encode (device) + obfuscated encryption
(device ChaCha20 r, r^n mod n^2) of the whole batch.  N GPUs = N independent shards (weak
scaling, one process per GPU, no collective in the timed region).  Also reported (every
rank; rank 0 prints): decrypt and ct-add throughput on the same data, the end-to-end rate
with host->device and device->host copies, a decrypt round-trip check, key-holder (CRT)
encryption, ct x pt, the SecureBoost histogram (unpacked and gh-packed), the Hetero-LR
gradient step, for N>1 the ciphertext all-gather and the cross-rank histogram fold, the
roofline of the dominant kernel and, at N=1, the CPU baseline (libgmp port of the
reference call sequence).  `config5` is BASELINE config 5 in weak form: 12.5M elements per
rank (100M at 8 GPUs), then the gather to rank 0 and the all-gather.  Progress goes to
stderr, one line per leg; the JSON line is the only stdout.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--n ELEMENTS] [--config5-per-rank M]
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

KEY_FIXTURE = os.path.join(ROOT, "tests", "golden", "paillier_2048.json")
# gfx950 integer MAC peak: 256 CU x 128 lanes/clk x 2.4 GHz at v_mad_u64_u32's half rate
# (measured half rate in profiles/r01_probe_alu.txt); one MAC32 = 32x32->64 multiply-add.
PEAK_TMAC32 = 256 * 128 * 2.4e9 / 2 / 1e12
PEAK_HBM_GBS = 8000.0
# host CPUs one GPU's box may use (the pool's share per GPU of an 8-GPU host); the CPU
# baseline's worker pool is capped there and the whole host is projected from it
CPU_SHARE_PER_GPU = 16
# limbs per lane of the Montgomery engine (28-bit limbs, fate_amd/csrc/mont27_dev.h)
ENGINE_LL = 37


_T_START = time.perf_counter()


def progress(msg: str) -> None:
    """One line per leg on stderr (the JSON line stays alone on stdout): a run that prints
    nothing for minutes is taken to be hung by the GPU harness."""
    r = os.environ.get("RANK", "0")
    print(f"[bench r{r} {time.perf_counter() - _T_START:7.1f}s] {msg}", file=sys.stderr, flush=True)


def mac32_per_mont(L: int) -> int:
    return 2 * L * L + L


def enc_mac32_per_elem(key_bits: int) -> float:
    # fixed-window (w=5) modexp with an E-bit exponent = E + ceil(E/5) + 16
    # Montgomery products, + 1 for the nude-ciphertext product; L = limbs of n^2.
    E = key_bits
    L = key_bits // 16
    return (E + math.ceil(E / 5) + 16 + 1) * mac32_per_mont(L)


def enc_products_per_elem(key_bits: int) -> int:
    E = key_bits
    return E + math.ceil(E / 5) + 16 + 1


def sliding_window_schedule(e: int, w: int = 6):
    """(squarings, general products) of powm27's sliding-window schedule for exponent e
    (fate_amd/csrc/kernels27.h): table build (X^2 as a general product + 2^(w-1)-1 products),
    then one squaring per bit below the first window and one product per later window."""
    bits = [(e >> i) & 1 for i in range(e.bit_length())]
    sq, mul = 0, 1 + (1 << (w - 1)) - 1
    i = len(bits) - 1
    j = max(i - w + 1, 0)
    while not bits[j]:
        j += 1
    i = j - 1
    while i >= 0:
        if not bits[i]:
            sq += 1
            i -= 1
            continue
        j = max(i - w + 1, 0)
        while not bits[j]:
            j += 1
        sq += i - j + 1
        mul += 1
        i = j - 1
    return sq, mul


def sliding_window_products(e: int, w: int = 6) -> int:
    sq, mul = sliding_window_schedule(e, w)
    return sq + mul


def enc_mad27_per_elem(key_bits: int, n: int) -> float:
    # issued v_mad_u64_u32 of the reduced-radix engine (fate_amd/csrc/mont27_dev.h), summed
    # over an element's TPI lanes: a general product is NL rows x 2 NL MACs; a squaring
    # (mont_sqr) NL rows x TPI x (LL/2 + 1 + LL) MACs.  28-bit limbs, LL = 37 per lane:
    # NL = 148 for 4096-bit n^2 (mont27_dev.h).
    # Products: to-Montgomery, the sliding-window r^n, x C_nude.
    TPI = key_bits // 16 // 32
    NL = ENGINE_LL * TPI
    sq, mul = sliding_window_schedule(n)
    return (1 + mul + 1) * 2 * NL * NL + sq * NL * TPI * (ENGINE_LL // 2 + 1 + ENGINE_LL)


def kh_direct_z(p: int, q: int) -> bool:
    """Whether the library draws the key holder's obfuscation as (z_p, z_q) directly
    (k_draw_z): FPHE_KH_DIRECT_Z unset or nonzero, and gcd(q, p-1) =
    gcd(p, q-1) = 1 (p, q prime: neither divides the other's predecessor)."""
    return os.environ.get("FPHE_KH_DIRECT_Z", "1") != "0" and (p - 1) % q != 0 and (q - 1) % p != 0


def enc_crt_mac32_per_elem(key_bits: int, direct: bool = True) -> float:
    # key-holder encrypt, the w=5 fixed-window formula of SURVEY.md §8(d) for the modexps it
    # runs, + 4 products of the recombination over n^2.  With the direct draw (k_draw_z,
    # any key size): per half z^p mod p^2 over the key/32-limb p^2, a (key/2)-bit exponent.
    # Otherwise, keys above 1024 bits (the split, FPHE_KH_SPLIT): per half z =
    # r^(q mod (p-1)) mod p over the key/64-limb p first; up to 1024 bits: one (n mod
    # s(s-1))-bit (~key_bits) exponent mod s^2 per half
    rec = 4 * mac32_per_mont(key_bits // 16)
    E = key_bits // 2
    if direct:
        return 2 * (E + math.ceil(E / 5) + 16) * mac32_per_mont(key_bits // 32) + rec
    if key_bits > 1024:
        per_half = (E + math.ceil(E / 5) + 16) * (mac32_per_mont(key_bits // 64) + mac32_per_mont(key_bits // 32))
        return 2 * per_half + rec
    E = key_bits
    return 2 * (E + math.ceil(E / 5) + 16) * mac32_per_mont(key_bits // 32) + rec


def dec_mac32_per_elem(key_bits: int) -> float:
    E = key_bits // 2
    L = key_bits // 32
    return 2 * (E + math.ceil(E / 5) + 16) * mac32_per_mont(L)


def _profile_order(path: str):
    """Natural order of profile names (r02z7 < r02z16): digit runs compare as numbers."""
    import re
    return [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", os.path.basename(path))]


def _pmc_profile(kind: str, pattern: str):
    """The committed PMC profile of this build: the one profiles/current_pmc.json names for
    `kind`, else the newest matching file in natural order."""
    import glob
    cur = os.path.join(ROOT, "profiles", "current_pmc.json")
    if os.path.exists(cur):
        with open(cur) as f:
            name = json.load(f).get(kind)
        if name and os.path.exists(os.path.join(ROOT, name)):
            return os.path.join(ROOT, name)
    paths = sorted(glob.glob(os.path.join(ROOT, "profiles", "**", pattern), recursive=True), key=_profile_order)
    return paths[-1] if paths else None


def pmc_traffic_per_elem():
    """HBM bytes per element of k_encrypt27 from the committed rocprofv3 PMC passes
    (FETCH_SIZE and WRITE_SIZE in separate runs, FETCH_SIZE doubled per the calibration
    probe tools/probe/fetch_calib.hip), or None when no such profile is present."""
    path = _pmc_profile("encrypt27", "*pmc_encrypt27.json")
    if not path:
        return None, None
    with open(path) as f:
        d = json.load(f)
    return float(d["hbm_bytes_per_elem"]), os.path.relpath(path, ROOT)


def pmc_ops_traffic(op: str):
    """HBM bytes per element of the decrypt / ct_add / ct_mul kernels (per term for iupdate)
    from the committed PMC passes (tools/pmc_ops_summary.py), or (None, None)."""
    path = _pmc_profile("ops", "*pmc_ops.json")
    if not path:
        return None, None
    with open(path) as f:
        d = json.load(f)
    if op not in d:
        return None, None
    return float(d[op]["hbm_bytes_per_elem"]), os.path.relpath(path, ROOT)


def _traffic(op: str, n: int):
    """roofline.traffic for n elements of op (HBM bytes per launch from the PMC profile)."""
    b, _ = pmc_ops_traffic(op)
    return None if b is None else round(b * n)


def cpu_baseline(p: int, q: int, seconds: float = 3.0):
    """The libgmp restatement of the reference's per-element call sequence (oracle/gmp_ref.c)
    timed the way FATE runs it: one worker process per core (oracle/cpu_baseline.py), for
    encrypt (the headline), decrypt and ct-add.  Runs as a child process: its forked
    workers must not inherit this GPU-initialised process."""
    import subprocess
    procs = int(os.environ.get("FPHE_CPU_PROCS", "0"))
    cmd = [sys.executable, "-m", "oracle.cpu_baseline", "--p", hex(p), "--q", hex(q), "--seconds", str(seconds),
           "--max-procs", str(CPU_SHARE_PER_GPU)]
    if procs:
        cmd += ["--procs", str(procs)]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=600)
    if r.returncode != 0:
        raise RuntimeError(r.stderr.strip()[-300:])
    d = json.loads(r.stdout.strip().splitlines()[-1])
    ops = d["ops"]
    return {
        "value": ops["encrypt"]["per_s"],
        "unit": "encrypts/s",
        "cores": d["procs"],
        "kind": "port",
        "per_core": ops["encrypt"]["per_process_per_s"],
        "single_process_per_s": {k: ops[k]["single_process_per_s"] for k in ops},
        "decrypt_per_s": ops["decrypt"]["per_s"],
        "ct_add_per_s": ops["add"]["per_s"],
        "ct_add_hetero_lr_gaps_per_s": ops["add_gap"]["per_s"],
        "ct_mul_per_s": ops["mul"]["per_s"],
        "iupdate_per_s": ops["iupdate"]["per_s"],
        "cpu_model": d["cpu_model"],
        "machine_cores": d["machine_cores"],
        "usable_cores": d["usable_cores"],
        "cgroup_cpu_max": d["cgroup_cpu_max"],
        "cpu_share": {"cores": d["procs"], "affinity": d["usable_cores"], "cgroup_quota_cpus": d["cgroup_quota_cpus"],
                      "rule": (f"the GPU box is a 1-GPU slice of a {d['topology']['hw_threads']}-thread host; the worker "
                               f"pool is the CPU quota of this process's cgroup ({d['cgroup_cpu_max']}) when one is "
                               f"set, capped at the pool's per-GPU share of {CPU_SHARE_PER_GPU}; the whole host is "
                               f"projected from it (host_projection)")},
        "topology": d["topology"],
        "smt": d["smt"],
        "host_projection": d["host_projection"],
        "sample": (f"{d['procs']} worker processes (one per core, FATE's process pool), libgmp mpz_* in the "
                   f"reference's call order (oracle/gmp_ref.c), 2048-bit key: {ops['encrypt']['elements']} "
                   f"obfuscated encryptions, {ops['decrypt']['elements']} CRT decryptions, "
                   f"{ops['add']['elements']} aligned ct-adds (mpz_mul + tdiv_r), {ops['add_gap']['elements']} ct-adds "
                   f"with the Hetero-LR exponent-gap mix (+ mpz_powm by 16^gap), {ops['mul']['elements']} ct x pt "
                   f"by float32 weights in [-1, 2) (mpz_powm by the significand, mpz_invert first for a third), "
                   f"{ops['iupdate']['elements']} iupdate scatter-adds of SecureBoost-shaped g, h terms into 256 "
                   f"slots (sequential Ciphertext::add with decrese_exp_to)"),
    }


def hbm_block(alg_bytes: float, ms: float, traffic=None, source=None) -> dict:
    """HBM view of one timed launch: the algorithmic bytes' rate and, when the committed
    rocprofv3 FETCH_SIZE / WRITE_SIZE passes cover the kernel (`traffic`, bytes per launch at
    this size), the counter bytes' rate (hbm_counter_GBps, north_star's "achieved HBM GB/s from
    rocprof") and their ratio to the algorithmic bytes (re-reads and spills)."""
    sec = ms / 1e3
    out = {"achieved": round(alg_bytes / sec / 1e9, 3), "peak": PEAK_HBM_GBS, "unit": "GB/s",
           "algorithmic_bytes": round(alg_bytes)}
    if traffic is not None:
        out.update({"counter_bytes": round(traffic), "hbm_counter_GBps": round(traffic / sec / 1e9, 3),
                    "counter_frac_of_peak": round(traffic / sec / 1e9 / PEAK_HBM_GBS, 4),
                    "counter_over_algorithmic": round(traffic / alg_bytes, 2), "counter_source": source})
    return out


def valu_roofline(kernel: str, mac32: float, ms: float, hbm_bytes: float, traffic=None, traffic_source=None,
                  **extra) -> dict:
    """A roofline block in SURVEY.md §8(d)'s MAC32 accounting for one timed launch."""
    achieved = mac32 / (ms / 1e3) / 1e12
    return {"bound": "valu", "kernel": kernel, "achieved": round(achieved, 3), "peak": round(PEAK_TMAC32, 3),
            "unit": "TMAC32/s", "frac": round(achieved / PEAK_TMAC32, 4), "kernel_ms": round(ms, 3),
            "traffic": None if traffic is None else round(traffic), "traffic_source": traffic_source,
            "hbm": hbm_block(hbm_bytes, ms, traffic, traffic_source), **extra}


class ClockMeter:
    """The shader clock a timed leg ran at: fphe_clock_stamp queues 2048
    one-wave workgroups on the leg's stream just before and just after it (~10 us each); each
    writes its CU's shader-clock cycle counter and the constant-rate counter, so (cycles1 -
    cycles0) / (wall1 - wall0) per CU stamped on both sides is that CU's mean clock over the
    leg (the counters of different CUs are not synchronised).  The rooflines price at 2.4 GHz;
    `frac_at_measured_clock` = frac x 2.4 / measured GHz separates a slow box's clock from the
    code."""

    BLOCKS = 2048
    SLOTS = 64

    def __init__(self, dev, stream):
        import ctypes
        from fate_amd import _lib
        self._c, self._lib = ctypes, _lib
        self.lib = _lib.load()
        self.stream = stream
        self.buf = torch.zeros((self.SLOTS, 3 * self.BLOCKS), dtype=torch.int64, device=dev)
        self.k = 0
        self.khz = ctypes.c_uint32(0)

    def stamp(self) -> int:
        i = self.k % self.SLOTS
        self.k += 1
        c = self._c
        self._lib.check(self.lib.fphe_clock_stamp(c.c_void_p(self.buf[i].data_ptr()), self.BLOCKS, c.byref(self.khz),
                                                  c.c_void_p(self.stream.cuda_stream)), "fphe_clock_stamp")
        return i

    def ghz(self, i0: int, i1: int):
        """Median (and spread) over CUs of the mean shader clock (GHz) between two stamps (call
        after a synchronize); None when no CU was stamped on both sides."""
        a = self.buf[i0].view(-1, 3).cpu().numpy().astype(np.uint64)
        b = self.buf[i1].view(-1, 3).cpu().numpy().astype(np.uint64)

        def first(rows):
            cu, idx = np.unique(rows[:, 0], return_index=True)
            return dict(zip(cu.tolist(), idx.tolist()))

        fa, fb = first(a), first(b)
        per = []
        for cu in set(fa) & set(fb):
            ra, rb = a[fa[cu]], b[fb[cu]]
            dc = int(rb[1]) - int(ra[1])
            dw = (int(rb[2]) - int(ra[2])) / (self.khz.value * 1e3)
            if dw > 0 and dc > 0:
                per.append(dc / dw / 1e9)
        if not per or not self.khz.value:
            return None
        per.sort()
        return {"GHz": round(per[len(per) // 2], 4), "p10": round(per[len(per) // 10], 4),
                "p90": round(per[(9 * len(per)) // 10], 4), "cus": len(per)}


def at_clock(frac: float, clock) -> dict:
    """frac rescaled to the measured clock (the roofline's peak prices 2.4 GHz)."""
    if not clock:
        return {"clock": None, "frac_at_measured_clock": None}
    return {"clock": clock, "frac_at_measured_clock": round(frac * 2.4 / clock["GHz"], 4)}


def timed_reps(fn, reps: int, stream, dev, meter: "ClockMeter") -> dict:
    """`reps` launches of fn on `stream`, each bracketed by HIP events, queued back to back
    (timed reps after warm-up), with clock stamps around them all."""
    evs = []
    s0 = meter.stamp()
    for _ in range(reps):
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        fn()
        e1.record(stream)
        evs.append((e0, e1))
    s1 = meter.stamp()
    torch.cuda.synchronize(dev)
    ms = [a.elapsed_time(b) for a, b in evs]
    return {"reps": reps, "mean_ms": sum(ms) / len(ms), "min_ms": min(ms), "max_ms": max(ms),
            "clock": meter.ghz(s0, s1)}


def rep_fields(r: dict) -> dict:
    return {"timed_reps": r["reps"], "kernel_ms_min": round(r["min_ms"], 3), "kernel_ms_max": round(r["max_ms"], 3)}


def add_kernel_leg(P, pk, a, b, N, stream, dev, meter=None) -> dict:
    """The ct-add kernel alone (k_add27 through fphe_add_ordered, launched on `stream`) on the
    Hetero-LR-shaped operands, in the exponent-gap order _add computes.  §8(d): an aligned
    add is one mulmod over L = 128 32-bit limbs (32,896 MAC32); each step of exponent gap
    adds 4 squarings of the same size (decrese_exp_to, fixedpoint_paillier/src/lib.rs:
    250-258); literal-1 operands cost nothing.  Algorithmic HBM bytes: two operands read,
    one result written, 517 B each (+ the 4-B order entry)."""
    import ctypes
    from fate_amd import _lib
    gaps = (a.exp[:N] - b.exp[:N]).abs()
    order = P._add_order(a.exp[:N], b.exp[:N], a.L2)
    out = P.CiphertextVector.empty(N, a.L2, dev)
    lib = _lib.load()
    ctx = pk._key.ctx(dev)

    def launch():
        _lib.check(lib.fphe_add_ordered(ctx, P._ptr(a.C), P._ptr(a.sign), P._ptr(a.exp), P._ptr(b.C), P._ptr(b.sign),
                                        P._ptr(b.exp), 1, N, P._ptr(order), P._ptr(out.C), P._ptr(out.sign),
                                        P._ptr(out.exp), None, ctypes.c_void_p(stream.cuda_stream)),
                   "fphe_add_ordered")

    # warm-up: ~30 ms of launches back to back, so the timed ones run at the clock a busy
    # pipeline sees (the shader clock ramps over the first ~25 ms of a burst,
    # profiles/r04/r04j2_clock_probe.txt); the first launch is timed too, as `cold_kernel_ms`
    c0 = torch.cuda.Event(enable_timing=True)
    c1 = torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize(dev)
    c0.record(stream)
    launch()
    c1.record(stream)
    for _ in range(5):
        launch()
    reps = timed_reps(launch, 10, stream, dev, meter)
    ms = reps["mean_ms"]
    L = a.L2
    mac = N * (1 + 4 * float(gaps.double().mean())) * mac32_per_mont(L)
    hist = torch.bincount(gaps.cpu()).tolist()
    # issued MACs: the final product (general; Montgomery-resident operands need no
    # to-Montgomery product) and the wave-max squarings
    TPI = L // 32
    NL = ENGINE_LL * TPI
    per_wave = 64 // TPI
    gs = gaps[order.long()] if order is not None else gaps
    pad = (-N) % per_wave
    if pad:
        gs = torch.cat([gs, gs.new_zeros(pad)])
    wave_sq = 4 * gs.view(-1, per_wave).amax(1).double().sum().item() * per_wave
    mads = N * 2 * NL * NL + wave_sq * NL * TPI * (ENGINE_LL // 2 + 1 + ENGINE_LL)
    blk = valu_roofline("k_add27<128> (exponent-gap order)", mac, ms, N * (3 * (L * 4 + 5) + 4),
                        traffic=_traffic("ct_add", N), traffic_source=pmc_ops_traffic("ct_add")[1],
                        per_elem_mac32=round(mac / N, 1), gap_histogram=hist, sorted=order is not None)
    blk["cold_kernel_ms"] = round(c0.elapsed_time(c1), 3)
    blk["warmup_launches"] = 6
    blk.update(rep_fields(reps))
    blk.update(at_clock(blk["frac"], reps["clock"]))
    blk["issue"] = {"mad64_per_elem": round(mads / N, 1), "achieved": round(mads / (ms / 1e3) / 1e12, 3),
                    "peak": round(PEAK_TMAC32, 3), "unit": "Tmad/s",
                    "frac": round(mads / (ms / 1e3) / 1e12 / PEAK_TMAC32, 4)}
    return blk


def iupdate_roofline(src, positions, stride: int, nslots: int, seconds: float, key_bits: int) -> dict:
    """rooflines.iupdate: the SecureBoost histogram's scatter ct-add
    (CiphertextVector::iupdate, fixedpoint_paillier/src/lib.rs:724-735) in SURVEY.md §8(d)'s
    MAC32 accounting, over the whole call (end to end: grouping, folds, exponent merge, the
    final add into the histogram).  Credit: one mulmod over L = 128 per scatter-add (an aligned
    Ciphertext::add), plus the exponent alignment at its least: 4 squarings per base-16 step
    between each slot's largest and least term exponent (a Horner merge of the slot's
    per-exponent partials; the reference's sequential adds align far more often).  Issued
    work: one 28-bit general product per term (2 x 148^2 mads) plus the alignment squarings
    actually run (each partial to its slot's least exponent) -- not counted here."""
    dev = src.device
    ns, npos = positions.shape
    pos = positions.to(dev).reshape(-1).long()
    ii = torch.arange(ns * npos, device=dev) // npos
    t = torch.arange(stride, device=dev)
    srci = (ii[:, None] * stride + t).reshape(-1)
    slot = (pos[:, None] * stride + t).reshape(-1)
    e = src.exp[srci].long()
    emax = torch.full((nslots,), -(1 << 40), dtype=torch.long, device=dev).scatter_reduce(0, slot, e, "amax")
    emin = torch.full((nslots,), 1 << 40, dtype=torch.long, device=dev).scatter_reduce(0, slot, e, "amin")
    used = emax > -(1 << 40)
    align_sq = int((4 * (emax - emin))[used].sum())
    terms = int(slot.numel())
    L = key_bits // 16
    mac = (terms + align_sq) * mac32_per_mont(L)
    # counter bytes: the fold's row copy and balanced level (the bulk of the call's traffic),
    # per term from the committed PMC passes, over the whole call's time
    blk = valu_roofline("fphe_fold_segments (k_gr_* grouping, k_segfold27 + k_fold27 levels, k_align_rows27) + k_add27",
                        mac, seconds * 1e3, terms * (key_bits // 4 + 5) + nslots * 3 * (key_bits // 4 + 5),
                        traffic=_traffic("iupdate", terms) if key_bits == 2048 else None,
                        traffic_source=pmc_ops_traffic("iupdate")[1],
                        per_term_mac32=round(mac / terms, 1), terms=terms, slots=nslots,
                        alignment_squarings=align_sq, scope="end to end (the whole iupdate call)")
    blk["scatter_adds_per_s"] = round(terms / seconds, 1)
    return blk


def hist_packed_leg(P, pk, sk, coder, N, HF, NB, key_bits, rank, dev):
    """SecureBoost histogram on the reference's default gh-packed path (BASELINE config 4
    (ii); ml/ensemble/learner/decision_tree/hetero/guest.py:195-235, binary task): the guest
    packs (g + 1, h) at precision 52 with shift_bit = compute_offset_bit(N, 2, 1), encrypts
    one ciphertext per sample under its own key; the host folds them into HF x NB bins
    (iupdate, all exponents 0), scans each feature (chunking_cumsum_with_step) and squeezes
    (pack_squeeze, histogram/values/_cipher.py:141) total_pack_num = (key_bits - 2) //
    (2 shift_bit) bins per ciphertext; the guest decrypts and unpacks
    (_histogram_splits.py:95-104).  Checked against the float64 cumulative histogram."""
    g0 = torch.Generator().manual_seed(4242 + rank)
    p = torch.sigmoid(torch.randn(N, generator=g0, dtype=torch.float64))
    y = (torch.rand(N, generator=g0, dtype=torch.float64) < 0.5).double()
    g, h = p - y, p * (1 - p)
    bins = torch.randint(0, NB, (N, HF), generator=g0)
    positions = bins + torch.arange(HF) * NB
    shift = int(math.log2(2 ** 52 * N * 2) + 1)
    squeeze_num = (key_bits - 2) // (shift * 2)
    vals = torch.stack([g + 1.0, h], 1).reshape(-1).to(dev)
    t = {}

    def timed(name, f):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        r = f()
        torch.cuda.synchronize(dev)
        t[name] = round(time.perf_counter() - t0, 4)
        return r

    pv = timed("pack_s", lambda: coder.pack_floats(vals, shift, 2, 52))
    en = timed("encrypt_s", lambda: pk.encrypt_encoded(pv, True))
    hist = P.CiphertextVector.zeros(HF * NB, pk._key.L2, dev)
    timed("iupdate_s", lambda: hist.iupdate(en, positions, 1, pk))
    timed("cumsum_s", lambda: hist.chunking_cumsum_with_step(pk, [NB] * HF, 1))
    sq = timed("squeeze_s", lambda: hist.pack_squeeze(squeeze_num, shift * 2, pk))
    dec = timed("decrypt_s", lambda: sk.decrypt_to_encoded(sq))
    got = torch.tensor(coder.unpack_floats(dec, shift, 2 * squeeze_num, 52, HF * NB * 2), dtype=torch.float64)
    want = torch.zeros(HF * NB, 2, dtype=torch.float64)
    for f in range(HF):
        want[:, 0].index_add_(0, positions[:, f], g + 1.0)
        want[:, 1].index_add_(0, positions[:, f], h)
    want = want.view(HF, NB, 2).cumsum(1).reshape(-1)
    return {"samples": N, "features": HF, "bins": NB, "shift_bit": shift, "squeeze_num": squeeze_num,
            "squeezed_ciphertexts": sq.count, **t,
            "scatter_adds_per_s": round(N * HF / t["iupdate_s"], 1),
            "allclose": bool(torch.allclose(got, want, rtol=1e-12, atol=1e-9))}


def hetero_lr_leg(P, pk, sk, coder, N, F, rank, dev):
    """Hetero-LR gradient step, arbiter-centralised (BASELINE config 3;
    ml/glm/hetero/coordinated_lr/guest.py:304-318 and host.py:242):
      host   enc(0.25 Xw_h) under the arbiter's public key       (N obfuscated encrypts)
      guest  enc(d) = enc(Xw_h') + (0.25 Xw - 0.5 y)              (add_plain: N ct-adds)
      host   enc(g_h) = X_h^T enc(d)                               (rmatmul: F x N ct x pt + folds)
      arbiter decrypts the F gradient entries.
    Checked against the float64 computation on the same float32 inputs."""
    g0 = torch.Generator().manual_seed(31337 + rank)
    xw = torch.randn(N, generator=g0)
    y = (torch.rand(N, generator=g0) < 0.5).float() * 2 - 1
    d_plain = (0.25 * xw - 0.5 * y).to(dev)
    xw_h = (0.25 * torch.randn(N, generator=g0)).to(dev)
    Xh = torch.randn(N, F, generator=g0).to(dev)
    t = {}

    def timed(name, f):
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        r = f()
        torch.cuda.synchronize(dev)
        t[name] = round(time.perf_counter() - t0, 4)
        return r

    enc_xw = timed("host_encrypt_s", lambda: pk.encrypt_encoded(coder.encode_f32_vec(xw_h), True))
    # evaluator.add_plain (protocol/phe/paillier.py:185-191): encode + encrypt(obfuscate=False) + add
    enc_d = timed("guest_add_plain_s",
                  lambda: enc_xw.add(pk, pk.encrypt_encoded(coder.encode_f32_vec(d_plain), False)))
    pt = coder.encode_f32_vec(Xh.t().contiguous().reshape(-1))
    grad = timed("host_rmatmul_s", lambda: enc_d.rmatmul(pk, pt, [N, 1], [F, N]))
    got = timed("arbiter_decrypt_s", lambda: coder.decode_f64_vec(sk.decrypt_to_encoded(grad))).cpu()
    dd = (d_plain.double() + xw_h.double()).cpu()
    want = Xh.double().cpu().t() @ dd
    dec_d = coder.decode_f64_vec(sk.decrypt_to_encoded(enc_d)).cpu()
    return {"samples": N, "features": F, **t,
            "ct_x_pt_per_s": round(N * F / t["host_rmatmul_s"], 1),
            "d_allclose": bool(torch.allclose(dec_d, dd, rtol=1e-12, atol=0)),
            "gradient_allclose": bool(torch.allclose(got, want, rtol=1e-9, atol=1e-9))}


def config5_leg(P, pk, sk, coder, dev, stream, meter, per_rank: int, rank: int, world: int, barrier) -> dict:
    """BASELINE config 5 in weak form (12.5M elements per GPU, 100M at 8 GPUs):
    each rank encrypts its contiguous shard [rank * per_rank, (rank + 1) * per_rank) of one
    float32 vector (randn * 4, the bench's distribution, seeded by the shard's start), one
    timed pass bracketed by a barrier and a device synchronise, max over ranks; then the
    exchange step of python/fate/arch/tensor/distributed/_tensor.py:365-395 over RCCL: the
    whole vector onto rank 0 (the federation sender; fate_amd.dist.gather_tiles_to, point to
    point) and onto every rank (the all-gather, fate_amd.dist.gather_tiles).  A 4,096-element
    sample decrypts to its inputs' bits."""
    s0 = rank * per_rank
    g = torch.Generator().manual_seed(20241218 + s0)
    x = torch.randn(per_rank, generator=g, dtype=torch.float32) * 4
    if rank == 0:
        x[:8] = torch.tensor([0.0, -0.0, 1e-30, -1e-30, 3.4e38, -3.4e38, 1.0, -1.0])[:per_rank]
    xd = x.to(dev)
    barrier()
    st0 = meter.stamp()
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    ct = pk.encrypt_encoded(coder.encode_f32_vec(xd), True)
    e1.record(stream)
    st1 = meter.stamp()
    barrier()
    secs = time.perf_counter() - t0
    kms = e0.elapsed_time(e1)
    clock = meter.ghz(st0, st1)
    nchk = min(per_rank, 4096)
    y = coder.decode_f32_vec(sk.decrypt_to_encoded(ct._gather(torch.arange(nchk)))).cpu().numpy().view(np.uint32)
    xb = x[:nchk].numpy().view(np.uint32).copy()
    xb[xb == 0x80000000] = 0
    ok = bool(np.array_equal(y, xb))
    del xd, x
    out = {"elements_per_rank": per_rank, "elements_total": per_rank * world, "ranks": world,
           "scaling": "weak", "seconds": None, "encrypts_per_s": None,
           "per_rank": {"encrypt_kernel_ms": [round(kms, 3)], "clock_GHz": [clock["GHz"] if clock else None]},
           "sample_roundtrip_bit_exact": ok}
    if world > 1:
        import torch.distributed as tdist
        tt = torch.tensor([secs, kms, clock["GHz"] if clock else float("nan"), 1.0 if ok else 0.0],
                          dtype=torch.float64, device=dev)
        allr = [torch.empty_like(tt) for _ in range(world)]
        tdist.all_gather(allr, tt)
        secs = max(float(v[0]) for v in allr)
        ks = [float(v[1]) for v in allr]
        out["per_rank"] = {"encrypt_kernel_ms": [round(v, 3) for v in ks],
                           "clock_GHz": [round(float(v[2]), 4) for v in allr],
                           "kernel_ms_spread": round(max(ks) / min(ks), 4)}
        out["sample_roundtrip_bit_exact"] = all(float(v[3]) == 1.0 for v in allr)
        from fate_amd.dist import gather_tiles, gather_tiles_to
        per_elem = ct.C.shape[1] * 4 + 1 + 4
        for name, fn in (("gather_to_rank0", lambda: gather_tiles_to(ct.C, ct.sign, ct.exp, ct.count, 0, trim=False)),
                         ("allgather", lambda: gather_tiles(ct.C, ct.sign, ct.exp, ct.count, trim=False))):
            torch.cuda.empty_cache()
            barrier()
            tg = time.perf_counter()
            got = fn()
            barrier()
            gs = time.perf_counter() - tg
            tt = torch.tensor([gs], dtype=torch.float64, device=dev)
            tdist.all_reduce(tt, op=tdist.ReduceOp.MAX)
            gs = float(tt.item())
            total = sum(got[3]) if got is not None else per_rank * world
            recv = (total - ct.count) * per_elem
            out[name] = {"seconds": round(gs, 4), "elements": int(total), "bytes_per_elem": per_elem,
                         "recv_GB": round(recv / 1e9, 2), "recv_GBps": round(recv / gs / 1e9, 2),
                         "encrypt_plus_exchange_per_s": round(per_rank * world / (secs + gs), 1)}
            del got
    out["seconds"] = round(secs, 4)
    out["encrypts_per_s"] = round(per_rank * world / secs, 1)
    out["kernel_ms_rank0"] = round(kms, 3)
    out["frac"] = round(per_rank * enc_mac32_per_elem(pk.n.bit_length()) / (kms / 1e3) / 1e12 / PEAK_TMAC32, 4)
    out.update(at_clock(out["frac"], clock))
    del ct
    torch.cuda.empty_cache()
    return out


def launch_ranks(nproc: int) -> int:
    """`bench.py --gpus N` (N > 1) started without a launcher: run the same command line as N
    ranks under torch.distributed.run (one process per GPU, rendezvous on 127.0.0.1) and
    return its exit code.  Called before anything touches the GPU; the ranks are child
    processes, not an exec of this one."""
    import socket
    import subprocess
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return subprocess.call(rank_command(nproc, port, sys.argv[1:]))


def rank_command(nproc: int, port: int, argv) -> list:
    """The torch.distributed.run command line launch_ranks starts: one node, `nproc` ranks,
    rendezvous on 127.0.0.1:port, this script with the same arguments.  torchrun's own
    parser would take "--n" as an abbreviation of its options, so it is passed as --elements."""
    args = ["--elements" if a == "--n" else ("--elements=" + a[4:] if a.startswith("--n=") else a) for a in argv]
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
            "--master-addr", "127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + args


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--n", "--elements", type=int, default=1 << 20, dest="n", help="elements per GPU")
    ap.add_argument("--total", type=int, default=0,
                    help="BASELINE config 5: this many elements in all, split over the ranks (strong "
                         "scaling), then the ciphertext all-gather; replaces --n")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip decrypt/add/e2e legs")
    ap.add_argument("--no-gather", action="store_true", help="N>1: skip the ciphertext all-gather leg")
    ap.add_argument("--config4-samples", type=int, default=10_000_000,
                    help="BASELINE config 4 leg (histogram_config4): samples in all, split over the ranks; 0 skips it")
    ap.add_argument("--config5-per-rank", type=int, default=12_500_000,
                    help="BASELINE config 5 leg (config5): elements per rank (weak: 100M at 8 GPUs), "
                         "then gather to rank 0 and all-gather; 0 skips it")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started {world} rank(s)")
    dist = world > 1
    if dist:
        import torch.distributed as tdist
        local = local % max(1, torch.cuda.device_count())  # identity with one rank per GPU
        torch.cuda.set_device(local)
        # FPHE_DIST_BACKEND=gloo: rehearse the N>1 path with several ranks on one GPU
        backend = os.environ.get("FPHE_DIST_BACKEND", "nccl")
        if backend == "nccl":
            tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            tdist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    from fate_amd import paillier as P

    with open(KEY_FIXTURE) as f:
        fx = json.load(f)
    p, q = int(fx["p"], 16), int(fx["q"], 16)
    # the headline is the public-key path (what paillier::PK::encrypt computes from n alone);
    # pk_kh is the key-holder PK that keygen hands the party owning the private key
    sk, pk, coder = P.keypair_from_primes(p, q, keyholder=False)
    pk_kh = P.keypair_from_primes(p, q, keyholder=True)[1]
    key_bits = pk.n.bit_length()

    strong = args.total > 0
    if strong:
        # BASELINE config 5: contiguous tile-aligned shards of one vector (fate_amd.dist)
        from fate_amd.dist import shard_bounds
        s0, s1 = shard_bounds(args.total, rank, world)
        N, seed = s1 - s0, 20241218 + s0
    else:
        N, seed = args.n, 20241218 + rank
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(N, generator=g, dtype=torch.float32) * 4
    x[:8] = torch.tensor([0.0, -0.0, 1e-30, -1e-30, 3.4e38, -3.4e38, 1.0, -1.0])[:N]
    xd = x.to(dev)
    stream = torch.cuda.current_stream(dev)

    def barrier():
        torch.cuda.synchronize(dev)
        if dist:
            tdist.barrier()

    def step():
        pv = coder.encode_f32_vec(xd)
        return pk.encrypt_encoded(pv, True)

    progress(f"inputs ready: {N} elements per rank")
    # warmup (also allocates the modexp scratch)
    ct = None
    for _ in range(max(args.warmup, 0)):
        ct = step()
    barrier()

    progress("warm-up done")
    # timed region; HIP events on the stream the kernels are launched on, and shader-clock
    # stamps (fphe_clock_stamp: two one-wave launches, microseconds) around the steps
    meter = ClockMeter(dev, stream)
    ev_enc = []
    st_enc0 = meter.stamp()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        pv = coder.encode_f32_vec(xd)
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        ct = pk.encrypt_encoded(pv, True)
        e1.record(stream)
        ev_enc.append((e0, e1))
    st_enc1 = meter.stamp()
    barrier()
    elapsed = time.perf_counter() - t0
    enc_ms_all = [a.elapsed_time(b) for a, b in ev_enc]
    enc_kernel_ms = sum(enc_ms_all) / max(len(ev_enc), 1)
    enc_clock = meter.ghz(st_enc0, st_enc1)
    per_rank = None
    if dist:
        tt = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        tdist.all_reduce(tt, op=tdist.ReduceOp.MAX)
        elapsed = float(tt.item())
        # per-rank kernel time and clock: the driver's scaling run can
        # then tell a rank's imbalance from its box's clock
        mine = torch.tensor([enc_kernel_ms, enc_clock["GHz"] if enc_clock else float("nan")], dtype=torch.float64,
                            device=dev)
        allr = [torch.empty_like(mine) for _ in range(world)]
        tdist.all_gather(allr, mine)
        ks = [float(v[0]) for v in allr]
        cs = [float(v[1]) for v in allr]
        per_rank = {"encrypt_kernel_ms": [round(v, 3) for v in ks], "clock_GHz": [round(v, 4) for v in cs],
                    "kernel_ms_min": round(min(ks), 3), "kernel_ms_max": round(max(ks), 3),
                    "kernel_ms_spread": round(max(ks) / min(ks), 4),
                    "clock_GHz_min": round(min(cs), 4), "clock_GHz_max": round(max(cs), 4)}
    progress(f"timed encrypt: {args.steps} steps in {elapsed:.1f} s")
    value = (args.total if strong else world * N) * args.steps / elapsed

    # BASELINE config 5's exchange step, outside the timed region: every rank's ciphertext
    # shard all-gathered over RCCL/xGMI (fate_amd.dist.gather_tiles), so the whole vector
    # sits on each rank as the federation sender needs it.  Reported beside `value`.
    gather_info = {}
    if dist and not args.no_gather:
        from fate_amd.dist import gather_tiles, gather_tiles_to
        # onto rank 0 only (the federation sender: fate_amd.dist.gather_tiles_to, point to
        # point), then onto every rank (the all-gather)
        barrier()
        tg = time.perf_counter()
        got = gather_tiles_to(ct.C, ct.sign, ct.exp, ct.count, 0, trim=False)
        barrier()
        g1 = time.perf_counter() - tg
        tt = torch.tensor([g1], dtype=torch.float64, device=dev)
        tdist.all_reduce(tt, op=tdist.ReduceOp.MAX)
        g1 = float(tt.item())
        total0 = sum(got[3]) if got is not None else 0
        del got
        torch.cuda.empty_cache()
        barrier()
        tg = time.perf_counter()
        Cg, sg, eg, counts = gather_tiles(ct.C, ct.sign, ct.exp, ct.count, trim=False)
        total = sum(counts)
        barrier()
        gs = time.perf_counter() - tg
        tt = torch.tensor([gs], dtype=torch.float64, device=dev)
        tdist.all_reduce(tt, op=tdist.ReduceOp.MAX)
        gs = float(tt.item())
        # ciphertext bytes each rank receives (limbs + sign + exp of the other ranks' shards)
        per_elem = ct.C.shape[1] * 4 + 1 + 4
        recv = (total - ct.count) * per_elem
        gather_info = {
            "allgather": {"seconds": round(gs, 4), "elements": int(total), "bytes_per_elem": per_elem,
                          "recv_GBps_per_rank": round(recv / gs / 1e9, 2),
                          "encrypt_plus_allgather_per_s": round((args.total if strong else world * N)
                                                                / (elapsed / args.steps + gs), 1)},
            "gather_to_rank0": {"seconds": round(g1, 4), "elements": int(total0),
                                "recv_GBps_rank0": round((total0 - ct.count) * per_elem / g1 / 1e9, 2),
                                "encrypt_plus_gather_per_s": round((args.total if strong else world * N)
                                                                   / (elapsed / args.steps + g1), 1)},
        }
        del Cg, sg, eg

    extras = {}
    if not args.no_extras and not strong:
        # decrypt (device-resident), with the bit-exact round trip check; one untimed pass
        # first, so the timed one does not include growing the context's scratch buffer
        # (the timed pass is queued right behind it, no host sync between: the shader clock
        # ramps over the first ~25 ms of a burst and drops within milliseconds of idling,
        # profiles/r04/r04j2_clock_probe.txt)
        ec0 = torch.cuda.Event(enable_timing=True); ec1 = torch.cuda.Event(enable_timing=True)
        ec0.record(stream)
        sk.decrypt_to_encoded(ct)
        ec1.record(stream)
        dec_reps = timed_reps(lambda: sk.decrypt_to_encoded(ct), 5, stream, dev, meter)
        pt = sk.decrypt_to_encoded(ct)
        y = coder.decode_f32_vec(pt)
        torch.cuda.synchronize(dev)
        dec_ms = dec_reps["mean_ms"]
        dec_cold_ms = ec0.elapsed_time(ec1)  # the first pass: cold clock, growing scratch
        e0 = torch.cuda.Event(enable_timing=True); e1 = torch.cuda.Event(enable_timing=True)
        xb = x.numpy().view(np.uint32).copy()
        xb[xb == 0x80000000] = 0  # -0.0 encodes to significand 0 -> decodes +0.0 (reference)
        roundtrip_ok = bool(np.array_equal(y.cpu().numpy().view(np.uint32), xb))
        progress("decrypt leg done")
        # ct-add (Hetero-LR aggregate shape): enc(x) + enc(0.25*x') elementwise, exps differ
        ct2 = pk.encrypt_encoded(coder.encode_f32_vec(torch.flip(xd, [0]) * 0.25), True)
        for _ in range(4):  # untimed: first-call costs of the sort, the output's allocation, the clock
            ct.add(pk, ct2)
        # the whole add call (order + kernel), 5 reps queued back to back (no gap read-back:
        # both operands come from the encoder, whose exponent range the kernel covers)
        add_reps = timed_reps(lambda: ct.add(pk, ct2), 5, stream, dev, meter)
        s = ct.add(pk, ct2)
        torch.cuda.synchronize(dev)
        add_ms = add_reps["mean_ms"]
        add_kernel = add_kernel_leg(P, pk, ct, ct2, N, stream, dev, meter)
        # end-to-end from host f32 to the reference's signed ciphertext integers in pinned host
        # memory (export out of the Montgomery-resident form included), one pass
        xh = x.pin_memory()
        Ch = torch.empty((N, ct.L2), dtype=torch.int32, pin_memory=True)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        ce = pk.encrypt_encoded(coder.encode_f32_vec(xh.to(dev, non_blocking=True)), True)
        mag_e, neg_e, exp_e = ce.export_signed(pk)
        Ch.copy_(mag_e, non_blocking=True)
        sh = neg_e.cpu(); eh = exp_e.cpu()
        torch.cuda.synchronize(dev)
        e2e = time.perf_counter() - t0
        del mag_e, neg_e, exp_e, Ch
        # ... and to the bytes that leave the party: the reference's pickle
        # state of the vector, bincode(CiphertextVector) of the signed integers
        # (paillier.rs:219-226), formatted on the device (fate_amd.wire) and copied into a
        # pinned host buffer -- what the federation transport sends
        from fate_amd import wire
        wire_cap = 8 + N * (4 + 8 + 4 + 1 + 8 * ct.L2)  # the widest record: a full-width hex integer
        Wh = torch.empty(wire_cap, dtype=torch.uint8, pin_memory=True)
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        cw = pk.encrypt_encoded(coder.encode_f32_vec(xh.to(dev, non_blocking=True)), True)
        whead, wrec = wire.ciphertext_vector_records(cw, pk)
        Wh[8:8 + wrec.numel()].copy_(wrec, non_blocking=True)
        torch.cuda.synchronize(dev)
        e2e_wire = time.perf_counter() - t0
        Wh[:8] = torch.frombuffer(bytearray(whead), dtype=torch.uint8)
        wire_bytes = 8 + wrec.numel()
        # the wire step alone (export + format + D2H), on the same vector
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        whead, wrec = wire.ciphertext_vector_records(cw, pk)
        Wh[8:8 + wrec.numel()].copy_(wrec, non_blocking=True)
        torch.cuda.synchronize(dev)
        wire_only = time.perf_counter() - t0
        # round trip of a sample of the bytes through the host parser (the reference's layout)
        nchk = min(N, 4096)
        hchk, rchk = wire.ciphertext_vector_records(cw._gather(torch.arange(nchk)), pk)
        back, used = wire.ciphertext_vector_from_bincode(hchk + bytes(rchk.cpu().numpy()), pk)
        wire_ok = used == 8 + rchk.numel() and torch.equal(back.C[: (nchk + 63) // 64], cw.C[: (nchk + 63) // 64]) \
            and torch.equal(back.sign[:nchk], cw.sign[:nchk]) and torch.equal(back.exp[:nchk], cw.exp[:nchk])
        e2e_wire_block = {"encrypts_per_s": round(N / e2e_wire, 1), "seconds": round(e2e_wire, 4),
                          "wire_bytes": int(wire_bytes), "wire_only_s": round(wire_only, 4),
                          "wire_only_GBps": round(wire_bytes / wire_only / 1e9, 3), "sample_round_trip_ok": bool(wire_ok),
                          "scope": "host f32 (pinned) -> H2D -> device encode + obfuscated encrypt -> export of the "
                                   "signed integers -> device bincode formatting -> D2H into pinned host bytes"}
        del cw, wrec, Wh, back
        progress("ct-add, end-to-end and wire legs done")
        # ct x pt (SecureBoost GOSS-style weights; negatives take the device inverse branch)
        gw = torch.Generator().manual_seed(777 + rank)
        wts = (torch.rand(N, generator=gw, dtype=torch.float32) * 3.0 - 1.0).to(dev)
        pw = coder.encode_f32_vec(wts)
        n_neg = int((wts < 0).sum().item())
        torch.cuda.synchronize(dev)
        ec0 = torch.cuda.Event(enable_timing=True); ec1 = torch.cuda.Event(enable_timing=True)
        ec0.record(stream)
        ct.mul(pk, pw)  # untimed: grows the context scratch to the op's size (and warms the clock)
        ec1.record(stream)
        mul_reps = timed_reps(lambda: ct.mul(pk, pw), 5, stream, dev, meter)
        m = ct.mul(pk, pw)
        torch.cuda.synchronize(dev)
        mul_ms = mul_reps["mean_ms"]
        mul_cold_ms = ec0.elapsed_time(ec1)
        # SecureBoost histogram (BASELINE config 4 shape at one GPU): (g, h) interleaved with
        # stride 2, HF features x 32 bins, iupdate = per-bin ct-add fold on the device
        HF, NB = 4, 32
        gb = torch.Generator().manual_seed(99 + rank)
        bins = torch.randint(0, NB, (N, HF), generator=gb)
        positions = bins + torch.arange(HF) * NB
        # the bin indexes are input data, resident in HBM like the ciphertexts (the binning
        # step that makes them runs on the device too); the host-list rate is reported beside
        positions_d = positions.to(dev, torch.int32)
        # SecureBoost-shaped gradients (as tools/bench_legs/secureboost_full.py): g = p - y,
        # h = p (1 - p), encrypted by the guest (key holder, untimed), interleaved (g, h)
        psig = torch.sigmoid(torch.randn(N, generator=gb, dtype=torch.float64))
        ylab = (torch.rand(N, generator=gb, dtype=torch.float64) < 0.5).double()
        g_sb, h_sb = (psig - ylab).float(), (psig * (1 - psig)).float()
        gh = pk_kh.encrypt_encoded(coder.encode_f32_vec(torch.stack([g_sb, h_sb], 1).reshape(-1).to(dev)), True)

        def run_hist(src, wg, wh):
            # untimed full-size pass first, as for the other legs: the call's stream-ordered
            # scratch (term keys, element-major rows, partials: ~0.6 GB here) is mapped into
            # the device pool there, not in the timed call
            P.CiphertextVector.zeros(HF * NB * 2, pk._key.L2, dev).iupdate(src, positions_d, 2, pk)
            hh = P.CiphertextVector.zeros(HF * NB * 2, pk._key.L2, dev)
            torch.cuda.synchronize(dev)
            s0h = meter.stamp()
            t0h = time.perf_counter()
            hh.iupdate(src, positions_d, 2, pk)
            s1h = meter.stamp()
            torch.cuda.synchronize(dev)
            secs = time.perf_counter() - t0h
            hist_clock.append(meter.ghz(s0h, s1h))
            # property check: decrypted bins == float64 sums of the encoded inputs
            hd = coder.decode_f64_vec(sk.decrypt_to_encoded(hh)).cpu().reshape(HF * NB, 2)
            want = torch.zeros(HF * NB, 2, dtype=torch.float64)
            for f in range(HF):
                want[:, 0].index_add_(0, positions[:, f], wg)
                want[:, 1].index_add_(0, positions[:, f], wh)
            fin = torch.isfinite(want)
            return hh, secs, bool(torch.allclose(hd[fin], want[fin], rtol=1e-9, atol=1e-6)), want

        progress("ct x pt leg done")
        hist_clock = []
        hist, hist_s, hist_ok, want = run_hist(gh, g_sb.double(), h_sb.double())
        hist_h = P.CiphertextVector.zeros(HF * NB * 2, pk._key.L2, dev)
        torch.cuda.synchronize(dev)
        t0h = time.perf_counter()
        hist_h.iupdate(gh, positions, 2, pk)  # positions as a host tensor: + the H2D copy
        torch.cuda.synchronize(dev)
        hist_host_s = time.perf_counter() - t0h
        # positions as the reference's caller hands them over: Vec<Vec<usize>>, one Python list per
        # sample (HistogramIndexer.get_positions, arch/histogram/_histogram_local.py:68-82), read
        # by the host helper; the lists are made before the clock starts
        pos_lists = positions.tolist()
        hist_h = P.CiphertextVector.zeros(HF * NB * 2, pk._key.L2, dev)
        torch.cuda.synchronize(dev)
        t0h = time.perf_counter()
        hist_h.iupdate(gh, pos_lists, 2, pk)
        torch.cuda.synchronize(dev)
        hist_list_s = time.perf_counter() - t0h
        del hist_h, pos_lists
        iupdate_block = iupdate_roofline(gh, positions, 2, HF * NB * 2, hist_s, key_bits)
        iupdate_block.update(at_clock(iupdate_block["frac"], hist_clock[0]))
        # the same call 5 times back to back (no host sync between calls; each still reads
        # back its own small bookkeeping): the shader clock ramps up over the first ~25 ms of
        # a full-chip burst (profiles/r04/r04j2_clock_probe.txt), so one cold 18-ms call runs
        # below the clock a busy pipeline sees.  Reported beside, `frac` stays the cold call's.
        hs5 = [P.CiphertextVector.zeros(HF * NB * 2, pk._key.L2, dev) for _ in range(5)]
        torch.cuda.synchronize(dev)
        s0h = meter.stamp()
        t0h = time.perf_counter()
        for h5 in hs5:
            h5.iupdate(gh, positions_d, 2, pk)
        s1h = meter.stamp()
        torch.cuda.synchronize(dev)
        sus_s = (time.perf_counter() - t0h) / 5
        del hs5
        sus_frac = iupdate_roofline(gh, positions, 2, HF * NB * 2, sus_s, key_bits)["frac"]
        iupdate_block["sustained"] = {"calls": 5, "mean_s": round(sus_s, 5), "frac": sus_frac,
                                      **at_clock(sus_frac, meter.ghz(s0h, s1h))}
        # the same fold over the encrypt leg's vector and its mirror (x with the edge values
        # 0, +-1e-30, +-3.4e38 among the first inputs): exponent gaps up to 31 force one
        # 124-squaring alignment chain, a ~4.8 ms critical path on a single wave
        gh_edge = P.Evaluator.cat([ct, ct2])._gather(torch.stack([torch.arange(N), N + torch.arange(N)], 1).reshape(-1))
        he, hist_edge_s, hist_edge_ok, _ = run_hist(gh_edge, x.double(), torch.flip(x, [0]).double() * 0.25)
        # the same data without the edge values (their 8 samples' g, and the 8 mirrored h, are
        # replaced by copies of neighbouring elements): what the edge values alone cost
        sel = torch.arange(2 * N)
        sel[0:16:2] = torch.arange(16, 32, 2)
        sel[2 * N - 15::2] = torch.arange(2 * N - 31, 2 * N - 15, 2)
        gh_ne = gh_edge._gather(sel)
        wg_ne, wh_ne = x.double().clone(), torch.flip(x, [0]).double() * 0.25
        wg_ne[:8] = wg_ne[8:16].clone()
        wh_ne[N - 8:] = wh_ne[N - 16:N - 8].clone()
        hne, hist_ne_s, hist_ne_ok, _ = run_hist(gh_ne, wg_ne, wh_ne)
        hist_edge = {"iupdate_s": round(hist_edge_s, 5), "allclose": hist_edge_ok,
                     "roofline_frac": iupdate_roofline(gh_edge, positions, 2, HF * NB * 2, hist_edge_s, key_bits)["frac"],
                     "iupdate_s_same_data_without_edge_values": round(hist_ne_s, 5),
                     "allclose_without_edge_values": hist_ne_ok,
                     "edge_over_without": round(hist_edge_s / hist_ne_s, 3)}
        del he, gh_edge, hne, gh_ne
        hist_mgpu = None
        if dist:
            # config 4 across GPUs: each rank folded its own samples; the
            # partial histograms are all-gathered over RCCL and folded again with ct-add
            # (RCCL has no modular product; ciphertext folds are order independent)
            try:
                from fate_amd.dist import fold_across_ranks
                barrier()
                acc, t_gather, t_fold = fold_across_ranks(pk, hist)
                wd = want.to(dev)  # the float64 reference sums, gathered as device tensors like the shards
                wants = [torch.empty_like(wd) for _ in range(world)]
                tdist.all_gather(wants, wd)
                want_all = sum(w.cpu() for w in wants)
                got_all = coder.decode_f64_vec(sk.decrypt_to_encoded(acc)).cpu().reshape(HF * NB, 2)
                fin_all = torch.isfinite(want_all)
                hist_mgpu = {"ranks": world, "gather_s": round(t_gather, 4), "fold_s": round(t_fold, 4),
                             "allclose": bool(torch.allclose(got_all[fin_all], want_all[fin_all], rtol=1e-9,
                                                             atol=1e-6))}
                del acc
            except Exception as exc:  # report, do not take the scaling run down
                hist_mgpu = {"error": repr(exc)[:200]}
        progress("histogram legs done")
        packed = hist_packed_leg(P, pk_kh, sk, coder, N, HF, NB, key_bits, rank, dev)
        hlr = hetero_lr_leg(P, pk, sk, coder, N, 4, rank, dev)
        progress("packed histogram and Hetero-LR legs done")
        # 1024-bit keys (the reference's own tests and configs[0] use them)
        with open(os.path.join(ROOT, "tests", "golden", "paillier_1024.json")) as f:
            fx1 = json.load(f)
        sk1, pk1, coder1 = P.keypair_from_primes(int(fx1["p"], 16), int(fx1["q"], 16), keyholder=False)
        pv1 = coder1.encode_f32_vec(xd)
        # untimed full-size passes first: the new context's scratch and the outputs are
        # allocated there, not in the timed calls
        # (timed passes queued behind them with no host sync: the clock, see the decrypt leg)
        sk1.decrypt_to_encoded(pk1.encrypt_encoded(pv1, True))
        enc1 = timed_reps(lambda: pk1.encrypt_encoded(pv1, True), 5, stream, dev, meter)
        c1 = pk1.encrypt_encoded(pv1, True)
        dec1 = timed_reps(lambda: sk1.decrypt_to_encoded(c1), 5, stream, dev, meter)
        d1 = sk1.decrypt_to_encoded(c1)
        torch.cuda.synchronize(dev)
        enc1_ms, dec1_ms = enc1["mean_ms"], dec1["mean_ms"]
        e2 = torch.cuda.Event(enable_timing=True); e3 = torch.cuda.Event(enable_timing=True)
        y1 = coder1.decode_f32_vec(d1)
        ef1 = round(N * enc_mac32_per_elem(1024) / (enc1_ms / 1e3) / 1e12 / PEAK_TMAC32, 4)
        df1 = round(N * dec_mac32_per_elem(1024) / (dec1_ms / 1e3) / 1e12 / PEAK_TMAC32, 4)
        k1024 = {"encrypt_per_s": round(N / (enc1_ms / 1e3), 1), "decrypt_per_s": round(N / (dec1_ms / 1e3), 1),
                 "roundtrip_bit_exact": bool(np.array_equal(y1.cpu().numpy().view(np.uint32), xb)),
                 "encrypt_roofline_frac": ef1, "decrypt_roofline_frac": df1,
                 "encrypt_reps": {**rep_fields(enc1), **at_clock(ef1, enc1["clock"])},
                 "decrypt_reps": {**rep_fields(dec1), **at_clock(df1, dec1["clock"])}}
        del c1, d1, y1, pv1
        # 4096-bit keys (the TPI-8 geometry; he_param.key_length is a job parameter): rates on
        # the first 2^16 elements (a 4096-bit encrypt is ~8x a 2048-bit one), round trip
        k4096 = None
        kpath = os.path.join(ROOT, "tests", "golden", "key_4096.json")
        if os.path.exists(kpath):
            with open(kpath) as f:
                fx4 = json.load(f)
            sk4, pk4, coder4 = P.keypair_from_primes(int(fx4["p"], 16), int(fx4["q"], 16), keyholder=False)
            n4 = min(N, 1 << 16)
            pv4 = coder4.encode_f32_vec(xd[:n4])
            sk4.decrypt_to_encoded(pk4.encrypt_encoded(pv4, True))  # untimed: scratch growth
            e0.record(stream)
            c4 = pk4.encrypt_encoded(pv4, True)
            e1.record(stream)
            e2.record(stream)
            d4 = sk4.decrypt_to_encoded(c4)
            e3.record(stream)
            torch.cuda.synchronize(dev)
            enc4_ms = e0.elapsed_time(e1)
            dec4_ms = e2.elapsed_time(e3)
            y4 = coder4.decode_f32_vec(d4)
            k4096 = {"elements": n4, "encrypt_per_s": round(n4 / (enc4_ms / 1e3), 1),
                     "decrypt_per_s": round(n4 / (dec4_ms / 1e3), 1),
                     "roundtrip_bit_exact": bool(np.array_equal(y4.cpu().numpy().view(np.uint32), xb[:n4])),
                     "encrypt_roofline_frac": round(n4 * enc_mac32_per_elem(4096) / (enc4_ms / 1e3) / 1e12 / PEAK_TMAC32, 4),
                     "decrypt_roofline_frac": round(n4 * dec_mac32_per_elem(4096) / (dec4_ms / 1e3) / 1e12 / PEAK_TMAC32, 4)}
            del c4, d4, y4, pv4
        progress("1024- and 4096-bit legs done")
        # key-holder encryption (CRT halves): throughput, round trip, and identity with the
        # public-key path on a subset with the same injected r
        torch.cuda.synchronize(dev)
        e0.record(stream)
        ck = pk_kh.encrypt_encoded(coder.encode_f32_vec(xd), True)
        e1.record(stream)
        torch.cuda.synchronize(dev)
        crt_ms = e0.elapsed_time(e1)
        yk = coder.decode_f32_vec(sk.decrypt_to_encoded(ck))
        crt_roundtrip = bool(np.array_equal(yk.cpu().numpy().view(np.uint32), xb))
        nsub = min(N, 4096)
        rr = np.random.default_rng(5 + rank)
        rsub = [1 + int.from_bytes(rr.bytes(key_bits // 8), "little") % (pk.n - 1) for _ in range(nsub)]
        psub = coder.encode_f32_vec(xd[:nsub])
        cpub = pk.encrypt_encoded(psub, True, r=rsub)
        ckh = pk_kh.encrypt_encoded(psub, True, r=rsub)
        crt_same = bool(torch.equal(cpub.C, ckh.C) and torch.equal(cpub.sign, ckh.sign))
        del ck, yk, cpub, ckh
        extras = {
            "encrypt_keyholder_crt_per_s": round(N / (crt_ms / 1e3), 1),
            "encrypt_keyholder_crt_roofline_frac": round(N * enc_crt_mac32_per_elem(key_bits, kh_direct_z(sk.p, sk.q))
                                                         / (crt_ms / 1e3) / 1e12 / PEAK_TMAC32, 4),
            "encrypt_keyholder_direct_z": kh_direct_z(sk.p, sk.q),
            "encrypt_keyholder_crt_roundtrip_bit_exact": crt_roundtrip,
            "encrypt_keyholder_crt_equals_public_4096": crt_same,
            "ct_mul_per_s": round(N / (mul_ms / 1e3), 1),
            "histogram_scatter_adds_per_s": round(N * HF * 2 / hist_s, 1),
            "histogram_iupdate_s": round(hist_s, 5),
            "histogram_iupdate_host_positions_s": round(hist_host_s, 5),
            "histogram_iupdate_list_positions_s": round(hist_list_s, 5),
            "histogram_edge_values": hist_edge,
            "histogram_config": f"{N} samples x {HF} features x {NB} bins x (g,h), SecureBoost-shaped g = p - y, "
                                f"h = p(1 - p) (key-holder encryptions, untimed), iupdate fold on device",
            "histogram_allclose": hist_ok,
            "histogram_packed": packed,
            "histogram_multi_gpu": hist_mgpu,
            "hetero_lr_gradient": hlr,
            "key_1024": k1024,
            "key_4096": k4096,
            "decrypt_per_s": round(N / (dec_ms / 1e3), 1),
            "ct_add_per_s": round(N / (add_ms / 1e3), 1),
            "e2e_host_encrypts_per_s": round(N / e2e, 1),
            "e2e_wire_bytes": e2e_wire_block,
            "ct_add_reps": rep_fields(add_reps),
            "roundtrip_bit_exact": roundtrip_ok,
            "decrypt_roofline_frac": round(N * dec_mac32_per_elem(key_bits) / (dec_ms / 1e3) / 1e12 / PEAK_TMAC32, 4),
            "rooflines": {
                "decrypt": valu_roofline("k_pow_half27<128,6,false,false> + k_decrypt_crt<128>",
                                         N * dec_mac32_per_elem(key_bits), dec_ms,
                                         N * (key_bits // 4 + 4 + key_bits // 8),
                                         traffic=_traffic("decrypt", N), traffic_source=pmc_ops_traffic("decrypt")[1],
                                         cold_kernel_ms=round(dec_cold_ms, 3), **rep_fields(dec_reps)),
                "iupdate": iupdate_block,
                "ct_add": add_kernel,
                # §8(d): float significands (E = 56): (56 + 12 + 16) mulmods over L = 128, + 3
                # for each negative weight (the inverse branch); the whole op is timed:
                # classify, batch inverse of the negative-weight elements, the powm
                "ct_mul": valu_roofline("k_mul_prep + k_binv_pre27/k_inv_n27/k_inv_lift27/k_binv_post27 + k_mul27<128,4>",
                                        (N * (56 + 12 + 16) + 3 * n_neg) * mac32_per_mont(key_bits // 16), mul_ms,
                                        N * 2 * (key_bits // 4 + 5) + N * 13, traffic=_traffic("ct_mul", N),
                                        traffic_source=pmc_ops_traffic("ct_mul")[1], negative_weights=n_neg,
                                        cold_kernel_ms=round(mul_cold_ms, 3), **rep_fields(mul_reps)),
            },
        }
        for _k, _r in (("decrypt", dec_reps), ("ct_mul", mul_reps)):
            extras["rooflines"][_k].update(at_clock(extras["rooflines"][_k]["frac"], _r["clock"]))
        del pt, y, ct2, s, ce, m, gh, hist
        # BASELINE config 4 at its stated size (10M samples x 10 features x 32 bins, 2048-bit):
        # unpacked ct x pt + the 200M-term iupdate, packed iupdate + cumsum + squeeze, sharded
        # over the ranks with the cross-rank fold (tools/bench_legs/secureboost_full.py)
        progress("key-holder leg done")
        if args.config4_samples > 0:
            import importlib.util
            spec = importlib.util.spec_from_file_location(
                "secureboost_full", os.path.join(ROOT, "tools", "bench_legs", "secureboost_full.py"))
            sbf = importlib.util.module_from_spec(spec)
            spec.loader.exec_module(sbf)
            torch.cuda.empty_cache()
            extras["histogram_config4"] = sbf.config4(P, pk_kh, sk, coder, dev, total=args.config4_samples, rank=rank,
                                                      world=world, iupdate_roofline=iupdate_roofline)
            torch.cuda.empty_cache()

    progress("extras done")
    # BASELINE config 5 (every line, so the driver's scaling run measures it): 12.5M per rank
    if args.config5_per_rank > 0 and not strong:
        del ct
        torch.cuda.empty_cache()
        extras["config5"] = config5_leg(P, pk, sk, coder, dev, stream, meter, args.config5_per_rank, rank, world,
                                        barrier)

    if rank != 0:
        if dist:
            tdist.barrier()
            tdist.destroy_process_group()
        return

    mac_launch = N * enc_mac32_per_elem(key_bits)
    achieved = mac_launch / (enc_kernel_ms / 1e3) / 1e12
    # algorithmic HBM bytes per element: f32 sig/exp/neg read (13 B) + C (512 B) + sign (1 B) written
    hbm_bytes = N * (8 + 1 + 4 + key_bits // 4 + 1)
    mad27 = N * enc_mad27_per_elem(key_bits, pk.n) / (enc_kernel_ms / 1e3) / 1e12
    tb, tsrc = pmc_traffic_per_elem()
    roofline = {
        "bound": "valu",
        "kernel": "k_encrypt27<128,6> (+k_draw_r)",
        "achieved": round(achieved, 3),
        "peak": round(PEAK_TMAC32, 3),
        "unit": "TMAC32/s",
        "frac": round(achieved / PEAK_TMAC32, 4),
        # HBM bytes per launch from PMC counters (separate --pmc runs, calibrated; dominated
        # by the window-table scratch, see the profile's note); None if not profiled
        "traffic": round(tb * N) if tb is not None else None,
        "traffic_source": tsrc,
        "per_elem_mac32": enc_mac32_per_elem(key_bits),
        "kernel_ms": round(enc_kernel_ms, 3),
        # instruction-issue view of the same launch: 27-bit-limb MACs issued (one
        # v_mad_u64_u32 each) against the same half-rate mad peak
        "issue": {"mad64_per_elem": enc_mad27_per_elem(key_bits, pk.n), "achieved": round(mad27, 3),
                  "peak": round(PEAK_TMAC32, 3), "unit": "Tmad/s", "frac": round(mad27 / PEAK_TMAC32, 4)},
        "hbm": hbm_block(hbm_bytes, enc_kernel_ms, round(tb * N) if tb is not None else None, tsrc),
        "kernel_ms_per_step": [round(v, 3) for v in enc_ms_all],
    }
    roofline.update(at_clock(roofline["frac"], enc_clock))
    out = {
        "metric": "Paillier-2048 encrypts/sec device-resident",
        "value": round(value, 1),
        "unit": "encrypts/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "strong" if strong else "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic",
        "config": ({"workload": f"paillier2048_encrypt_f32_{args.total}_strong", "key_bits": key_bits,
                    "elements_total": args.total, "elements_rank0": N, "obfuscate": True,
                    "parallelism": f"shard{world}"} if strong else
                   {"workload": "paillier2048_encrypt_f32_" + ("1M" if N == 1 << 20 else str(N)), "key_bits": key_bits,
                    "elements_per_gpu": N,
                    "obfuscate": True, "parallelism": f"shard{world}"}),
        "roofline": roofline,
    }
    if per_rank is not None:
        out["per_rank"] = per_rank
    out.update(gather_info)
    out.update(extras)
    progress("config 5 leg done; CPU baseline next" if world == 1 else "config 5 leg done")
    if world == 1 and not args.no_cpu_baseline and not strong:
        try:
            cb = cpu_baseline(p, q)
            # GPU / CPU ratios: against the measured worker pool, one process, and the
            # projected whole host (north_star target: >= 10x on 2048-bit encrypt)
            sp = cb["single_process_per_s"]
            hp = cb["host_projection"]["encrypt_per_s"]
            ratios = {"encrypt_vs_pool": value / cb["value"], "encrypt_vs_1_process": value / sp["encrypt"],
                      "encrypt_vs_host_projection": value / hp if hp else None}
            if extras:
                # the host projection scales every op's pool rate by the encrypt projection's
                # host/pool factor (cores x SMT uplift)
                host = hp / cb["value"]
                gpu = {"decrypt": extras["decrypt_per_s"], "ct_add_hetero_lr": extras["ct_add_per_s"],
                       "ct_mul": extras["ct_mul_per_s"], "iupdate": extras["histogram_scatter_adds_per_s"]}
                cpu = {"decrypt": cb["decrypt_per_s"], "ct_add_hetero_lr": cb["ct_add_hetero_lr_gaps_per_s"],
                       "ct_mul": cb["ct_mul_per_s"], "iupdate": cb["iupdate_per_s"]}
                for k in gpu:
                    ratios[f"{k}_vs_pool"] = gpu[k] / cpu[k]
                    ratios[f"{k}_vs_host_projection"] = gpu[k] / (cpu[k] * host)
            cb["gpu_over_cpu"] = {k: (round(v, 2) if v is not None else None) for k, v in ratios.items()}
            out["cpu_baseline"] = cb
        except Exception as exc:  # GMP missing on the box: say so, do not fake a number
            out["cpu_baseline"] = {"value": None, "unit": "encrypts/s", "cores": 0, "kind": "port",
                                   "sample": f"unavailable: {exc}"}
    print(json.dumps(out))
    if dist:
        tdist.barrier()
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
