"""ctypes wrapper of oracle/build/libgmpref.so -- TEST INFRASTRUCTURE ONLY.

Cross-checks the pure-Python restatement against libgmp (the library rug wraps) and times
the CPU baseline for bench.py (cpu_baseline.kind = "port").
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import Optional

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "libgmpref.so")
_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        lib = ctypes.CDLL(LIB)
        lib.gref_new.restype = ctypes.c_void_p
        lib.gref_new.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p]
        lib.gref_free.argtypes = [ctypes.c_void_p]
        for name in ("gref_encrypt",):
            getattr(lib, name).argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int,
                                           ctypes.c_char_p, ctypes.c_size_t]
        lib.gref_decrypt.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_size_t]
        lib.gref_add_ct.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p,
                                    ctypes.c_size_t]
        lib.gref_powm.argtypes = [ctypes.c_char_p] * 4 + [ctypes.c_size_t]
        lib.gref_tdiv_r.argtypes = [ctypes.c_char_p] * 3 + [ctypes.c_size_t]
        P, L_, I = ctypes.c_void_p, ctypes.c_long, ctypes.c_int
        lib.gref_fold.argtypes = [P, I, P, P, P, P, P, L_, P, P, P, L_, I]
        lib.gref_mul.argtypes = [P, I, P, P, P, I, P, P, P, L_, P, P, P, I]
        lib.gref_squeeze.argtypes = [P, I, P, P, L_, I, ctypes.c_ulong, P, P, P]
        lib.gref_cumsum.argtypes = [P, I, P, P, P, L_, P, L_, L_]
        lib.gref_bench.restype = ctypes.c_double
        lib.gref_bench.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_long, ctypes.c_int, ctypes.c_ulong]
        _lib = lib
    return _lib


def _h(v: int) -> bytes:
    return (("-" + hex(-v)[2:]) if v < 0 else hex(v)[2:]).encode()


def _int(buf) -> int:
    s = buf.value.decode()
    return -int(s[1:], 16) if s.startswith("-") else int(s, 16)


class GmpKey:
    def __init__(self, n: int, p: Optional[int] = None, q: Optional[int] = None):
        lib = load()
        self.n = n
        self.ctx = lib.gref_new(_h(n), _h(p) if p else None, _h(q) if q else None)
        self.cap = 4 * n.bit_length() // 4 + 16

    def __del__(self):
        try:
            load().gref_free(self.ctx)
        except Exception:
            pass

    def encrypt(self, m: int, r: Optional[int], obfuscate: bool) -> int:
        out = ctypes.create_string_buffer(self.cap)
        load().gref_encrypt(self.ctx, _h(m), _h(r or 1), 1 if obfuscate else 0, out, self.cap)
        return _int(out)

    def decrypt(self, c: int) -> int:
        out = ctypes.create_string_buffer(self.cap)
        load().gref_decrypt(self.ctx, _h(c), out, self.cap)
        return _int(out)

    def add_ct(self, a: int, b: int) -> int:
        out = ctypes.create_string_buffer(self.cap)
        load().gref_add_ct(self.ctx, _h(a), _h(b), out, self.cap)
        return _int(out)

    # ---- bulk vector checkers: numpy (words [count, L] uint32, neg [count] uint8,
    # exp [count] int32) -- the reference's signed integers, as fphe_export_signed writes them
    def fold(self, src, terms, slots, acc, threads: int = 0):
        """acc[slots[k]] = Ciphertext::add(acc[slots[k]], src[terms[k]]) for k ascending (the
        reference's iupdate / intervals_sum / matmul loops).  src and acc are (words, neg, exp)
        triples; returns the new acc triple."""
        sw, sn, se = _vec(src)
        aw, an, ae = (x.copy() for x in _vec(acc))
        t = np.ascontiguousarray(terms, dtype=np.int64)
        s_ = np.ascontiguousarray(slots, dtype=np.int64)
        if t.shape != s_.shape or (t.size and (t.min() < 0 or t.max() >= len(sn) or s_.min() < 0
                                               or s_.max() >= len(an))):
            raise ValueError("gref_fold: bad term/slot indexes")
        rc = load().gref_fold(self.ctx, sw.shape[1], _p(sw), _p(sn), _p(se), _p(t), _p(s_), t.size, _p(aw), _p(an),
                              _p(ae), len(an), _threads(threads))
        if rc:
            raise RuntimeError(f"gref_fold rc={rc}")
        return aw, an, ae

    def mul(self, src, pt, threads: int = 0):
        """Ciphertext::mul element-wise; pt = (signed significand words [count, Lp], neg, exp)."""
        sw, sn, se = _vec(src)
        pw, pn, pe = _vec(pt)
        n = len(sn)
        ow, on, oe = np.zeros_like(sw), np.zeros(n, np.uint8), np.zeros(n, np.int32)
        rc = load().gref_mul(self.ctx, sw.shape[1], _p(sw), _p(sn), _p(se), pw.shape[1], _p(pw), _p(pn), _p(pe), n,
                             _p(ow), _p(on), _p(oe), _threads(threads))
        if rc:
            raise RuntimeError(f"gref_mul rc={rc}")
        return ow, on, oe

    def squeeze(self, src, pack_num: int, shift_bit: int):
        sw, sn, _ = _vec(src)
        n = len(sn)
        m = -(-n // pack_num)
        ow, on, oe = np.zeros((m, sw.shape[1]), np.uint32), np.zeros(m, np.uint8), np.zeros(m, np.int32)
        rc = load().gref_squeeze(self.ctx, sw.shape[1], _p(sw), _p(sn), n, pack_num, shift_bit, _p(ow), _p(on), _p(oe))
        if rc:
            raise RuntimeError(f"gref_squeeze rc={rc}")
        return ow, on, oe

    def cumsum(self, vec, chunk_sizes, step: int):
        w, ng, ex = (x.copy() for x in _vec(vec))
        ch = np.ascontiguousarray(chunk_sizes, dtype=np.int64)
        rc = load().gref_cumsum(self.ctx, w.shape[1], _p(w), _p(ng), _p(ex), len(ng), _p(ch), ch.size, step)
        if rc:
            raise RuntimeError(f"gref_cumsum rc={rc}")
        return w, ng, ex

    def bench(self, op: str, per_thread: int, threads: int = 1, seed: int = 1) -> float:
        """Wall seconds for threads x per_thread elements of op in {'encrypt', 'decrypt', 'add',
        'add_gap'} ('add_gap': ct-add with the Hetero-LR exponent-gap mix, see gmp_ref.c)."""
        code = {"encrypt": 0, "decrypt": 1, "add": 2, "add_gap": 3, "mul": 4, "iupdate": 5}[op]
        return load().gref_bench(self.ctx, code, per_thread, threads, seed)


def _vec(v):
    w, ng, ex = v
    return (np.ascontiguousarray(w, dtype=np.uint32), np.ascontiguousarray(ng, dtype=np.uint8),
            np.ascontiguousarray(ex, dtype=np.int32))


def _p(a):
    return ctypes.c_void_p(a.ctypes.data)


def _threads(k: int) -> int:
    """Worker threads: k, else the CPUs this process may use (the GPU box's cgroup quota is 16
    of a many-core host), at most 16."""
    if k > 0:
        return k
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            return max(1, min(16, int(q) // int(per)))
    except (OSError, ValueError):
        pass
    return max(1, min(16, len(os.sched_getaffinity(0))))


def to_vec(cs, exps, L: int):
    """Python signed ints + exps -> the (words, neg, exp) triple."""
    w = np.zeros((len(cs), L), np.uint32)
    for i, c in enumerate(cs):
        m = abs(int(c))
        w[i] = np.frombuffer(m.to_bytes(4 * L, "little"), dtype=np.uint32)
    return w, np.array([1 if c < 0 else 0 for c in cs], np.uint8), np.array(list(exps), np.int32)


def from_vec(v):
    """(words, neg, exp) -> (Python signed ints, exps)."""
    w, ng, ex = _vec(v)
    nb = 4 * w.shape[1]
    raw = w.tobytes()
    mags = [int.from_bytes(raw[i * nb:(i + 1) * nb], "little") for i in range(w.shape[0])]
    return [-m if s else m for m, s in zip(mags, ng.tolist())], ex.tolist()


def powm(b: int, e: int, m: int) -> int:
    cap = 2 * m.bit_length() // 4 + 16
    out = ctypes.create_string_buffer(cap)
    load().gref_powm(_h(b), _h(e), _h(m), out, cap)
    return _int(out)


def tdiv_r(a: int, m: int) -> int:
    cap = a.bit_length() // 4 + 16
    out = ctypes.create_string_buffer(cap)
    load().gref_tdiv_r(_h(a), _h(m), out, cap)
    return _int(out)


def _batch(args):
    """Pool worker (spawn-safe: imports nothing but this module): encrypt or decrypt a batch."""
    op, n, p, q, items = args
    key = GmpKey(n, p, q)
    if op == "encrypt":
        return [key.encrypt(m, r, r is not None) for m, r in items]
    return [key.decrypt(c) for c in items]


def parallel(op: str, n: int, p: int, q: int, items, procs: int = 16):
    """op over items in `procs` spawned worker processes (fresh interpreters: safe beside a
    GPU-initialised parent), order preserved.  op "encrypt": items are (m, r or None);
    "decrypt": items are signed ciphertexts."""
    import multiprocessing as mp
    items = list(items)
    if not items:
        return []
    k = max(1, -(-len(items) // procs))
    chunks = [items[i:i + k] for i in range(0, len(items), k)]
    with mp.get_context("spawn").Pool(min(procs, len(chunks))) as pool:
        parts = pool.map(_batch, [(op, n, p, q, c) for c in chunks])
    return [x for part in parts for x in part]
