"""ctypes wrapper of oracle/build/libgmpref.so -- TEST INFRASTRUCTURE ONLY.

Cross-checks the pure-Python restatement against libgmp (the library rug wraps) and times
the CPU baseline for bench.py (cpu_baseline.kind = "port").
"""
from __future__ import annotations

import ctypes
import os
import subprocess
from typing import Optional

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

    def bench(self, op: str, per_thread: int, threads: int = 1, seed: int = 1) -> float:
        """Wall seconds for threads x per_thread elements of op in {'encrypt', 'decrypt', 'add',
        'add_gap'} ('add_gap': ct-add with the Hetero-LR exponent-gap mix, see gmp_ref.c)."""
        code = {"encrypt": 0, "decrypt": 1, "add": 2, "add_gap": 3, "mul": 4, "iupdate": 5}[op]
        return load().gref_bench(self.ctx, code, per_thread, threads, seed)


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
