"""MI355X mirror of the reference's native surface ``fate_utils.paillier``.

Reference: rust/fate_utils/crates/fate_utils/src/paillier/paillier.rs (pyo3 classes
PK, SK, Coder, Ciphertext, CiphertextVector, PlaintextVector, Evaluator, keygen), backed
by rust/fate_utils/crates/fixedpoint_paillier/src/lib.rs.

Vectors live in GPU memory (HBM) in the tile-major SoA layout of include/fate_phe.h:
limb j of element e is word ((e//64)*L + j)*64 + e%64 of a torch int32 tensor shaped
[ntiles, L, 64].  Per-element sign (uint8) and exponent (int32) arrays are padded to
ntiles*64.  All arithmetic runs in libfatephe.so; there is no CPU compute path --
without a HIP device the constructors of device vectors raise.
"""
from __future__ import annotations

import contextlib
import ctypes
import itertools
import os
import threading
from typing import Dict, List, Optional, Sequence, Tuple

import numpy as np
import torch

from . import _lib
from ._keygen import keygen_primes

WAVE = 64
BASE = 16
MAX_INT_FRACTION = 2


class PanicException(BaseException):
    """Raised where the reference Rust code panics (pyo3 surfaces those as
    ``pyo3_runtime.PanicException``, a BaseException subclass)."""


def _ntiles(n: int) -> int:
    return (n + WAVE - 1) // WAVE


def _device(device=None) -> torch.device:
    if device is not None:
        d = torch.device(device)
        if d.type != "cuda":
            raise ValueError("fate_amd vectors live on a HIP device (torch 'cuda')")
        return d if d.index is not None else torch.device("cuda", torch.cuda.current_device())
    if not torch.cuda.is_available():
        raise RuntimeError("fate_amd requires a HIP device (torch.cuda.is_available() is False)")
    return torch.device("cuda", torch.cuda.current_device())


def _stream(device: torch.device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def _ptr(t: Optional[torch.Tensor]):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def _permute(C_in, s_in, e_in, L: int, idx: torch.Tensor, nspace: int, scatter: bool, C_out, s_out, e_out,
             dev) -> None:
    """fphe_permute: gather (out[i] = in[idx[i]]) or scatter (out[idx[i]] = in[i]) of
    tile-major element vectors on the device (include/fate_phe.h)."""
    idx = idx.to(device=dev, dtype=torch.int64).contiguous()
    n = idx.numel()
    if n == 0:
        return
    # shapes the kernel's addressing assumes (tile-major [nt, L, 64], flat sign/exp)
    side_in, side_out = (n, nspace) if scatter else (nspace, n)
    for t, elems in ((C_in, side_in), (C_out, side_out)):
        if t is not None and (not t.is_contiguous() or t.dim() != 3 or t.shape[1] != L or t.shape[2] != WAVE
                              or t.shape[0] * WAVE < elems):
            raise ValueError(f"fphe_permute: bad tile tensor {tuple(t.shape)} for {elems} elements of {L} words")
    for t, elems in ((s_in, side_in), (e_in, side_in), (s_out, side_out), (e_out, side_out)):
        if t is not None and (not t.is_contiguous() or t.numel() < elems):
            raise ValueError("fphe_permute: bad sign/exp tensor")
    with torch.cuda.device(dev):  # a context-less entry point: launches on the current device
        _lib.check(_lib.load().fphe_permute(_ptr(C_in), _ptr(s_in), _ptr(e_in), L, _ptr(idx), n, nspace,
                                            1 if scatter else 0, _ptr(C_out), _ptr(s_out), _ptr(e_out),
                                            ctypes.c_void_p(_stream(dev))), "fphe_permute")


def _index_array(indexes) -> np.ndarray:
    """Vec<usize> (a list, tuple, array or tensor of integers) as an int64 array; a negative
    index is pyo3's usize extraction error."""
    if isinstance(indexes, torch.Tensor):
        a = indexes.detach().cpu().numpy()
    else:
        a = np.asarray(indexes if isinstance(indexes, (list, tuple, np.ndarray)) else list(indexes))
    if a.size == 0:
        return np.zeros(0, dtype=np.int64)
    if a.dtype == np.bool_ or not np.issubdtype(a.dtype, np.integer):
        raise TypeError("indexes must be integers")
    a = a.astype(np.int64, copy=False).reshape(-1)
    if bool((a < 0).any()):
        raise OverflowError("can't convert negative int to unsigned")
    return a


def _check_indexes(idx: np.ndarray, n: int) -> None:
    """The reference indexes a Vec: the first index outside [0, n) panics (slice_indexes,
    fixedpoint_paillier/src/lib.rs:457-463)."""
    bad = np.flatnonzero(idx >= n)
    if bad.size:
        raise PanicException(f"index out of bounds: the len is {n} but the index is {int(idx[bad[0]])}")


def _cycle_walk(idx: np.ndarray, n: int) -> np.ndarray:
    """CiphertextVector::i_shuffle's swaps (lib.rs:473-490) replayed on positions by the host
    helper: perm[k] = the element that ends at k; the reference's first out-of-bounds access
    panics with its message."""
    idx = np.ascontiguousarray(idx, dtype=np.int64)
    perm = np.empty(n, dtype=np.int64)
    visited = np.empty(n, dtype=np.uint8)
    bad = np.zeros(2, dtype=np.int64)
    if _lib.load_py().fphe_cycle_walk(idx.ctypes.data, idx.size, n, perm.ctypes.data, visited.ctypes.data,
                                      bad.ctypes.data):
        raise PanicException(f"index out of bounds: the len is {int(bad[0])} but the index is {int(bad[1])}")
    return perm


# --------------------------------------------------------------------------------------
# host <-> tile-layout conversion (plumbing; not on the hot path)
# --------------------------------------------------------------------------------------
def ints_to_limbs(values: Sequence[int], limbs: int) -> np.ndarray:
    """Non-negative ints -> uint32 [count, limbs] little-endian."""
    nb = 4 * limbs
    buf = b"".join(int(v).to_bytes(nb, "little") for v in values)
    return np.frombuffer(buf, dtype=np.uint32).reshape(len(values), limbs) if values else \
        np.zeros((0, limbs), dtype=np.uint32)


def limbs_to_ints(arr: np.ndarray) -> List[int]:
    """uint32 [count, limbs] -> Python ints."""
    arr = np.ascontiguousarray(arr, dtype=np.uint32)
    raw = arr.tobytes()
    nb = arr.shape[1] * 4
    return [int.from_bytes(raw[i * nb:(i + 1) * nb], "little") for i in range(arr.shape[0])]


def rows_to_tiles(rows: np.ndarray) -> np.ndarray:
    """uint32 [count, L] -> uint32 [ntiles, L, 64] (zero padded)."""
    count, L = rows.shape
    nt = _ntiles(count)
    pad = np.zeros((nt * WAVE, L), dtype=np.uint32)
    pad[:count] = rows
    return np.ascontiguousarray(pad.reshape(nt, WAVE, L).transpose(0, 2, 1))


def tiles_to_rows(tiles: np.ndarray, count: int) -> np.ndarray:
    nt, L, _ = tiles.shape
    return np.ascontiguousarray(tiles.transpose(0, 2, 1).reshape(nt * WAVE, L)[:count])


def tiles_to_cols(t: torch.Tensor) -> torch.Tensor:
    """[nt, L, 64] -> [L, nt*64] (element-major view, materialised)."""
    nt, L, _ = t.shape
    return t.permute(1, 0, 2).reshape(L, nt * WAVE)


def cols_to_tiles(c: torch.Tensor) -> torch.Tensor:
    L, n = c.shape
    nt = _ntiles(n)
    if n != nt * WAVE:
        c = torch.cat([c, c.new_zeros((L, nt * WAVE - n))], dim=1)
    return c.reshape(L, nt, WAVE).permute(1, 0, 2).contiguous()


def gather_rows(t: torch.Tensor, idx: torch.Tensor) -> torch.Tensor:
    """Elements idx of a tile-major [nt, L, 64] tensor as rows [len(idx), L] (only the
    gathered elements move)."""
    return t[idx // WAVE, :, idx % WAVE]


def rows_to_tile_tensor(rows: torch.Tensor) -> torch.Tensor:
    """[n, L] rows -> tile-major [ceil(n/64), L, 64] (zero padded)."""
    n, L = rows.shape
    nt = _ntiles(n)
    if n != nt * WAVE:
        rows = torch.cat([rows, rows.new_zeros((nt * WAVE - n, L))], dim=0)
    return rows.reshape(nt, WAVE, L).permute(0, 2, 1).contiguous()


def _pad_flat(x: torch.Tensor, n: int) -> torch.Tensor:
    nt = _ntiles(n)
    if x.shape[0] == nt * WAVE:
        return x.contiguous()
    out = x.new_zeros(nt * WAVE)
    out[: x.shape[0]] = x
    return out


# --------------------------------------------------------------------------------------
# per-device key contexts
# --------------------------------------------------------------------------------------
MIN_KEY_BITS, MAX_KEY_BITS = 256, 4096


def supports(key_bits: int) -> bool:
    """Key sizes this backend runs: even, MIN_KEY_BITS..MAX_KEY_BITS.  The reference takes any
    even size (paillier/src/lib.rs:72-87); FATE's integration keeps its CPU path for the
    others."""
    return MIN_KEY_BITS <= key_bits <= MAX_KEY_BITS and key_bits % 2 == 0


class _KeyCtx:
    """Owns one fphe_ctx per HIP device for a key (public, or public+private)."""

    def __init__(self, n: int, p: Optional[int] = None, q: Optional[int] = None):
        self.n, self.p, self.q = n, p, q
        self.key_bits = n.bit_length()
        if not supports(self.key_bits):
            raise ValueError(f"unsupported key size {self.key_bits}: this backend runs even sizes "
                             f"{MIN_KEY_BITS}..{MAX_KEY_BITS} (larger keys stay on the CPU fate_utils path)")
        # geometry: the 1024-, 2048- or 4096-bit kernels, n zero-padded up to it
        self.L1 = 32 if self.key_bits <= 1024 else (64 if self.key_bits <= 2048 else 128)
        self.L2 = 2 * self.L1
        self._ctx: Dict[int, ctypes.c_void_p] = {}
        self._one: Dict[int, torch.Tensor] = {}
        self._lock = threading.Lock()
        self._closed = False
        self.rng_key = (ctypes.c_uint32 * 8)(*np.frombuffer(os.urandom(32), dtype=np.uint32).tolist())
        self._nonce = itertools.count(1)

    def next_nonce(self) -> int:
        return (os.getpid() << 40) ^ next(self._nonce)

    def mont_one(self, device: torch.device) -> torch.Tensor:
        """M(1) = R mod n^2, the stored words of the literal 1 (int32 [L2] on `device`):
        device vectors are Montgomery-resident (fphe_ctx_mont_one, include/fate_phe.h)."""
        idx = device.index
        t = self._one.get(idx)
        if t is None:
            w = (ctypes.c_uint32 * self.L2)()
            _lib.check(_lib.load().fphe_ctx_mont_one(self.ctx(device), w), "fphe_ctx_mont_one")
            t = self._one[idx] = torch.tensor(np.frombuffer(w, dtype=np.uint32).view(np.int32), device=device)
        return t

    def ctx(self, device: torch.device) -> ctypes.c_void_p:
        idx = device.index
        with self._lock:
            c = self._ctx.get(idx)
            if c is not None:
                return c
            lib = _lib.load()
            nw = (ctypes.c_uint32 * self.L1)(*ints_to_limbs([self.n], self.L1)[0].tolist())
            pw = qw = None
            if self.p is not None:
                lq = self.L1 // 2
                pw = (ctypes.c_uint32 * lq)(*ints_to_limbs([self.p], lq)[0].tolist())
                qw = (ctypes.c_uint32 * lq)(*ints_to_limbs([self.q], lq)[0].tolist())
            if self._closed:
                raise RuntimeError("key context used after its teardown (process exit): stop the threads "
                                   "that use fate_amd before the interpreter exits")
            out = ctypes.c_void_p()
            _lib.check(lib.fphe_ctx_create(idx, self.key_bits, nw, pw, qw, ctypes.byref(out)), "fphe_ctx_create")
            with _OPTIONS_LOCK:
                for opt, val in _PATH_OPTIONS.items():
                    _lib.check(lib.fphe_ctx_set_option(out, opt, val), "fphe_ctx_set_option")
            self._ctx[idx] = out
            global _TEARDOWN_REGISTERED
            if not _TEARDOWN_REGISTERED:
                import atexit
                atexit.register(_teardown_contexts)
                _TEARDOWN_REGISTERED = True
            return out

    def close(self) -> None:
        """Destroy this key's device contexts (device memory, side stream, events) after the
        work queued on their devices has finished.  Called for every key by the atexit hook
        :func:`_teardown_contexts`, while HIP and torch are still fully up.  Afterwards ctx()
        raises instead of creating a context.  A thread still inside a call at exit holds the
        raw context pointer: threads that use this backend (daemon threads included) must be
        stopped before the interpreter exits."""
        with self._lock:
            ctxs, self._ctx = self._ctx, {}
            self._one = {}
            self._closed = True  # ctx() refuses to create new contexts from now on
        for idx, c in ctxs.items():
            try:
                torch.cuda.synchronize(idx)
            except Exception:
                pass
            _lib.load().fphe_ctx_destroy(c)

    # No __del__: keys live in _KEYS for the life of the process, and device frees from a
    # finaliser would run at interpreter shutdown in no defined order against the HIP/torch
    # runtime's own teardown.  _teardown_contexts frees them first.


_KEYS: Dict[Tuple[int, Optional[int]], _KeyCtx] = {}
_KEYS_LOCK = threading.Lock()
_TEARDOWN_REGISTERED = False


def _teardown_contexts() -> None:
    """atexit hook, registered at the first context creation -- after torch's import, so it
    runs before torch's own exit hooks (atexit is LIFO) and long before the C++ static
    destructors of the HIP runtime (__cxa_finalize, after Py_Finalize): every device context
    is destroyed while the runtime is intact, and none is left for process teardown."""
    with _KEYS_LOCK:
        keys = list(_KEYS.values())
    for k in keys:
        try:
            k.close()
        except Exception:
            pass


# ---- path options (fphe_ctx_set_option) -----------------------------------------------------
# Which of two kernels with the same integer results runs a call: small calls take the
# one-element-per-wave latency kernels (wide_dev.h), larger ones the throughput kernels the
# bench times.  Options set here apply to every existing and future context of the process.
_OPTION_IDS = {
    "wide_decrypt_max": _lib.OPT_WIDE_DECRYPT_MAX,
    "wide_encrypt_max": _lib.OPT_WIDE_ENCRYPT_MAX,
    "wide_kh_encrypt_max": _lib.OPT_WIDE_KH_ENCRYPT_MAX,
    "kh_direct_z": _lib.OPT_KH_DIRECT_Z,
}
_PATH_OPTIONS: Dict[int, int] = {}
_OPTIONS_LOCK = threading.RLock()


_OPTION_ENV = {"wide_decrypt_max": ("FPHE_WIDE_DECRYPT_MAX", 4096),
               "wide_encrypt_max": ("FPHE_WIDE_ENCRYPT_MAX", 2048),
               "wide_kh_encrypt_max": ("FPHE_WIDE_KH_ENCRYPT_MAX", 4096),
               "kh_direct_z": ("FPHE_KH_DIRECT_Z", 1),
               "wide_squeeze_max": ("FPHE_WIDE_SQUEEZE_MAX", 4096)}


def _option_default(name: str) -> int:
    """A new context's value of `name` (fphe_ctx_create: the env variable, else the default)."""
    env, dflt = _OPTION_ENV[name]
    return int(os.environ.get(env, dflt))


def set_path_options(**options: Optional[int]) -> Dict[str, Optional[int]]:
    """Set path options on every context of the process, existing and future; None restores
    the default.  Returns the previous settings (None where the default applied), so
    ``set_path_options(**prev)`` undoes a call.  Names: ``wide_decrypt_max``,
    ``wide_encrypt_max``, ``wide_kh_encrypt_max`` (0 = never the latency kernel),
    ``kh_direct_z`` (0 = the key holder draws r, not (z_p, z_q)) and ``wide_squeeze_max``
    (``pack_squeeze`` chunks on the one-launch kernel)."""
    global WIDE_SQUEEZE_MAX_CHUNKS
    for name in options:
        if name not in _OPTION_ENV:
            raise ValueError(f"unknown path option {name!r}")
    prev: Dict[str, Optional[int]] = {}
    with _OPTIONS_LOCK:
        for name, val in options.items():
            if name == "wide_squeeze_max":
                prev[name] = None if WIDE_SQUEEZE_MAX_CHUNKS == _option_default(name) else WIDE_SQUEEZE_MAX_CHUNKS
                WIDE_SQUEEZE_MAX_CHUNKS = _option_default(name) if val is None else int(val)
                continue
            opt = _OPTION_IDS[name]
            prev[name] = _PATH_OPTIONS.get(opt)
            if val is None:
                _PATH_OPTIONS.pop(opt, None)
            else:
                _PATH_OPTIONS[opt] = int(val)
        with _KEYS_LOCK:
            keys = list(_KEYS.values())
        for k in keys:
            with k._lock:
                ctxs = list(k._ctx.values())
            for c in ctxs:
                for name, val in options.items():
                    if name in _OPTION_IDS:
                        v = _option_default(name) if val is None else int(val)
                        _lib.check(_lib.load().fphe_ctx_set_option(c, _OPTION_IDS[name], v), "fphe_ctx_set_option")
    return prev


@contextlib.contextmanager
def path_options(**options: Optional[int]):
    """``with path_options(...)``: :func:`set_path_options` for the block, undone after it."""
    prev = set_path_options(**options)
    try:
        yield
    finally:
        set_path_options(**prev)


# every latency path off: each call runs the throughput kernels the bench times
THROUGHPUT_PATHS = dict(wide_decrypt_max=0, wide_encrypt_max=0, wide_kh_encrypt_max=0, wide_squeeze_max=0)


def path_option(device: torch.device, key: "_KeyCtx", name: str) -> int:
    """The effective value of a path option on `key`'s context on `device`."""
    v = ctypes.c_int64()
    _lib.check(_lib.load().fphe_ctx_get_option(key.ctx(device), _OPTION_IDS[name], ctypes.byref(v)),
               "fphe_ctx_get_option")
    return v.value


def _key_for(n: int, p: Optional[int] = None, q: Optional[int] = None) -> _KeyCtx:
    """One device context per (key, public/private) per process, shared by PK/SK/Coder."""
    with _KEYS_LOCK:
        k = _KEYS.get((n, p))
        if k is None:
            k = _KEYS[(n, p)] = _KeyCtx(n, p, q)
        return k


# ---- pickling helpers -------------------------------------------------------------------
# The reference pickles every object as bincode bytes, returned by pyo3 as Vec<u8> (a list of
# ints) and read back from any sequence of ints.  The state here is `bytes` (accepted by the
# reference's __setstate__, which extracts Vec<u8> from any sequence; pickles 8x smaller than
# a list); FPHE_PICKLE_STATE=list gives the reference's exact list form.
#
# A reference ciphertext vector's state is key-less: signed integers (paillier.rs:219-226).
# Unpickled here it stays in that form ("raw": C holds the magnitudes, sign the negative
# flags) until an operation supplies the key -- every arithmetic op takes the PK, and decrypt
# the SK -- which converts it to (C mod n^2, sign) on the device.  Permutations (slice,
# shuffle, cat, ...) move raw elements as they are.  No key is ever guessed.
_UNPICKLED = threading.local()


def _pickle_state(b: bytes):
    return list(b) if os.environ.get("FPHE_PICKLE_STATE") == "list" else b


def _isqrt_exact(ns: int) -> Optional[int]:
    import math
    r = math.isqrt(ns)
    return r if r * r == ns else None


class unpickle_key:
    """``with unpickle_key(pk): pickle.loads(...)`` -- read ciphertext vector states under this
    key right away (their signed integers become (C mod n^2, sign) during the load).  Without
    it a vector is converted when the first operation hands it a key."""

    def __init__(self, pk: "PK"):
        self.n = pk.n

    def __enter__(self):
        self.prev = getattr(_UNPICKLED, "forced", None)
        _UNPICKLED.forced = self.n
        return self

    def __exit__(self, *exc):
        _UNPICKLED.forced = self.prev
        return False


def _resolve(v: "CiphertextVector", n: int) -> None:
    """Give a raw (unpickled, key-less) vector its key: the signed integers become (C mod n^2,
    sign) in place (fphe_import_signed); |value| >= n^2 raises ValueError as a corrupt state."""
    if not getattr(v, "raw", False):
        return
    key = _key_for(n)
    L2 = key.L2
    dev = v.device
    if v.lit:  # a zeros() vector: M(1) everywhere, no import (sign 0, exp 0 as made)
        v.C = key.mont_one(dev).view(1, -1, 1).expand(v.C.shape[0], L2, WAVE).contiguous()
        v.sign.zero_()
        v.n, v.raw, v.lit = n, False, False
        return
    from .wire import _check_below
    rows = tiles_to_cols(v.C).t()[: v.count]  # [count, Lw] element-major magnitudes
    if rows.shape[1] > L2:
        if bool((rows[:, L2:] != 0).any()):
            raise ValueError("CiphertextVector state: |value| >= n^2")
        rows = rows[:, :L2]
    elif rows.shape[1] < L2:
        rows = torch.cat([rows, rows.new_zeros((rows.shape[0], L2 - rows.shape[1]))], 1)
    rows = rows.contiguous()
    if v.count:
        _check_below(rows, n * n)
    cv = CiphertextVector.import_signed(PK(n), rows, v.sign[: v.count].contiguous(), v.exp[: v.count])
    v.C, v.sign, v.exp, v.n, v.raw = cv.C, cv.sign, cv.exp, n, False
    del dev


# Coder::encode_f64's exponent range (fixedpoint_paillier/src/lib.rs:148-168): floor((e - 53) / 4)
# for frexp exponents e in [-1073, 1024], and -14 for zero; float32 inputs are widened first
ENCODE_EXP_RANGE = (-282, 242)


def _ebound_union(a, b):
    """Exponent bounds (lo, hi) of vectors, joined; None (unknown) absorbs.  A host-side
    bound lets ct-add skip the read-back of the largest exponent gap when no gap can exceed
    the kernel's exact range (encoder-made vectors and what adds, folds, negations and
    permutations make of them); unpickled and crafted vectors carry None and are checked."""
    if a is None or b is None:
        return None
    return (min(a[0], b[0]), max(a[1], b[1]))


def _resolve_args(n: int, *objs) -> None:
    """Give every key-less vector among an operation's arguments its key.  Sequences are entered
    only when they hold vectors (cat's list, iadd_slice's ciphertexts): a histogram's position
    lists (Vec<Vec<usize>>) are never walked element by element."""
    for a in objs:
        if isinstance(a, CiphertextVector):
            _resolve(a, n)
        elif isinstance(a, Ciphertext):
            _resolve(a.vec, n)
        elif isinstance(a, (list, tuple)) and a and isinstance(a[0], (CiphertextVector, Ciphertext)):
            _resolve_args(n, *a)


def _fit_limbs(v: "CiphertextVector", L2: int) -> "CiphertextVector":
    """Zero-extend / truncate limb rows to the key's L2 (exact for values < n^2; used for
    ``zeros()`` vectors, which are created before the key is known)."""
    if v.L2 == L2:
        return v
    if v.L2 > L2:
        C = v.C[:, :L2, :].contiguous()
    else:
        C = torch.cat([v.C, v.C.new_zeros((v.C.shape[0], L2 - v.L2, WAVE))], dim=1)
    return CiphertextVector(C, v.sign, v.exp, v.count, v.n, v.raw)


_ERR_MESSAGES = [
    (_lib.EF_ENCODE_NONFINITE, "called `Option::unwrap()` on a `None` value"),
    (_lib.EF_DECODE_CORRUPTED, "Attempted to decode corrupted number"),
    (_lib.EF_DECODE_OVERFLOW, "Overflow detected in decrypted number"),
    (_lib.EF_MUL_INVALID_PT, "invalid plaintext"),
    (_lib.EF_NOT_INVERTIBLE, "called `Option::unwrap()` on a `None` value (non-invertible)"),
    (_lib.EF_DECODE_I128, "cant't convert to i128"),
]


def _raise_err(err: torch.Tensor) -> None:
    v = int(err.item())
    if v:
        for bit, msg in _ERR_MESSAGES:
            if v & bit:
                raise PanicException(msg)


# --------------------------------------------------------------------------------------
# vectors
# --------------------------------------------------------------------------------------
class PlaintextVector:
    """Encoded plaintexts (``fixedpoint_paillier::PlaintextVector``, lib.rs:364-367):
    significand magnitude limbs P [ntiles, lp, 64], negative flags, base-16 exponents."""

    # ebound: (lo, hi) a host-side bound on every exponent, or None (unknown); see _ebound
    __slots__ = ("P", "neg", "exp", "count", "ebound")

    def __init__(self, P: torch.Tensor = None, neg: torch.Tensor = None, exp: torch.Tensor = None, count: int = 0):
        self.P, self.neg, self.exp, self.count = P, neg, exp, count
        self.ebound = None

    @property
    def lp(self) -> int:
        return self.P.shape[1]

    @property
    def device(self) -> torch.device:
        return self.P.device

    def __len__(self) -> int:
        return self.count

    # host view -------------------------------------------------------------------
    def to_ints(self) -> Tuple[List[int], List[int]]:
        """(signed significands, exps) on the host."""
        rows = tiles_to_rows(self.P.cpu().numpy().view(np.uint32), self.count)
        mags = limbs_to_ints(rows)
        neg = self.neg[: self.count].cpu().numpy()
        sig = [-m if (g and m) else m for m, g in zip(mags, neg)]
        return sig, self.exp[: self.count].cpu().tolist()

    @staticmethod
    def from_ints(sig: Sequence[int], exp: Sequence[int], device=None, lp: Optional[int] = None) -> "PlaintextVector":
        dev = _device(device)
        count = len(sig)
        mags = [abs(int(s)) for s in sig]
        need = max([1] + [(m.bit_length() + 31) // 32 for m in mags])
        lp = max(lp or 0, need, 1)
        tiles = rows_to_tiles(ints_to_limbs(mags, lp))
        P = torch.from_numpy(tiles.view(np.int32)).to(dev)
        neg = _pad_flat(torch.tensor([1 if s < 0 else 0 for s in sig], dtype=torch.uint8), count).to(dev)
        ex = _pad_flat(torch.tensor(list(exp), dtype=torch.int32), count).to(dev)
        v = PlaintextVector(P, neg, ex, count)
        v.ebound = (min(exp), max(exp)) if count else (0, 0)
        return v

    def get_stride(self, index: int, stride: int) -> "PlaintextVector":
        """``PlaintextVector.get_stride`` (paillier.rs:406-408; lib.rs:912-917)."""
        return self._gather(torch.arange(index * stride, index * stride + stride, device=self.device))

    def tolist(self) -> List["Plaintext"]:
        return [Plaintext(self._gather(torch.tensor([i], device=self.device))) for i in range(self.count)]

    def _gather(self, idx: torch.Tensor) -> "PlaintextVector":
        n = int(idx.numel())
        nt = _ntiles(n)
        dev = self.device
        out = PlaintextVector(torch.zeros((nt, self.lp, WAVE), dtype=self.P.dtype, device=dev),
                              torch.zeros(nt * WAVE, dtype=self.neg.dtype, device=dev),
                              torch.zeros(nt * WAVE, dtype=self.exp.dtype, device=dev), n)
        out.ebound = self.ebound
        _permute(self.P, self.neg, self.exp, self.lp, idx, self.count, False, out.P, out.neg, out.exp, dev)
        return out

    def __str__(self):
        return f"PlaintextVector(len={self.count}, lp={self.lp})"

    # pickling: the reference's state, bincode(PlaintextVector) (paillier.rs:395-402)
    def __getstate__(self):
        from . import wire
        return _pickle_state(wire.plaintext_vector_to_bincode(self))

    def __setstate__(self, state):
        from . import wire
        v = wire.plaintext_vector_from_bincode(bytes(state))
        self.P, self.neg, self.exp, self.count = v.P, v.neg, v.exp, v.count
        self.ebound = v.ebound


class Plaintext:
    """Scalar plaintext (``fate_utils.paillier.Plaintext``): a length-1 vector."""

    __slots__ = ("vec",)

    def __init__(self, vec: PlaintextVector):
        self.vec = vec


class CiphertextVector:
    """Encrypted vector (``fixedpoint_paillier::CiphertextVector``, lib.rs:353-356):
    C [ntiles, L2, 64] the key's Montgomery-resident residues M(c) = c R mod n^2 of the
    canonical ciphertexts c, sign (reference integer = c - n^2), exp (base-16 exponent).
    Every product kernel works on M(.) directly (include/fate_phe.h)."""

    # n: the key's modulus (set by encrypt and by every op that takes a PK); M(.) is
    # meaningful under that key only, and pickling needs it to write the reference's signed
    # integers.  raw: a key-less vector -- unpickled, or zeros() -- not yet given its key (C =
    # magnitudes of the reference's signed integers, sign = negative flags; see _resolve)
    # lit: a raw vector still exactly as zeros() made it (every element the literal 1, exp 0):
    # its key is given by writing M(1), not by importing integers (_resolve)
    # ebound: (lo, hi) a host-side bound on every exponent, or None (unknown); see _ebound
    __slots__ = ("C", "sign", "exp", "count", "n", "raw", "lit", "ebound")

    def __init__(self, C: torch.Tensor = None, sign: torch.Tensor = None, exp: torch.Tensor = None, count: int = 0,
                 n: Optional[int] = None, raw: bool = False):
        self.C, self.sign, self.exp, self.count, self.n, self.raw = C, sign, exp, count, n, raw
        self.lit = False
        self.ebound = None

    # ---- construction / host views -----------------------------------------------
    @property
    def device(self) -> torch.device:
        return self.C.device

    @property
    def L2(self) -> int:
        return self.C.shape[1]

    def __len__(self) -> int:
        return self.count

    def __str__(self) -> str:
        return f"CiphertextVector(len={self.count}, limbs={self.L2})"

    __repr__ = __str__

    @staticmethod
    def empty(count: int, L2: int, device) -> "CiphertextVector":
        nt = _ntiles(count)
        return CiphertextVector(torch.empty((nt, L2, WAVE), dtype=torch.int32, device=device),
                                torch.zeros(nt * WAVE, dtype=torch.uint8, device=device),
                                torch.zeros(nt * WAVE, dtype=torch.int32, device=device), count)

    @staticmethod
    def zeros(size: int, L2: int = 128, device=None) -> "CiphertextVector":
        """``CiphertextVector::zeros`` (lib.rs:434-437): literal 1 with exp 0 (:244-249).  As in
        the reference it knows no key: a key-less (raw) vector of the integer 1, which the first
        operation that supplies a key turns into M(1) (:func:`_resolve`)."""
        dev = _device(device)
        v = CiphertextVector.empty(size, L2, dev)
        v.C.zero_()
        v.C[:, 0, :] = 1
        v.raw = True
        v.lit = True
        v.ebound = (0, 0)
        return v

    def to_signed_ints(self, ns: Optional[int] = None) -> Tuple[List[int], List[int]]:
        """Reference (signed rug::Integer, exp) pairs, for parity checks and the wire (ns may
        be omitted for a raw vector, or one whose signs are all 0)."""
        if not self.raw:
            n = self.n if self.n is not None else (_isqrt_exact(ns) if ns is not None else None)
            if n is None:
                raise TypeError("to_signed_ints: a keyed vector without its key")
            mag, neg, exp = self.export_signed(PK(n))
            mags = limbs_to_ints(mag.cpu().numpy().view(np.uint32))
            sg = neg.cpu().numpy()
            return [-m if s else m for m, s in zip(mags, sg)], exp.cpu().tolist()
        rows = tiles_to_rows(self.C.cpu().numpy().view(np.uint32), self.count)
        mags = limbs_to_ints(rows)
        sg = self.sign[: self.count].cpu().numpy()
        return [-m if s else m for m, s in zip(mags, sg)], self.exp[: self.count].cpu().tolist()

    @staticmethod
    def from_signed_ints(cs: Sequence[int], exps: Sequence[int], ns: int, L2: int, device=None) -> "CiphertextVector":
        """The reference's signed integers (|c| < n^2) under the key of modulus^2 ns, on the
        device in the Montgomery-resident form (fphe_import_signed)."""
        dev = _device(device)
        count = len(cs)
        tiles = rows_to_tiles(ints_to_limbs([abs(c) for c in cs], L2))
        C = torch.from_numpy(tiles.view(np.int32)).to(dev)
        sign = _pad_flat(torch.tensor([1 if c < 0 else 0 for c in cs], dtype=torch.uint8), count).to(dev)
        ex = _pad_flat(torch.tensor(list(exps), dtype=torch.int32), count).to(dev)
        v = CiphertextVector(C, sign, ex, count, None, raw=True)
        n = _isqrt_exact(ns)
        if n is None:
            raise ValueError("from_signed_ints: ns is not the square of a modulus")
        _resolve(v, n)
        return v

    def export_signed(self, pk: "PK") -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        """The reference's signed integers on the device (fphe_export_signed): magnitudes as
        element-major LSF uint32 words [count, L2], negative flags [count], exponents."""
        dev = self.device
        _resolve(self, pk.n)
        v = _fit_limbs(self, pk._key.L2)
        mag = torch.empty((self.count, v.L2), dtype=torch.int32, device=dev)
        neg = torch.empty(self.count, dtype=torch.uint8, device=dev)
        _lib.check(_lib.load().fphe_export_signed(pk._key.ctx(dev), _ptr(v.C), _ptr(v.sign), self.count, _ptr(mag),
                                                  _ptr(neg), ctypes.c_void_p(_stream(dev))), "fphe_export_signed")
        return mag, neg, self.exp[: self.count].clone()

    @staticmethod
    def import_signed(pk: "PK", mag: torch.Tensor, neg: torch.Tensor, exp: torch.Tensor) -> "CiphertextVector":
        """Inverse of :meth:`export_signed` (fphe_import_signed); |value| < n^2."""
        dev = mag.device
        n = int(mag.shape[0])
        if mag.dim() != 2 or mag.shape[1] != pk._key.L2 or neg.numel() != n or exp.numel() != n:
            raise ValueError("import_signed: magnitudes [count, L2], flags and exponents [count]")
        out = CiphertextVector.empty(n, pk._key.L2, dev)
        mag, neg = mag.contiguous(), neg.contiguous()  # held across the launch
        _lib.check(_lib.load().fphe_import_signed(pk._key.ctx(dev), _ptr(mag), _ptr(neg), n,
                                                  _ptr(out.C), _ptr(out.sign), ctypes.c_void_p(_stream(dev))),
                   "fphe_import_signed")
        out.exp[:n] = exp.to(dev, torch.int32)
        out.n = pk.n
        return out

    # ---- pickling: the reference's state, bincode(CiphertextVector) (paillier.rs:219-226) --
    def signed_rows(self) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        """The reference's signed integers as (element-major magnitudes [count, L2], negative
        flags, exps) on the device, from the key this vector carries (a raw vector needs none)."""
        if self.raw:
            mag = tiles_to_cols(self.C).t()[: self.count].contiguous()
            return mag, self.sign[: self.count].contiguous(), self.exp[: self.count].clone()
        if self.n is None:
            raise TypeError("CiphertextVector: a keyed vector without its key; build it through a PK operation "
                            "before pickling")
        return self.export_signed(PK(self.n))

    def __getstate__(self):
        from . import wire
        return _pickle_state(wire.ciphertext_vector_to_bincode(self))

    def __setstate__(self, state):
        from . import wire
        buf = bytes(state)
        forced = getattr(_UNPICKLED, "forced", None)
        v, used = wire.ciphertext_vector_from_bincode(buf, PK(forced) if forced is not None else None)
        if used != len(buf):
            raise ValueError("bincode CiphertextVector: trailing bytes")
        self.C, self.sign, self.exp, self.count, self.n, self.raw = v.C, v.sign, v.exp, v.count, v.n, v.raw
        self.lit = False
        self.ebound = None  # crafted or foreign exponents: every add checks its gaps

    def __copy__(self) -> "CiphertextVector":
        """A device-side clone (the key and raw state travel; no wire round trip)."""
        v = CiphertextVector(self.C.clone(), self.sign.clone(), self.exp.clone(), self.count, self.n, self.raw)
        v.ebound = self.ebound
        return v

    def __deepcopy__(self, memo) -> "CiphertextVector":
        return self.__copy__()

    # ---- element plumbing (torch indexing; no arithmetic) ---------------------------
    def _gather(self, idx: torch.Tensor) -> "CiphertextVector":
        n = int(idx.numel())
        nt = _ntiles(n)
        dev = self.device
        out = CiphertextVector(torch.zeros((nt, self.L2, WAVE), dtype=torch.int32, device=dev),
                               torch.zeros(nt * WAVE, dtype=torch.uint8, device=dev),
                               torch.zeros(nt * WAVE, dtype=torch.int32, device=dev), n, self.n, self.raw)
        out.ebound = self.ebound
        _permute(self.C, self.sign, self.exp, self.L2, idx, self.count, False, out.C, out.sign, out.exp, dev)
        return out

    def _assign(self, idx: torch.Tensor, src: "CiphertextVector") -> None:
        """self[idx[i]] = src[i] (in place; only the assigned elements move)."""
        idx = idx.to(self.device, torch.long)
        if idx.numel() == 0:
            return
        if src.raw != self.raw:
            if self.n is not None:
                _resolve(src, self.n)
            elif src.n is not None:
                _resolve(self, src.n)
            else:
                raise TypeError("assigning between an unpickled (key-less) vector and a keyed one without a key")
        self.lit = False
        self.ebound = _ebound_union(self.ebound, src.ebound)
        if self.L2 != src.L2:
            # a zeros() vector is sized before the key is known (evaluator.zeros(size, dtype),
            # protocol/phe/paillier.py:347-349): adopt the key's limb count, exactly
            self.C = _fit_limbs(self, src.L2).C
        _permute(src.C, src.sign, src.exp, self.L2, idx, self.count, True, self.C, self.sign, self.exp, self.device)

    def slice(self, start: int, size: int) -> "CiphertextVector":
        """``CiphertextVector::slice`` (lib.rs:452-455)."""
        if start + size > self.count:
            raise PanicException(f"range end index {start + size} out of range for slice of length {self.count}")
        return self._gather(torch.arange(start, start + size))

    def slice_indexes(self, indexes: Sequence[int]) -> "CiphertextVector":
        """``CiphertextVector::slice_indexes`` (lib.rs:457-463)."""
        idx = _index_array(indexes)
        _check_indexes(idx, self.count)
        return self._gather(torch.from_numpy(idx))

    def cat(self, others: Sequence["CiphertextVector"]) -> "CiphertextVector":
        """``CiphertextVector::cat`` (lib.rs:465-471)."""
        return Evaluator.cat([self, *others])

    def shuffle(self, indexes: Sequence[int]) -> "CiphertextVector":
        """``CiphertextVector::shuffle`` (lib.rs:492-497): result[i] = data[indexes[i]] for a
        permutation, realised as a gather (same result as the reference's cycle walk)."""
        out = CiphertextVector(self.C.clone(), self.sign.clone(), self.exp.clone(), self.count, self.n, self.raw)
        out.i_shuffle(indexes)
        return out

    def i_shuffle(self, indexes: Sequence[int]) -> None:
        """``CiphertextVector::i_shuffle`` (lib.rs:473-490).  The reference's cycle walk, swap
        for swap, runs on positions (:func:`_cycle_walk`), then one gather moves the
        ciphertexts: new[i] = old[indexes[i]] for a permutation, and the reference's own result
        (or index panic) for any other list."""
        perm = _cycle_walk(_index_array(indexes), self.count)
        g = self._gather(torch.from_numpy(perm))
        self.C, self.sign, self.exp = g.C, g.sign, g.exp
        self.lit = False

    def intervals_slice(self, intervals: Sequence[Tuple[int, int]]) -> "CiphertextVector":
        """``CiphertextVector::intervals_slice`` (lib.rs:499-513): the intervals' elements, in
        order.  The first interval that fails decides the error, as the reference's loop: an end
        past the data is its anyhow error (RuntimeError), a start past the end the slice panic."""
        s, e = _interval_array(intervals)
        n = self.count
        bad = torch.nonzero((e > n) | (s > e)).squeeze(1)
        if bad.numel():
            i = int(bad[0])
            si, ei = int(s[i]), int(e[i])
            if ei > n:
                raise RuntimeError(f"end index out of range: start={si}, end={ei}, data_size={n}")
            raise PanicException(f"slice index starts at {si} but ends at {ei}")
        idx, _ = _interval_items(s, e)
        return self._gather(idx)

    def tolist(self) -> List["CiphertextVector"]:
        return [self._gather(torch.tensor([i])) for i in range(self.count)]

    # ---- arithmetic (device kernels) ----------------------------------------------
    def add(self, pk: "PK", other: "CiphertextVector") -> "CiphertextVector":
        """``CiphertextVector::add`` (lib.rs:797-805)."""
        return _add(pk, self, other, broadcast=False)

    def add_scalar(self, pk: "PK", other: "Ciphertext") -> "CiphertextVector":
        """``CiphertextVector::add_scalar`` (lib.rs:807-810)."""
        return _add(pk, self, other.vec, broadcast=True)

    def iadd(self, pk: "PK", other: "CiphertextVector") -> None:
        """``CiphertextVector::iadd`` (lib.rs:748-752)."""
        r = _add(pk, self, other, broadcast=False, count=min(self.count, other.count))
        self._overwrite_prefix(r)

    def idouble(self, pk: "PK") -> None:
        """``CiphertextVector::idouble`` (lib.rs:753-758): x.add(x)."""
        r = _add(pk, self, self, broadcast=False)
        self.C, self.sign, self.exp = r.C, r.sign, r.exp

    def iadd_vec(self, other: "CiphertextVector", sa: int, sb: int, size: Optional[int], pk: "PK") -> None:
        """``CiphertextVector::iadd_vec`` (lib.rs:634-677)."""
        if size is None:  # self.data[sa..] zipped with other.data[sb..]: either start may panic
            if sa > self.count:
                raise PanicException(f"range start index {sa} out of range for slice of length {self.count}")
            if sb > other.count:
                raise PanicException(f"range start index {sb} out of range for slice of length {other.count}")
            size = min(self.count - sa, other.count - sb)
        else:
            if sa + size > self.count:
                raise RuntimeError(f"end index out of range: sa={sa}, ea={sa + size}, data_size={self.count}")
            if sb + size > other.count:
                raise RuntimeError(f"end index out of range: sb={sb}, eb={sb + size}, data_size={other.count}")
        if size <= 0:
            return
        a = self.slice(sa, size)
        b = other.slice(sb, size)
        self._assign(torch.arange(sa, sa + size), _add(pk, a, b, broadcast=False))

    def neg(self, pk: "PK") -> "CiphertextVector":
        """Element-wise ``Ciphertext::neg`` (lib.rs:259-264): (invert(c, n^2), exp)."""
        return _neg(pk, self)

    def sub(self, pk: "PK", other: "CiphertextVector") -> "CiphertextVector":
        """``CiphertextVector::sub`` (lib.rs:812-820): x.add(y.neg())."""
        return _add(pk, self, _neg(pk, other), broadcast=False)

    def sub_scalar(self, pk: "PK", other: "Ciphertext") -> "CiphertextVector":
        """``CiphertextVector::sub_scalar`` (lib.rs:822-825)."""
        return _add(pk, self, _neg(pk, other.vec), broadcast=True)

    def rsub(self, pk: "PK", other: "CiphertextVector") -> "CiphertextVector":
        """``CiphertextVector::rsub`` (lib.rs:827-835): y.sub(x) = y.add(x.neg())."""
        n = min(self.count, other.count)
        return _add(pk, other, _neg(pk, self, count=n), broadcast=False, count=n)

    def rsub_scalar(self, pk: "PK", other: "Ciphertext") -> "CiphertextVector":
        """``CiphertextVector::rsub_scalar`` (lib.rs:837-840): other.sub(x) = other.add(x.neg())."""
        neg = _neg(pk, self)
        return _add(pk, neg, other.vec, broadcast=True)

    def isub(self, pk: "PK", other: "CiphertextVector") -> None:
        """In-place sub (x.sub_assign(y) over zip, lib.rs:289-292)."""
        r = self.sub(pk, other)
        self._overwrite_prefix(r)

    def isub_vec(self, other: "CiphertextVector", sa: int, sb: int, size: Optional[int], pk: "PK") -> None:
        """``CiphertextVector::isub_vec`` (lib.rs:679-722)."""
        if size is None:  # self.data[sa..] zipped with other.data[sb..]: either start may panic
            if sa > self.count:
                raise PanicException(f"range start index {sa} out of range for slice of length {self.count}")
            if sb > other.count:
                raise PanicException(f"range start index {sb} out of range for slice of length {other.count}")
            size = min(self.count - sa, other.count - sb)
        else:
            if sa + size > self.count:
                raise RuntimeError(f"end index out of range: sa={sa}, ea={sa + size}, data_size={self.count}")
            if sb + size > other.count:
                raise RuntimeError(f"end index out of range: sb={sb}, eb={sb + size}, data_size={other.count}")
        if size <= 0:
            return
        a = self.slice(sa, size)
        b = other.slice(sb, size)
        self._assign(torch.arange(sa, sa + size), a.sub(pk, b))

    def mul(self, pk: "PK", other: PlaintextVector) -> "CiphertextVector":
        """``CiphertextVector::mul`` (lib.rs:842-850)."""
        return _mul(pk, self, other, broadcast=False)

    def mul_scalar(self, pk: "PK", other: Plaintext) -> "CiphertextVector":
        """``CiphertextVector::mul_scalar`` (lib.rs:852-859)."""
        return _mul(pk, self, other.vec, broadcast=True)

    # ---- SecureBoost / Hetero-LR vector ops (fixedpoint_paillier/src/lib.rs:417-909) -----
    # Folds and scans are trees of the device ct-add kernel.  Ciphertext addition is
    # associative and commutative bit for bit (tests/test_oracle.py),
    # so a tree gives the reference's sequential result.
    def iadd_slice(self, pk: "PK", position: int, other: Sequence["Ciphertext"]) -> None:
        """``CiphertextVector::iadd_slice`` (lib.rs:509-513)."""
        if not other:
            return
        o = Evaluator.cat([c.vec for c in other])
        idx = torch.arange(position, position + o.count)
        self._assign(idx, _add(pk, self._gather(idx), o, broadcast=False))

    def iadd_vec_self(self, sa: int, sb: int, size: Optional[int], pk: "PK") -> None:
        """``CiphertextVector::iadd_vec_self`` (lib.rs:521-568), including its in-place
        cascade when the two ranges overlap (iadd_i_j, :417-424)."""
        self._self_op(sa, sb, size, pk, sub=False)

    def isub_vec_self(self, sa: int, sb: int, size: Optional[int], pk: "PK") -> None:
        """``CiphertextVector::isub_vec_self`` (lib.rs:569-632)."""
        self._self_op(sa, sb, size, pk, sub=True)

    def _self_op(self, sa: int, sb: int, size: Optional[int], pk: "PK", sub: bool) -> None:
        n = self.count
        if sa == sb:
            if size is not None and sa + size > n:
                raise RuntimeError(f"end index out of range: sa={sa}, s={size}, data_size={n}")
            if size is None and sa > n:  # self.data[sa..]
                raise PanicException(f"range start index {sa} out of range for slice of length {n}")
            end = n if size is None else sa + size
            if end <= sa:
                return
            idx = torch.arange(sa, end)
            if sub:  # x - x -> Ciphertext::zero() (lib.rs:578-588)
                z = CiphertextVector.zeros(end - sa, self.L2, self.device)
                self._assign(idx, z)
            else:  # i_double: powm(c, 2) (lib.rs:294-299), = add(x, x)
                x = self._gather(idx)
                self._assign(idx, _add(pk, x, x, broadcast=False))
            return
        w0, r0 = max(sa, sb), min(sa, sb)
        if size is not None and w0 + size > n:
            nm = "sb" if sa < sb else "sa"
            raise RuntimeError(f"end index out of range: {nm}={w0}, s={size}, data_size={n}")
        if size is None and w0 > n:  # iadd_i_j(w0, r0, len - w0): the first data[w0] is out of bounds
            raise PanicException(f"index out of bounds: the len is {n} but the index is {w0}")
        s = (n - w0) if size is None else size
        d = w0 - r0
        # data[w0+k] op= data[r0+k] for k ascending; reads of r0+k >= w0 see earlier writes:
        # process k in rounds of d so every round reads only finished values.
        for start in range(0, s, d):
            k = torch.arange(start, min(start + d, s))
            x, y = self._gather(w0 + k), self._gather(r0 + k)
            self._assign(w0 + k, x.sub(pk, y) if sub else _add(pk, x, y, broadcast=False))

    def iupdate(self, other: "CiphertextVector", indexes, stride: int, pk: "PK") -> None:
        """``CiphertextVector::iupdate`` (lib.rs:724-735): data[pos*stride+t] += other[i*stride+t]
        for every position pos listed for sample i, folded per target slot on the device."""
        if isinstance(indexes, np.ndarray) and indexes.ndim == 2:
            indexes = torch.from_numpy(indexes)
        elif not isinstance(indexes, torch.Tensor):
            # the reference's Vec<Vec<usize>> (SecureBoost: one list per sample), read once by the
            # host helper; every sample listing the same number of positions -- one per feature,
            # the usual histogram -- makes it the [samples, positions] matrix of the tensor path
            lens, pos = _position_lists(indexes)
            if lens.size and lens[0] > 0 and bool((lens == lens[0]).all()):
                indexes = torch.from_numpy(pos).view(lens.size, int(lens[0]))
            else:
                ii = torch.from_numpy(np.repeat(np.arange(lens.size, dtype=np.int64), lens))
                self._scatter_fold(other, ii.to(self.device), torch.from_numpy(pos).to(self.device), stride, pk)
                return
        if (isinstance(indexes, torch.Tensor) and indexes.dim() == 2 and indexes.numel()
                and not indexes.is_floating_point() and not indexes.is_complex() and indexes.dtype != torch.bool):
            # [samples, positions] integer tensor (SecureBoost's bin indexes): the term lists
            # straight from it, in the reference's sample-major order, in four launches
            # (sample i's ids are implied: only the positions need a range check)
            ns, npos = indexes.shape
            st = max(int(stride), 1)
            if ns * st > other.count:
                raise PanicException("index out of bounds")
            pp = indexes.to(device=self.device)
            if pp.dtype not in (torch.int32, torch.int64):
                pp = pp.to(torch.int64)
            pp = pp.contiguous()
            src = torch.empty(ns * npos * st, dtype=torch.int32, device=self.device)
            slot = torch.empty_like(src)
            # one launch, no read-back: a position out of [0, count / stride) becomes slot -1,
            # which the fold reports (FPHE_ERR_ARG -> the reference's index panic)
            with torch.cuda.device(self.device):  # context-less: launches on the current device
                _lib.check(_lib.load().fphe_positions_terms(_ptr(pp), int(pp.dtype == torch.int64), ns, npos, st,
                                                            self.count, _ptr(src), _ptr(slot),
                                                            ctypes.c_void_p(_stream(self.device))),
                           "fphe_positions_terms")
            self._fold_terms(other, src, slot, pk)
            return
        ii, pp = _flatten_positions(indexes, self.device)
        self._scatter_fold(other, ii, pp, stride, pk)

    def iupdate_with_masks(self, other: "CiphertextVector", indexes, masks, stride: int, pk: "PK") -> None:
        """``CiphertextVector::iupdate_with_masks`` (lib.rs:736-747): the k-th position list
        belongs to the k-th sample whose mask is true."""
        if isinstance(masks, torch.Tensor):
            m = masks.to(torch.bool)
        elif isinstance(masks, np.ndarray):
            m = torch.from_numpy(masks.astype(bool, copy=False).reshape(-1))
        else:  # Vec<bool>: a Python list, read in C by numpy (3x a tensor from the list)
            m = torch.from_numpy(np.fromiter(masks, dtype=bool))
        vpos = torch.nonzero(m.to(self.device)).squeeze(1).to(torch.int32)
        ii, pp = _flatten_positions(indexes, self.device)
        if ii.numel():
            if int(ii.max()) >= vpos.numel():  # more position lists than true masks: the reference's zip stops
                keep = ii < vpos.numel()
                ii, pp = ii[keep], pp[keep]
            ii = vpos[ii.long()]
        self._scatter_fold(other, ii, pp, stride, pk)

    def _scatter_fold(self, other: "CiphertextVector", ii: torch.Tensor, pp: torch.Tensor, stride: int,
                      pk: "PK") -> None:
        """data[pp*stride+t] += other[ii*stride+t] for all listed pairs, in the reference's
        order (sample-major).  The terms are folded per slot straight out of ``other``
        (fphe_fold reads them by index), then added to the slot's current value:
        fold(data[s], t_1, ..., t_k) = add(data[s], fold(t_1, ..., t_k)), literal-1 rule
        included."""
        if ii.numel() == 0:
            return
        dev = self.device
        stride = max(int(stride), 1)
        # positions are usize in the reference: out of [0, len / stride) it panics on the index
        # (lib.rs:724-735).  Checked in 64 bits before any narrowing, so a huge position cannot
        # wrap onto a valid slot; the samples likewise against `other`
        lo, hi = torch.aminmax(pp.to(torch.int64))
        lo, hi, imax = torch.stack([lo, hi, ii.max().to(torch.int64)]).tolist()  # one read-back
        if lo < 0 or (hi + 1) * stride > self.count or (imax + 1) * stride > other.count:
            raise PanicException("index out of bounds")
        # int32 index arithmetic (fphe_fold_segments takes int32 indexes): half the bytes of the
        # int64 expansion on 8M-term histograms; every value is now < 2^31
        ii, pp = ii.to(dev, torch.int32), pp.to(dev, torch.int32)
        t = torch.arange(stride, device=dev, dtype=torch.int32)
        src = (ii[:, None] * stride + t).reshape(-1)
        slot = (pp[:, None] * stride + t).reshape(-1)
        self._fold_terms(other, src, slot, pk)

    def _fold_terms(self, other: "CiphertextVector", src: torch.Tensor, slot: torch.Tensor, pk: "PK") -> None:
        """data[slot[k]] += other[src[k]] for every term k (int32, range-checked by the caller),
        folded per slot in term order."""
        # one ciphertext per slot (the literal 1 where no term lands: add's identity), then
        # data[s] = add(data[s], fold(terms of s)) for every slot at once
        # the error flags of the fold and of the add are read back once both are queued: no
        # host sync between the launches
        ferr, aerr = [], []
        folded, present = _fold_to_segments(pk, other, slot, self.count, index=src, with_present=True, deferred=ferr)
        if getattr(_FRESH_ONES, "v", None) is self:
            # a zeros() vector, the literal 1 in every slot (the operation was entered with it:
            # _keyed, which leaves it key-less): add(1, x) = x (the literal-1 rule,
            # lib.rs:301-308, exponent and sign included), so the folded slots replace it and no
            # ct-add runs -- SecureBoost's histograms start as zeros()
            if not _fold_failed(ferr):
                # fphe_fold_segments already wrote the literal 1 (M(1), sign 0, exp 0) into every
                # segment no term reaches -- what the vector holds there -- so the fold is the
                # result, and the vector takes the key with it (no M(1) fill first)
                self.C, self.sign, self.exp = folded.C, folded.sign, folded.exp
                self.n, self.raw, self.lit = pk.n, False, False
                self.ebound = _ebound_union(self.ebound, other.ebound)
                return
            # an exponent gap beyond the device merge: the exact torch path
            _resolve(self, pk.n)
            cur = _fit_limbs(self, pk._key.L2)
            folded, present = _fold_dense(pk, other, slot, self.count, src)
            r = folded
        else:
            cur = _fit_limbs(self, pk._key.L2)
            r = _add(pk, cur, folded, broadcast=False, deferred=aerr)
            if _fold_failed(ferr):  # an exponent gap beyond the device merge: the exact torch path
                folded, present = _fold_dense(pk, other, slot, self.count, src)
                r = _add(pk, cur, folded, broadcast=False)
            elif _fold_failed(aerr):  # a gap beyond k_add27's range: pre-aligned, exact
                r = _add(pk, cur, folded, broadcast=False)
        # slots no term reaches keep their value as it was (exponent of a literal 1 included:
        # the reference never touches them)
        keep = present[: r.sign.numel()] == 0
        r.C = torch.where(keep.view(-1, 1, WAVE), cur.C, r.C)
        r.sign = torch.where(keep, cur.sign, r.sign)
        r.exp = torch.where(keep, cur.exp, r.exp)
        self.C, self.sign, self.exp = r.C, r.sign, r.exp
        self.ebound = _ebound_union(cur.ebound, other.ebound)

    def chunking_cumsum_with_step(self, pk: "PK", chunk_sizes: Sequence[int], step: int) -> None:
        """``CiphertextVector::chunking_cumsum_with_step`` (lib.rs:760-771): within each chunk,
        data[i+j] += data[i+j-step] for j ascending -- an inclusive scan with stride `step`,
        run as a Hillis-Steele scan (log2(chunk/step) rounds of the ct-add kernel)."""
        sizes = [int(c) for c in chunk_sizes]
        step = int(step)
        n = self.count
        # the reference touches data[i + j] for j in step..size: a chunk no longer than the step
        # touches nothing (even past the data), a longer one panics at its first index >= len
        i = 0
        for c in sizes:
            if c > step and i + c > n:
                raise PanicException(f"index out of bounds: the len is {n} but the index is {max(n, i + step)}")
            i += c
        total = sum(sizes)
        if total == 0 or step <= 0:  # step 0: each element adds the literal 1, i.e. stays
            return
        starts = torch.repeat_interleave(torch.tensor([0] + list(itertools.accumulate(sizes))[:-1]),
                                         torch.tensor(sizes))
        rel = torch.arange(total) - starts
        shift = step
        while shift < max(sizes):
            idx = torch.nonzero(rel >= shift).squeeze(1)
            if idx.numel() == 0:
                break
            x, y = self._gather(idx), self._gather(idx - shift)
            self._assign(idx, _add(pk, x, y, broadcast=False))
            shift *= 2

    def intervals_sum_with_step(self, pk: "PK", intervals: Sequence[Tuple[int, int]], step: int
                                ) -> "CiphertextVector":
        """``CiphertextVector::intervals_sum_with_step`` (lib.rs:773-788): out[i*step + c] =
        fold of data[s+k] over k = c (mod step), s+k < e, from zero."""
        s, e = _interval_array(intervals)
        n = self.count
        bad = torch.nonzero((e > n) | (s > e)).squeeze(1)
        if bad.numel():  # &self.data[s..e] of the first failing interval (lib.rs:781)
            i = int(bad[0])
            si, ei = int(s[i]), int(e[i])
            if si > ei:
                raise PanicException(f"slice index starts at {si} but ends at {ei}")
            raise PanicException(f"range end index {ei} out of range for slice of length {n}")
        step = int(step)
        nout = s.numel() * step
        idx, rel = _interval_items(s, e)
        if idx.numel() == 0 or step == 0:  # step 0: empty chunks, (0..0).cycle() adds nothing
            return CiphertextVector.zeros(nout, self.L2, self.device)
        seg = torch.repeat_interleave(torch.arange(s.numel(), dtype=torch.int64) * step, e - s) + rel % step
        return _fold_to_segments(pk, self, seg, nout, index=idx)

    def pack_squeeze(self, pack_num: int, offset_bit: int, pk: "PK") -> "CiphertextVector":
        """``CiphertextVector::pack_squeeze`` (paillier.rs:241; lib.rs:439-450): per chunk of
        pack_num, acc = x0; acc = acc^(2^offset_bit) * y mod n^2 for each further y; exp 0."""
        n = self.count
        if pack_num == 0:  # self.data.chunks(0)
            raise PanicException("chunk size must be non-zero")
        nch = -(-n // pack_num) if pack_num > 0 else 0
        if 0 < nch <= WIDE_SQUEEZE_MAX_CHUNKS and pack_num > 1:
            # few chunks: the whole squeeze in one launch, one chunk per wave (fphe_pack_squeeze)
            dev = self.device
            src = _fit_limbs(self, pk._key.L2)
            out = CiphertextVector.empty(nch, pk._key.L2, dev)
            _lib.check(_lib.load().fphe_pack_squeeze(pk._key.ctx(dev), _ptr(src.C), _ptr(src.sign), n, pack_num,
                                                     int(offset_bit), _ptr(out.C), _ptr(out.sign),
                                                     ctypes.c_void_p(_stream(dev))), "fphe_pack_squeeze")
            out.n = pk.n
            out.ebound = (0, 0)
            return out
        heads = torch.arange(0, n, pack_num)
        acc = self._gather(heads)
        for j in range(1, pack_num):
            ch = torch.nonzero(heads + j < n).squeeze(1)
            if ch.numel() == 0:
                break
            y = self._gather(heads[ch] + j)
            acc._assign(ch, _sqmul(pk, acc._gather(ch), y, offset_bit))
        acc.exp.zero_()
        acc.ebound = (0, 0)
        return acc

    def matmul(self, pk: "PK", other: PlaintextVector, lshape, rshape) -> "CiphertextVector":
        """``CiphertextVector::matmul`` (lib.rs:861-880): out[i,j] = sum_k self[i,k] * other[k,j]."""
        I, K = int(lshape[0]), int(lshape[1])
        J = int(rshape[1])
        i, j, k = torch.meshgrid(torch.arange(I), torch.arange(J), torch.arange(K), indexing="ij")
        return _matmul_terms(pk, self, other, (i * K + k).reshape(-1), (k * J + j).reshape(-1),
                             (i * J + j).reshape(-1), I * J)

    def rmatmul(self, pk: "PK", other: PlaintextVector, lshape, rshape) -> "CiphertextVector":
        """``CiphertextVector::rmatmul`` (lib.rs:882-908): out[i,j] = sum_k other[i,k] * self[k,j]
        with self (lshape) = [K, Jl], other (rshape) = [I, K]."""
        Jl = int(lshape[1])
        I, K = int(rshape[0]), int(rshape[1])
        i, j, k = torch.meshgrid(torch.arange(I), torch.arange(Jl), torch.arange(K), indexing="ij")
        return _matmul_terms(pk, self, other, (k * Jl + j).reshape(-1), (i * K + k).reshape(-1),
                             (i * Jl + j).reshape(-1), I * Jl)

    def _overwrite_prefix(self, r: "CiphertextVector") -> None:
        if r.count == self.count:
            self.C, self.sign, self.exp = r.C, r.sign, r.exp
            self.ebound = r.ebound
        else:
            self._assign(torch.arange(0, r.count), r)


_FRESH_ONES = threading.local()  # .v: the in-place target known to hold only literal 1s (_keyed)
# the in-place methods whose fold replaces a zeros() target (_fold_terms): _keyed leaves such a
# target key-less on entry, so its M(1) fill is never made only to be replaced
_FRESH_TARGETS = frozenset({"iupdate", "iupdate_with_masks"})


def _keyed(fn):
    """Stamp the key's modulus on the vectors an operation returns (and on an in-place
    target that had none, e.g. a ``zeros()`` histogram): from its PK argument, else from
    the input vector."""
    import functools

    @functools.wraps(fn)
    def w(self, *args, **kw):
        pk = next((a for a in itertools.chain(args, kw.values()) if isinstance(a, PK)), None)
        # an in-place target that is still a zeros() vector (the literal 1 everywhere) for the
        # length of this call only: _fold_terms then replaces its slots instead of adding
        fresh = isinstance(self, CiphertextVector) and self.raw and self.lit
        if pk is not None:  # unpickled operands get their key before any arithmetic
            if fresh and fn.__name__ in _FRESH_TARGETS:
                _resolve_args(pk.n, *args, *kw.values())
            else:
                _resolve_args(pk.n, self, *args, *kw.values())
        prev = getattr(_FRESH_ONES, "v", None)
        _FRESH_ONES.v = self if fresh else None
        try:
            r = fn(self, *args, **kw)
        finally:
            _FRESH_ONES.v = prev
        n = pk.n if pk is not None else self.n
        if n is not None and not self.raw:
            if self.n is None:
                self.n = n
            for v in (r if isinstance(r, list) else [r]):
                if isinstance(v, CiphertextVector) and v.n is None and not v.raw:
                    v.n = n
                elif isinstance(v, Ciphertext) and v.vec.n is None and not v.vec.raw:
                    v.vec.n = n
        return r
    return w


for _name in ("slice", "slice_indexes", "cat", "shuffle", "i_shuffle", "intervals_slice", "tolist", "add",
              "add_scalar", "iadd", "idouble", "iadd_vec", "neg", "sub", "sub_scalar", "rsub", "rsub_scalar", "isub",
              "isub_vec", "mul", "mul_scalar", "iadd_slice", "iadd_vec_self", "isub_vec_self", "iupdate",
              "iupdate_with_masks", "chunking_cumsum_with_step", "intervals_sum_with_step", "pack_squeeze", "matmul",
              "rmatmul", "_gather"):
    setattr(CiphertextVector, _name, _keyed(getattr(CiphertextVector, _name)))


class Ciphertext:
    """Scalar ciphertext (``fate_utils.paillier.Ciphertext``): a length-1 vector."""

    __slots__ = ("vec",)

    def __init__(self, vec: CiphertextVector):
        self.vec = vec


# --------------------------------------------------------------------------------------
# kernel launchers
# --------------------------------------------------------------------------------------
ADD_SORT_MIN = 4096  # elements; below this the sort costs more than it saves
ADD_CHUNK = 1 << 22  # elements per fphe_add_ordered call (its C vector must stay < 4 GiB)


def _add_order(ea: torch.Tensor, eb: torch.Tensor, L2: int) -> Optional[torch.Tensor]:
    """Launch order for fphe_add_ordered that groups equal exponent gaps.

    Aligning the higher-exponent operand costs 4*|ea - eb| Montgomery squarings
    (decrese_exp_to, fixedpoint_paillier/src/lib.rs:250-258), and k_add27 runs every element
    of a wave for the wave's largest gap (the lanes of a wave share one instruction stream).
    With float data the gaps differ from element to element, so most waves pay for an
    outlier; sorted by gap, a wave's elements need the same number of squarings.  The kernel
    reads and writes the elements in place through the order (no gather or scatter
    copies).  k_add27 cuts the slots into ADD_REGIONS equal runs of wave tiles, one per XCD,
    and the order keeps each run's elements in it: first the few with gaps >= 3, largest
    first (a gap-31 tile is ~25 ordinary tiles long and must start early), then block by
    block (4096 elements) the rest by gap.  The slots an XCD works on at once therefore map to
    neighbouring elements, whose operand words share 128-byte lines in that XCD's L2 (HBM
    traffic 5.8 -> 3.9 KB per element).  fphe_add_order builds it with a device counting sort:
    no host synchronisation.  FPHE_ADD_REGION_SORT=0 selects round 2's global stable sort by
    gap (A/B).  Returns the int32 permutation."""
    if not _ADD_REGION_SORT:
        d = (ea.to(torch.int32) - eb.to(torch.int32)).abs().clamp(max=63)
        return torch.sort((63 - d).to(torch.uint8), stable=True)[1].to(torch.int32)
    # the device counting sort of fphe_add_order (three small launches, ~0.05 ms per 1M):
    # runs of whole wave tiles per XCD, gaps >= 3 at the head of each run (largest first),
    # then the rest by gap within blocks of 4096 elements
    m = ea.numel()
    ea32 = ea.to(torch.int32).contiguous()
    eb32 = eb.to(torch.int32).contiguous()
    order = torch.empty(m, dtype=torch.int32, device=ea.device)
    with torch.cuda.device(ea.device):  # context-less: launches on the current device
        _lib.check(_lib.load().fphe_add_order(_ptr(ea32), _ptr(eb32), m, L2, _ptr(order),
                                              ctypes.c_void_p(_stream(ea.device))), "fphe_add_order")
    return order


def _prealign(pk: "PK", a: CiphertextVector, b: CiphertextVector, n: int
              ) -> Tuple[CiphertextVector, CiphertextVector]:
    """Operands whose exponent gap exceeds MAX_GAP (the add kernel's exact range, kMaxGap):
    the higher-exponent one, unless either is the literal 1 (add's identity, returned as it
    is), is raised to 16^(gap - MAX_GAP) and its exponent lowered by as much, in fphe_align
    steps of at most MAX_GAP -- decrese_exp_to (fixedpoint_paillier/src/lib.rs:250-258) split
    into powers that compose: x^(16^(g1 + g2)) = (x^(16^g1))^(16^g2).  The add that follows
    then has gaps <= MAX_GAP and returns the reference's integers.  Gaps beyond MAX_EXACT_GAP
    (4 x 2^20 squarings per element) raise ValueError instead of running for hours.
    Returns copies; the inputs are untouched."""
    dev = a.device
    gap = a.exp[:n].to(torch.int64) - b.exp[:n].to(torch.int64)
    lit = _is_literal_one(pk, a)[:n] | _is_literal_one(pk, b)[:n]
    big = (gap.abs() > MAX_GAP) & ~lit
    idx = torch.nonzero(big).squeeze(1)
    if idx.numel() == 0:
        return a, b
    g = gap[idx]
    if int(g.abs().max()) > MAX_EXACT_GAP:
        raise ValueError(f"exponent gap {int(g.abs().max())} beyond {MAX_EXACT_GAP} in ct-add "
                         f"(4 squarings per step): corrupt exponents")
    a, b = a.__copy__(), b.__copy__()
    for side, sel in ((a, g > 0), (b, g < 0)):
        sidx = idx[sel]
        if sidx.numel() == 0:
            continue
        steps = g[sel].abs() - MAX_GAP
        sub = side._gather(sidx)
        rem = steps.clone()
        while int(rem.max()) > 0:
            st = rem.clamp(max=MAX_GAP)
            e0 = sub.exp.clone()
            sub = _align(pk, sub, st)
            sub.exp.copy_(e0)
            rem -= st
        sub.exp[: sidx.numel()] -= steps.to(torch.int32)
        sub.ebound = None
        side._assign(sidx.to(dev), sub)
    return a, b


# FPHE_CHECK_EBOUND=1 (the GPU test suite sets it): whenever ct-add trusts the host-side
# exponent bounds instead of reading the gaps back, read the exponents anyway and fail if one
# lies outside its vector's bound.  A stale bound would otherwise give a silently wrong sum.
CHECK_EBOUND = os.environ.get("FPHE_CHECK_EBOUND") == "1"


def _check_ebound(v: "CiphertextVector", exp: torch.Tensor) -> None:
    if exp.numel() == 0:
        return
    lo, hi = int(exp.min()), int(exp.max())
    if lo < v.ebound[0] or hi > v.ebound[1]:
        raise AssertionError(f"stale exponent bound: exponents span [{lo}, {hi}], ebound {v.ebound}")


def _add(pk: "PK", a: CiphertextVector, b: CiphertextVector, broadcast: bool, count: Optional[int] = None,
         reorder: bool = True, deferred: Optional[list] = None) -> CiphertextVector:
    """deferred: a list to append the kernel's device error flags to instead of checking the
    gaps first (no read-back here); the caller tests them with :func:`_fold_failed` once its
    later launches are queued and redoes the add without `deferred` if a gap was beyond
    MAX_GAP (the flagged elements are unspecified)."""
    dev = a.device
    a, b = _fit_limbs(a, pk._key.L2), _fit_limbs(b, pk._key.L2)
    n = a.count if count is None else count
    if not broadcast and b.count < n:
        n = b.count  # zip() semantics of the reference (lib.rs:797-805)
    out = CiphertextVector.empty(n, a.L2, dev)
    # the sum's exponent is the lesser of its operands' (lib.rs:301-333)
    out.ebound = _ebound_union(a.ebound, b.ebound)
    if n == 0:
        return out
    err = None
    if deferred is not None:
        err = torch.zeros(1, dtype=torch.int32, device=dev)
        deferred.append(err)
    elif out.ebound is not None and out.ebound[1] - out.ebound[0] <= MAX_GAP:
        # every gap is within the kernel's exact range: no read-back
        if CHECK_EBOUND:
            _check_ebound(a, a.exp[:n])
            _check_ebound(b, b.exp[:1] if broadcast else b.exp[:n])
    else:
        # the kernel is exact for exponent gaps up to MAX_GAP (one read-back of the largest gap)
        eb = b.exp[:1].expand(n) if broadcast else b.exp[:n]
        if int((a.exp[:n].to(torch.int64) - eb.to(torch.int64)).abs().max()) > MAX_GAP:
            if broadcast:
                b, broadcast = b._gather(torch.zeros(n, dtype=torch.long)), False
            a, b = _prealign(pk, a, b, n)
    lib = _lib.load()
    ctx = pk._key.ctx(dev)
    stream = ctypes.c_void_p(_stream(dev))
    for s0 in range(0, n, ADD_CHUNK):  # whole tiles per chunk
        m = min(ADD_CHUNK, n - s0)
        t0, t1 = s0 // WAVE, _ntiles(s0 + m)
        e0, e1 = s0, t1 * WAVE
        order = None
        if reorder and not broadcast and m >= ADD_SORT_MIN:
            order = _add_order(a.exp[s0:s0 + m], b.exp[s0:s0 + m], a.L2)
        bC, bs, be = (b.C, b.sign, b.exp) if broadcast else (b.C[t0:t1], b.sign[e0:e1], b.exp[e0:e1])
        _lib.check(lib.fphe_add_ordered(ctx, _ptr(a.C[t0:t1]), _ptr(a.sign[e0:e1]), _ptr(a.exp[e0:e1]), _ptr(bC),
                                        _ptr(bs), _ptr(be), 0 if broadcast else 1, m, _ptr(order),
                                        _ptr(out.C[t0:t1]), _ptr(out.sign[e0:e1]), _ptr(out.exp[e0:e1]), _ptr(err),
                                        stream),
                   "fphe_add_ordered")
        del order  # the launch is stream-ordered: the allocator reuses the block only after it
    return out


def _flatten_positions(indexes, dev=None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Vec<Vec<usize>> of positions per sample -> (sample ids, positions), flat on `dev`: sample
    ids int64, positions in their own integer type (int32 for a device int32 tensor), range-checked
    and narrowed by the caller (:meth:`CiphertextVector._scatter_fold`).  A [samples, positions]
    tensor is expanded on the device (no host-side index arrays)."""
    if isinstance(indexes, torch.Tensor):
        if indexes.dim() != 2:
            raise ValueError("positions tensor must be 2-D [samples, positions]")
        ns, npos = indexes.shape
        pp = indexes.to(device=dev).reshape(-1)
        if pp.dtype not in (torch.int32, torch.int64):
            pp = pp.to(torch.int64)
        ii = torch.arange(ns * npos, device=dev, dtype=torch.int64) // max(npos, 1)
        return ii, pp
    lens, pos = _position_lists(indexes)
    ii = torch.from_numpy(np.repeat(np.arange(lens.size, dtype=np.int64), lens))
    return ii.to(dev), torch.from_numpy(pos).to(dev)


def _interval_array(intervals) -> Tuple[torch.Tensor, torch.Tensor]:
    """Vec<(usize, usize)> as (starts, ends) int64 tensors; a negative bound is pyo3's usize
    extraction error."""
    iv = torch.tensor([(int(a), int(b)) for a, b in intervals], dtype=torch.int64).reshape(-1, 2)
    if iv.numel() and bool((iv < 0).any()):
        raise OverflowError("can't convert negative int to unsigned")
    return iv[:, 0], iv[:, 1]


def _interval_items(s: torch.Tensor, e: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """The element indexes of consecutive intervals [s_i, e_i) (s <= e), concatenated, and each
    one's offset inside its interval."""
    lens = e - s
    total = int(lens.sum()) if lens.numel() else 0
    if total == 0:
        z = torch.zeros(0, dtype=torch.int64)
        return z, z
    rel = torch.arange(total, dtype=torch.int64) - torch.repeat_interleave(torch.cumsum(lens, 0) - lens, lens)
    return torch.repeat_interleave(s, lens) + rel, rel


def _position_lists(indexes) -> Tuple[np.ndarray, np.ndarray]:
    """Vec<Vec<usize>> -> (positions per sample, every position in the reference's sample-major
    order), int64 arrays, read by the host helper (fate_amd/csrc/host_positions.c) in two passes
    over the Python objects.  A non-integer position raises TypeError, as pyo3's extraction
    does; ranges are checked by the callers."""
    if not isinstance(indexes, (list, tuple)):
        indexes = list(indexes)
    lib = _lib.load_py()
    lens = np.empty(len(indexes), dtype=np.int64)
    total = lib.fphe_py_positions_lens(indexes, lens.ctypes.data, lens.size)
    pos = np.empty(total, dtype=np.int64)
    lib.fphe_py_positions_fill(indexes, pos.ctypes.data, total)
    return lens, pos


# pack_squeeze takes the one-chunk-per-wave kernel (fphe_pack_squeeze) up to this many chunks:
# beyond it the throughput kernel's full waves issue the squarings more cheaply
WIDE_SQUEEZE_MAX_CHUNKS = int(os.environ.get("FPHE_WIDE_SQUEEZE_MAX", "4096"))
ADD_REGIONS = 8  # kAddRegions in fate_phe.hip: runs of k_add27 wave tiles, one per XCD
# FPHE_ADD_REGION_SORT=0: one global gap sort (round-2 order; same-box A/B in tools/)
_ADD_REGION_SORT = os.environ.get("FPHE_ADD_REGION_SORT", "1") != "0"
FOLD_MAX = 64  # terms per chunk of fphe_fold (kFoldMax in kernels27.h)
FOLD_TARGET_CHUNKS = 32768


def _run_starts(head: torch.Tensor) -> torch.Tensor:
    """For run-head flags, the index of each position's run start (a cumsum and a gather;
    cheaper on the device than cummax-with-indices)."""
    heads = torch.nonzero(head).squeeze(1)
    return heads[torch.cumsum(head.to(torch.int32), 0) - 1]


def _fold_chunks(pk: "PK", src: CiphertextVector, ordv: torch.Tensor, keys: torch.Tensor
                 ) -> Tuple[CiphertextVector, torch.Tensor]:
    """One fphe_fold pass: the terms src[ordv[i]] carry sorted group keys keys[i]; every run of
    equal keys is cut into chunks of <= FOLD_MAX terms and each chunk becomes one partial.
    Returns the partials (in key order) and their keys."""
    dev = src.device
    n = keys.numel()
    pos = torch.arange(n, device=dev)
    head = torch.ones(n, dtype=torch.bool, device=dev)
    head[1:] = keys[1:] != keys[:-1]
    gstart = _run_starts(head)
    # chunk length: 64 while that still gives every wave slot of the chip work (~32K chunks
    # of 16-element waves), shorter on the later, smaller rounds so their sequential depth
    # (one product per term) stays low
    k = max(8, min(FOLD_MAX, -(-n // FOLD_TARGET_CHUNKS)))
    cstart = torch.nonzero(head | ((pos - gstart) % k == 0)).squeeze(1)
    nch = cstart.numel()
    clen = torch.diff(cstart, append=torch.tensor([n], device=dev)).to(torch.int32)
    out = CiphertextVector.empty(nch, pk._key.L2, dev)
    rows = src.C.permute(0, 2, 1).contiguous()  # element-major copy for the gathers
    lib = _lib.load()
    # operands bound to names: a temporary passed as _ptr(t.to(...)) would go back to the
    # caching allocator before the launch and could share its block with the next one
    ord64, cst = ordv.to(torch.int64).contiguous(), cstart.contiguous()
    _lib.check(lib.fphe_fold(pk._key.ctx(dev), _ptr(rows), _ptr(src.sign), _ptr(src.exp),
                             _ptr(ord64), _ptr(cst), _ptr(clen), nch,
                             _ptr(out.C), _ptr(out.sign), _ptr(out.exp), ctypes.c_void_p(_stream(dev))), "fphe_fold")
    return out, keys[cstart]


def _fold_segments(pk: "PK", src: CiphertextVector, seg: torch.Tensor, index: Optional[torch.Tensor] = None
                   ) -> Tuple[CiphertextVector, torch.Tensor]:
    """Fold the terms src[index[i]] (index defaults to all of src) by segment id seg[i]: the
    reference's sequential ct-add folds, which are order-independent.
    Terms are sorted by (segment, exponent): equal-exponent runs are folded as plain
    products by fphe_fold (chunks of 64, repeated until one partial per (segment,
    exponent)), then each segment's per-exponent partials are merged by the aligning ct-add
    tree.  Returns one ciphertext per non-empty segment with the segment ids (ascending)."""
    dev = src.device
    src = _fit_limbs(src, pk._key.L2)
    seg = seg.to(dev, torch.long)
    n = seg.numel()
    if n == 0:
        return CiphertextVector.empty(0, pk._key.L2, dev), seg
    index = torch.arange(n, device=dev) if index is None else index.to(dev, torch.long)
    texp = src.exp[index]
    key = seg * (1 << 32) + (texp.to(torch.long) + (1 << 31))
    key, order = torch.sort(key)
    cur, ckeys = _fold_chunks(pk, src, index[order], key)
    while bool((ckeys[1:] == ckeys[:-1]).any()):
        cur, ckeys = _fold_chunks(pk, cur, torch.arange(cur.count, device=dev), ckeys)
    merged = _merge_exponents(pk, cur, ckeys) if MERGE_BY_ALIGN else None
    res, ids = merged if merged is not None else _fold_tree(pk, cur, ckeys >> 32)
    # A segment whose terms are all the literal 1 folds to 1: add(1, y) returns y, so the
    # reference's sequential fold ends on its LAST term, exponent included (lib.rs:303-308).
    lit = _is_literal_one(pk, res)
    if bool(lit.any()):
        pos = torch.arange(n, device=dev)
        last = torch.zeros(int(seg.max()) + 1, dtype=torch.long, device=dev)
        last.scatter_reduce_(0, seg, pos, reduce="amax", include_self=False)
        li = torch.nonzero(lit).squeeze(1)
        res.exp[li] = texp[last[ids[li]]]
    return res, ids


def _fold_failed(errs: Sequence[torch.Tensor]) -> bool:
    """Did a device fold meet an exponent gap beyond its exact range (FPHE_EF_EXP_RANGE)?
    Reads the flags back (synchronises); the caller then folds with :func:`_fold_dense`."""
    return any(int(e.item()) & _lib.EF_EXP_RANGE for e in errs)


def _literal_ones(pk: "PK", count: int, dev) -> CiphertextVector:
    """``count`` literal 1s (exp 0) under pk's key: M(1) words, sign 0."""
    v = CiphertextVector.empty(count, pk._key.L2, dev)
    v.C.copy_(pk._key.mont_one(dev).view(1, -1, 1).expand_as(v.C))
    v.n = pk.n
    v.ebound = (0, 0)
    return v


def _fold_dense(pk: "PK", src: CiphertextVector, seg: torch.Tensor, nseg: int, idx: Optional[torch.Tensor]):
    """out[s] for every s < nseg by the torch grouping of :func:`_fold_segments` (exact for any
    exponent gap up to MAX_EXACT_GAP): the fallback of fphe_fold_segments for key spaces too
    large for its counting sort and for gaps beyond its alignment range.  Returns (out, present)."""
    dev = src.device
    res, ids = _fold_segments(pk, src, seg.long(), index=None if idx is None else idx.long())
    res.n = pk.n
    out = _literal_ones(pk, nseg, dev)
    out._assign(ids, res)
    present = torch.zeros(_ntiles(nseg) * WAVE, dtype=torch.uint8, device=dev)
    present[ids] = 1
    return out, present


def _fold_to_segments(pk: "PK", src: CiphertextVector, seg: torch.Tensor, nseg: int,
                      index: Optional[torch.Tensor] = None, with_present: bool = False, deferred: list = None):
    """out[s] = the reference's sequential ct-add fold of the terms src[index[t]] with seg[t] == s,
    for every s < nseg (the literal 1, exp 0, where no term lands) -- fphe_fold_segments, which
    groups, folds and merges the exponents on the device.  Falls back to the torch grouping of
    :func:`_fold_segments` when the (segment, exponent) key space is too large for it.
    with_present: also return the per-segment uint8 flags "some term landed here".
    deferred: a list to append the device error flags to instead of reading them back here
    (the caller then calls :func:`_fold_failed` once its follow-up launches are queued, and
    folds with :func:`_fold_dense` if it reports a gap beyond the device merge's range)."""
    dev = src.device
    T = seg.numel()
    if T > FOLD_MAX_TERMS:
        return _fold_chunked(pk, src, seg, nseg, index, with_present)
    src = _fit_limbs(src, pk._key.L2)
    L2 = pk._key.L2
    seg = seg.to(dev, torch.int32).contiguous()
    idx = None if index is None else index.to(dev, torch.int32).contiguous()
    if idx is not None and idx.numel() != T:
        raise ValueError("fold: index and segment arrays differ in length")
    # fphe_fold_segments writes every word of these first (k_gr_init_out: the literal 1, exp 0,
    # not present, tile padding included), so none is zeroed here
    nt = _ntiles(nseg)
    out = CiphertextVector(torch.empty((nt, L2, WAVE), dtype=torch.int32, device=dev),
                           torch.empty(nt * WAVE, dtype=torch.uint8, device=dev),
                           torch.empty(nt * WAVE, dtype=torch.int32, device=dev), nseg, pk.n)
    present = torch.empty(nt * WAVE, dtype=torch.uint8, device=dev)
    if nseg == 0:
        if T:
            raise PanicException("index out of bounds")
        return (out, present) if with_present else out
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    st = _lib.load().fphe_fold_segments(pk._key.ctx(dev), _ptr(src.C), _ptr(src.sign), _ptr(src.exp), src.count,
                                        _ptr(idx), _ptr(seg), T, nseg, _ptr(out.C), _ptr(out.sign), _ptr(out.exp),
                                        _ptr(present), _ptr(err), ctypes.c_void_p(_stream(dev)))
    if st == _lib.FPHE_ERR_RANGE:
        out, present = _fold_dense(pk, src, seg, nseg, idx)
        return (out, present) if with_present else out
    if st == _lib.FPHE_ERR_ARG:
        raise PanicException("index out of bounds")
    _lib.check(st, "fphe_fold_segments")
    if deferred is not None:
        deferred.append(err)
    elif _fold_failed([err]):
        out, present = _fold_dense(pk, src, seg, nseg, idx)
    return (out, present) if with_present else out


# fphe_fold_segments counts its terms in int32 (include/fate_phe.h): a longer term list is
# folded in chunks of this many (module-level so the GPU tests can exercise the split small)
FOLD_MAX_TERMS = (1 << 31) - 1


def _fold_chunked(pk: "PK", src: CiphertextVector, seg: torch.Tensor, nseg: int,
                  index: Optional[torch.Tensor], with_present: bool):
    """_fold_to_segments over more than FOLD_MAX_TERMS terms: fold consecutive chunks and add
    each chunk's per-segment result onto the running one where both hold terms.  The reference's
    fold is sequential, so fold(t_1..t_k) = add(fold(t_1..t_j), fold(t_j+1..t_k)) with add's
    literal-1 rule giving the right exponent when either side folded to the literal 1; a segment
    a chunk does not reach keeps its running value."""
    out = present = None
    for a in range(0, seg.numel(), FOLD_MAX_TERMS):
        b = min(a + FOLD_MAX_TERMS, seg.numel())
        f, p = _fold_to_segments(pk, src, seg[a:b], nseg, None if index is None else index[a:b], with_present=True)
        if out is None:
            out, present = f, p
            continue
        r = _add(pk, out, f, broadcast=False)
        both = (present != 0) & (p != 0)
        take = torch.where(both, 2, torch.where(p != 0, 1, 0))[: r.sign.numel()]
        pick = lambda x0, x1, x2, t: torch.where(t == 2, x2, torch.where(t == 1, x1, x0))
        out.C = pick(out.C, f.C, r.C, take.view(-1, 1, WAVE))
        out.sign = pick(out.sign, f.sign, r.sign, take)
        out.exp = pick(out.exp, f.exp, r.exp, take)
        present = present | p
    return (out, present) if with_present else out


def _is_literal_one(pk: "PK", v: CiphertextVector) -> torch.Tensor:
    """Per element: is the signed ciphertext integer exactly 1 (the reference's zero), i.e. is
    C = M(1) with sign 0 (Montgomery-resident words)."""
    one = pk._key.mont_one(v.device).view(1, -1, 1)
    lit = (v.C == one).all(dim=1).reshape(-1)[: v.count]
    return lit & (v.sign[: v.count] == 0)


# merge a segment's per-exponent partials by one alignment pass + product folds (True), or by
# the pairwise ct-add tree (False: ceil(log2(partials)) launches, each as long as its largest
# exponent gap)
MERGE_BY_ALIGN = True
MAX_GAP = 1 << 16  # kMaxGap of fate_amd/csrc/kernels27.h: the add / align kernels' exact range
# larger gaps are split into fphe_align steps (_prealign) up to this many, else ValueError
MAX_EXACT_GAP = 1 << 20


def _merge_exponents(pk: "PK", cur: CiphertextVector, ckeys: torch.Tensor
                     ) -> Optional[Tuple[CiphertextVector, torch.Tensor]]:
    """One ciphertext per segment from its per-exponent partials (keys (segment << 32) |
    (exp + 2^31), ascending, one partial per key).  The reference's sequential adds raise
    every term to 16^(e - e_min), e_min the least exponent of the segment's non-literal
    terms, and multiply (decrese_exp_to + add, fixedpoint_paillier/src/lib.rs:250-258,
    301-333; order-independent); a term that was raised loses its sign
    (powm is canonical), so the product's sign is the XOR over the e_min terms.  Literal-1
    partials are add's identity: they stay out of e_min and fold as 1.  So: one fphe_align
    pass over all partials (largest gaps first), then plain product folds (fphe_fold) of
    each segment, all at e_min.  Segments of literal-1 partials only fold to 1 (the caller
    restores the reference's exponent for those)."""
    dev = cur.device
    n = cur.count
    seg = ckeys >> 32
    exp = (ckeys & 0xFFFFFFFF) - (1 << 31)
    lit = _is_literal_one(pk, cur)
    big = 1 << 40
    _, inv = torch.unique_consecutive(seg, return_inverse=True)
    emin = torch.full((int(inv.max()) + 1,), big, dtype=torch.long, device=dev)
    emin.scatter_reduce_(0, inv, torch.where(lit, torch.full_like(exp, big), exp), reduce="amin")
    em = emin[inv]
    gap = torch.where(lit | (em == big), torch.zeros_like(exp), exp - em)
    if int(gap.max()) > MAX_GAP:  # fphe_align's contract (kMaxGap in kernels27.h): the caller
        return None               # merges by the pairwise ct-add tree, exact for such gaps
    tgt = torch.where(em == big, torch.zeros_like(em), em)
    order = torch.argsort(gap, descending=True, stable=True)
    src = cur._gather(order)
    aligned = _align(pk, src, gap[order])
    aligned.exp[:n] = tgt[order].to(torch.int32)
    key2, o2 = torch.sort(seg[order] * (1 << 32) + (tgt[order] + (1 << 31)))
    res, k2 = _fold_chunks(pk, aligned, o2, key2)
    while bool((k2[1:] == k2[:-1]).any()):
        res, k2 = _fold_chunks(pk, res, torch.arange(res.count, device=dev), k2)
    return res, k2 >> 32


def _align(pk: "PK", a: CiphertextVector, gap: torch.Tensor) -> CiphertextVector:
    """(a^(16^gap) mod n^2, sign 0 where gap > 0, exp unchanged) on the device (fphe_align)."""
    dev = a.device
    a = _fit_limbs(a, pk._key.L2)
    n = a.count
    out = CiphertextVector.empty(n, a.L2, dev)
    if n == 0:
        return out
    out.exp[:n] = a.exp[:n]
    g32 = gap.to(device=dev, dtype=torch.int32).contiguous()
    lib = _lib.load()
    _lib.check(lib.fphe_align(pk._key.ctx(dev), _ptr(a.C), _ptr(a.sign), _ptr(g32), n, _ptr(out.C), _ptr(out.sign),
                              ctypes.c_void_p(_stream(dev))), "fphe_align")
    return out


def _fold_tree(pk: "PK", src: CiphertextVector, seg: torch.Tensor) -> Tuple[CiphertextVector, torch.Tensor]:
    """Fold src by segment id with the ct-add kernel, as a pairwise tree inside each
    segment (ceil(log2(longest segment)) launches).  Returns one folded ciphertext per
    non-empty segment, with the segment ids (ascending)."""
    dev = src.device
    seg = seg.to(dev, torch.long)
    order = torch.argsort(seg, stable=True)
    ids = seg[order]
    cur = src._gather(order)
    while ids.numel() > 1:
        n = ids.numel()
        pos = torch.arange(n, device=dev)
        head = torch.ones(n, dtype=torch.bool, device=dev)
        head[1:] = ids[1:] != ids[:-1]
        start = _run_starts(head)
        left = pos[(pos - start) % 2 == 0]
        nxt = torch.clamp(left + 1, max=n - 1)
        has = (left + 1 < n) & (ids[nxt] == ids[left])
        if not bool(has.any()):
            break
        pl = left[has]
        summed = _add(pk, cur._gather(pl), cur._gather(pl + 1), broadcast=False)
        new = cur._gather(left)
        new._assign(torch.nonzero(has).squeeze(1), summed)
        cur, ids = new, ids[left]
    return cur, ids


def _matmul_terms(pk: "PK", a: CiphertextVector, b: PlaintextVector, ai: torch.Tensor, bi: torch.Tensor,
                  oi: torch.Tensor, nout: int, chunk: int = 1 << 22) -> CiphertextVector:
    """out[o] = fold over terms t with oi[t] == o of a[ai[t]] * b[bi[t]], from zero; the
    products run through the ct x pt kernel, the folds through the ct-add kernel, in chunks
    of `chunk` terms so the materialised products stay bounded."""
    out = CiphertextVector.zeros(nout, a.L2, a.device)
    for s0 in range(0, ai.numel(), chunk):
        sl = slice(s0, s0 + chunk)
        prod = _mul(pk, a._gather(ai[sl]), b._gather(bi[sl].to(b.device)), broadcast=False)
        folded = _fold_to_segments(pk, prod, oi[sl], nout)
        # the running partial sums come first: fold(out, terms) = add(out, fold(terms))
        out = folded if s0 == 0 else _add(pk, out, folded, broadcast=False)
    return out


def _sqmul(pk: "PK", a: CiphertextVector, b: CiphertextVector, nsq: int) -> CiphertextVector:
    """(a^(2^nsq) * b mod n^2, sign of b) on the device (fphe_sqmul)."""
    dev = a.device
    a, b = _fit_limbs(a, pk._key.L2), _fit_limbs(b, pk._key.L2)
    n = min(a.count, b.count)
    out = CiphertextVector.empty(n, a.L2, dev)
    if n == 0:
        return out
    lib = _lib.load()
    ctx = pk._key.ctx(dev)
    _lib.check(lib.fphe_sqmul(ctx, _ptr(a.C), _ptr(b.C), _ptr(b.sign), int(nsq), n, _ptr(out.C), _ptr(out.sign),
                              ctypes.c_void_p(_stream(dev))), "fphe_sqmul")
    return out


def _neg(pk: "PK", a: CiphertextVector, count: Optional[int] = None) -> CiphertextVector:
    """(invert(C, n^2), sign 0, exp) on the device (fphe_neg)."""
    dev = a.device
    a = _fit_limbs(a, pk._key.L2)
    n = a.count if count is None else count
    out = CiphertextVector.empty(n, a.L2, dev)
    if n == 0:
        return out
    lib = _lib.load()
    ctx = pk._key.ctx(dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    _lib.check(lib.fphe_neg(ctx, _ptr(a.C), n, _ptr(out.C), _ptr(err), ctypes.c_void_p(_stream(dev))), "fphe_neg")
    out.exp[:n] = a.exp[:n]
    out.ebound = a.ebound
    if int(err.item()) & _lib.EF_NOT_INVERTIBLE:
        raise PanicException("called `Option::unwrap()` on a `None` value")  # invert().unwrap() (math/src/rug/mod.rs:30-35)
    return out


def _mul(pk: "PK", a: CiphertextVector, p: PlaintextVector, broadcast: bool) -> CiphertextVector:
    dev = a.device
    a = _fit_limbs(a, pk._key.L2)
    n = a.count if broadcast else min(a.count, p.count)
    out = CiphertextVector.empty(n, a.L2, dev)
    if n == 0:
        return out
    lib = _lib.load()
    ctx = pk._key.ctx(dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    P = p.P if p.lp <= pk._key.L1 else p.P[:, : pk._key.L1].contiguous()
    _lib.check(lib.fphe_mul(ctx, _ptr(a.C), _ptr(a.sign), _ptr(a.exp), _ptr(P), P.shape[1], _ptr(p.neg),
                            _ptr(p.exp), 0 if broadcast else 1, n, _ptr(out.C), _ptr(out.sign), _ptr(out.exp),
                            _ptr(err), ctypes.c_void_p(_stream(dev))), "fphe_mul")
    if a.ebound is not None and p.ebound is not None:  # exp = exp_c + exp_pt (lib.rs:345-348)
        out.ebound = (a.ebound[0] + p.ebound[0], a.ebound[1] + p.ebound[1])
    v = int(err.item())
    if v & _lib.EF_MUL_INVALID_PT:
        raise PanicException("invalid plaintext")
    if v & _lib.EF_NOT_INVERTIBLE:
        raise PanicException("called `Option::unwrap()` on a `None` value")  # invert().unwrap() (math/src/rug/mod.rs:30-35)
    return out


# --------------------------------------------------------------------------------------
# keys and coder
# --------------------------------------------------------------------------------------
class PK:
    """``fate_utils.paillier.PK`` (paillier.rs:50-75; fixedpoint_paillier::PK lib.rs:18-34).

    A PK made by :func:`keygen` in the process that holds the private key carries a
    reference to that key's device context (never pickled: ``__getstate__`` is ``n``
    only, as the reference's).  Its obfuscated encryptions then run the key-holder path
    (``fphe_encrypt_crt``: r^n mod n^2 from two half-width CRT modexps), which yields the
    same ciphertext integers as the public-key path for the same r.  ``PK(n)`` -- and any
    unpickled PK -- is public-only.  ``FPHE_KEYHOLDER_CRT=0`` disables the CRT path."""

    def __init__(self, n: Optional[int] = None):
        self.n = n
        self._priv: Optional[_KeyCtx] = None
        if n is not None:
            self._init(n)

    def _init(self, n: int):
        self.n = n
        self.ns = n * n
        self.max_int = n // MAX_INT_FRACTION
        self._key = _key_for(n)

    def _bind_private(self, p: int, q: int) -> "PK":
        self._priv = _key_for(self.n, *((p, q) if p < q else (q, p)))
        return self

    @property
    def keyholder(self) -> bool:
        return self._priv is not None and os.environ.get("FPHE_KEYHOLDER_CRT", "1") != "0"

    def encrypt_encoded(self, plaintext_vector: PlaintextVector, obfuscate: bool,
                        r: Optional[Sequence[int]] = None) -> CiphertextVector:
        """``PK.encrypt_encoded`` (paillier.rs:51-57 -> lib.rs:370-381).  ``r`` (our extension)
        injects the obfuscation nonces (parity mode); default draws them on the device."""
        pv = plaintext_vector
        dev = pv.device
        k = self._key
        n = pv.count
        out = CiphertextVector.empty(n, k.L2, dev)
        out.n = self.n
        if n == 0:
            return out
        if pv.lp > k.L1:
            raise PanicException("plaintext does not fit the key")
        rt = None
        if r is not None:
            if len(r) != n:
                raise ValueError("need one r per element")
            rt = torch.from_numpy(rows_to_tiles(ints_to_limbs(list(r), k.L1)).view(np.int32)).to(dev)
        lib = _lib.load()
        stream = ctypes.c_void_p(_stream(dev))
        if obfuscate and self.keyholder:
            kp = self._priv
            _lib.check(lib.fphe_encrypt_crt(kp.ctx(dev), _ptr(pv.P), pv.lp, _ptr(pv.neg), n, _ptr(rt), kp.rng_key,
                                            kp.next_nonce(), _ptr(out.C), _ptr(out.sign), stream),
                       "fphe_encrypt_crt")
        else:
            _lib.check(lib.fphe_encrypt(k.ctx(dev), _ptr(pv.P), pv.lp, _ptr(pv.neg), n, 1 if obfuscate else 0,
                                        _ptr(rt), k.rng_key, k.next_nonce(), _ptr(out.C), _ptr(out.sign), stream),
                       "fphe_encrypt")
        out.exp[:n] = pv.exp[:n]
        out.n = self.n
        out.ebound = pv.ebound
        return out

    def encrypt_encoded_scalar(self, plaintext: Plaintext, obfuscate: bool) -> Ciphertext:
        """``PK.encrypt_encoded_scalar`` (paillier.rs:58-60)."""
        return Ciphertext(self.encrypt_encoded(plaintext.vec, obfuscate))

    # pickling: the reference's state, bincode(fixedpoint_paillier::PK) (paillier.rs:67-74)
    def __getstate__(self):
        from . import wire
        return _pickle_state(wire.pk_to_bincode(self))

    def __setstate__(self, state):
        from . import wire
        self._priv = None
        self._init(wire.pk_from_bincode(bytes(state)).n)


class SK:
    """``fate_utils.paillier.SK`` (paillier.rs:77-99; paillier::SK lib.rs:55-69, 124-177)."""

    def __init__(self, p: Optional[int] = None, q: Optional[int] = None):
        if p is not None:
            self._init(p, q)

    def _init(self, p: int, q: int):
        if p == q:
            raise PanicException("p == q")
        self.p, self.q = (p, q) if p < q else (q, p)
        self.n = self.p * self.q
        self._key = _key_for(self.n, self.p, self.q)

    def decrypt_to_encoded(self, data: CiphertextVector) -> PlaintextVector:
        """``SK.decrypt_to_encoded`` (paillier.rs:79-81 -> lib.rs:392-399)."""
        dev = data.device
        k = self._key
        _resolve(data, self.n)
        data = _fit_limbs(data, k.L2)
        n = data.count
        nt = _ntiles(n)
        P = torch.empty((nt, k.L1, WAVE), dtype=torch.int32, device=dev)
        out = PlaintextVector(P, torch.zeros(nt * WAVE, dtype=torch.uint8, device=dev),
                              data.exp.clone(), n)
        if n == 0:
            return out
        lib = _lib.load()
        _lib.check(lib.fphe_decrypt(k.ctx(dev), _ptr(data.C), n, _ptr(P), ctypes.c_void_p(_stream(dev))),
                   "fphe_decrypt")
        return out

    def decrypt_to_encoded_scalar(self, data: Ciphertext) -> Plaintext:
        return Plaintext(self.decrypt_to_encoded(data.vec))

    # pickling: bincode(fixedpoint_paillier::SK) (paillier.rs:91-98)
    def __getstate__(self):
        from . import wire
        return _pickle_state(wire.sk_to_bincode(self))

    def __setstate__(self, state):
        from . import wire
        sk = wire.sk_from_bincode(bytes(state))
        self._init(sk.p, sk.q)


class Coder:
    """``fate_utils.paillier.Coder`` (paillier.rs:101-204; fixedpoint_paillier::Coder lib.rs:53-193)."""

    def __init__(self, n: Optional[int] = None):
        if n is not None:
            self._init(n)

    def _init(self, n: int):
        self.n = n
        self.max_int = n // MAX_INT_FRACTION
        self._key = _key_for(n)

    # pickling: bincode(fixedpoint_paillier::Coder) (paillier.rs:128-135)
    def __getstate__(self):
        from . import wire
        return _pickle_state(wire.coder_to_bincode(self.n))

    def __setstate__(self, state):
        from . import wire
        self._init(wire.coder_from_bincode(bytes(state)))

    # ---- vector encode (device) ------------------------------------------------------
    def _encode_float(self, arr, dtype: torch.dtype, device=None) -> PlaintextVector:
        dev = _device(device if device is not None else (arr.device if isinstance(arr, torch.Tensor)
                                                         and arr.is_cuda else None))
        x = torch.as_tensor(arr).detach().flatten().to(dtype=dtype, device=dev).contiguous()
        n = x.numel()
        nt = _ntiles(n)
        P = torch.zeros((nt, 2, WAVE), dtype=torch.int32, device=dev)
        neg = torch.zeros(nt * WAVE, dtype=torch.uint8, device=dev)
        ex = torch.zeros(nt * WAVE, dtype=torch.int32, device=dev)
        out = PlaintextVector(P, neg, ex, n)
        if n == 0:
            return out
        err = torch.zeros(1, dtype=torch.int32, device=dev)
        lib = _lib.load()
        fn = lib.fphe_encode_f32 if dtype == torch.float32 else lib.fphe_encode_f64
        _lib.check(fn(self._key.ctx(dev), _ptr(x), n, _ptr(P), _ptr(neg), _ptr(ex), _ptr(err),
                      ctypes.c_void_p(_stream(dev))), "fphe_encode")
        _raise_err(err)
        out.ebound = ENCODE_EXP_RANGE
        return out

    def encode_f32_vec(self, data, device=None) -> PlaintextVector:
        """``Coder.encode_f32_vec`` (paillier.rs:162-169)."""
        return self._encode_float(data, torch.float32, device)

    def encode_f64_vec(self, data, device=None) -> PlaintextVector:
        """``Coder.encode_f64_vec`` (paillier.rs:145-152)."""
        return self._encode_float(data, torch.float64, device)

    def _encode_int(self, data, device=None) -> PlaintextVector:
        # encode_i64 / encode_i32 (lib.rs:68-78, 119-129): sig = v (v >= 0) or n + v, exp 0
        dev = _device(device if device is not None else (data.device if isinstance(data, torch.Tensor)
                                                         and data.is_cuda else None))
        x = torch.as_tensor(data).detach().flatten().to(dtype=torch.int64, device=dev).contiguous()
        n = x.numel()
        nt = _ntiles(n)
        L1 = self._key.L1
        out = PlaintextVector(torch.zeros((nt, L1, WAVE), dtype=torch.int32, device=dev),
                              torch.zeros(nt * WAVE, dtype=torch.uint8, device=dev),
                              torch.zeros(nt * WAVE, dtype=torch.int32, device=dev), n)
        if n == 0:
            return out
        lib = _lib.load()
        _lib.check(lib.fphe_encode_i64(self._key.ctx(dev), _ptr(x), n, _ptr(out.P), _ptr(out.neg), _ptr(out.exp),
                                       ctypes.c_void_p(_stream(dev))), "fphe_encode_i64")
        out.ebound = (0, 0)
        return out

    def encode_i64_vec(self, data, device=None) -> PlaintextVector:
        """``Coder.encode_i64_vec`` (paillier.rs:182-189)."""
        return self._encode_int(data, device)

    def encode_i32_vec(self, data, device=None) -> PlaintextVector:
        """``Coder.encode_i32_vec`` (paillier.rs:193-200)."""
        return self._encode_int(data, device)

    # ---- vector decode (device) -------------------------------------------------------
    def _decode_float(self, data: PlaintextVector, dtype: torch.dtype) -> torch.Tensor:
        dev = data.device
        n = data.count
        out = torch.empty(n, dtype=dtype, device=dev)
        if n == 0:
            return out
        err = torch.zeros(1, dtype=torch.int32, device=dev)
        lib = _lib.load()
        fn = lib.fphe_decode_f32 if dtype == torch.float32 else lib.fphe_decode_f64
        P = data.P
        _lib.check(fn(self._key.ctx(dev), _ptr(P), P.shape[1], _ptr(data.exp), n, _ptr(out), _ptr(err),
                      ctypes.c_void_p(_stream(dev))), "fphe_decode")
        _raise_err(err)
        return out

    def decode_f32_vec(self, data: PlaintextVector) -> torch.Tensor:
        """``Coder.decode_f32_vec`` (paillier.rs:173-181); returns a device tensor."""
        return self._decode_float(data, torch.float32)

    def decode_f64_vec(self, data: PlaintextVector) -> torch.Tensor:
        """``Coder.decode_f64_vec`` (paillier.rs:153-161); returns a device tensor."""
        return self._decode_float(data, torch.float64)

    def _mantissa(self, sig: int) -> int:
        if sig > self.n:
            raise PanicException("Attempted to decode corrupted number")
        if sig <= self.max_int:
            return sig
        if sig >= self.n - self.max_int:
            return sig - self.n
        raise PanicException("Overflow detected in decrypted number")

    def _decode_int(self, data: PlaintextVector, dtype: torch.dtype) -> torch.Tensor:
        dev = data.device
        n = data.count
        out = torch.empty(n, dtype=dtype, device=dev)
        if n == 0:
            return out
        err = torch.zeros(1, dtype=torch.int32, device=dev)
        lib = _lib.load()
        fn = lib.fphe_decode_i64 if dtype == torch.int64 else lib.fphe_decode_i32
        _lib.check(fn(self._key.ctx(dev), _ptr(data.P), data.P.shape[1], _ptr(data.exp), n, _ptr(out), _ptr(err),
                      ctypes.c_void_p(_stream(dev))), "fphe_decode_int")
        _raise_err(err)
        return out

    def decode_i64_vec(self, data: PlaintextVector) -> List[int]:
        """``Coder.decode_i64_vec`` (paillier.rs:190-192; decode_i64 lib.rs:130-142)."""
        return self._decode_int(data, torch.int64).cpu().tolist()

    def decode_i32_vec(self, data: PlaintextVector) -> List[int]:
        """``Coder.decode_i32_vec`` (paillier.rs:201-203): decode_f64 as i32 (lib.rs:143-146)."""
        return self._decode_int(data, torch.int32).cpu().tolist()

    def pack_floats(self, float_tensor, offset_bit: int, pack_num: int, precision: int,
                    device=None) -> PlaintextVector:
        """``Coder.pack_floats`` (paillier.rs:135-138; lib.rs:79-93), on the device."""
        dev = _device(device if device is not None else (float_tensor.device if isinstance(float_tensor, torch.Tensor)
                                                         and float_tensor.is_cuda else None))
        x = torch.as_tensor(float_tensor).detach().flatten().to(dtype=torch.float64, device=dev).contiguous()
        n = (x.numel() + pack_num - 1) // pack_num
        nt = _ntiles(n)
        L1 = self._key.L1
        out = PlaintextVector(torch.zeros((nt, L1, WAVE), dtype=torch.int32, device=dev),
                              torch.zeros(nt * WAVE, dtype=torch.uint8, device=dev),
                              torch.zeros(nt * WAVE, dtype=torch.int32, device=dev), n)
        if n == 0:
            return out
        err = torch.zeros(1, dtype=torch.int32, device=dev)
        lib = _lib.load()
        _lib.check(lib.fphe_pack_f64(self._key.ctx(dev), _ptr(x), x.numel(), offset_bit, pack_num, precision,
                                     _ptr(out.P), _ptr(out.neg), _ptr(out.exp), _ptr(err),
                                     ctypes.c_void_p(_stream(dev))), "fphe_pack_f64")
        _raise_err(err)
        out.ebound = (0, 0)
        return out

    def unpack_floats(self, packed: PlaintextVector, offset_bit: int, pack_num: int, precision: int,
                      total_num: int) -> List[float]:
        """``Coder.unpack_floats`` (paillier.rs:140-142; lib.rs:94-118), on the device."""
        dev = packed.device
        out = torch.zeros(total_num, dtype=torch.float64, device=dev)
        if total_num and packed.count:
            lib = _lib.load()
            _lib.check(lib.fphe_unpack_f64(self._key.ctx(dev), _ptr(packed.P), packed.P.shape[1], packed.count,
                                           offset_bit, pack_num, precision, total_num, _ptr(out),
                                           ctypes.c_void_p(_stream(dev))), "fphe_unpack_f64")
        return out.cpu().tolist()

    # ---- scalars (length-1 vectors) ---------------------------------------------------
    def encode_f64(self, data: float) -> Plaintext:
        return Plaintext(self.encode_f64_vec(torch.tensor([data], dtype=torch.float64)))

    def encode_f32(self, data: float) -> Plaintext:
        return Plaintext(self.encode_f32_vec(torch.tensor([data], dtype=torch.float32)))

    def encode_i64(self, data: int) -> Plaintext:
        return Plaintext(self.encode_i64_vec(torch.tensor([data], dtype=torch.int64)))

    def encode_i32(self, data: int) -> Plaintext:
        return Plaintext(self.encode_i32_vec(torch.tensor([data], dtype=torch.int64)))

    def decode_f64(self, data: Plaintext) -> float:
        return float(self.decode_f64_vec(data.vec)[0].item())

    def decode_f32(self, data: Plaintext) -> float:
        return float(self.decode_f32_vec(data.vec)[0].item())

    def decode_i64(self, data: Plaintext) -> int:
        return self.decode_i64_vec(data.vec)[0]

    def decode_i32(self, data: Plaintext) -> int:
        return self.decode_i32_vec(data.vec)[0]


class Evaluator:
    """``fate_utils.paillier.Evaluator`` (paillier.rs:414-432)."""

    @staticmethod
    def cat(vec_list: Sequence[CiphertextVector]) -> CiphertextVector:
        n = next((v.n for v in vec_list if v.n is not None), None)
        if n is not None:  # key-less parts (unpickled, zeros()) join a keyed vector under its key
            _resolve_args(n, list(vec_list))
        elif any(v.raw for v in vec_list) and not all(v.raw for v in vec_list if v.count):
            # Montgomery-resident words of an unknown key cannot join signed integers
            raise TypeError("cat of a key-less vector with a vector of unknown key")
        out = Evaluator._cat(vec_list)
        out.n = n
        out.raw = n is None and any(v.raw for v in vec_list if v.count)
        return out

    @staticmethod
    def _cat(vec_list: Sequence[CiphertextVector]) -> CiphertextVector:
        vecs = [v for v in vec_list if v.count > 0]
        if not vecs:
            return CiphertextVector.zeros(0, vec_list[0].L2 if vec_list else 128)
        L2 = max(v.L2 for v in vecs)
        vecs = [_fit_limbs(v, L2) for v in vecs]
        n = sum(v.count for v in vecs)
        if all(v.count % WAVE == 0 for v in vecs[:-1]):  # tile-aligned: concatenate tiles as they are
            C = torch.cat([v.C[: _ntiles(v.count)] for v in vecs], dim=0)
            return CiphertextVector(C,
                                    _pad_flat(torch.cat([v.sign[: v.count] for v in vecs]), n),
                                    _pad_flat(torch.cat([v.exp[: v.count] for v in vecs]), n), n)
        # otherwise each part is scattered to its offset (fphe_permute)
        dev = vecs[0].device
        nt = _ntiles(n)
        out = CiphertextVector(torch.zeros((nt, L2, WAVE), dtype=torch.int32, device=dev),
                               torch.zeros(nt * WAVE, dtype=torch.uint8, device=dev),
                               torch.zeros(nt * WAVE, dtype=torch.int32, device=dev), n)
        off = 0
        for v in vecs:
            _permute(v.C, v.sign, v.exp, L2, torch.arange(off, off + v.count, device=dev), n, True, out.C, out.sign,
                     out.exp, dev)
            off += v.count
        return out

    @staticmethod
    def slice_indexes(a: CiphertextVector, indexes: Sequence[int]) -> CiphertextVector:
        return a.slice_indexes(indexes)


def keygen(bit_length: int) -> Tuple[SK, PK, Coder]:
    """``fate_utils.paillier.keygen`` (paillier.rs:206-210; fixedpoint_paillier::keygen lib.rs:408-413).
    Odd sizes fail as the reference's assert does; even sizes outside :func:`supports` raise
    ``ValueError`` before any key is drawn."""
    if bit_length % 2 == 0 and not supports(bit_length):
        raise ValueError(f"unsupported key size {bit_length}: even {MIN_KEY_BITS}..{MAX_KEY_BITS} run on MI355X")
    p, q = keygen_primes(bit_length)
    return SK(p, q), PK(p * q)._bind_private(p, q), Coder(p * q)


def keypair_from_primes(p: int, q: int, keyholder: bool = True) -> Tuple[SK, PK, Coder]:
    """Deterministic key construction for tests / fixtures.  ``keyholder=False`` gives a
    public-only PK (the encrypting party without the private key)."""
    pk = PK(p * q)
    if keyholder:
        pk._bind_private(p, q)
    return SK(p, q), pk, Coder(p * q)
