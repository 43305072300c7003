"""Wire format of the reference's pickled PHE objects: ``bincode(serde(...))``.

``fate_utils.paillier`` pickles every object as ``bincode::serialize(&self.0)``
(``crates/fate_utils/src/paillier/paillier.rs:67-74`` PK, ``:91-98`` SK, ``:128-135`` Coder,
``:219-226`` CiphertextVector, ``:395-402`` PlaintextVector).  bincode 1.3's default
``serialize`` is fixint little endian: ``i32`` = 4 bytes, a ``Vec`` or ``String`` = ``u64``
length + items, structs and newtypes (``BInt``, ``CT``, ``PT``;
``math/src/rug/mod.rs:11``, ``paillier/src/lib.rs:7,47``) are their fields in order.  rug's
serde support writes an ``Integer`` as the struct ``{radix: i32, value: String}`` with radix 10
when the magnitude has at most 32 significant bits and 16 (lowercase) otherwise, ``-`` for
negatives; this module writes the same and reads any radix 2..36.

Parity status: the struct field order is read off the reference
(``paillier/src/lib.rs:49-69``, ``fixedpoint_paillier/src/lib.rs:18-57,237-241,353-367``);
the rug Integer record layout follows rug 1.20's published serde code and is **unpinned**:
there is no rug, bincode or fate_utils build in this image to produce reference bytes.

Ciphertext vectors are formatted and parsed on the device (``fphe_wire_*`` in
``include/fate_phe.h``): one record length per element, an exclusive scan, then one thread
per (element, 32-bit word) writing or reading that word's 8 hex digits.  The host only walks
the record headers (``fphe_wire_scan``) when parsing.
"""
from __future__ import annotations

import ctypes
import struct
from typing import List, Optional, Tuple

import numpy as np
import torch

from . import _lib
from .paillier import (MAX_INT_FRACTION, CiphertextVector, PK, PlaintextVector, SK, _device, _ptr, _stream)

_DIGITS = "0123456789abcdefghijklmnopqrstuvwxyz"
MIN_RECORD = 4 + 8 + 1 + 4  # radix, length, one digit, exponent


def radix_of(v: int) -> int:
    """rug's serde radix for an Integer: decimal up to 32 significant bits, else hex."""
    return 10 if abs(v).bit_length() <= 32 else 16


# ---- scalar big integers (keys, coders, plaintexts) ------------------------------------
def bint(v: int) -> bytes:
    """One rug ``Integer`` record: i32 radix | u64 len | ``-``? digits (see radix_of)."""
    r = radix_of(v)
    digits = str(abs(v)) if r == 10 else format(abs(v), "x")
    b = (("-" if v < 0 else "") + digits).encode("ascii")
    return struct.pack("<iQ", r, len(b)) + b


def parse_digits(txt: str, radix: int) -> int:
    """rug-style digit string (optional leading ``-``, then digits of ``radix`` only) to an int;
    ``ValueError`` for anything else (Python's int() would also accept ``_``, spaces, ``+``)."""
    neg = txt.startswith("-")
    body = txt[1:] if neg else txt
    if not body or any(c not in _DIGITS[:radix] for c in body.lower()):
        raise ValueError(f"bincode: {txt[:40]!r} is not a radix-{radix} integer")
    v = int(body, radix)
    return -v if neg else v


class Reader:
    """Sequential bincode reader over a bytes buffer; raises ``ValueError`` when truncated."""

    def __init__(self, buf: bytes, pos: int = 0):
        self.buf, self.pos = memoryview(buf), pos

    def _take(self, n: int) -> memoryview:
        if self.pos + n > len(self.buf):
            raise ValueError("bincode: truncated buffer")
        out = self.buf[self.pos: self.pos + n]
        self.pos += n
        return out

    def i32(self) -> int:
        return struct.unpack("<i", self._take(4))[0]

    def u64(self) -> int:
        return struct.unpack("<Q", self._take(8))[0]

    def bint(self) -> int:
        radix = self.i32()
        if not 2 <= radix <= 36:
            raise ValueError(f"bincode: Integer radix {radix} outside 2..36")
        try:
            s = bytes(self._take(self.u64())).decode("ascii")
        except UnicodeDecodeError as exc:
            raise ValueError("bincode: non-ASCII Integer digits") from exc
        return parse_digits(s, radix)

    def done(self) -> None:
        if self.pos != len(self.buf):
            raise ValueError("bincode: trailing bytes")


def _sk_fields(p: int, q: int) -> List[int]:
    """``paillier::SK`` fields in declaration order, as ``SK::new`` computes them
    (``paillier/src/lib.rs:56-69,124-150``; p < q)."""
    p, q = (p, q) if p < q else (q, p)
    n, ps, qs = p * q, p * p, q * q
    g = n + 1
    hp = pow((pow(g, p - 1, ps) - 1) // p, -1, p)
    hq = pow((pow(g, q - 1, qs) - 1) // q, -1, q)
    return [p, q, n, p - 1, q - 1, ps, qs, pow(p, -1, q), hp, hq]


def pk_to_bincode(pk: PK) -> bytes:
    """``fixedpoint_paillier::PK {pk: paillier::PK {n, ns}, max_int}`` (lib.rs:18-22)."""
    return bint(pk.n) + bint(pk.n * pk.n) + bint(pk.n // MAX_INT_FRACTION)


def pk_from_bincode(buf: bytes) -> PK:
    r = Reader(buf)
    n, ns, max_int = r.bint(), r.bint(), r.bint()
    r.done()
    if ns != n * n or max_int != n // MAX_INT_FRACTION:
        raise ValueError("bincode PK: inconsistent n / ns / max_int")
    return PK(n)


def sk_to_bincode(sk: SK) -> bytes:
    """``fixedpoint_paillier::SK {sk: paillier::SK {p, q, n, p_minus_one, ...}}``."""
    return b"".join(bint(v) for v in _sk_fields(sk.p, sk.q))


def sk_from_bincode(buf: bytes) -> SK:
    r = Reader(buf)
    vals = [r.bint() for _ in range(10)]
    r.done()
    if vals != _sk_fields(vals[0], vals[1]):
        raise ValueError("bincode SK: fields inconsistent with p, q")
    return SK(vals[0], vals[1])


def coder_to_bincode(n: int) -> bytes:
    """``Coder {n, max_int}`` (fixedpoint_paillier/src/lib.rs:54-58)."""
    return bint(n) + bint(n // MAX_INT_FRACTION)


def coder_from_bincode(buf: bytes) -> int:
    r = Reader(buf)
    n, max_int = r.bint(), r.bint()
    r.done()
    if max_int != n // MAX_INT_FRACTION:
        raise ValueError("bincode Coder: inconsistent max_int")
    return n


def plaintext_vector_to_bincode(pv: PlaintextVector) -> bytes:
    """``PlaintextVector {data: Vec<Plaintext {significant, exp}>}`` (lib.rs:358-367)."""
    sigs, exps = pv.to_ints()
    return struct.pack("<Q", len(sigs)) + b"".join(bint(s) + struct.pack("<i", e) for s, e in zip(sigs, exps))


def plaintext_vector_from_bincode(buf: bytes, device=None) -> PlaintextVector:
    r = Reader(buf)
    n = r.u64()
    if n > (len(buf) - 8) // MIN_RECORD:
        raise ValueError("bincode PlaintextVector: element count larger than the buffer holds")
    sigs, exps = [], []
    for _ in range(n):
        sigs.append(r.bint())
        exps.append(r.i32())
    r.done()
    return PlaintextVector.from_ints(sigs, exps, device=device)


# ---- ciphertext vectors, on the device --------------------------------------------------
def ciphertext_vector_records(cv: CiphertextVector, pk: Optional[PK] = None) -> Tuple[bytes, torch.Tensor]:
    """The bincode of ``cv`` as (the 8-byte length header, the records as a DEVICE uint8
    tensor): each record is ``Ciphertext {significant_encryped, exp}`` of the reference's signed
    integer (under ``pk``, else the key the vector carries), formatted on the device.  The
    caller moves the records to where they go (a pinned buffer, the transport)."""
    n = cv.count
    head = struct.pack("<Q", n)
    dev = cv.device
    if n == 0:
        return head, torch.empty(0, dtype=torch.uint8, device=dev)
    lib = _lib.load()
    mag, neg, exp = cv.export_signed(pk) if pk is not None else cv.signed_rows()
    L = int(mag.shape[1])
    s = ctypes.c_void_p(_stream(dev))
    rec_len = torch.empty(n, dtype=torch.int64, device=dev)
    radix = torch.empty(n, dtype=torch.uint8, device=dev)
    with torch.cuda.device(dev):  # context-less entry points launch on the current device
        _lib.check(lib.fphe_wire_lengths(_ptr(mag), _ptr(neg), L, n, _ptr(rec_len), _ptr(radix), s),
                   "fphe_wire_lengths")
    ends = torch.cumsum(rec_len, 0)
    total = int(ends[-1].item())
    rec_off = ends - rec_len
    out = torch.empty(total, dtype=torch.uint8, device=dev)
    exp = exp.to(torch.int32).contiguous()
    with torch.cuda.device(dev):
        _lib.check(lib.fphe_wire_encode(_ptr(mag), _ptr(neg), _ptr(exp), L, n, _ptr(rec_off), _ptr(rec_len),
                                        _ptr(radix), _ptr(out), s), "fphe_wire_encode")
    return head, out


def ciphertext_vector_to_bincode(cv: CiphertextVector, pk: Optional[PK] = None) -> bytes:
    """``CiphertextVector {data: Vec<Ciphertext {significant_encryped, exp}>}``
    (fixedpoint_paillier/src/lib.rs:237-241,353-356) of the reference's signed integers
    (under ``pk``, else the key the vector carries)."""
    head, out = ciphertext_vector_records(cv, pk)
    if out.numel() == 0:
        return head
    res = bytearray(8 + out.numel())
    res[:8] = head
    torch.from_numpy(np.frombuffer(res, dtype=np.uint8)[8:]).copy_(out)  # D2H straight into the result
    return bytes(res)


# magnitude widths (32-bit words) of the kernels' geometries: n^2 of <= 1024-, <= 2048- and
# <= 4096-bit keys; a key-less (raw) vector is read at the smallest one that holds its values
RAW_WIDTHS = (64, 128, 256)


def _digit_bits(dig_len: np.ndarray, radix: np.ndarray) -> int:
    """An upper bound of the bit length of the widest record."""
    if dig_len.size == 0:
        return 0
    return int(np.max(np.ceil(dig_len * np.log2(np.maximum(radix, 2)))))


def ciphertext_vector_from_bincode(buf: bytes, pk: Optional[PK] = None, device=None
                                   ) -> Tuple[CiphertextVector, int]:
    """Parse a ``CiphertextVector`` starting at ``buf[0]``; returns (vector, bytes consumed).
    Radix-16 records and radix-10 records of up to 19 digits (what rug writes) are decoded on
    the device; any other radix (valid for rug's parser) is parsed on the host.  With ``pk``
    the vector is converted under that key (ValueError for |c| >= n^2); without, it stays in
    the reference's key-less signed form (``raw``) until an operation supplies the key.
    Raises ``ValueError`` on a malformed record."""
    dev = _device(device)
    if len(buf) < 8:
        raise ValueError("bincode: truncated buffer")
    n = struct.unpack_from("<Q", buf, 0)[0]
    L = pk._key.L2 if pk is not None else RAW_WIDTHS[0]
    if n == 0:
        return CiphertextVector.empty(0, L, dev), 8
    if n > (len(buf) - 8) // MIN_RECORD:  # before sizing anything by an untrusted count
        raise ValueError("bincode CiphertextVector: element count larger than the buffer holds")
    lib = _lib.load()
    raw = np.frombuffer(buf, dtype=np.uint8)
    dig_off = np.empty(n, dtype=np.int64)
    dig_len = np.empty(n, dtype=np.int32)
    neg = np.empty(n, dtype=np.uint8)
    exp = np.empty(n, dtype=np.int32)
    radix = np.empty(n, dtype=np.int32)
    end = ctypes.c_size_t(0)
    st = lib.fphe_wire_scan(raw.ctypes.data, raw.size, 8, n, dig_off.ctypes.data, dig_len.ctypes.data,
                            neg.ctypes.data, exp.ctypes.data, radix.ctypes.data, ctypes.byref(end))
    if st != _lib.FPHE_OK:
        raise ValueError("bincode CiphertextVector: malformed or truncated record")
    used = int(end.value)
    if pk is None:
        bits = _digit_bits(dig_len, radix)
        fits = [w for w in RAW_WIDTHS if 32 * w >= bits]
        L = fits[0] if fits else RAW_WIDTHS[-1]  # wider than any supported n^2: rejected below
    s = ctypes.c_void_p(_stream(dev))
    dbuf = torch.from_numpy(raw[:used].copy()).to(dev)
    mag = torch.zeros((n, L), dtype=torch.int32, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    on_device = (radix == 16) | ((radix == 10) & (dig_len <= 19))
    if on_device.all():
        d_off = torch.from_numpy(dig_off).to(dev)  # held until the launch is queued
        d_len = torch.from_numpy(dig_len).to(dev)
        d_rdx = torch.from_numpy(radix).to(dev)
        with torch.cuda.device(dev):  # context-less: launches on the current device
            _lib.check(lib.fphe_wire_decode(_ptr(dbuf), _ptr(d_off), _ptr(d_len), _ptr(d_rdx), L, n, _ptr(mag),
                                            _ptr(err), s), "fphe_wire_decode")
    else:
        words = np.zeros((n, L), dtype=np.uint32)
        for e in range(n):
            try:
                txt = bytes(raw[dig_off[e]: dig_off[e] + dig_len[e]]).decode("ascii")
            except UnicodeDecodeError as exc:
                raise ValueError("bincode CiphertextVector: non-ASCII digits") from exc
            v = parse_digits(txt, int(radix[e]))  # the sign was taken off by the scan
            if v < 0 or v.bit_length() > 32 * L:
                raise ValueError("bincode CiphertextVector: malformed value or wider than n^2")
            words[e] = np.frombuffer(v.to_bytes(4 * L, "little"), dtype=np.uint32)
        mag = torch.from_numpy(words.view(np.int32)).to(dev)
    if int(err.item()):
        raise ValueError("bincode CiphertextVector: bad digit or value wider than n^2")
    negd, expd = torch.from_numpy(neg).to(dev), torch.from_numpy(exp).to(dev)
    if pk is None:
        from .paillier import _pad_flat, rows_to_tile_tensor
        return CiphertextVector(rows_to_tile_tensor(mag), _pad_flat(negd, n), _pad_flat(expd, n), n, None,
                                raw=True), used
    _check_below(mag, pk.n * pk.n)
    cv = CiphertextVector.import_signed(pk, mag, negd, expd)
    return cv, used


def _check_below(mag: torch.Tensor, bound: int) -> None:
    """Every magnitude (element-major LSF uint32 words) < bound, compared word-wise from the top."""
    L = mag.shape[1]
    b = torch.from_numpy(np.frombuffer(bound.to_bytes(4 * L, "little"), dtype=np.uint32).astype(np.int64)).to(mag.device)
    m = mag.to(torch.int64) & 0xFFFFFFFF
    diff = (m != b).flip(1)
    first = torch.argmax(diff.to(torch.int8), dim=1)  # most significant differing word
    idx = (L - 1 - first).unsqueeze(1)
    less = m.gather(1, idx).squeeze(1) < b[idx.squeeze(1)]
    if not bool((diff.any(1) & less).all()):
        raise ValueError("bincode CiphertextVector: |value| >= n^2")
