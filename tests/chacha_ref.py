"""Pure-Python ChaCha20 block function (RFC 8439 §2.3) -- test infrastructure for the
device CSPRNG (fate_amd/csrc/chacha_dev.h), pinned by RFC 8439 §2.3.2's published vector
(tests/test_host.py) before it is used to check the device."""
from typing import List, Sequence

M = 0xFFFFFFFF


def _rotl(x: int, n: int) -> int:
    return ((x << n) | (x >> (32 - n))) & M


def _qr(s: List[int], a: int, b: int, c: int, d: int) -> None:
    s[a] = (s[a] + s[b]) & M; s[d] = _rotl(s[d] ^ s[a], 16)
    s[c] = (s[c] + s[d]) & M; s[b] = _rotl(s[b] ^ s[c], 12)
    s[a] = (s[a] + s[b]) & M; s[d] = _rotl(s[d] ^ s[a], 8)
    s[c] = (s[c] + s[d]) & M; s[b] = _rotl(s[b] ^ s[c], 7)


def chacha20_block(key: Sequence[int], counter: int, nonce: Sequence[int]) -> List[int]:
    """key: 8 LE words, counter: 32-bit, nonce: 3 LE words -> 16 output words."""
    init = [0x61707865, 0x3320646E, 0x79622D32, 0x6B206574, *key, counter & M, *nonce]
    s = list(init)
    for _ in range(10):
        _qr(s, 0, 4, 8, 12); _qr(s, 1, 5, 9, 13); _qr(s, 2, 6, 10, 14); _qr(s, 3, 7, 11, 15)
        _qr(s, 0, 5, 10, 15); _qr(s, 1, 6, 11, 12); _qr(s, 2, 7, 8, 13); _qr(s, 3, 4, 9, 14)
    return [(a + b) & M for a, b in zip(s, init)]


def _le_words(bs: bytes) -> List[int]:
    return [int.from_bytes(bs[i:i + 4], "little") for i in range(0, len(bs), 4)]


# RFC 8439 §2.3.2: key 00:01:..:1f, nonce 00:00:00:09:00:00:00:4a:00:00:00:00, counter 1;
# the state after the block function (the serialized keystream 10 f1 e7 e4 d1 3b 59 15 ...)
RFC8439_232 = (
    _le_words(bytes(range(32))),
    1,
    _le_words(bytes([0, 0, 0, 0x09, 0, 0, 0, 0x4A, 0, 0, 0, 0])),
    [0xE4E7F110, 0x15593BD1, 0x1FDD0F50, 0xC47120A3, 0xC7F4D1C7, 0x0368C033, 0x9AAA2204, 0x4E6CD4C3,
     0x466482D2, 0x09AA9F07, 0x05D7C214, 0xA2028BD9, 0xD19C12B5, 0xB94E16DE, 0xE883D0CB, 0x4E3C50A2],
)
RFC8439_232_SERIALIZED = bytes.fromhex(
    "10f1e7e4d13b5915500fdd1fa32071c4c7d1f4c733c068030422aa9ac3d46c4e"
    "d2826446079faa0914c2d705d98b02a2b5129cd1de164eb9cbd083e8a2503c4e")


# ---- vectorised block function and the library's draws (test infrastructure) ----------------
# The device draws (fate_phe.hip draw_r / draw_below) restated on the host, so that tests can
# recompute the obfuscation a device-drawn encryption used and check its ciphertexts against
# the oracle's encryption with that r.  Pinned against chacha20_block in tests/test_host.py.
def chacha20_blocks_np(key: Sequence[int], counters, nonces):
    """counters: uint32 [N]; nonces: uint32 [N, 3] -> uint32 [N, 16] (one block per row)."""
    import numpy as np
    counters = np.asarray(counters, dtype=np.uint32)
    nonces = np.asarray(nonces, dtype=np.uint32)
    n = counters.shape[0]
    init = np.empty((16, n), dtype=np.uint32)
    init[0:4] = np.array([0x61707865, 0x3320646E, 0x79622D32, 0x6B206574], dtype=np.uint32)[:, None]
    init[4:12] = np.array(list(key), dtype=np.uint32)[:, None]
    init[12] = counters
    init[13:16] = nonces.T
    s = init.copy()

    def rotl(x, k):
        return (x << np.uint32(k)) | (x >> np.uint32(32 - k))

    def qr(a, b, c, d):
        s[a] += s[b]; s[d] = rotl(s[d] ^ s[a], 16)
        s[c] += s[d]; s[b] = rotl(s[b] ^ s[c], 12)
        s[a] += s[b]; s[d] = rotl(s[d] ^ s[a], 8)
        s[c] += s[d]; s[b] = rotl(s[b] ^ s[c], 7)

    with np.errstate(over="ignore"):
        for _ in range(10):
            qr(0, 4, 8, 12); qr(1, 5, 9, 13); qr(2, 6, 10, 14); qr(3, 7, 11, 15)
            qr(0, 5, 10, 15); qr(1, 6, 11, 12); qr(2, 7, 8, 13); qr(3, 4, 9, 14)
        s += init
    return s.T.copy()


DRAW_Z_TAG, DRAW_HALF_TAG = 1 << 31, 1 << 30


def draw_below_host(key: Sequence[int], nonce: int, count: int, bound: int, nwords: int, tag: int = 0,
                    ebase: int = 0) -> List[int]:
    """Element e's draw of the library: uniform in [1, bound - 1] by rejection from e's ChaCha20
    stream (counter = attempt * NB + b | (e >> 32) << 16 | tag, nonce = (e mod 2^32, nonce hi,
    nonce lo)), nwords = the kernel's word count (L1 for r, L1 / 2 for z_p / z_q).  bound = n
    with tag 0 is draw_r (random.rs:22-25's range); bound = p or q with DRAW_Z_TAG (| DRAW_HALF_TAG
    for q) is draw_below of k_draw_z."""
    import numpy as np
    nb = (nwords + 15) // 16
    bits = bound.bit_length()
    out: List[int] = [0] * count
    todo = np.arange(count, dtype=np.int64)
    attempt = 0
    while todo.size:
        e = todo + ebase
        words = np.empty((todo.size, nb * 16), dtype=np.uint32)
        nonces = np.stack([(e & 0xFFFFFFFF).astype(np.uint32),
                           np.full(todo.size, (nonce >> 32) & 0xFFFFFFFF, dtype=np.uint32),
                           np.full(todo.size, nonce & 0xFFFFFFFF, dtype=np.uint32)], axis=1)
        for b in range(nb):
            ctr = ((attempt * nb + b) | ((e >> 32) << 16) | tag).astype(np.uint32)
            words[:, 16 * b:16 * b + 16] = chacha20_blocks_np(key, ctr, nonces)
        words = words[:, :nwords]
        keep = []
        for i, row in zip(todo.tolist(), words):
            x = int.from_bytes(row.astype("<u4").tobytes(), "little") & ((1 << bits) - 1)
            if x < bound - 1:
                out[i] = x + 1
            else:
                keep.append(i)
        todo = np.array(keep, dtype=np.int64)
        attempt += 1
    return out
