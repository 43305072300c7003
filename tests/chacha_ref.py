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
