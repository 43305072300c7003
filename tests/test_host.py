"""CPU tests of the host side: the C-ABI library loads and exports every symbol declared in
include/fate_phe.h (no compute calls without a GPU), tile-layout plumbing, key
generation, and the product path refuses to run without the HIP extension / device."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    with open(os.path.join(ROOT, "include", "fate_phe.h")) as f:
        text = f.read()
    return sorted(set(re.findall(r"\b(fphe_[a-z0-9_]+)\s*\(", text)))


def test_header_symbols_listed_in_binding():
    from fate_amd import _lib
    assert header_symbols() == sorted(_lib.EXPORTED_SYMBOLS)


def test_library_exports_every_header_symbol():
    from fate_amd import _lib
    assert os.path.exists(_lib.LIB_PATH), "build libfatephe.so first (__graft_entry__.build())"
    lib = ctypes.CDLL(_lib.LIB_PATH)
    for name in header_symbols():
        assert hasattr(lib, name), name
    assert _lib.load() is not None


def test_header_is_plain_c_and_links(tmp_path):
    """include/fate_phe.h is a plain C header (what a cgo / Rust FFI binding includes) and a
    C program linking only libfatephe.so and the HIP runtime builds against it
    (tests/c_abi/abi_roundtrip.c, run on the GPU by tests/test_gpu_c_abi.py)."""
    import subprocess
    inc = os.path.join(ROOT, "include")
    subprocess.run(["gcc", "-std=c11", "-Wall", "-Wextra", "-Werror", "-fsyntax-only", "-x", "c",
                    os.path.join(inc, "fate_phe.h")], check=True)
    out = tmp_path / "abi_roundtrip"
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "tests", "c_abi"), f"abi_roundtrip"], check=True)
    subprocess.run(["gcc", "-O2", "-std=c11", "-Wall", "-Wextra", "-Werror", "-D__HIP_PLATFORM_AMD__", f"-I{inc}",
                    "-I/opt/rocm/include", "-o", str(out), os.path.join(ROOT, "tests", "c_abi", "abi_roundtrip.c"),
                    "-L" + os.path.join(ROOT, "fate_amd", "lib"), "-lfatephe", "-L/opt/rocm/lib", "-lamdhip64"],
                   check=True)
    assert out.exists()


def test_tile_layout_roundtrip():
    from fate_amd import paillier as P
    rng = np.random.default_rng(0)
    for count, L in [(1, 4), (63, 8), (64, 8), (65, 16), (300, 128)]:
        rows = rng.integers(0, 2 ** 32, size=(count, L), dtype=np.uint64).astype(np.uint32)
        tiles = P.rows_to_tiles(rows)
        assert tiles.shape == ((count + 63) // 64, L, 64)
        assert np.array_equal(P.tiles_to_rows(tiles, count), rows)
        t = torch.from_numpy(tiles.view(np.int32))
        cols = P.tiles_to_cols(t)
        assert np.array_equal(cols[:, :count].numpy().view(np.uint32), rows.T)
        assert torch.equal(P.cols_to_tiles(cols), t)
    vals = [0, 1, 2 ** 32 - 1, 2 ** 64 + 5, 2 ** 255 - 19]
    assert P.limbs_to_ints(P.ints_to_limbs(vals, 8)) == vals


def test_keygen_sizes():
    from fate_amd._keygen import keygen_primes, is_probable_prime
    p, q = keygen_primes(1024)
    assert p < q and (p * q).bit_length() == 1024
    assert is_probable_prime(p) and is_probable_prime(q)
    assert not is_probable_prime(p * q)


def test_no_cpu_fallback_without_device():
    """The product path fails loudly instead of computing on the CPU."""
    if torch.cuda.is_available():
        pytest.skip("device present")
    from fate_amd import paillier as P
    with pytest.raises(RuntimeError):
        P.CiphertextVector.zeros(4)
    coder = P.Coder(int("f" * 256, 16))
    with pytest.raises((RuntimeError, ValueError)):
        coder.encode_f32_vec(torch.zeros(4))


def test_protocol_surface_matches_reference():
    """fate_amd.protocol exposes the reference plugin names (paillier.py:33-399)."""
    from fate_amd import protocol
    for name in ("keygen", "evaluator", "SK", "PK", "Coder"):
        assert hasattr(protocol, name)
    # the TensorEvaluator static methods of protocol/phe/paillier.py:179-399
    for m in ("add", "add_plain", "add_plain_scalar", "sub", "sub_plain", "sub_plain_scalar", "rsub",
              "rsub_plain", "rsub_plain_scalar", "mul_plain", "mul_plain_scalar", "matmul", "rmatmul", "zeros",
              "i_add", "i_sub", "slice", "i_shuffle", "shuffle", "i_update", "i_update_with_masks",
              "intervals_slice", "cat", "chunking_cumsum_with_step", "pack_squeeze"):
        assert callable(getattr(protocol.evaluator, m)), m
    for m in ("encode_tensor", "decode_tensor", "encode_vec", "decode_vec", "encode", "encode_f32_vec",
              "decode_f32_vec", "encode_i64_vec", "decode_i64_vec"):
        assert callable(getattr(protocol.Coder, m))


def test_ciphertext_vector_surface_matches_reference():
    """fate_amd.paillier.CiphertextVector has the pyo3 methods of paillier.rs:213-387."""
    from fate_amd.paillier import CiphertextVector
    for m in ("zeros", "pack_squeeze", "slice", "slice_indexes", "cat", "i_shuffle", "shuffle", "intervals_slice",
              "iadd_slice", "iadd_vec_self", "isub_vec_self", "iadd_vec", "isub_vec", "iupdate",
              "iupdate_with_masks", "iadd", "idouble", "chunking_cumsum_with_step", "intervals_sum_with_step",
              "tolist", "add", "add_scalar", "sub", "sub_scalar", "rsub", "rsub_scalar", "mul", "mul_scalar",
              "matmul", "rmatmul", "__len__"):
        assert callable(getattr(CiphertextVector, m)), m


def test_tile_gather_assign_cat_plumbing():
    from fate_amd import paillier as P
    """Layout helpers of the tile-major format agree with the element-major view (host logic,
    CPU tensors); the device gather/scatter (fphe_permute) is checked in test_gpu_edges."""
    t = torch.randint(0, 2**31 - 1, (5, 7, 64), dtype=torch.int32)
    idx = torch.tensor([3, 200, 64, 0, 319, 5])
    cols = P.tiles_to_cols(t)
    rows = P.gather_rows(t, idx)
    assert torch.equal(rows, cols[:, idx].T)
    assert torch.equal(P.rows_to_tile_tensor(rows), P.cols_to_tiles(cols[:, idx]))


def test_chacha20_reference_pinned_by_rfc8439():
    """The Python ChaCha20 restatement the device CSPRNG is checked against reproduces RFC
    8439 §2.3.2 (state words and serialized keystream)."""
    from tests.chacha_ref import RFC8439_232, RFC8439_232_SERIALIZED, chacha20_block
    key, counter, nonce, want = RFC8439_232
    got = chacha20_block(key, counter, nonce)
    assert got == want
    assert b"".join(w.to_bytes(4, "little") for w in got) == RFC8439_232_SERIALIZED


def test_chacha20_vectorised_and_draws_match_scalar():
    """The vectorised block function (tests/chacha_ref.chacha20_blocks_np) equals the scalar
    one on RFC 8439's vector and other counters / nonces, and draw_below_host follows the
    library's stream layout: element e, attempt 0 reads blocks (b | tag, (e, nonce hi, lo)),
    keeps bits(bound) bits and accepts x < bound - 1 as r = x + 1 (random.rs:22-25)."""
    import numpy as np
    from tests.chacha_ref import (DRAW_Z_TAG, RFC8439_232, chacha20_block, chacha20_blocks_np,
                                  draw_below_host)
    key, counter, nonce, want = RFC8439_232
    ctrs = [counter, 0, 7, 0xFFFFFFFF, 1 << 31]
    nonces = [nonce, [1, 2, 3], [0, 0, 0], [0xFFFFFFFF] * 3, [5, 0xDEADBEEF, 9]]
    got = chacha20_blocks_np(key, ctrs, nonces)
    assert got[0].tolist() == want
    for i in range(len(ctrs)):
        assert got[i].tolist() == chacha20_block(key, ctrs[i], nonces[i])
    bound = (1 << 200) - 12345  # acceptance ~1: attempt 0 for every element
    nonce64 = (7 << 32) | 11
    r = draw_below_host(key, nonce64, 5, bound, 8, DRAW_Z_TAG)
    for e in range(5):
        w = chacha20_block(key, DRAW_Z_TAG, [e, 7, 11])[:8]
        x = int.from_bytes(np.array(w, dtype="<u4").tobytes(), "little") & ((1 << 200) - 1)
        assert r[e] == (x + 1 if x < bound - 1 else r[e])
        assert 1 <= r[e] < bound


def test_chacha20_symbol_exported():
    from fate_amd import _lib
    assert "fphe_chacha20_blocks" in _lib.EXPORTED_SYMBOLS


def test_key_size_gate():
    """Even sizes 256..4096 run on the device geometries (1024-, 2048-, 4096-bit); others
    decline at keygen (ValueError) before any prime is drawn; odd sizes fail like the
    reference's assert (paillier/src/lib.rs:73)."""
    import pytest
    from fate_amd import paillier as P
    from fate_amd import protocol as PR
    assert all(PR.supports(b) for b in (256, 512, 1024, 1030, 1536, 2048, 2050, 3072, 4096))
    assert not any(PR.supports(b) for b in (254, 1023, 4098, 8192))
    with pytest.raises(ValueError):
        PR.keygen(4098)
    with pytest.raises(AssertionError):
        P.keygen(1023)
    pk = P.PK(P.keygen(512)[1].n)
    assert pk._key.L1 == 32 and pk._key.L2 == 64
    assert P.PK((1 << 3071) + 1)._key.L2 == 256


def test_path_options_set_and_restore():
    """fate_amd.paillier.path_options (fphe_ctx_set_option on every context; none exist on the
    CPU): the block's settings, then the previous ones again; None means the library default;
    an unknown name raises before anything changes."""
    import pytest
    from fate_amd import paillier as P
    before_sq = P.WIDE_SQUEEZE_MAX_CHUNKS
    before = dict(P._PATH_OPTIONS)
    with P.path_options(**P.THROUGHPUT_PATHS, kh_direct_z=0):
        assert P._PATH_OPTIONS[P._OPTION_IDS["wide_decrypt_max"]] == 0
        assert P._PATH_OPTIONS[P._OPTION_IDS["kh_direct_z"]] == 0
        assert P.WIDE_SQUEEZE_MAX_CHUNKS == 0
        with P.path_options(wide_decrypt_max=7):
            assert P._PATH_OPTIONS[P._OPTION_IDS["wide_decrypt_max"]] == 7
        assert P._PATH_OPTIONS[P._OPTION_IDS["wide_decrypt_max"]] == 0
    assert P._PATH_OPTIONS == before and P.WIDE_SQUEEZE_MAX_CHUNKS == before_sq
    with pytest.raises(ValueError, match="unknown path option"):
        P.set_path_options(wide_decrypt_max=1, no_such_option=3)
    assert P._PATH_OPTIONS == before
    # the library's enum values (include/fate_phe.h)
    from fate_amd import _lib
    hdr = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "fate_phe.h")).read()
    for name in ("WIDE_DECRYPT_MAX", "WIDE_ENCRYPT_MAX", "WIDE_KH_ENCRYPT_MAX", "KH_DIRECT_Z"):
        assert f"FPHE_OPT_{name} = {getattr(_lib, 'OPT_' + name)}," in hdr


def test_position_lists_host_helper():
    """The reference's Vec<Vec<usize>> position lists (paillier.rs:261-283) read by the CPython
    helper (fate_amd/csrc/host_positions.c): same order as walking them in Python, ragged and
    empty lists, tuples, numpy integers and iterables; a non-integer position is a TypeError
    (pyo3's usize extraction), a non-sequence sample likewise."""
    import itertools
    import random

    from fate_amd import paillier as P
    rng = random.Random(3)
    lists = [[rng.randrange(1 << 20) for _ in range(rng.randrange(0, 5))] for _ in range(2000)]
    lists[7] = (3, 1, 2)
    lists[8] = [np.int64(5), np.int32(9)]
    lens, pos = P._position_lists(lists)
    assert lens.tolist() == [len(x) for x in lists]
    assert pos.tolist() == [int(v) for v in itertools.chain.from_iterable(lists)]
    lens, pos = P._position_lists(iter([[1, 2], [], [3]]))
    assert lens.tolist() == [2, 0, 1] and pos.tolist() == [1, 2, 3]
    lens, pos = P._position_lists([])
    assert lens.size == 0 and pos.size == 0
    ii, pp = P._flatten_positions([[4], [], [5, 6]], None)
    assert ii.tolist() == [0, 2, 2] and pp.tolist() == [4, 5, 6]
    with pytest.raises(TypeError):
        P._position_lists([[1, 2.5]])
    with pytest.raises(TypeError):
        P._position_lists([[1], 7])
    with pytest.raises(OverflowError):
        P._position_lists([[1 << 70]])


def test_interval_bounds_follow_the_reference():
    """intervals_slice's checks in the reference's order (lib.rs:499-513): the first failing
    interval decides; an end past the data is the anyhow error (RuntimeError), a start past its
    end the slice panic; a negative bound is pyo3's usize error.  Checked before any device
    work, so a CPU-resident vector shows them."""
    from fate_amd import paillier as P
    v = P.CiphertextVector(torch.zeros((1, 128, 64), dtype=torch.int32), torch.zeros(64, dtype=torch.uint8),
                           torch.zeros(64, dtype=torch.int32), 10)
    with pytest.raises(RuntimeError, match="end index out of range: start=3, end=11, data_size=10"):
        v.intervals_slice([(0, 2), (3, 11), (5, 4)])
    with pytest.raises(P.PanicException, match="slice index starts at 5 but ends at 4"):
        v.intervals_slice([(0, 2), (5, 4), (3, 11)])
    with pytest.raises(OverflowError):
        v.intervals_slice([(-1, 2)])
    s, e = P._interval_array([(2, 5), (0, 0), (7, 9)])
    idx, rel = P._interval_items(s, e)
    assert idx.tolist() == [2, 3, 4, 7, 8] and rel.tolist() == [0, 1, 2, 0, 1]



def _ref_i_shuffle(data, indexes):
    """The oracle's transcription of the reference walk (oracle/paillier_oracle.py i_shuffle,
    lib.rs:473-490), on a copy; IndexError where Rust panics."""
    from oracle import paillier_oracle as O
    data = list(data)
    O.i_shuffle(data, indexes)
    return data

def test_i_shuffle_cycle_walk_matches_reference():
    """i_shuffle's walk replayed on positions by the host helper equals the reference's walk on
    the data for permutations (new[i] = old[indexes[i]]) and for any other index list
    (duplicates, fixed points, longer lists); a short list or an index past the data panics
    where the reference does (the first out-of-bounds access, with its message)."""
    import random

    from fate_amd import paillier as P
    rng = random.Random(8)
    for n in (1, 2, 7, 64, 1000):
        perm = list(range(n))
        rng.shuffle(perm)
        got = P._cycle_walk(np.array(perm), n)
        assert got.tolist() == _ref_i_shuffle(range(n), perm) == perm
        for _ in range(20):
            ix = [rng.randrange(n) for _ in range(n + rng.randrange(3))]
            assert P._cycle_walk(np.array(ix), n).tolist() == _ref_i_shuffle(range(n), ix)
    for ix, n in (([1, 2], 3), ([0, 5, 1], 3), ([2, 0, 7, 1], 4)):
        try:
            _ref_i_shuffle(range(n), ix)
            raise AssertionError("the reference walk should fail")
        except IndexError:
            pass
        with pytest.raises(P.PanicException, match="index out of bounds"):
            P._cycle_walk(np.array(ix), n)
    with pytest.raises(OverflowError):
        P._index_array([3, -1])
    with pytest.raises(TypeError):
        P._index_array([1.5])
    assert P._index_array(torch.tensor([4, 2])).tolist() == [4, 2]


def test_open_ended_ranges_panic_as_the_reference():
    """Range checks that fire before any device work, in the reference's order and words:
    iadd_vec / isub_vec with size None slice data[sa..] and other[sb..] (lib.rs:634-722),
    iadd_vec_self with size None (:521-568), and chunking_cumsum_with_step, whose chunks no
    longer than the step touch nothing (:763-774)."""
    from fate_amd import paillier as P

    def vec(count):
        nt = (count + 63) // 64
        return P.CiphertextVector(torch.zeros((nt, 128, 64), dtype=torch.int32),
                                  torch.zeros(nt * 64, dtype=torch.uint8), torch.zeros(nt * 64, dtype=torch.int32),
                                  count)
    pk = P.PK((1 << 1023) + 1155)  # any odd n: the key is never used before the checks fire
    a, b = vec(10), vec(6)
    with pytest.raises(P.PanicException, match="range start index 11 out of range for slice of length 10"):
        a.iadd_vec(b, 11, 0, None, pk)
    with pytest.raises(P.PanicException, match="range start index 7 out of range for slice of length 6"):
        a.isub_vec(b, 0, 7, None, pk)
    with pytest.raises(P.PanicException, match="range start index 12 out of range for slice of length 10"):
        a.iadd_vec_self(12, 12, None, pk)
    with pytest.raises(P.PanicException, match="the len is 10 but the index is 13"):
        a.isub_vec_self(2, 13, None, pk)
    with pytest.raises(P.PanicException, match="the len is 10 but the index is 10"):
        a.chunking_cumsum_with_step(pk, [5, 7], 2)
    with pytest.raises(P.PanicException, match="the len is 10 but the index is 12"):
        a.chunking_cumsum_with_step(pk, [10, 9], 2)
    a.chunking_cumsum_with_step(pk, [2, 2, 2, 2, 2, 2, 1], 2)  # past the data, but no chunk longer than the step


def test_pack_squeeze_zero_pack_num_panics():
    """pack_squeeze's self.data.chunks(pack_num) (lib.rs:439-450) panics for 0, before any
    device work."""
    from fate_amd import paillier as P
    v = P.CiphertextVector(torch.zeros((1, 128, 64), dtype=torch.int32), torch.zeros(64, dtype=torch.uint8),
                           torch.zeros(64, dtype=torch.int32), 5)
    with pytest.raises(P.PanicException, match="chunk size must be non-zero"):
        v.pack_squeeze(0, 10, P.PK((1 << 1023) + 1155))
