"""Drop-in replacement for ``fate.arch.protocol.phe.paillier`` on MI355X.

Mirrors python/fate/arch/protocol/phe/paillier.py:33-399 (SK / PK / Coder wrappers,
``keygen(key_size)`` and the ``evaluator`` TensorEvaluator plugin, type.py:24) with the
same method names, argument meaning and error behaviour, over :mod:`fate_amd.paillier`
(the mirror of ``fate_utils.paillier``).  A FATE deployment selects it where
``PHECipherBuilder.setup`` imports ``fate.arch.protocol.phe.paillier``
(python/fate/arch/context/_cipher.py:111-124); see INTEGRATION.md.

Route A (:mod:`fate_amd.compat`) runs FATE's own adapter file unchanged; this module is
Route B and keeps only what differs from that file: tensors may be CUDA (HIP) tensors --
encoding reads them in place in HBM instead of calling ``.numpy()`` (paillier.py:159-161),
decoding returns a tensor on the requested device -- and :func:`supports` gates key sizes.
The pass-through methods are generated from name tables rather than written out.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch

from . import paillier as _p
from .paillier import CiphertextVector, PlaintextVector

V = torch.Tensor
EV = CiphertextVector
FV = PlaintextVector


class SK:
    def __init__(self, sk: _p.SK):
        self.sk = sk

    def decrypt_to_encoded(self, vec: EV) -> FV:
        return self.sk.decrypt_to_encoded(vec)


class PK:
    def __init__(self, pk: _p.PK):
        self.pk = pk

    def encrypt_encoded(self, vec: FV, obfuscate: bool) -> EV:
        return self.pk.encrypt_encoded(vec, obfuscate)

    def encrypt_encoded_scalar(self, val, obfuscate) -> EV:
        return self.pk.encrypt_encoded_scalar(val, obfuscate)


# dtype -> the fate_utils Coder method suffix (paillier.py:79-93, 128-140)
_SUFFIX = {torch.float64: "f64", torch.float32: "f32", torch.int64: "i64", torch.int32: "i32"}


def _suffix(dtype) -> str:
    if dtype not in _SUFFIX:
        raise NotImplementedError(f"{dtype} not supported")
    return _SUFFIX[dtype]


class Coder:
    def __init__(self, coder: _p.Coder):
        self.coder = coder

    def pack_floats(self, float_tensor: V, offset_bit: int, pack_num: int, precision: int) -> FV:
        """paillier.py:56-57 (device tensor in, no .tolist() round trip)."""
        return self.coder.pack_floats(float_tensor.detach(), offset_bit, pack_num, precision)

    def unpack_floats(self, packed: FV, offset_bit: int, pack_num: int, precision: int, total_num: int) -> V:
        """paillier.py:59-60."""
        return torch.tensor(self.coder.unpack_floats(packed, offset_bit, pack_num, precision, total_num))

    def encode_tensor(self, tensor: V, dtype: torch.dtype = None) -> FV:
        # paillier.py:68-69 encodes by tensor.dtype and ignores `dtype`
        return self.encode_vec(tensor.flatten(), dtype=tensor.dtype)

    def decode_tensor(self, tensor: FV, dtype: torch.dtype, shape: torch.Size = None, device=None) -> V:
        data = self.decode_vec(tensor, dtype)
        if shape is not None:
            data = data.reshape(shape)
        if device is not None:
            data = data.to(device.to_torch_device() if hasattr(device, "to_torch_device") else device)
        return data

    def encode_vec(self, vec: V, dtype: torch.dtype = None) -> FV:
        if dtype is None:
            dtype = vec.dtype
        elif dtype != vec.dtype:
            vec = vec.to(dtype=dtype)
        return getattr(self, f"encode_{_suffix(dtype)}_vec")(vec)

    def decode_vec(self, vec: FV, dtype: torch.dtype) -> V:
        return getattr(self, f"decode_{_suffix(dtype)}_vec")(vec)

    def encode(self, val, dtype=None):
        if isinstance(val, torch.Tensor):
            assert val.ndim == 0, "only scalar supported"
            dtype = val.dtype
            val = val.item()
        return getattr(self.coder, f"encode_{_suffix(dtype)}")(val)


def _coder_methods() -> None:
    """encode_X / decode_X pass through; encode_X_vec flattens the (device) tensor in place;
    decode_X_vec returns a CPU tensor, as paillier.py's torch.tensor does (paillier.py:141-171:
    integer lists become int64 tensors, decode_vec included)."""
    for sfx in _SUFFIX.values():
        for kind in ("encode", "decode"):
            name = f"{kind}_{sfx}"
            setattr(Coder, name, lambda self, val, _n=name: getattr(self.coder, _n)(val))
        setattr(Coder, f"encode_{sfx}_vec",
                lambda self, vec, _n=f"encode_{sfx}_vec": getattr(self.coder, _n)(vec.detach().flatten()))
        if sfx in ("f64", "f32"):
            dec = lambda self, vec, _n=f"decode_{sfx}_vec": getattr(self.coder, _n)(vec).cpu()
        else:
            dec = lambda self, vec, _n=f"decode_{sfx}_vec": torch.tensor(getattr(self.coder, _n)(vec))
        setattr(Coder, f"decode_{sfx}_vec", dec)


_coder_methods()


def supports(key_size: int) -> bool:
    """Whether this backend runs keys of ``key_size`` bits (even, 256..4096).  The
    ``PHECipherBuilder.setup`` branch in INTEGRATION.md keeps FATE's CPU module for the rest
    (the reference accepts any even size, paillier/src/lib.rs:72-87)."""
    return _p.supports(key_size)


def keygen(key_size):
    """paillier.py:174-176.  ValueError for sizes :func:`supports` rejects."""
    sk, pk, coder = _p.keygen(key_size)
    return SK(sk), PK(pk), Coder(coder)


def _encrypted(b, pk: PK, coder: Coder, output_dtype, scalar: bool) -> EV:
    """The plain operand of add/sub/rsub_plain(_scalar): encoded, encrypted without
    obfuscation (paillier.py:187-262)."""
    if scalar:
        return pk.encrypt_encoded_scalar(coder.encode(b, dtype=output_dtype), obfuscate=False)
    return pk.encrypt_encoded(coder.encode_tensor(b, dtype=output_dtype or b.dtype), obfuscate=False)


class evaluator:
    """paillier.py:179-399 (TensorEvaluator[EV, V, PK, Coder]).  add / sub / rsub and their
    _plain / _plain_scalar forms are generated below."""

    @staticmethod
    def mul_plain(a: EV, b: V, pk: PK, coder: Coder, output_dtype=None):
        return a.mul(pk.pk, coder.encode_tensor(b, dtype=output_dtype or b.dtype))

    @staticmethod
    def mul_plain_scalar(a: EV, b, pk: PK, coder: Coder, output_dtype):
        return a.mul_scalar(pk.pk, coder.encode(b, dtype=output_dtype))

    @staticmethod
    def matmul(a: EV, b: V, a_shape, b_shape, pk: PK, coder: Coder, output_dtype):
        return a.matmul(pk.pk, coder.encode_tensor(b, dtype=output_dtype), a_shape, b_shape)

    @staticmethod
    def rmatmul(a: EV, b: V, a_shape, b_shape, pk: PK, coder: Coder, output_dtype):
        return a.rmatmul(pk.pk, coder.encode_tensor(b, dtype=output_dtype), a_shape, b_shape)

    @staticmethod
    def zeros(size, dtype) -> EV:
        return CiphertextVector.zeros(size)

    @staticmethod
    def i_add(pk: PK, a: EV, b: EV, sa=0, sb=0, size: Optional[int] = None) -> None:
        if a is b:
            a.iadd_vec_self(sa, sb, size, pk.pk)
        else:
            a.iadd_vec(b, sa, sb, size, pk.pk)

    @staticmethod
    def i_sub(pk: PK, a: EV, b: EV, sa=0, sb=0, size: Optional[int] = None) -> None:
        if a is b:
            a.isub_vec_self(sa, sb, size, pk.pk)
        else:
            a.isub_vec(b, sa, sb, size, pk.pk)

    @staticmethod
    def i_update(pk: PK, a: EV, b: EV, positions, stride: int) -> None:
        a.iupdate(b, positions, stride, pk.pk)

    @staticmethod
    def i_update_with_masks(pk: PK, a: EV, b: EV, positions, masks, stride: int) -> None:
        a.iupdate_with_masks(b, positions, masks, stride, pk.pk)

    @staticmethod
    def chunking_cumsum_with_step(pk: PK, a: EV, chunk_sizes: List[int], step: int):
        return a.chunking_cumsum_with_step(pk.pk, chunk_sizes, step)

    @staticmethod
    def intervals_sum_with_step(pk: PK, a: EV, intervals: List[Tuple[int, int]], step: int):
        return a.intervals_sum_with_step(pk.pk, intervals, step)

    @staticmethod
    def pack_squeeze(a: EV, pack_num: int, shift_bit: int, pk: PK) -> EV:
        return a.pack_squeeze(pack_num, shift_bit, pk.pk)

    @staticmethod
    def slice(a: EV, start: int, size: int) -> EV:
        return a.slice(start, size)

    @staticmethod
    def i_shuffle(pk: PK, a: EV, indices: torch.LongTensor) -> None:
        a.i_shuffle(indices)  # a tensor is read as an array, not a Python list

    @staticmethod
    def shuffle(pk: PK, a: EV, indices: torch.LongTensor) -> EV:
        return a.shuffle(indices)

    @staticmethod
    def intervals_slice(a: EV, intervals: List[Tuple[int, int]]) -> EV:
        return a.intervals_slice(intervals)

    @staticmethod
    def cat(list: List[EV]) -> EV:
        return _p.Evaluator.cat(list)


def _evaluator_arith() -> None:
    """add / sub / rsub (EV op EV), op_plain (tensor; output_dtype defaults to b.dtype) and
    op_plain_scalar (scalar) -- paillier.py:183-262, one pattern per op."""
    for op in ("add", "sub", "rsub"):
        setattr(evaluator, op, staticmethod(lambda a, b, pk, _o=op: getattr(a, _o)(pk.pk, b)))
        setattr(evaluator, f"{op}_plain", staticmethod(
            lambda a, b, pk, coder, output_dtype=None, _o=op:
            getattr(a, _o)(pk.pk, _encrypted(b, pk, coder, output_dtype, False))))
        setattr(evaluator, f"{op}_plain_scalar", staticmethod(
            lambda a, b, pk, coder, output_dtype, _o=op:
            getattr(a, f"{_o}_scalar")(pk.pk, _encrypted(b, pk, coder, output_dtype, True))))


_evaluator_arith()
