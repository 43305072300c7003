"""Drop-in replacement for ``fate.arch.protocol.phe.paillier`` on MI355X.

Mirrors python/fate/arch/protocol/phe/paillier.py:33-399 (SK / PK / Coder wrappers,
``keygen(key_size)`` and the ``evaluator`` TensorEvaluator plugin, type.py:24) with the
same method names, argument meaning and error behaviour, over :mod:`fate_amd.paillier`
(the mirror of ``fate_utils.paillier``).  A FATE deployment selects it where
``PHECipherBuilder.setup`` imports ``fate.arch.protocol.phe.paillier``
(python/fate/arch/context/_cipher.py:111-124); see INTEGRATION.md.

Differences by design: tensors may be CUDA (HIP) tensors -- encoding reads them in place
in HBM instead of calling ``.numpy()`` (paillier.py:159-161), and decoding returns a
tensor on the requested device.
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
        if dtype == torch.float64:
            return self.coder.encode_f64_vec(vec)
        if dtype == torch.float32:
            return self.coder.encode_f32_vec(vec)
        if dtype == torch.int64:
            return self.coder.encode_i64_vec(vec)
        if dtype == torch.int32:
            return self.coder.encode_i32_vec(vec)
        raise NotImplementedError(f"{vec.dtype} not supported")

    def decode_vec(self, vec: FV, dtype: torch.dtype) -> V:
        if dtype == torch.float64:
            return self.coder.decode_f64_vec(vec).cpu()
        if dtype == torch.float32:
            return self.coder.decode_f32_vec(vec).cpu()
        if dtype == torch.int64:
            return torch.tensor(self.coder.decode_i64_vec(vec), dtype=torch.int64)
        if dtype == torch.int32:
            return torch.tensor(self.coder.decode_i32_vec(vec), dtype=torch.int32)
        raise NotImplementedError(f"{dtype} not supported")

    def encode(self, val, dtype=None):
        if isinstance(val, torch.Tensor):
            assert val.ndim == 0, "only scalar supported"
            dtype = val.dtype
            val = val.item()
        if dtype == torch.float64:
            return self.coder.encode_f64(val)
        if dtype == torch.float32:
            return self.coder.encode_f32(val)
        if dtype == torch.int64:
            return self.coder.encode_i64(val)
        if dtype == torch.int32:
            return self.coder.encode_i32(val)
        raise NotImplementedError(f"{dtype} not supported")

    def encode_f64(self, val: float):
        return self.coder.encode_f64(val)

    def decode_f64(self, val):
        return self.coder.decode_f64(val)

    def encode_i64(self, val: int):
        return self.coder.encode_i64(val)

    def decode_i64(self, val):
        return self.coder.decode_i64(val)

    def encode_f32(self, val: float):
        return self.coder.encode_f32(val)

    def decode_f32(self, val):
        return self.coder.decode_f32(val)

    def encode_i32(self, val: int):
        return self.coder.encode_i32(val)

    def decode_i32(self, val):
        return self.coder.decode_i32(val)

    def encode_f64_vec(self, vec: torch.Tensor):
        return self.coder.encode_f64_vec(vec.detach().flatten())

    def decode_f64_vec(self, vec):
        return self.coder.decode_f64_vec(vec).cpu()

    def encode_i64_vec(self, vec: torch.Tensor):
        return self.coder.encode_i64_vec(vec.detach().flatten())

    def decode_i64_vec(self, vec):
        return torch.tensor(self.coder.decode_i64_vec(vec))

    def encode_f32_vec(self, vec: torch.Tensor):
        return self.coder.encode_f32_vec(vec.detach().flatten())

    def decode_f32_vec(self, vec):
        return self.coder.decode_f32_vec(vec).cpu()

    def encode_i32_vec(self, vec: torch.Tensor):
        return self.coder.encode_i32_vec(vec.detach().flatten())

    def decode_i32_vec(self, vec):
        return torch.tensor(self.coder.decode_i32_vec(vec))


def supports(key_size: int) -> bool:
    """Whether this backend runs keys of ``key_size`` bits (even, 256..4096).  The
    ``PHECipherBuilder.setup`` branch in INTEGRATION.md keeps FATE's CPU module for the rest
    (the reference accepts any even size, paillier/src/lib.rs:72-87)."""
    return _p.supports(key_size)


def keygen(key_size):
    """paillier.py:174-176.  ValueError for sizes :func:`supports` rejects."""
    sk, pk, coder = _p.keygen(key_size)
    return SK(sk), PK(pk), Coder(coder)


class evaluator:
    """paillier.py:179-399 (TensorEvaluator[EV, V, PK, Coder])."""

    @staticmethod
    def add(a: EV, b: EV, pk: PK):
        return a.add(pk.pk, b)

    @staticmethod
    def add_plain(a: EV, b: V, pk: PK, coder: Coder, output_dtype=None):
        if output_dtype is None:
            output_dtype = b.dtype
        encoded = coder.encode_tensor(b, dtype=output_dtype)
        encrypted = pk.encrypt_encoded(encoded, obfuscate=False)
        return a.add(pk.pk, encrypted)

    @staticmethod
    def add_plain_scalar(a: EV, b, pk: PK, coder: Coder, output_dtype):
        encoded = coder.encode(b, dtype=output_dtype)
        encrypted = pk.encrypt_encoded_scalar(encoded, obfuscate=False)
        return a.add_scalar(pk.pk, encrypted)

    @staticmethod
    def sub(a: EV, b: EV, pk: PK):
        return a.sub(pk.pk, b)

    @staticmethod
    def sub_plain(a: EV, b: V, pk: PK, coder: Coder, output_dtype=None):
        if output_dtype is None:
            output_dtype = b.dtype
        encoded = coder.encode_tensor(b, dtype=output_dtype)
        encrypted = pk.encrypt_encoded(encoded, obfuscate=False)
        return a.sub(pk.pk, encrypted)

    @staticmethod
    def sub_plain_scalar(a: EV, b, pk: PK, coder: Coder, output_dtype):
        encoded = coder.encode(b, dtype=output_dtype)
        encrypted = pk.encrypt_encoded_scalar(encoded, obfuscate=False)
        return a.sub_scalar(pk.pk, encrypted)

    @staticmethod
    def rsub(a: EV, b: EV, pk: PK):
        return a.rsub(pk.pk, b)

    @staticmethod
    def rsub_plain(a: EV, b: V, pk: PK, coder: Coder, output_dtype=None):
        if output_dtype is None:
            output_dtype = b.dtype
        encoded = coder.encode_tensor(b, dtype=output_dtype)
        encrypted = pk.encrypt_encoded(encoded, obfuscate=False)
        return a.rsub(pk.pk, encrypted)

    @staticmethod
    def rsub_plain_scalar(a: EV, b, pk: PK, coder: Coder, output_dtype):
        encoded = coder.encode(b, dtype=output_dtype)
        encrypted = pk.encrypt_encoded_scalar(encoded, obfuscate=False)
        return a.rsub_scalar(pk.pk, encrypted)

    @staticmethod
    def mul_plain(a: EV, b: V, pk: PK, coder: Coder, output_dtype=None):
        if output_dtype is None:
            output_dtype = b.dtype
        encoded = coder.encode_tensor(b, dtype=output_dtype)
        return a.mul(pk.pk, encoded)

    @staticmethod
    def mul_plain_scalar(a: EV, b, pk: PK, coder: Coder, output_dtype):
        encoded = coder.encode(b, dtype=output_dtype)
        return a.mul_scalar(pk.pk, encoded)

    @staticmethod
    def matmul(a: EV, b: V, a_shape, b_shape, pk: PK, coder: Coder, output_dtype):
        encoded = coder.encode_tensor(b, dtype=output_dtype)
        return a.matmul(pk.pk, encoded, a_shape, b_shape)

    @staticmethod
    def rmatmul(a: EV, b: V, a_shape, b_shape, pk: PK, coder: Coder, output_dtype):
        encoded = coder.encode_tensor(b, dtype=output_dtype)
        return a.rmatmul(pk.pk, encoded, a_shape, b_shape)

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
        a.i_shuffle(indices.tolist() if isinstance(indices, torch.Tensor) else indices)

    @staticmethod
    def shuffle(pk: PK, a: EV, indices: torch.LongTensor) -> EV:
        return a.shuffle(indices.tolist() if isinstance(indices, torch.Tensor) else indices)

    @staticmethod
    def intervals_slice(a: EV, intervals: List[Tuple[int, int]]) -> EV:
        return a.intervals_slice(intervals)

    @staticmethod
    def cat(list: List[EV]) -> EV:
        return _p.Evaluator.cat(list)
