"""ctypes binding of libfatephe.so (include/fate_phe.h).

The library is built in-tree by ``__graft_entry__.build()`` (or ``make -C fate_amd``)
into ``fate_amd/lib/libfatephe.so``.  There is no CPU fallback: if the shared object
is missing or a HIP device is absent, every compute entry point raises.
"""
from __future__ import annotations

import ctypes
import os
import threading
from typing import Optional

_HERE = os.path.dirname(os.path.abspath(__file__))
# FPHE_LIB_PATH selects another build of the same library (A/B measurements in tools/)
LIB_PATH = os.environ.get("FPHE_LIB_PATH") or os.path.join(_HERE, "lib", "libfatephe.so")

FPHE_OK = 0
FPHE_ERR_ARG = 1
FPHE_ERR_HIP = 2
FPHE_ERR_NO_SK = 3
FPHE_ERR_KEY = 4
FPHE_ERR_RANGE = 5

EF_ENCODE_NONFINITE = 0x01
EF_DECODE_CORRUPTED = 0x02
EF_DECODE_OVERFLOW = 0x04
EF_MUL_INVALID_PT = 0x08
EF_NOT_INVERTIBLE = 0x10
EF_DECODE_I128 = 0x20
EF_EXP_RANGE = 0x40

# fphe_ctx_set_option / fphe_ctx_get_option (include/fate_phe.h)
OPT_WIDE_DECRYPT_MAX = 1
OPT_WIDE_ENCRYPT_MAX = 2
OPT_WIDE_KH_ENCRYPT_MAX = 3
OPT_KH_DIRECT_Z = 4

# every symbol declared in include/fate_phe.h
EXPORTED_SYMBOLS = (
    "fphe_ctx_create", "fphe_ctx_destroy", "fphe_ctx_limbs", "fphe_ctx_mont_one",
    "fphe_ctx_set_option", "fphe_ctx_get_option",
    "fphe_encode_f32", "fphe_encode_f64", "fphe_decode_f32", "fphe_decode_f64",
    "fphe_encode_i64", "fphe_decode_i64", "fphe_decode_i32", "fphe_pack_f64", "fphe_unpack_f64",
    "fphe_encrypt", "fphe_encrypt_crt", "fphe_decrypt", "fphe_add", "fphe_add_ordered", "fphe_add_order", "fphe_mul", "fphe_neg", "fphe_sqmul", "fphe_align",
    "fphe_fold", "fphe_fold_segments", "fphe_permute", "fphe_export_signed", "fphe_import_signed",
    "fphe_wire_lengths", "fphe_wire_encode", "fphe_wire_scan", "fphe_wire_decode", "fphe_chacha20_blocks",
    "fphe_clock_stamp", "fphe_pack_squeeze", "fphe_positions_terms",
)

_lock = threading.Lock()
_lib: Optional[ctypes.CDLL] = None

c_u32p = ctypes.POINTER(ctypes.c_uint32)
vp = ctypes.c_void_p


class NativeLibraryMissing(RuntimeError):
    pass


def load() -> ctypes.CDLL:
    """Load (once) and type the native library.  Raises NativeLibraryMissing."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise NativeLibraryMissing(
                f"{LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
        lib = ctypes.CDLL(LIB_PATH)
        st = ctypes.c_int
        lib.fphe_ctx_create.argtypes = [ctypes.c_int, ctypes.c_uint32, c_u32p, c_u32p, c_u32p, ctypes.POINTER(vp)]
        lib.fphe_ctx_create.restype = st
        lib.fphe_ctx_destroy.argtypes = [vp]
        lib.fphe_ctx_destroy.restype = st
        lib.fphe_ctx_limbs.argtypes = [vp, c_u32p, c_u32p]
        lib.fphe_ctx_limbs.restype = st
        if hasattr(lib, "fphe_ctx_mont_one"):  # an A/B build from before it (FPHE_LIB_PATH) lacks it
            lib.fphe_ctx_mont_one.argtypes = [vp, c_u32p]
            lib.fphe_ctx_mont_one.restype = st
        if hasattr(lib, "fphe_ctx_set_option"):  # an A/B build from before it (FPHE_LIB_PATH) lacks it
            lib.fphe_ctx_set_option.argtypes = [vp, ctypes.c_int, ctypes.c_int64]
            lib.fphe_ctx_set_option.restype = st
            lib.fphe_ctx_get_option.argtypes = [vp, ctypes.c_int, ctypes.POINTER(ctypes.c_int64)]
            lib.fphe_ctx_get_option.restype = st
        for name in ("fphe_encode_f32", "fphe_encode_f64"):
            f = getattr(lib, name)
            f.argtypes = [vp, vp, ctypes.c_size_t, vp, vp, vp, vp, vp]
            f.restype = st
        for name in ("fphe_decode_f32", "fphe_decode_f64"):
            f = getattr(lib, name)
            f.argtypes = [vp, vp, ctypes.c_uint32, vp, ctypes.c_size_t, vp, vp, vp]
            f.restype = st
        lib.fphe_encode_i64.argtypes = [vp, vp, ctypes.c_size_t, vp, vp, vp, vp]
        lib.fphe_encode_i64.restype = st
        for name in ("fphe_decode_i64", "fphe_decode_i32"):
            f = getattr(lib, name)
            f.argtypes = [vp, vp, ctypes.c_uint32, vp, ctypes.c_size_t, vp, vp, vp]
            f.restype = st
        lib.fphe_pack_f64.argtypes = [vp, vp, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                      vp, vp, vp, vp, vp]
        lib.fphe_pack_f64.restype = st
        lib.fphe_unpack_f64.argtypes = [vp, vp, ctypes.c_uint32, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_uint32,
                                        ctypes.c_uint32, ctypes.c_size_t, vp, vp]
        lib.fphe_unpack_f64.restype = st
        lib.fphe_encrypt.argtypes = [vp, vp, ctypes.c_uint32, vp, ctypes.c_size_t, ctypes.c_int, vp,
                                     c_u32p, ctypes.c_uint64, vp, vp, vp]
        lib.fphe_encrypt.restype = st
        lib.fphe_encrypt_crt.argtypes = [vp, vp, ctypes.c_uint32, vp, ctypes.c_size_t, vp, c_u32p, ctypes.c_uint64,
                                         vp, vp, vp]
        lib.fphe_encrypt_crt.restype = st
        lib.fphe_decrypt.argtypes = [vp, vp, ctypes.c_size_t, vp, vp]
        lib.fphe_decrypt.restype = st
        lib.fphe_add.argtypes = [vp, vp, vp, vp, vp, vp, vp, ctypes.c_int, ctypes.c_size_t, vp, vp, vp, vp, vp]
        lib.fphe_add.restype = st
        lib.fphe_add_ordered.argtypes = [vp, vp, vp, vp, vp, vp, vp, ctypes.c_int, ctypes.c_size_t, vp, vp, vp, vp,
                                         vp, vp]
        lib.fphe_add_ordered.restype = st
        lib.fphe_mul.argtypes = [vp, vp, vp, vp, vp, ctypes.c_uint32, vp, vp, ctypes.c_int, ctypes.c_size_t,
                                 vp, vp, vp, vp, vp]
        lib.fphe_mul.restype = st
        lib.fphe_neg.argtypes = [vp, vp, ctypes.c_size_t, vp, vp, vp]
        lib.fphe_neg.restype = st
        lib.fphe_sqmul.argtypes = [vp, vp, vp, vp, ctypes.c_uint32, ctypes.c_size_t, vp, vp, vp]
        lib.fphe_sqmul.restype = st
        lib.fphe_align.argtypes = [vp, vp, vp, vp, ctypes.c_size_t, vp, vp, vp]
        lib.fphe_align.restype = st
        lib.fphe_fold.argtypes = [vp, vp, vp, vp, vp, vp, vp, ctypes.c_size_t, vp, vp, vp, vp]
        lib.fphe_fold.restype = st
        lib.fphe_fold_segments.argtypes = [vp, vp, vp, vp, ctypes.c_size_t, vp, vp, ctypes.c_size_t, ctypes.c_size_t,
                                           vp, vp, vp, vp, vp, vp]
        lib.fphe_fold_segments.restype = st
        if hasattr(lib, "fphe_positions_terms"):  # an A/B build from before it (FPHE_LIB_PATH) lacks it
            lib.fphe_positions_terms.argtypes = [vp, ctypes.c_int, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int32,
                                                 ctypes.c_size_t, vp, vp, vp]
            lib.fphe_positions_terms.restype = st
        if hasattr(lib, "fphe_add_order"):  # an A/B build from before it (FPHE_LIB_PATH) lacks it
            lib.fphe_add_order.argtypes = [vp, vp, ctypes.c_size_t, ctypes.c_uint32, vp, vp]
            lib.fphe_add_order.restype = st
        lib.fphe_permute.argtypes = [vp, vp, vp, ctypes.c_uint32, vp, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int,
                                     vp, vp, vp, vp]
        lib.fphe_permute.restype = st
        for name in ("fphe_export_signed", "fphe_import_signed"):
            getattr(lib, name).argtypes = [vp, vp, vp, ctypes.c_size_t, vp, vp, vp]
            getattr(lib, name).restype = st
        sz = ctypes.c_size_t
        lib.fphe_chacha20_blocks.argtypes = [vp, ctypes.c_uint32, vp, sz, vp, vp]
        lib.fphe_chacha20_blocks.restype = st
        lib.fphe_clock_stamp.argtypes = [vp, ctypes.c_uint32, vp, vp]
        lib.fphe_clock_stamp.restype = st
        lib.fphe_pack_squeeze.argtypes = [vp, vp, vp, sz, ctypes.c_uint32, ctypes.c_uint32, vp, vp, vp]
        lib.fphe_pack_squeeze.restype = st
        lib.fphe_wire_lengths.argtypes = [vp, vp, ctypes.c_uint32, sz, vp, vp, vp]
        lib.fphe_wire_encode.argtypes = [vp, vp, vp, ctypes.c_uint32, sz, vp, vp, vp, vp, vp]
        lib.fphe_wire_scan.argtypes = [vp, sz, sz, sz, vp, vp, vp, vp, vp, vp]
        lib.fphe_wire_decode.argtypes = [vp, vp, vp, vp, ctypes.c_uint32, sz, vp, vp, vp]
        for name in ("fphe_wire_lengths", "fphe_wire_encode", "fphe_wire_scan", "fphe_wire_decode"):
            getattr(lib, name).restype = st
        _lib = lib
        return lib


# host helper (fate_amd/csrc/host_positions.c): CPython-API marshalling of position lists and
# i_shuffle's cycle walk, called with the GIL held (ctypes.PyDLL), no device code
PY_LIB_PATH = os.path.join(_HERE, "lib", "libfphe_py.so")
_pylib: Optional[ctypes.PyDLL] = None


def load_py() -> ctypes.PyDLL:
    """Load (once) the host helper library.  Raises NativeLibraryMissing."""
    global _pylib
    with _lock:
        if _pylib is not None:
            return _pylib
        if not os.path.exists(PY_LIB_PATH):
            raise NativeLibraryMissing(
                f"{PY_LIB_PATH} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`")
        lib = ctypes.PyDLL(PY_LIB_PATH)
        lib.fphe_py_positions_lens.argtypes = [ctypes.py_object, vp, ctypes.c_int64]
        lib.fphe_py_positions_lens.restype = ctypes.c_int64
        lib.fphe_py_positions_fill.argtypes = [ctypes.py_object, vp, ctypes.c_int64]
        lib.fphe_py_positions_fill.restype = ctypes.c_int64
        lib.fphe_cycle_walk.argtypes = [vp, ctypes.c_int64, ctypes.c_int64, vp, vp, vp]
        lib.fphe_cycle_walk.restype = ctypes.c_int
        _pylib = lib
        return lib


def check(status: int, what: str) -> None:
    if status == FPHE_OK:
        return
    if status == FPHE_ERR_ARG:
        raise ValueError(f"{what}: invalid argument")
    if status == FPHE_ERR_NO_SK:
        raise ValueError(f"{what}: context has no private key")
    if status == FPHE_ERR_KEY:
        raise ValueError(f"{what}: key material rejected")
    raise RuntimeError(f"{what}: HIP runtime error (status {status})")
