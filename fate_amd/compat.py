"""``fate_utils.paillier`` alias: run FATE's own Paillier adapter on this backend.

FATE imports its native module as ``from fate_utils.paillier import CiphertextVector,
PlaintextVector, Coder, Evaluator, PK, SK, keygen`` (python/fate/arch/protocol/phe/
paillier.py:18-23) and its federation unpickler admits only classes under the ``fate.`` and
``fate_utils.`` module prefixes (arch/federation/api/_serdes.py:280, 311-333).
:func:`install` registers ``fate_utils`` / ``fate_utils.paillier`` modules whose classes are
this backend's, with ``__module__ = "fate_utils.paillier"``: FATE's adapter then runs on the
MI355X kernels unchanged, and pickles name ``fate_utils.paillier.<Class>`` with the
reference's bincode state (``fate_amd.paillier`` ``__getstate__``), so a CPU party running the
Rust ``fate_utils`` and a GPU party running this backend exchange ciphertexts both ways.

Host-side return types follow the pyo3 signatures (paillier.rs:101-204): ``decode_f64_vec`` /
``decode_f32_vec`` return numpy arrays (``into_pyarray``), ``decode_i64_vec`` /
``decode_i32_vec`` lists.  Call :func:`install` before anything imports ``fate_utils``; it
refuses to shadow a real ``fate_utils`` build.
"""
from __future__ import annotations

import sys
import types

from . import paillier as _p

MODULE = "fate_utils.paillier"


class Coder(_p.Coder):
    """``fate_utils.paillier.Coder`` with the pyo3 host return types."""

    def decode_f64_vec(self, data):
        return _p.Coder.decode_f64_vec(self, data).cpu().numpy()

    def decode_f32_vec(self, data):
        return _p.Coder.decode_f32_vec(self, data).cpu().numpy()


def keygen(bit_length: int):
    """``fate_utils.paillier.keygen`` (paillier.rs:206-210)."""
    sk, pk, coder = _p.keygen(bit_length)
    c = Coder.__new__(Coder)
    c._init(coder.n)
    return sk, pk, c


CLASSES = {"PK": _p.PK, "SK": _p.SK, "Coder": Coder, "Ciphertext": _p.Ciphertext,
           "CiphertextVector": _p.CiphertextVector, "Plaintext": _p.Plaintext,
           "PlaintextVector": _p.PlaintextVector, "Evaluator": _p.Evaluator}


def install() -> types.ModuleType:
    """Register the alias modules (idempotent); returns ``fate_utils.paillier``."""
    have = sys.modules.get(MODULE)
    if have is not None:
        if getattr(have, "_fate_amd_alias", False):
            return have
        raise RuntimeError("a real fate_utils.paillier is already imported; not shadowing it")
    pkg = sys.modules.get("fate_utils")
    if pkg is None:
        pkg = types.ModuleType("fate_utils")
        pkg.__path__ = []  # a package, so "fate_utils.paillier" resolves as a submodule
        pkg._fate_amd_alias = True
        sys.modules["fate_utils"] = pkg
    elif not getattr(pkg, "_fate_amd_alias", False):
        raise RuntimeError("a real fate_utils is already imported; not shadowing it")
    mod = types.ModuleType(MODULE)
    mod._fate_amd_alias = True
    for name, cls in CLASSES.items():
        cls.__module__ = MODULE
        cls.__qualname__ = name
        setattr(mod, name, cls)
    keygen.__module__ = MODULE
    mod.keygen = keygen
    pkg.paillier = mod
    sys.modules[MODULE] = mod
    return mod
