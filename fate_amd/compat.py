"""``fate_utils.paillier`` alias: run FATE's own Paillier adapter on this backend.

FATE imports its native module as ``from fate_utils.paillier import CiphertextVector,
PlaintextVector, Coder, Evaluator, PK, SK, keygen`` (python/fate/arch/protocol/phe/
paillier.py:18-23) and its federation unpickler admits only classes under the ``fate.`` and
``fate_utils.`` module prefixes (arch/federation/api/_serdes.py:280, 311-333).
:func:`install` registers ``fate_utils`` / ``fate_utils.paillier`` modules whose classes are
alias subclasses of this backend's, named ``fate_utils.paillier.<Class>``, and pickle reducers
(``copyreg``) under which this backend's objects pickle as those aliases with the reference's
bincode state (``fate_amd.paillier`` ``__getstate__``).  FATE's adapter then runs on the MI355X
kernels unchanged, and a CPU party running the Rust ``fate_utils`` and a GPU party running this
backend exchange ciphertexts both ways.  ``fate_amd.paillier``'s own classes are not modified.
Importing ``fate_amd`` also appends a meta-path finder that serves these aliases for
``import fate_utils[.paillier]`` only when no real ``fate_utils`` is importable, so a process
that never called :func:`install` still loads such pickles.

Host-side return types follow the pyo3 signatures (paillier.rs:101-204): ``decode_f64_vec`` /
``decode_f32_vec`` return numpy arrays (``into_pyarray``), ``decode_i64_vec`` /
``decode_i32_vec`` lists.  Call :func:`install` before anything imports ``fate_utils``; it
refuses to shadow a real ``fate_utils`` build.
"""
from __future__ import annotations

import copyreg
import importlib.abc
import importlib.machinery
import sys
import types

from . import paillier as _p

MODULE = "fate_utils.paillier"


class Coder(_p.Coder):
    """``fate_utils.paillier.Coder`` with the pyo3 host return types."""

    __module__ = MODULE

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


keygen.__module__ = MODULE


def _alias(name: str, base: type) -> type:
    """A subclass of `base` named ``fate_utils.paillier.<name>`` (no new state)."""
    ns = {"__module__": MODULE, "__qualname__": name, "__doc__": base.__doc__}
    if "__slots__" in base.__dict__:
        ns["__slots__"] = ()
    return type(name, (base,), ns)


CLASSES = {name: _alias(name, getattr(_p, name))
           for name in ("PK", "SK", "Ciphertext", "CiphertextVector", "Plaintext", "PlaintextVector", "Evaluator")}
CLASSES["Coder"] = Coder
BASES = {name: getattr(_p, name) for name in CLASSES}


def _reducer(name: str, alias: type):
    """Pickle a base-class object as `alias`.  The five classes the reference pickles (PK, SK,
    Coder, CiphertextVector, PlaintextVector: paillier.rs:62-74, 86-98, 124-134, 214-226,
    391-402) as pyo3 does: the class called with no arguments (its ``#[new]``), then
    ``__setstate__`` with the bincode state.  Ciphertext / Plaintext (not picklable in the
    reference) as the class called on their vector; Evaluator (no state) as the class."""
    if name in ("Ciphertext", "Plaintext"):
        return lambda obj: (alias, (obj.vec,))
    if name == "Evaluator":
        return lambda obj: (alias, ())
    return lambda obj: (alias, (), obj.__getstate__())


def install() -> types.ModuleType:
    """Register the alias modules and the pickle reducers (idempotent); returns
    ``fate_utils.paillier``.  Refuses to shadow a real ``fate_utils``."""
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
        setattr(mod, name, cls)
        base = BASES[name]
        if base is not cls:
            copyreg.pickle(base, _reducer(name, cls))
    mod.keygen = keygen
    pkg.paillier = mod
    sys.modules[MODULE] = mod
    return mod


class _AliasLoader(importlib.abc.Loader):
    def create_module(self, spec):
        install()
        return sys.modules[spec.name]

    def exec_module(self, module):
        pass


class AliasFinder(importlib.abc.MetaPathFinder):
    """Last on ``sys.meta_path``: resolves ``fate_utils`` / ``fate_utils.paillier`` to the
    aliases only when every other finder (a real ``fate_utils`` build among them) found
    nothing."""

    def find_spec(self, name, path=None, target=None):
        if name not in ("fate_utils", MODULE):
            return None
        return importlib.machinery.ModuleSpec(name, _AliasLoader(), is_package=(name == "fate_utils"))
