"""fate_amd -- MI355X-native Paillier PHE backend for FATE (the secure-aggregation hot path).

Public modules:
  fate_amd.paillier  -- mirror of the reference's native ``fate_utils.paillier`` surface
  fate_amd.protocol  -- drop-in for ``fate.arch.protocol.phe.paillier`` (keygen + evaluator)
  fate_amd.dist      -- element sharding across GPUs (one process per GPU)
The compute lives in fate_amd/lib/libfatephe.so (HIP, gfx950); see include/fate_phe.h.
"""
__all__ = ["paillier", "protocol"]


def _register_alias_finder() -> None:
    """Serve fate_utils.paillier aliases (fate_amd.compat) to imports -- unpickling a ciphertext
    a route-A party sent, for instance -- when no real fate_utils is importable.  Appended
    last, so a real build always wins; nothing is imported until such an import happens."""
    import importlib.abc
    import importlib.machinery
    import sys

    class _LazyAliasFinder(importlib.abc.MetaPathFinder):
        def find_spec(self, name, path=None, target=None):
            if name not in ("fate_utils", "fate_utils.paillier"):
                return None
            from .compat import AliasFinder
            return AliasFinder().find_spec(name, path, target)

    if not any(type(f).__name__ == "_LazyAliasFinder" for f in sys.meta_path):
        sys.meta_path.append(_LazyAliasFinder())


_register_alias_finder()
