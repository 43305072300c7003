"""fate_amd -- MI355X-native Paillier PHE backend for FATE (the secure-aggregation hot path).

Public modules:
  fate_amd.paillier  -- mirror of the reference's native ``fate_utils.paillier`` surface
  fate_amd.protocol  -- drop-in for ``fate.arch.protocol.phe.paillier`` (keygen + evaluator)
  fate_amd.dist      -- element sharding across GPUs (one process per GPU)
The compute lives in fate_amd/lib/libfatephe.so (HIP, gfx950); see include/fate_phe.h.
"""
__all__ = ["paillier", "protocol"]
