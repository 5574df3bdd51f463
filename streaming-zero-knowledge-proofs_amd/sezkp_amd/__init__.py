"""sezkp_amd — MI355X-native STARK v1 prover hot path (host side).

Python mirror of the reference's `ProvingBackend`/`StarkV1` surface over the
C ABI in include/sezkp_stark.h. All compute runs in lib/libsezkp_stark.so
(HIP kernels for gfx950); importing fails loudly when it is not built.
"""
from ._lib import LIB_PATH, SezkpError, lib  # noqa: F401  (raises ImportError if the .so is missing)
from .backend import STAGES, ProofArtifact, ProverContext, ShardedProverContext, StarkV1  # noqa: F401
from .blocks import BlockSoA, partition, reference_blocks, reference_trace, simulate, synthetic_blocks  # noqa: F401

__all__ = ["StarkV1", "ProverContext", "ShardedProverContext", "ProofArtifact", "BlockSoA", "SezkpError", "simulate", "partition",
           "synthetic_blocks", "reference_blocks", "reference_trace", "STAGES", "LIB_PATH", "lib"]
