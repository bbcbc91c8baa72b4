"""pfs_amd — MI355X-native PFS chunk-ingest path (CDC rolling hash + BLAKE2b content hash).

Product modules: ``cdc`` (batch GPU API), ``chunk`` (chunk.Writer mirror), ``distributed``
(file sharding + RCCL gather of the chunk-ref index).  Native code: ``libpfscdc.so``
(HIP kernels for gfx950 + C ABI in ``include/pfscdc.h``).
"""
from .cdc import ChunkParams, Chunker, ScanResult, synthetic_bytes  # noqa: F401

__all__ = ["ChunkParams", "Chunker", "ScanResult", "synthetic_bytes"]
