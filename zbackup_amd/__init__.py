"""zbackup_amd -- MI355X-native rolling-hash chunking engine for zbackup's dedup hot path.

The product is libzchunk.so (HIP kernels for gfx950 + the boundary resolver,
C ABI in include/zchunk.h).  This package builds it in-tree and exposes the
Python mirror of the reference's BackupCreator interface.
"""
from ._lib import ZC_BYTES, ZC_CHUNK_DUP, ZC_CHUNK_NEW, ZcError, load  # noqa: F401
from .chunker import (META_DTYPE, RECORD_DTYPE, BackupCreator, Sha256, anchor_def, chunk_id_blob,  # noqa: F401
                      fill_splitmix64, serialize_instruction)

__all__ = ["BackupCreator", "Sha256", "ZcError", "RECORD_DTYPE", "chunk_id_blob", "serialize_instruction",
           "fill_splitmix64", "load", "META_DTYPE", "anchor_def", "ZC_CHUNK_NEW", "ZC_CHUNK_DUP", "ZC_BYTES"]
