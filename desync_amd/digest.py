"""Chunk ID digests (digest.go:11-29, nullchunk.go:17-23).

``Digest`` is the package-global algorithm (SHA-512/256 by default, SHA-256
alternative), as in the reference.  It selects the algorithm; the chunk IDs of
the product paths are computed on the GPU with it (digest_kernel behind
dsx_chunk_ids, dsx_index_fd / dsx_index_host and dsx_stream_ids: IndexFromFile,
VerifyIndex, ChunkStream).  ``Digest.Sum`` here is the host form (hashlib) for
a single buffer a caller holds, as the reference's Digest.Sum is.
"""
from __future__ import annotations

import hashlib


class SHA512256:
    def Sum(self, data) -> bytes:
        return hashlib.new("sha512_256", data).digest()

    def Algorithm(self) -> str:
        return "sha512-256"


class SHA256:
    def Sum(self, data) -> bytes:
        return hashlib.sha256(data).digest()

    def Algorithm(self) -> str:
        return "sha256"


Digest = SHA512256()


def set_digest(name: str):
    """cmd/desync/config.go:281-291 (--digest sha512-256|sha256)."""
    global Digest
    if name == "sha512-256":
        Digest = SHA512256()
    elif name == "sha256":
        Digest = SHA256()
    else:
        raise ValueError(f"invalid digest algorithm '{name}'")


class NullChunk:
    """nullchunk.go:17-23 -- the all-zero max-size chunk and its ID."""

    def __init__(self, size: int):
        self.Data = bytes(size)
        self.ID = Digest.Sum(self.Data)


def NewNullChunk(size: int) -> NullChunk:
    return NullChunk(size)
