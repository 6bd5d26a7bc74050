"""desync_amd -- MI355X-native content-defined chunker (desync drop-in).

The chunking hot path of folbricht/desync (chunker.go Buzhash scan + cut
chain, make.go split-and-align) runs as hand-written gfx950 HIP kernels in
libdsx.so behind the C ABI of include/dsx.h.  This package is the host-side
mirror of the reference's Go API for that path:

    NewChunker / Chunker.Next / Advance / Min / Avg / Max   (chunker.go)
    NewHash / Hash (the exported legacy rolling hash)       (chunker.go:320-371)
    IndexFromFile, ChunkingStats                            (make.go)
    VerifyIndex                                             (verifyindex.go)
    ChunkStream, ChunkStorage                               (index.go, chunkstorage.go)
    ChopFile, ChunkInvalid                                  (chop.go, errors.go)
    Index, IndexChunk, Index.WriteTo, IndexFromReader       (index.go)
    Digest (SHA512256 / SHA256), NullChunk                  (digest.go)

There is no CPU fallback: without libdsx.so or a GPU, calls raise.
"""
from .chunker import ChunkerReadError, ChunkerWindowSize, Chunker, NewChunker, Params  # noqa: F401
from .digest import SHA256, SHA512256, NewNullChunk, NullChunk, set_digest  # noqa: F401
from .errors import ChunkInvalid, Interrupted  # noqa: F401
from .index import FormatIndex, Index, IndexChunk, IndexFromReader  # noqa: F401
from .stream import Chunk, ChunkStorage, ChunkStream, MemoryStore  # noqa: F401
from .make import ChunkingStats, IndexFromFile, VerifyError, VerifyIndex, chunk_ids, cut_device, cut_device_result, \
    cut_fd, cut_host, file_size, ids_fd, ids_host, index_fd, index_host  # noqa: F401
from .chop import ChopFile  # noqa: F401
from .hash import Hash, NewHash  # noqa: F401

__all__ = [
    "ChunkerWindowSize", "Chunker", "ChunkerReadError", "NewChunker", "Params", "SHA256", "SHA512256", "NullChunk",
    "NewNullChunk", "set_digest", "Interrupted", "FormatIndex", "Index", "IndexChunk",
    "IndexFromReader", "Chunk", "ChunkStorage", "ChunkStream", "MemoryStore", "ChunkingStats", "IndexFromFile", "cut_device", "cut_device_result",
    "cut_fd", "cut_host", "chunk_ids", "VerifyIndex", "VerifyError", "file_size", "index_fd",
    "index_host", "ids_fd", "ids_host", "ChopFile", "ChunkInvalid", "Hash", "NewHash",
]
