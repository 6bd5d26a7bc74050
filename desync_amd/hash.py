"""The exported legacy rolling ``Hash`` type of chunker.go:320-371.

Nothing in the reference calls it (the chunker inlines its own 2-byte loop,
chunker.go:259-271), but it is public API of the hot-path file, so a user of
the reference finds it here with the same names and semantics:

    NewHash(size, discriminator) Hash          chunker.go:331-338
    (*Hash).Roll(b byte)                       chunker.go:342-350
    (*Hash).Initialize(b []byte)               chunker.go:354-359
    (*Hash).IsBoundary() bool                  chunker.go:363-365
    (*Hash).Reset()                            chunker.go:368-371

It is a per-byte host utility (one Python call per byte), not a data path:
chunking a blob goes through the GPU (NewChunker, IndexFromFile).  The
substitution table is the one the kernels use (include/dsx_buzhash_table.h,
chunker.go:30-95).
"""
from __future__ import annotations

import os

_TABLE_H = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include",
                        "dsx_buzhash_table.h")


def _load_table():
    with open(_TABLE_H) as f:
        txt = f.read().split("#define DSX_BUZHASH_TABLE_INIT {")[1].split("}")[0]
    vals = [int(t.strip().rstrip("u"), 16)
            for t in txt.replace("\\", " ").replace("\n", " ").split(",") if t.strip()]
    if len(vals) != 256:
        raise RuntimeError(f"{_TABLE_H}: expected 256 table entries, found {len(vals)}")
    return tuple(vals)


hashTable = _load_table()


def _rotl32(x, r):
    r &= 31  # bits.RotateLeft32 rotates by k mod 32
    return ((x << r) | (x >> (32 - r))) & 0xFFFFFFFF if r else x


class Hash:
    """chunker.go:322-328: value, window ring, size, idx, discriminator."""

    __slots__ = ("value", "window", "size", "idx", "discriminator")

    def __init__(self, size, discriminator):
        self.value = 0
        self.window = bytearray(size)
        self.size = size
        self.idx = 0
        self.discriminator = discriminator & 0xFFFFFFFF

    def Roll(self, b):
        """Adds byte b; the byte that falls out of the window is removed
        (chunker.go:342-350)."""
        ob = self.window[self.idx]
        self.window[self.idx] = b
        self.idx = (self.idx + 1) % self.size
        self.value = (_rotl32(self.value, 1) ^ _rotl32(hashTable[ob], len(self.window))
                      ^ hashTable[b])

    def Initialize(self, b):
        """Hash of a full window (len(b) == size; chunker.go:354-359)."""
        for i, c in enumerate(bytes(b)):
            self.value ^= _rotl32(hashTable[c], self.size - i - 1)
        n = min(len(b), len(self.window))
        self.window[:n] = bytes(b)[:n]

    def IsBoundary(self):
        """value % discriminator == discriminator - 1 (chunker.go:363-365)."""
        return self.value % self.discriminator == (self.discriminator - 1) & 0xFFFFFFFF

    def Reset(self):
        """chunker.go:368-371: index and value back to 0 (the window bytes
        stay, as in the reference)."""
        self.idx = 0
        self.value = 0


def NewHash(size, discriminator):
    """chunker.go:331-338"""
    return Hash(size, discriminator)
