"""Index / IndexChunk and the caibx encoding (index.go, format.go, const.go).

Reference: ``Index`` / ``IndexChunk`` (index.go:20-32), ``(*Index).WriteTo``
(index.go:90-124) via ``FormatEncoder.Encode`` for FormatIndex / FormatTable
(format.go:582-620), ``IndexFromReader`` (index.go:36-87), constants
(const.go:23-25, 74-77).  All values little-endian uint64 (writer.go:16-22).
"""
from __future__ import annotations

import io
import struct
from collections.abc import MutableSequence
from dataclasses import dataclass, field

import numpy as np

CaFormatEntry = 0x1396FABCEA5BBB51
CaFormatIndex = 0x96824D9C7B129FF9
CaFormatTable = 0xE75B9E112F17417D
CaFormatTableTailMarker = 0x4B4F050E5549ECD1
CaFormatSHA512256 = 0x2000000000000000
CaFormatExcludeNoDump = 0x8000000000000000


_ITEM = np.dtype([("off", "<u8"), ("id", "S32")])


class InvalidFormat(ValueError):
    pass


@dataclass
class FormatIndex:
    FeatureFlags: int = 0
    ChunkSizeMin: int = 0
    ChunkSizeAvg: int = 0
    ChunkSizeMax: int = 0


@dataclass(slots=True)
class IndexChunk:
    ID: bytes
    Start: int
    Size: int


class ChunkArray(MutableSequence):
    """Index.Chunks of a contiguous chunk list held as arrays (chunk ends and
    32-byte IDs, as libdsx returns them): IndexChunk objects are built only
    when an element is read, and WriteTo packs the arrays directly.  Any
    change turns it into a plain list of IndexChunk first."""

    def __init__(self, ends, ids, start=0):
        self._ends = np.ascontiguousarray(ends, dtype=np.uint64)
        ids = np.frombuffer(ids, dtype=np.uint8) if isinstance(ids, (bytes, bytearray)) else ids
        self._ids = np.ascontiguousarray(ids, dtype=np.uint8).reshape(-1, 32)
        self._start = int(start)  # the first chunk's start (the stream position it began at)
        self._list = None

    def _chunk(self, i):
        e = int(self._ends[i])
        s = int(self._ends[i - 1]) if i else self._start
        return IndexChunk(self._ids[i].tobytes(), s, e - s)

    def _materialize(self):
        if self._list is None:
            el = self._ends.tolist()
            raw = self._ids.tobytes()
            self._list = [IndexChunk(raw[32 * i:32 * i + 32], s, e - s)
                          for i, (s, e) in enumerate(zip([self._start] + el[:-1], el))]
        return self._list

    def __len__(self):
        return len(self._list) if self._list is not None else len(self._ends)

    def __getitem__(self, i):
        if self._list is not None:
            return self._list[i]
        if isinstance(i, slice):
            return [self._chunk(k) for k in range(*i.indices(len(self._ends)))]
        n = len(self._ends)
        if i < 0:
            i += n
        if not 0 <= i < n:
            raise IndexError("chunk index out of range")
        return self._chunk(i)

    def __iter__(self):
        return iter(self._materialize())

    def __setitem__(self, i, v):
        self._materialize()[i] = v

    def __delitem__(self, i):
        del self._materialize()[i]

    def insert(self, i, v):
        self._materialize().insert(i, v)

    def __eq__(self, other):
        return list(self) == list(other)

    def __repr__(self):
        return f"ChunkArray({len(self)} chunks)"


@dataclass
class Index:
    Index: FormatIndex = field(default_factory=FormatIndex)
    Chunks: list = field(default_factory=list)

    def WriteTo(self, w) -> int:
        """index.go:90-124 -- returns the number of bytes written."""
        b = self.encode()
        w.write(b)
        return len(b)

    def encode(self) -> bytes:
        fi = self.Index
        out = bytearray(struct.pack("<6Q", 48, CaFormatIndex, fi.FeatureFlags, fi.ChunkSizeMin,
                                    fi.ChunkSizeAvg, fi.ChunkSizeMax))
        out += struct.pack("<2Q", 0xFFFFFFFFFFFFFFFF, CaFormatTable)
        # table items {end offset, ID} (format.go:596-605), packed in one go
        nc = len(self.Chunks)
        items = np.empty(nc, dtype=_ITEM)
        ca = self.Chunks if isinstance(self.Chunks, ChunkArray) and self.Chunks._list is None else None
        if nc and ca is not None:  # arrays as libdsx returned them
            items["off"] = ca._ends
            items["id"] = ca._ids.view("S32").reshape(-1)
        elif nc:
            items["off"] = np.cumsum(np.fromiter((c.Size for c in self.Chunks), np.uint64, nc))
            items["id"] = np.frombuffer(b"".join(bytes(c.ID) for c in self.Chunks), "S32")
        out += items.tobytes()
        n = 16 + 40 * nc
        # tail record: zero fill x2, index offset, table size, marker (format.go:607-614)
        out += struct.pack("<5Q", 0, 0, 48, n + 40, CaFormatTableTailMarker)
        return bytes(out)

    def Length(self) -> int:
        """index.go:127-133"""
        if not self.Chunks:
            return 0
        last = self.Chunks[-1]
        return last.Start + last.Size


def IndexFromReader(r, digest_algorithm="sha512-256") -> Index:
    """index.go:36-87 (decode a caibx)."""
    data = r.read() if hasattr(r, "read") else bytes(r)
    if len(data) < 64:
        raise InvalidFormat("reading index")
    size, typ, flags, mn, av, mx = struct.unpack_from("<6Q", data, 0)
    if typ != CaFormatIndex:
        raise InvalidFormat("input is not an index file")
    if digest_algorithm == "sha512-256" and not flags & CaFormatSHA512256:
        raise InvalidFormat("index file uses SHA256")
    if digest_algorithm == "sha256" and flags & CaFormatSHA512256:
        raise InvalidFormat("index file uses SHA512-256")
    tsize, ttyp = struct.unpack_from("<2Q", data, 48)
    if ttyp != CaFormatTable:
        raise InvalidFormat("index table not found in input")
    if tsize != 0xFFFFFFFFFFFFFFFF:
        raise InvalidFormat("expected size MAX_UINT64 in format table")
    off, last = 64, 0
    chunks = []
    while True:
        (o,) = struct.unpack_from("<Q", data, off)
        if o == 0:
            break
        cid = data[off + 8:off + 40]
        chunks.append(IndexChunk(ID=cid, Start=last, Size=o - last))
        if o - last > mx:
            raise InvalidFormat(f"chunk size {o - last} is larger than maximum {mx}")
        last = o
        off += 40
    z2, _idx, _tsz, marker = struct.unpack_from("<4Q", data, off + 8)
    if z2 != 0 or marker != CaFormatTableTailMarker:
        raise InvalidFormat("tail marker not found")
    return Index(FormatIndex(flags, mn, av, mx), chunks)


def catar_feature_flags(head: bytes) -> int:
    """make.go:49-61: FeatureFlags of a leading catar FormatEntry (size 64,
    format.go:161-172), else 0."""
    if len(head) < 24:
        return 0
    size, typ, ff = struct.unpack_from("<3Q", head, 0)
    if typ != CaFormatEntry:
        return 0
    if size != 64 or len(head) < 64:
        return 0
    return ff


def encode_to_bytes(index: Index) -> bytes:
    b = io.BytesIO()
    index.WriteTo(b)
    return b.getvalue()
