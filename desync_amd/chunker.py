"""Mirror of desync's Chunker API (chunker.go) over the MI355X engine.

Reference interface (chunker.go):
    func NewChunker(r io.Reader, min, avg, max uint64) (Chunker, error)   :134
    func (c *Chunker) Next() (uint64, []byte, error)                       :206
    func (c *Chunker) Advance(n int) error                                 :292
    func (c *Chunker) Min() / Avg() / Max() uint64                         :312-318
    const ChunkerWindowSize = 48                                           :11

Same argument meaning and error behaviour: NewChunker validates in the
reference order and raises ValueError with the reference's message; Next()
returns (start, b'') at the end of the stream; read errors propagate.
The boundary scan and cut chain run on the GPU (libdsx.so); this class only
moves bytes from the reader into the library (dsx_stream_push) and hands
out confirmed chunks (dsx_stream_pop).
"""
from __future__ import annotations

import ctypes

from . import _lib
from ._lib import check, lib

ChunkerWindowSize = 48
# reads per refill; the reference refills 10*max (chunker.go:179)
_READ_FACTOR = 10


class Params:
    """Validated chunker parameters (dsx_params_init <- chunker.go:134-171)."""

    def __init__(self, min_size, avg_size, max_size):
        p = _lib.Params()
        rc = lib().dsx_params_init(int(min_size), int(avg_size), int(max_size), ctypes.byref(p))
        if rc != 0:
            # reference messages, chunker.go:135-146
            raise ValueError(lib().dsx_strerror(rc).decode())
        self.c = p
        self.min, self.avg, self.max = int(min_size), int(avg_size), int(max_size)

    @property
    def discriminator(self):
        return int(self.c.discriminator)


class Chunker:
    """Content-defined chunker over a file-like reader (``read(n) -> bytes``)."""

    def __init__(self, reader, min_size, avg_size, max_size, ctx=None, device=0):
        self.params = Params(min_size, avg_size, max_size)
        self.r = reader
        # Like a Go Chunker (its own buffer and hash state, chunker.go:108-131)
        # every Chunker owns a library context: the stream state and device
        # scratch live there.  A caller-supplied ctx must not carry another
        # unfinished stream (dsx_stream_begin refuses: DSX_E_STATE).
        self._own = ctx is None
        self.ctx = _lib.Context(device) if ctx is None else ctx
        check(lib().dsx_stream_begin(self.ctx.h, ctypes.byref(self.params.c)), self.ctx.h)
        self._eof = False
        self._start = ctypes.c_uint64()
        self._size = ctypes.c_uint64()

    # -- reference API -----------------------------------------------------
    def Next(self):
        """(start, chunk bytes); (start, b'') when the stream is exhausted."""
        L = lib()
        h = self.ctx.h
        while True:
            rc = check(L.dsx_stream_pop(h, ctypes.byref(self._start), ctypes.byref(self._size)), h)
            if rc == 1:
                ptr = L.dsx_stream_chunk_data(h)
                n = self._size.value
                return self._start.value, ctypes.string_at(ptr, n)
            if self._eof:
                return self._start.value, b""
            self._fill()

    def Advance(self, n):
        """Skip n bytes and restart the hash as if the stream began there."""
        check(lib().dsx_stream_advance(self.ctx.h, int(n)), self.ctx.h)

    def Min(self):
        return self.params.min

    def Avg(self):
        return self.params.avg

    def Max(self):
        return self.params.max

    def close(self):
        """Release the stream (and the context, if this Chunker created it)."""
        if self.ctx is not None and self.ctx.h:
            lib().dsx_stream_end(self.ctx.h)
            if self._own:
                self.ctx.close()
        self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- pythonic aliases --------------------------------------------------
    next = Next
    advance = Advance

    def __iter__(self):
        while True:
            start, b = self.Next()
            if not b:
                return
            yield start, b

    # -- internals -------------------------------------------------------------
    def _fill(self):
        want = _READ_FACTOR * self.params.max
        data = self.r.read(want)  # reader errors propagate (chunker.go:208-211)
        if not data:
            self._eof = True
            check(lib().dsx_stream_push(self.ctx.h, None, 0, 1), self.ctx.h)
            return
        if not isinstance(data, bytes):
            data = bytes(data)
        # bytes are immutable and stay alive for the call: passed without a copy
        # (the library copies what it keeps, dsx.h)
        check(lib().dsx_stream_push(self.ctx.h, data, len(data), 0), self.ctx.h)


def NewChunker(reader, min_size, avg_size, max_size, **kw):
    """chunker.go:134 NewChunker."""
    return Chunker(reader, min_size, avg_size, max_size, **kw)
