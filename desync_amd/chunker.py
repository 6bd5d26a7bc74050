"""Mirror of desync's Chunker API (chunker.go) over the MI355X engine.

Reference interface (chunker.go):
    func NewChunker(r io.Reader, min, avg, max uint64) (Chunker, error)   :134
    func (c *Chunker) Next() (uint64, []byte, error)                       :206
    func (c *Chunker) Advance(n int) error                                 :292
    func (c *Chunker) Min() / Avg() / Max() uint64                         :312-318
    const ChunkerWindowSize = 48                                           :11

Same argument meaning and error behaviour: NewChunker validates in the
reference order and raises ValueError with the reference's message; Next()
returns (start, b'') at the end of the stream; the returned chunk is a
read-only view of library memory, valid until the next call (Next's rule,
chunker.go:202-205: copy it to keep it).  A reader error surfaces where the
reference's would: Next() raises ChunkerReadError carrying (start, chunk,
cause), the chunk being all bytes buffered after start (split(n, err),
chunker.go:207-211), and chunking starts over behind them.

The boundary scan and cut chain run on the GPU (libdsx.so); this class only
moves bytes from the reader into the library (straight into its pinned
buffer with readinto when the reader has it) and hands out confirmed chunks.
"""
from __future__ import annotations

import bisect
import ctypes
import itertools

from . import _lib
from ._lib import check, lib

ChunkerWindowSize = 48
# bytes per reader call (the library sends 8 MiB batches to the GPU)
_READ = 8 << 20
# confirmed chunks taken from the library per call (Next() then serves them
# without a library call per chunk)
_POP = 4096
_tokens = itertools.count()


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


class ChunkerReadError(IOError):
    """Next()'s (start, b, err) with err != nil: ``start`` and ``chunk`` (the
    buffered bytes, chunker.go:207-211) and the reader's exception as
    ``__cause__``."""

    def __init__(self, start, chunk, cause):
        super().__init__(f"read error after stream position {start + len(chunk)}: {cause!r}")
        self.start = start
        self.chunk = chunk
        self.__cause__ = cause


def _view(ptr, n):
    if n == 0:
        return memoryview(b"")
    return memoryview((ctypes.c_ubyte * n).from_address(ptr)).cast("B").toreadonly()


class Chunker:
    """Content-defined chunker over a file-like reader (``readinto(buf)`` or
    ``read(n)``)."""

    def __init__(self, reader, min_size, avg_size, max_size, ctx=None, device=0, zero_copy=False):
        self.params = Params(min_size, avg_size, max_size)
        # Next()'s chunk: a bytes copy by default.  zero_copy=True hands out a
        # read-only view of the library's pinned buffer instead (Go's aliasing
        # rule, chunker.go:202-205: valid until the next call on this
        # Chunker), which a caller must not keep: the library may move or free
        # that buffer, and a stale view is a dangling pointer, not stale data.
        self._zero_copy = bool(zero_copy)
        self.r = reader
        # Like a Go Chunker (its own buffer and hash state, chunker.go:108-131)
        # every Chunker owns a library context while it lives: the stream
        # state and device scratch live there.  Without a ctx it takes one
        # from the per-device pool and returns it on close(), so the buffers
        # sized by earlier streams are reused (a fresh context's allocations
        # cost more than chunking 512 MiB).  A caller-supplied ctx must not
        # carry another unfinished stream (dsx_stream_begin: DSX_E_STATE).
        self._own = ctx is None
        self.ctx = _lib.acquire_context(device) if ctx is None else ctx
        try:
            check(lib().dsx_stream_begin(self.ctx.h, ctypes.byref(self.params.c)), self.ctx.h)
        except BaseException:
            if self._own:  # (not pooled: it failed)
                self.ctx.close()
            self.ctx = None
            raise
        # (close() must not end a later Chunker's stream; a token, not self: a
        # reference from the context back to this Chunker would make a cycle,
        # and the cycle collector finalizes a pooled context with it)
        self._token = next(_tokens)
        self.ctx._stream_owner = self._token
        self._eof = False
        self._start = ctypes.c_uint64()
        self._size = ctypes.c_uint64()
        self._ptr = ctypes.c_void_p()
        # the reference's buffer bookkeeping, replayed to place reader errors
        # exactly: Next() refills when fewer than max bytes are buffered
        # (chunker.go:207) and reads up to 10*max (chunker.go:179)
        self._cur = 0       # start of the next chunk
        self._R = 0         # end of the reference's buffer
        self._pos = 0       # bytes received from the reader
        self._err = None    # pending reader exception ...
        self._E = 0         # ... raised at stream position _E
        self._synced = False
        # chunks popped from the library, served one per Next()
        self._ends = (ctypes.c_uint64 * _POP)()
        self._idbuf = None  # (EnableIDs) their IDs
        self._q, self._qi, self._qids = [], 0, b""
        self._n = ctypes.c_uint64()
        self._win, self._wbase = None, 0  # view of the library's held bytes
        self._last_id = None
        # read-ahead beyond the reference's buffer (0: none).  A consumer that
        # reads the stream to its end anyway (ChunkStream) sets it, so that the
        # next batches are on the GPU while it works through this one's chunks
        # instead of the read, the GPU and the consumer taking turns.
        self._ra = 0

    # -- reference API -----------------------------------------------------
    def Next(self):
        """(start, chunk bytes); (start, empty) when the stream is exhausted.
        With zero_copy the chunk is a view valid until the next call."""
        mx = self.params.max
        if self._R - self._cur < mx:  # the reference's fillBuffer
            target = self._cur + 10 * mx
            while self._pos < target and not self._eof and self._err is None:
                self._fill()  # (our reads run ahead of the reference's; make sure they do)
            if self._err is not None and target > self._E:
                return self._read_error()
            self._R = target
        if self._ra and self._pos - self._cur < self._ra // 2:
            target = self._cur + self._ra
            while self._pos < target and not self._eof and self._err is None:
                self._fill()
        if self._qi < len(self._q):
            return self._take()
        L, h = lib(), self.ctx.h
        while True:
            rc = check(L.dsx_stream_pop_many(h, self._ends, self._idbuf, _POP, ctypes.byref(self._start),
                                             ctypes.byref(self._n)), h)
            if rc == 1:
                k = self._n.value
                self._q, self._qi = self._ends[:k], 0
                if self._idbuf is not None:
                    self._qids = bytes(self._idbuf)[:32 * k]
                self._win = None
                return self._take()
            if self._eof:
                return self._start.value, (memoryview(b"") if self._zero_copy else b"")
            if self._err is not None:
                if self._synced:  # cannot happen: the next chunk ends before _E
                    raise RuntimeError("stream stalled behind a reader error")
                check(L.dsx_stream_commit(h, 0, _lib.DSX_STREAM_SYNC), h)
                self._synced = True
                continue
            self._fill()

    def _take(self):
        """The next popped chunk as a view of the library's buffer."""
        if self._win is None:  # (re)map the held bytes after any buffer call
            base, pos, n = ctypes.c_void_p(), ctypes.c_uint64(), ctypes.c_uint64()
            check(lib().dsx_stream_window(self.ctx.h, ctypes.byref(base), ctypes.byref(pos),
                                          ctypes.byref(n)), self.ctx.h)
            self._win, self._wbase = _view(base.value or 0, n.value), pos.value
        i = self._qi
        s, e = self._cur, self._q[i]
        self._qi = i + 1
        self._cur = e
        if self._idbuf is not None:
            self._last_id = self._qids[32 * i:32 * i + 32]
        v = self._win[s - self._wbase:e - self._wbase]
        return s, (v if self._zero_copy else v.tobytes())

    def _next_run(self):
        """What Next() would return over its next calls, up to the next point
        where it reads (the reference's fillBuffer check, or the read-ahead):
        a list of (start, bytes copy, ID or None), [] at the end of the
        stream.  The first chunk comes from Next() itself, so reader errors
        surface exactly where Next() raises them.  (ChunkStream: one call per
        run instead of one per chunk.)"""
        s, b = self.Next()
        if not b:
            return []
        out = [(s, b if not self._zero_copy else b.tobytes(), self._last_id)]
        q, qi, n = self._q, self._qi, len(self._q)
        if qi >= n or self._win is None:
            return out
        win, wb, ids = self._win, self._wbase, self._qids if self._idbuf is not None else None
        cur = self._cur
        k = self._run_end()
        while qi < k:
            e = q[qi]
            out.append((cur, win[cur - wb:e - wb].tobytes(),
                        ids[32 * qi:32 * qi + 32] if ids is not None else None))
            cur = e
            qi += 1
        self._qi, self._cur = qi, cur
        if ids is not None:
            self._last_id = out[-1][2]
        return out

    def _run_end(self):
        """After a Next() that took chunk qi-1 from the popped queue: the end
        k of the run of queued chunks qi..k-1 that Next() would return without
        reading.  Chunk j starts at q[j-1] and is in the run while the
        reference's fillBuffer check would not read (start <= R - max) and
        the read-ahead is not due (start <= pos - ra/2); starts only grow, so
        one bisection.  At the end of the stream (no read can happen, no
        reader error pending) fillBuffer only moves R: the whole queue is the
        run, and R moves as Next() would move it."""
        q, qi, n = self._q, self._qi, len(self._q)
        mx = self.params.max
        if self._eof and self._err is None:
            R = self._R
            for j in range(qi, n):
                if R - q[j - 1] < mx:
                    R = q[j - 1] + 10 * mx
            self._R = R
            return n
        limit = self._R - mx
        if self._ra:
            limit = min(limit, self._pos - self._ra // 2)
        return min(n, bisect.bisect_right(q, limit, qi - 1, n) + 1)

    def _next_block(self, clone=None, max_bytes=None):
        """_next_run's chunks as one block, with no per-chunk object: (start,
        ends, ids, data) -- ends the chunks' absolute end offsets (a list),
        ids their 32-byte IDs concatenated (b"" without IDs), data ONE copy
        of [start, ends[-1]) (``clone(view)`` of the library's bytes, default
        bytes(view)) -- or None at the end of the stream.  The same chunks as
        _next_run, up to the same point (the reference's fillBuffer check or
        the read-ahead) or max_bytes; the first comes from Next()."""
        clone = clone or bytes
        zc, self._zero_copy = self._zero_copy, True  # (the first chunk: a view, cloned below)
        try:
            s, b = self.Next()
        finally:
            self._zero_copy = zc
        if not b:
            return None
        q, qi, n = self._q, self._qi, len(self._q)
        ids = self._qids if self._idbuf is not None else None
        if qi >= n or self._win is None:
            return s, [s + len(b)], self._last_id or b"", clone(b)
        k = self._run_end()
        if max_bytes is not None:  # (at least the first chunk)
            k = max(qi, min(k, bisect.bisect_right(q, s + max_bytes, qi - 1, k)))
        end = q[k - 1]
        first = qi - 1
        data = clone(self._win[s - self._wbase:end - self._wbase])
        idb = ids[32 * first:32 * k] if ids is not None else b""
        self._qi, self._cur = k, end
        if ids is not None:
            self._last_id = ids[32 * (k - 1):32 * k]
        return s, q[first:k], idb, data

    def EnableIDs(self, algo=None):
        """Compute every chunk's Digest.Sum on the GPU next to its cut (for
        ChunkStream); only before the first Next().  ``algo``: "sha512-256"
        or "sha256" (default: the package-global Digest)."""
        from . import make
        check(lib().dsx_stream_ids(self.ctx.h, make._digest_code(algo)), self.ctx.h)
        self._idbuf = (ctypes.c_uint8 * (32 * _POP))()

    def ChunkID(self):
        """The 32-byte ID of the chunk the last Next() returned (EnableIDs)."""
        return self._last_id

    def Advance(self, n):
        """Skip n bytes and restart the hash as if the stream began there."""
        h = self.ctx.h
        check(lib().dsx_stream_unpop(h, self._cur), h)  # (chunks popped ahead go back)
        check(lib().dsx_stream_advance(h, int(n)), h)
        self._q, self._qi, self._win = [], 0, None
        self._cur += int(n)
        self._R = max(self._R, self._cur)

    def Min(self):
        return self.params.min

    def Avg(self):
        return self.params.avg

    def Max(self):
        return self.params.max

    def close(self):
        """Release the stream (and return the context to the pool, if this
        Chunker took it from there; a context whose stream did not end
        cleanly is closed instead)."""
        ctx, self.ctx = self.ctx, None
        if ctx is not None and ctx.h:
            rc = 0
            if getattr(ctx, "_stream_owner", None) == getattr(self, "_token", -1):
                rc = lib().dsx_stream_end(ctx.h)
                ctx._stream_owner = None
            if self._own:
                if rc == 0:
                    _lib.release_context(ctx)
                else:
                    ctx.close()

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
    def _read_error(self):
        L, h = lib(), self.ctx.h
        check(L.dsx_stream_unpop(h, self._cur), h)
        check(L.dsx_stream_flush(h, ctypes.byref(self._start), ctypes.byref(self._size)), h)
        start, n = self._start.value, self._size.value
        chunk = bytes(_view(L.dsx_stream_chunk_data(h), n))
        err, self._err, self._synced = self._err, None, False
        self._q, self._qi, self._win = [], 0, None
        self._cur = self._R = start + n
        raise ChunkerReadError(start, chunk, err)

    def _fill(self):
        L, h = lib(), self.ctx.h
        self._win = None  # the library may move its buffer
        check(L.dsx_stream_buffer(h, _READ, ctypes.byref(self._ptr)), h)
        try:
            if hasattr(self.r, "readinto"):
                got = self.r.readinto(_writable(self._ptr.value, _READ))
            else:
                data = self.r.read(_READ)
                got = len(data) if data else 0
                if got:
                    ctypes.memmove(self._ptr.value, data, got)
        except Exception as e:  # noqa: BLE001 -- any reader failure is Next's err
            self._err, self._E = e, self._pos
            return
        got = got or 0
        self._pos += got
        if got == 0:
            self._eof = True
        check(L.dsx_stream_commit(h, got, _lib.DSX_STREAM_EOF if got == 0 else 0), h)


def _writable(ptr, n):
    return memoryview((ctypes.c_ubyte * n).from_address(ptr)).cast("B")


def NewChunker(reader, min_size, avg_size, max_size, **kw):
    """chunker.go:134 NewChunker."""
    return Chunker(reader, min_size, avg_size, max_size, **kw)
