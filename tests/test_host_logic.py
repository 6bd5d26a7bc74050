"""Host-side logic of the desync_amd mirror that needs no GPU."""
import os
import stat
import struct

import pytest

from desync_amd import make


def test_file_size_regular(tmp_path):
    f = tmp_path / "x"
    f.write_bytes(b"a" * 12345)
    fd = os.open(str(f), os.O_RDONLY)
    try:
        assert make.file_size(fd) == 12345
    finally:
        os.close(fd)


def test_file_size_block_device(monkeypatch, tmp_path):
    """GetFileSize (ioctl_linux.go:63-84): a block device's st_size is 0, its
    size comes from the BLKGETSIZE64 ioctl (mocked: no loop devices here)."""
    import fcntl
    f = tmp_path / "dev"
    f.write_bytes(b"")
    real_fstat = os.fstat

    class St:
        def __init__(self, s):
            self.st_mode = stat.S_IFBLK | 0o660
            self.st_size = 0

    calls = []

    def fake_ioctl(fd, req, arg):
        calls.append(req)
        assert req == 0x80081272  # BLKGETSIZE64 = _IOR(0x12, 114, size_t)
        return struct.pack("Q", 7 << 30)

    monkeypatch.setattr(os, "fstat", lambda fd: St(real_fstat(fd)))
    monkeypatch.setattr(fcntl, "ioctl", fake_ioctl)
    fd = os.open(str(f), os.O_RDONLY)
    try:
        assert make.file_size(fd) == 7 << 30
    finally:
        os.close(fd)
    assert calls == [0x80081272]


def test_chunk_storage_dedup_and_retry():
    """chunkstorage.go: an ID is stored once; IDs the store has are skipped;
    a failed store unmarks the ID so it can be retried."""
    import pytest

    from desync_amd.stream import Chunk, ChunkStorage, MemoryStore

    class Flaky(MemoryStore):
        def __init__(self):
            super().__init__()
            self.calls = 0

        def StoreChunk(self, chunk):
            self.calls += 1
            if self.calls == 1:
                raise IOError("transient")
            super().StoreChunk(chunk)

    ws = Flaky()
    s = ChunkStorage(ws)
    a, b = Chunk(b"a" * 32, b"x"), Chunk(b"b" * 32, b"y")
    with pytest.raises(IOError):
        s.StoreChunk(a)
    s.StoreChunk(a)
    s.StoreChunk(a)
    s.StoreChunk(b)
    assert ws.calls == 3 and set(ws.chunks) == {b"a" * 32, b"b" * 32}
    ws2 = MemoryStore()
    ws2.chunks[b"b" * 32] = b"y"
    s2 = ChunkStorage(ws2)
    s2.StoreChunk(b)
    assert ws2.chunks == {b"b" * 32: b"y"}


def test_memory_store_keeps_its_own_bytes():
    """A store that keeps chunk bytes copies them (ChunkStream's Chunk.Data()
    is a read-only view into a pooled slab; keeping the view would pin the
    whole slab and change under a reused slab)."""
    from desync_amd.stream import Chunk, MemoryStore

    slab = bytearray(b"abcdefgh" * 4)
    ws = MemoryStore()
    ws.StoreChunk(Chunk(b"i" * 32, memoryview(slab)[8:16].toreadonly()))
    slab[8:16] = b"XXXXXXXX"  # the slab is reused
    got = ws.chunks[b"i" * 32]
    assert isinstance(got, bytes) and got == b"abcdefgh"


def test_legacy_hash_type():
    """chunker.go:320-371 (NewHash / Initialize / Roll / IsBoundary / Reset):
    after Initialize on a 48-byte window and Roll over the following bytes,
    the value is the window hash at every position (the oracle's
    restatement), and IsBoundary marks exactly the oracle's candidates."""
    import numpy as np

    from desync_amd.hash import NewHash, hashTable
    from oracle import oracle as o
    assert list(hashTable) == [int(v) for v in o.T]
    data = o.synth_uniform(9, 0, 20000)
    d = o.discriminator(1024)  # dense enough to see boundaries in 20 kB
    h = NewHash(48, d)
    h.Initialize(data[:48].tobytes())
    assert h.value == o.window_hash(data[:48])
    got = [48] if h.IsBoundary() else []
    for p in range(48, data.size):
        h.Roll(int(data[p]))
        if p % 997 == 0:
            assert h.value == o.window_hash(data[p - 47:p + 1])
        if h.IsBoundary():
            got.append(p + 1)
    assert got == o.candidates_np(data, d).tolist() and len(got) > 5
    h.Reset()
    assert h.value == 0 and h.idx == 0
    # a window size other than 48 (Roll rotates the outgoing term by size)
    g = NewHash(16, 7)
    g.Initialize(bytes(range(16)))
    ref = 0
    for i, c in enumerate(range(16)):
        ref ^= o.rotl32(int(o.T[c]), 15 - i)
    assert g.value == ref
    g.Roll(200)
    ref2 = 0
    for i, c in enumerate(list(range(1, 16)) + [200]):
        ref2 ^= o.rotl32(int(o.T[c]), 15 - i)
    assert g.value == ref2
    assert isinstance(g.IsBoundary(), (bool, np.bool_))


def test_chop_batches():
    """ChopFile's read batches (desync_amd.chop._batches): contiguous chunks
    up to 64 MiB per batch, a longer chunk alone, a gap starts a new batch;
    every chunk exactly once, in order."""
    from desync_amd import chop
    from desync_amd.index import IndexChunk
    MiB = 1 << 20
    sizes = [30 * MiB, 30 * MiB, 10 * MiB, 100 * MiB, 1, 5]
    chunks, pos = [], 0
    for s in sizes:
        chunks.append(IndexChunk(b"\0" * 32, pos, s))
        pos += s
    chunks.append(IndexChunk(b"\0" * 32, pos + 7, 3))  # (a gap: a new run)
    got = list(chop._batches(chunks, pos + 10))
    assert [i for i, _ in got] == [0, 2, 3, 4, 6]
    assert [len(b) for _, b in got] == [2, 1, 1, 2, 1]
    assert [c for _, b in got for c in b] == chunks
    for _, b in got:
        assert len(b) == 1 or b[-1].Start + b[-1].Size - b[0].Start <= chop._BATCH


def test_context_pool(monkeypatch):
    """_lib.acquire_context / release_context without a GPU (a stand-in
    Context): an idle context is handed out again under the same DSX_*
    settings only, stale ones are closed on the next acquire, at most
    _POOL_IDLE stay idle, and a context closed while idle is skipped."""
    from desync_amd import _lib

    made = []

    class FakeCtx:
        def __init__(self, device=0):
            self.h, self.device = object(), device
            made.append(self)

        def close(self):
            self.h = None

    monkeypatch.setattr(_lib, "Context", FakeCtx)
    monkeypatch.setattr(_lib, "_pool", {})
    for k in [k for k in os.environ if k.startswith("DSX_")]:
        monkeypatch.delenv(k)
    a = _lib.acquire_context(0)
    _lib.release_context(a)
    assert _lib.acquire_context(0) is a
    b = _lib.acquire_context(0)  # a is in use: a new one
    assert b is not a
    _lib.release_context(a)
    _lib.release_context(b)
    with _lib.pooled_context(0) as c:
        assert c in (a, b)
    monkeypatch.setenv("DSX_SCAN_NT", "0")
    d = _lib.acquire_context(0)
    assert d not in (a, b) and a.h is None and b.h is None  # stale ones closed
    _lib.release_context(d)
    e = _lib.acquire_context(1)  # another device's pool does not touch device 0's
    assert e is not d and d.h is not None
    _lib.release_context(e)
    many = [_lib.acquire_context(0) for _ in range(_lib._POOL_IDLE + 2)]
    for x in many:
        _lib.release_context(x)
    assert sum(x.h is not None for x in many) == _lib._POOL_IDLE
    idle = [x for x in many if x.h is not None]
    for x in idle[:-1]:
        x.close()  # closed while idle (reset_context_pool, another owner)
    assert _lib.acquire_context(0) is idle[-1]
    n = len(made)
    assert _lib.acquire_context(0) not in many and len(made) == n + 1


def test_clone_pool_reuses_released_slabs():
    """ChunkStream's clones (desync_amd.stream._ClonePool): a slab returns to
    the pool once the last chunk view of it is gone, a store that keeps its
    chunks' bytes makes the pool fall back to fresh copies, and every clone is
    a read-only copy of its source."""
    import gc

    import numpy as np

    from desync_amd import stream
    pool = stream._ClonePool(2)
    src = np.arange(1 << 20, dtype=np.uint64).view(np.uint8)
    a = pool.clone(memoryview(src))
    assert a.readonly and bytes(a[:64]) == src[:64].tobytes() and len(a) == src.size
    base_a = a.obj.base
    b = pool.clone(memoryview(src[:4096]))  # the second (and last) slab
    kept = b[100:200]  # a store keeping a chunk view holds b's slab
    del a
    gc.collect()
    c = pool.clone(memoryview(src[:8192]))  # a's slab, released
    assert c.obj.base is base_a
    d = pool.clone(memoryview(src[:16]))  # no free slab: a fresh copy
    assert isinstance(d.obj, bytes) and bytes(d) == src[:16].tobytes()
    assert bytes(kept) == src[100:200].tobytes()
    big = pool.clone(memoryview(np.zeros(stream._SLAB + 1, np.uint8)))  # larger than a slab
    assert isinstance(big.obj, bytes) and len(big) == stream._SLAB + 1


def test_host_copy_pool():
    """dsx_host_copy (ChunkStream's clone of a run): every size and thread
    count copies the bytes exactly, including the ragged last part and sizes
    below one part; overlapping ranges are refused.  Host only, no GPU."""
    import ctypes

    import numpy as np

    from desync_amd import _lib, stream
    L = _lib.lib()
    rng = np.random.default_rng(11)
    src = rng.integers(0, 256, (9 << 20) + 4321, dtype=np.uint8)
    for n in (0, 1, 4095, 1 << 20, (1 << 20) + 1, (3 << 20) + 12345, src.size):
        for threads in (0, 1, 2, 4, 16):
            dst = np.zeros(n + 64, np.uint8)
            assert L.dsx_host_copy(dst.ctypes.data, src.ctypes.data, n, threads) == 0
            assert np.array_equal(dst[:n], src[:n]) and not dst[n:].any(), (n, threads)
    buf = np.zeros(4 << 20, np.uint8)
    assert L.dsx_host_copy(buf.ctypes.data + 4096, buf.ctypes.data, 2 << 20, 4) == _lib.DSX_E_INVAL
    assert L.dsx_host_copy(None, ctypes.c_void_p(buf.ctypes.data), 16, 4) == _lib.DSX_E_INVAL
    # the clone pool's copies go through it
    pool = stream._ClonePool(1)
    v = pool.clone(memoryview(src[:(5 << 20) + 7]))
    assert bytes(v) == src[:(5 << 20) + 7].tobytes()


def test_host_sha512_256():
    """dsx_host_sha512_256, the host SHA-512/256 of the index pipeline's tail
    (digest.go:22): the AVX-512 multi-buffer form (when the CPU has it) and
    the scalar form against hashlib, over the padding edge lengths (111, 112,
    127, 128, 239, 240 ...), empty messages, groups of 8 with ragged lengths
    and a thread count above the group count.  Host only, no GPU."""
    import ctypes
    import hashlib

    import numpy as np

    from desync_amd import _lib
    L = _lib.lib()
    rng = np.random.default_rng(12)
    lens = [0, 1, 55, 111, 112, 113, 127, 128, 129, 239, 240, 241, 256, 1000, 65536, 262144]
    lens += [int(x) for x in rng.integers(0, 300000, 45)]
    bufs = [rng.integers(0, 256, n, dtype=np.uint8) for n in lens]
    ptrs = (ctypes.c_void_p * len(bufs))(*[b.ctypes.data if b.size else None for b in bufs])
    ln = (ctypes.c_uint64 * len(bufs))(*lens)
    want = [hashlib.new("sha512_256", b.tobytes()).digest() for b in bufs]
    for flags in (0, _lib.DSX_HOST_SHA_SCALAR):
        for threads in (1, 3, 64):
            out = np.zeros(32 * len(bufs), np.uint8)
            assert L.dsx_host_sha512_256(ptrs, ln, len(bufs), out.ctypes.data, threads, flags) == 0
            got = [out[32 * i:32 * i + 32].tobytes() for i in range(len(bufs))]
            assert got == want, (flags, threads)
    assert L.dsx_host_sha512_256(ptrs, ln, len(bufs), None, 1, 0) == _lib.DSX_E_INVAL
    assert L.dsx_host_sha512_256(ptrs, ln, len(bufs), out.ctypes.data, 1, 4) == _lib.DSX_E_INVAL


def test_chunkstream_store_workers():
    """ChunkStream's store workers over blocks of chunks (a stand-in chunker,
    no GPU): an ID repeated within and across hand-offs is stored once (the
    reference's ChunkStorage), a store that has an ID is not asked to store
    it, the index lists every chunk in order, and a failing store raises out
    of ChunkStream and no chunk is stored after it."""
    import hashlib

    import numpy as np

    from desync_amd import stream

    rng = np.random.default_rng(3)
    data = rng.integers(0, 256, 3 << 20, dtype=np.uint8).tobytes()
    sizes = rng.integers(1000, 9000, 600)
    ends = np.cumsum(sizes)
    ends = ends[ends < len(data)].tolist() + [len(data)]
    # IDs: every 7th chunk repeats the ID of the chunk before it
    ids = [hashlib.sha256(str(i - (i % 7 == 0 and i > 0)).encode()).digest() for i in range(len(ends))]

    class Blocks:
        def __init__(self, per):
            self.i, self.per = 0, per

        def EnableIDs(self):
            pass

        def _next_block(self, clone, max_bytes):
            i = self.i
            if i >= len(ends):
                return None
            k = min(len(ends), i + self.per)
            s = ends[i - 1] if i else 0
            self.i = k
            return s, ends[i:k], b"".join(ids[i:k]), clone(memoryview(data)[s:ends[k - 1]])

        def Min(self):
            return 1000

        def Avg(self):
            return 4000

        def Max(self):
            return 9000

    class Store:
        def __init__(self, fail_at=None, have=()):
            self.got, self.fail_at, self.have = {}, fail_at, set(have)

        def HasChunk(self, cid):
            return cid in self.have

        def StoreChunk(self, ch):
            if self.fail_at is not None and len(self.got) == self.fail_at:
                raise IOError("disk full")
            assert ch.ID() not in self.got
            self.got[ch.ID()] = bytes(ch.Data())

    for per in (1, 5, 64, 200):
        st = Store(have=ids[10:12])
        idx = stream.ChunkStream(None, Blocks(per), st, 3)
        assert [c.Start + c.Size for c in idx.Chunks] == ends
        assert [c.ID for c in idx.Chunks] == ids
        want = {}
        for i, e in enumerate(ends):
            if ids[i] not in ids[10:12]:
                want.setdefault(ids[i], data[(ends[i - 1] if i else 0):e])
        assert st.got == want, per
    st = Store(fail_at=40)
    with pytest.raises(IOError, match="disk full"):
        stream.ChunkStream(None, Blocks(64), st, 2)
    assert len(st.got) == 40


def test_chunk_array_start():
    """Index.Chunks as a ChunkArray whose first chunk starts past 0 (a stream
    that began at an offset): Start/Size of each element, materialised or
    not, and the caibx table of absolute chunk ends."""
    import numpy as np

    from desync_amd.index import ChunkArray
    ends = np.array([1500, 4000, 4100], np.uint64)
    ids = bytes(range(96))
    ca = ChunkArray(ends, ids, start=1000)
    assert (ca[0].Start, ca[0].Size) == (1000, 500) and ca[2].ID == bytes(range(64, 96))
    assert [(c.Start, c.Size) for c in ca] == [(1000, 500), (1500, 2500), (4000, 100)]


def test_smu_summary_window():
    """tools/smu_summary.py over synthetic SMU samples: energy from the
    accumulator over the --marks window, J/GiB above idle, PPT residency from
    the accumulation counters."""
    import importlib.util
    import json
    import os
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools",
                        "smu_summary.py")
    spec = importlib.util.spec_from_file_location("smu_summary", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    rows, e, t0 = [], 0.0, 1000.0
    for i in range(2000):  # 2 ms samples: 0.4 s idle at 250 W, 2 s at 1400 W, idle again
        t = t0 + 0.002 * i
        p = 1400.0 if 0.4 <= t - t0 < 2.4 else 250.0
        e += p * 0.002 / 15.259e-6
        r = {"t": t, "current_socket_power": p, "energy_accumulator": int(e),
             "accumulation_counter": i, "ppt_residency_acc": min(max(i - 200, 0), 400)}
        rows.append(r)
    static = {"energy": {"counter_resolution": 15.259}}
    out = mod.summarise(static, rows, {"t0": t0 + 0.5, "t1": t0 + 2.0, "bytes": 3 << 30})
    json.dumps(out)
    assert abs(out["mean_power_w"] - 1400) < 2 and out["idle_w"] == 250.0
    assert abs(out["j_per_gib"] - 1400 * 1.5 / 3) < 1
    assert abs(out["j_per_gib_above_idle"] - 1150 * 1.5 / 3) < 1
    assert abs(out["res_ppt"] - 350 / 750) < 0.01  # (PPT active over samples 200..599)


def _diag_lib():
    import ctypes
    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "desync_amd",
                        "libdsx_diag.so")
    if not os.path.exists(path):
        pytest.skip("libdsx_diag.so not built (make -C desync_amd/csrc diag)")
    lib = ctypes.CDLL(path)
    u64p = ctypes.POINTER(ctypes.c_uint64)
    lib.dsx_diag_index_plan.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_int, u64p, u64p,
                                        u64p, u64p, ctypes.c_int]
    lib.dsx_diag_index_plan.restype = ctypes.c_int
    lib.dsx_diag_index_pieces.argtypes = [ctypes.c_uint64] * 4 + [ctypes.c_int, u64p, u64p, ctypes.c_uint64]
    lib.dsx_diag_index_pieces.restype = ctypes.c_uint64
    return lib


@pytest.mark.parametrize("length,threads,fcut,fcut_end,shares", [
    # 1 GiB at the box's 12 feeder threads: two shares (the first half wholly
    # on the GPU), 44 KiB after them
    (1 << 30, 12, 65536, 45056, [(1 << 29, 262144), (3 << 28, 131072)]),
    # tests/test_gpu_index.py::test_index_host_tail_gpu_shares' cases
    ((320 << 20) + 4321, 28, 28672, 28672, [(((320 << 20) + 4321) // 2, 81920)]),
    ((640 << 20) + 4321, 28, 28672, 28672, [(((640 << 20) + 4321) // 2, 163840),
                                            (3 * ((640 << 20) + 4321) // 4, 81920)]),
    # too short for a share at 1/2; one thread: the cut clamps at 128 KiB
    (64 << 20, 12, 65536, 65536, []),
    (1 << 30, 1, 131072, 90112, [(1 << 29, 262144)]),
])
def test_index_share_plan(length, threads, fcut, fcut_end, shares):
    """The one-window IndexFromFile plan (dsx_index.cpp plan_shares,
    feed_cut_for, share_end_cut): the feeder's cut from its threads, the GPU's
    shares at 1/2, 3/4, ... with cut = the read time left / 45 ns per byte,
    stopping below 1.5 x the feeder's cut, and 11/16 of it after them."""
    import ctypes
    lib = _diag_lib()
    a, b = ctypes.c_uint64(), ctypes.c_uint64()
    at, cut = (ctypes.c_uint64 * 8)(), (ctypes.c_uint64 * 8)()
    n = lib.dsx_diag_index_plan(length, 256 << 10, threads, ctypes.byref(a), ctypes.byref(b), at, cut, 8)
    assert (a.value, b.value) == (fcut, fcut_end)
    got = [(at[i], cut[i]) for i in range(n)]
    assert [c for _, c in got] == [c for _, c in shares]
    assert all(abs(x - y) <= 1 for (x, _), (y, _) in zip(got, shares))


def test_index_piece_map():
    """The pieces run_index reads (IndexGeom + PieceMap): they tile the file;
    32 MiB slots, and with the tail feeder the last 32 MiB of the last window
    in 8 MiB pieces; windows stay whole multiples of the slot."""
    import ctypes
    import random
    lib = _diag_lib()
    slot, window = 32 << 20, 1 << 30
    rnd = random.Random(5)
    cases = [1, 4095, 4096, 8 << 20, (32 << 20) + 1, 1 << 30, (1 << 30) + 12345, (3 << 30) - 7]
    cases += [rnd.randrange(1, 5 << 30) for _ in range(40)]
    for length in cases:
        for feeds in (0, 1):
            cap = 4096
            off, size = (ctypes.c_uint64 * cap)(), (ctypes.c_uint64 * cap)()
            n = lib.dsx_diag_index_pieces(length, 256 << 10, slot, window, feeds, off, size, cap)
            assert 0 < n <= cap
            pos = 0
            for k in range(n):
                assert off[k] == pos and 0 < size[k] <= slot, (length, feeds, k)
                pos += size[k]
            assert pos == length
            piece = min(slot, max(length, 4096) + 4095 & ~4095)
            fine = [k for k in range(n) if size[k] < piece and off[k] + size[k] < length]
            if not feeds or piece <= 4 * 4096:
                assert not fine, (length, feeds)
            else:
                # the small pieces are the file's last 32 MiB (rounded down to
                # a slot), inside its last window
                assert all(off[k] >= length - (32 << 20) - piece for k in fine), (length, feeds)
