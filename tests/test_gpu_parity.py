"""GPU parity: the HIP path (through the C ABI) vs the CPU oracle.

Bit-exact for every cut.  Small inputs are compared cut-for-cut with the
oracle; the reference's goldens (caibx files) are matched byte for byte end
to end; at the BASELINE sizes the same comparison is made against the C
oracle on the same seeded bytes (regenerated on the CPU).
"""
import ctypes
import io
import os

import numpy as np
import pytest

from oracle import oracle as o

pytestmark = pytest.mark.gpu

MIN, AVG, MAX = 16 * 1024, 64 * 1024, 256 * 1024


def torch_dev(arr):
    import torch
    t = torch.from_numpy(np.array(arr, dtype=np.uint8, copy=True)).to("cuda")
    torch.cuda.synchronize()
    return t


def gpu_cut(dctx, arr, mn=MIN, av=AVG, mx=MAX):
    import desync_amd
    t = torch_dev(arr)
    return desync_amd.cut_device(t.data_ptr(), t.numel(), mn, av, mx, ctx=dctx)


# ---------------------------------------------------------------- predicate
@pytest.mark.parametrize("avg", [16 * 1024, 64 * 1024, 256 * 1024, 1024 * 1024, 8192, 4096, 1000])
@pytest.mark.parametrize("mode", [0, 1, 2, -1])
def test_boundary_predicate_ranges(dctx, avg, mode):
    """chunker_test.go:190-213 on the device: [0,3d) and [2^32-1-3d, 2^32)."""
    import desync_amd
    from desync_amd import _lib
    p = desync_amd.Params(max(48, avg // 4), avg, avg * 4)
    d = p.discriminator
    if mode == 1 and not (2048 < d < (1 << 24)):
        pytest.skip("float form is only used for 2048 < d < 2^24")
    if mode == 2 and d & (d - 1) == 0:
        pytest.skip("prefilter form needs d with an odd factor > 1")
    for h0, n in ((0, 3 * d), (2**32 - 1 - 3 * d, 3 * d + 1), (0x5A5A5A5A, 1 << 24)):
        bad = ctypes.c_uint64()
        _lib.check(_lib.lib().dsx_selftest_boundary(dctx.h, ctypes.byref(p.c), mode, h0, n,
                                                    ctypes.byref(bad)), dctx.h)
        assert bad.value == 0


@pytest.mark.parametrize("avg", [16 * 1024, 64 * 1024, 256 * 1024])
@pytest.mark.parametrize("mode", [1, 2])
def test_boundary_predicate_exhaustive(dctx, avg, mode):
    """All 2^32 hash values for the BASELINE discriminators."""
    import desync_amd
    from desync_amd import _lib
    p = desync_amd.Params(avg // 4, avg, avg * 4)
    bad = ctypes.c_uint64()
    _lib.check(_lib.lib().dsx_selftest_boundary(dctx.h, ctypes.byref(p.c), mode, 0, 1 << 32,
                                                ctypes.byref(bad)), dctx.h)
    assert bad.value == 0


# ---------------------------------------------------------------- goldens
GOLDEN_PAIRS = [
    ("chunker.input", "chunker.index"),
    ("blob1", "blob1.caibx"),
    ("blob2", "blob2.caibx"),
    ("tree.catar", "tree.caidx"),
]


@pytest.mark.parametrize("inp,idx", GOLDEN_PAIRS)
def test_device_cuts_match_golden(dctx, golden, inp, idx):
    data = np.frombuffer(golden(inp), np.uint8)
    d = o.decode_caibx(golden(idx))
    ends = gpu_cut(dctx, data, d["min"], d["avg"], d["max"])
    assert np.array_equal(ends, d["ends"])


@pytest.mark.parametrize("inp,idx", GOLDEN_PAIRS)
def test_index_from_file_bit_identical(dctx, golden, inp, idx, tmp_path):
    """desync make: IndexFromFile + WriteTo == the reference's caibx bytes."""
    import desync_amd
    ref = golden(idx)
    d = o.decode_caibx(ref)
    f = tmp_path / inp
    f.write_bytes(golden(inp))
    index, stats = desync_amd.IndexFromFile(None, str(f), 4, d["min"], d["avg"], d["max"])
    b = io.BytesIO()
    index.WriteTo(b)
    assert b.getvalue() == ref
    assert stats.ChunksAccepted == len(d["ends"])
    assert stats.ChunksProduced >= stats.ChunksAccepted  # (+ cuts a stitch repair replaced)


class _Progress:
    def __init__(self):
        self.total, self.added, self.finished = None, 0, False

    def SetTotal(self, n):
        self.total = n

    def Start(self):
        pass

    def Add(self, n):
        self.added += n

    def Finish(self):
        self.finished = True


@pytest.mark.parametrize("blob,idx", [("blob1", "blob1.caibx"), ("blob2", "blob2.caibx")])
def test_verify_index_golden(dctx, golden, tmp_path, blob, idx):
    """cmd/desync/verifyindex_test.go:10-31: the reference's own index verifies
    against its blob (IDs recomputed by dsx_chunk_ids), a one-byte change in
    any chunk is caught, and blob2.caibx does not verify blob1."""
    import desync_amd
    index = desync_amd.IndexFromReader(golden(idx))
    f = tmp_path / blob
    data = bytearray(golden(blob))
    f.write_bytes(bytes(data))
    pb = _Progress()
    assert desync_amd.VerifyIndex(None, str(f), index, 4, pb) is None
    assert pb.total == len(index.Chunks) == pb.added and pb.finished
    for c in (index.Chunks[0], index.Chunks[len(index.Chunks) // 2], index.Chunks[-1]):
        bad = bytearray(data)
        bad[c.Start + c.Size - 1] ^= 0x40
        f.write_bytes(bytes(bad))
        with pytest.raises(desync_amd.VerifyError, match="doesn't match its data"):
            desync_amd.VerifyIndex(None, str(f), index, 4)
    other = tmp_path / "other"
    other.write_bytes(golden("blob1" if blob == "blob2" else "blob2"))
    with pytest.raises(desync_amd.VerifyError):
        desync_amd.VerifyIndex(None, str(other), index, 1)


@pytest.mark.parametrize("algo", ["sha512-256", "sha256"])
def test_verify_index_roundtrip(dctx, tmp_path, algo):
    """IndexFromFile -> VerifyIndex over 5 MiB of seeded bytes, both digests;
    a hand-built index with a gap between chunks (non-contiguous runs) is
    verified per run and checked against hashlib."""
    import hashlib

    import desync_amd
    from desync_amd import digest
    data = o.synth_uniform(11, 0, 5 << 20)
    f = tmp_path / "blob"
    f.write_bytes(data.tobytes())
    prev = digest.Digest.Algorithm()
    desync_amd.set_digest(algo)
    try:
        index, _ = desync_amd.IndexFromFile(None, str(f), 2, 4096, 16384, 65536)
        desync_amd.VerifyIndex(None, str(f), index, 2)
        h = (lambda b: hashlib.new("sha512_256", b).digest()) if algo == "sha512-256" \
            else (lambda b: hashlib.sha256(b).digest())
        raw = data.tobytes()
        spans = [(0, 1000), (5000, 70000), (70000, 3), (4 << 20, (1 << 20) - 7)]
        hand = desync_amd.Index(index.Index, [desync_amd.IndexChunk(ID=h(raw[s:s + n]), Start=s, Size=n)
                                              for s, n in spans])
        hand.Chunks.append(desync_amd.IndexChunk(ID=h(raw[(5 << 20) - 7:]), Start=(5 << 20) - 7, Size=7))
        desync_amd.VerifyIndex(None, str(f), hand, 1)
        hand.Chunks[2] = desync_amd.IndexChunk(ID=h(b"x"), Start=70000, Size=3)
        with pytest.raises(desync_amd.VerifyError):
            desync_amd.VerifyIndex(None, str(f), hand, 1)
    finally:
        desync_amd.set_digest(prev)


def test_large_file_next(dctx, golden):
    """TestChunkerLargeFile through Chunker.Next (streaming path)."""
    import desync_amd
    from test_oracle_golden import LARGE_FILE
    import hashlib
    c = desync_amd.NewChunker(io.BytesIO(golden("chunker.input")), MIN, AVG, MAX, ctx=dctx)
    for start, size, sid in LARGE_FILE:
        s, b = c.Next()
        assert (s, len(b), hashlib.new("sha512_256", b).hexdigest()) == (start, size, sid)
    s, b = c.Next()
    assert b == b""


# ---------------------------------------------------------------- edge cases
def test_edge_cases(dctx):
    """chunker_test.go:69-131 on the device path."""
    import desync_amd
    import torch
    t = torch.zeros(16, dtype=torch.uint8, device="cuda")
    assert desync_amd.cut_device(t.data_ptr(), 0, MIN, AVG, MAX, ctx=dctx).size == 0
    assert gpu_cut(dctx, np.arange(16, dtype=np.uint8)).tolist() == [16]
    assert gpu_cut(dctx, np.zeros(1 << 20, np.uint8)).tolist() == [MAX * (i + 1) for i in range(4)]
    for size in (MIN, AVG, MAX):
        assert gpu_cut(dctx, np.zeros(size, np.uint8)).tolist() == [size]
    for size in (1, 47, 48, 49, MIN - 1, MIN + 1, MIN + 48, MIN + 49, MAX + 1, 2 * MAX - 1):
        data = o.synth_uniform(11, 0, size)
        assert np.array_equal(gpu_cut(dctx, data), o.chunk_stream(data, MIN, AVG, MAX)), size


def test_chunker_advance(dctx):
    """TestChunkerAdvance (chunker_test.go:134-175)."""
    import desync_amd
    null = bytes(MAX)
    data_a = b"a" * 128
    data_b = b"b" * (12 * MAX)
    inp = null + data_a + null + data_b
    c = desync_amd.NewChunker(io.BytesIO(inp), MIN, AVG, MAX, ctx=dctx)
    _, b = c.Next()
    assert b == null
    c.Advance(len(data_a))
    _, b = c.Next()
    assert b == null
    c.Advance(len(data_b))
    _, b = c.Next()
    assert b == b""


# ---------------------------------------------------------------- seeded random
@pytest.mark.parametrize("seed,size", [(1, 1 << 20), (2, 3 * (1 << 20) + 12345), (3, 17 << 20),
                                       (4, 64 << 20)])
def test_random_default_params(dctx, seed, size):
    data = o.synth_uniform(seed, 0, size)
    assert np.array_equal(gpu_cut(dctx, data), o.chunk_stream(data, MIN, AVG, MAX))


@pytest.mark.parametrize("avg", [16 * 1024, 64 * 1024, 256 * 1024, 8192, 4096, 2048, 1000, 192])
def test_random_avg_sweep(dctx, avg):
    mn, mx = max(48, avg // 4), avg * 4
    data = o.synth_uniform(5, 0, 9 << 20)
    assert np.array_equal(gpu_cut(dctx, data, mn, avg, mx), o.chunk_stream(data, mn, avg, mx))


@pytest.mark.parametrize("env", [{"DSX_LANE_TARGET": "384"}, {"DSX_LANE_TARGET": "2304"}, {}])
def test_scan_geometries(env, monkeypatch):
    """The line-aligned scan with short lane segments (DSX_LANE_TARGET: many
    regions per wave slot from the work queue) and device pointers off the
    128-B line grid: at the blob start (the 96-B-row scan_kernel) and inside
    it (shard pieces: grid origin before the piece start)."""
    import torch
    import desync_amd
    from desync_amd import _lib
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    ctx = _lib.Context(0)
    try:
        data = o.synth_uniform(31, 0, (24 << 20) + 333)
        assert np.array_equal(gpu_cut(ctx, data), o.chunk_stream(data, MIN, AVG, MAX))
        for off in (195, 73, 128):  # blobs starting off (or on) the line grid
            n = (8 << 20) + off
            arr = o.synth_uniform(32 + off, 0, n)
            tt = torch_dev(np.concatenate([np.zeros(off, np.uint8), arr]))
            got = desync_amd.cut_device(tt.data_ptr() + off, n, MIN, AVG, MAX, ctx=ctx)
            assert np.array_equal(got, o.chunk_stream(arr, MIN, AVG, MAX)), off
        # shard pieces at odd positions: the line grid starts before the piece
        _shard_protocol(o.synth_uniform(33, 0, (6 << 20) + 1001), 3, False)
    finally:
        ctx.close()


def test_odd_params(dctx):
    """min == avg == max, min = 48, max >> avg."""
    data = o.synth_uniform(6, 0, 3 << 20)
    for mn, av, mx in ((48, 48, 48), (48, 4096, 1 << 20), (1000, 1000, 1000), (4096, 4096, 65536),
                       (64, 100, 50000)):
        assert np.array_equal(gpu_cut(dctx, data, mn, av, mx), o.chunk_stream(data, mn, av, mx)), \
            (mn, av, mx)


def test_null_compositions(dctx):
    """make_test.go:16-80 inputs (random/null blocks of 4*max)."""
    rng = np.random.default_rng(7)
    null = np.zeros(4 * MAX, np.uint8)
    r1 = rng.integers(0, 256, 4 * MAX, dtype=np.uint8)
    r2 = rng.integers(0, 256, 4 * MAX, dtype=np.uint8)
    for parts in ([r1, r2, r1, r2, r1], [null] * 4 + [r1, r2], [r1, r2] + [null] * 4,
                  [r1] + [null] * 4 + [r2], [r1, null, null, null, r1, null, null, null, r2]):
        data = np.concatenate(parts)
        assert np.array_equal(gpu_cut(dctx, data), o.chunk_stream(data, MIN, AVG, MAX))


def test_periodic_dense_candidates(dctx):
    """Adversarial data with a boundary candidate every 48 bytes: chains never
    re-synchronise, exercising the dense-slot path and the sequential repair."""
    P = o.params(MIN, AVG, MAX)
    rng = np.random.default_rng(1)
    while True:  # find a 48-byte block whose periodic window hash is a candidate
        blk = rng.integers(0, 256, 48, dtype=np.uint8)
        if o.window_hash(bytes(blk)) % P.d == P.d - 1:
            break
    data = np.tile(blk, (3 << 20) // 48)
    assert np.array_equal(gpu_cut(dctx, data), o.chunk_stream(data, MIN, AVG, MAX))


def _window_with_hash(target, seed):
    """A 48-byte window whose rolling hash (chunker.go:225-228) is `target`:
    44 random bytes, the last 4 by meet-in-the-middle over two byte pairs."""
    rng = np.random.default_rng(seed)
    T = np.array([int(v) for v in o.T], dtype=np.uint64)
    rot = lambda v, r: ((v << np.uint64(r)) | (v >> np.uint64(32 - r))) & np.uint64(0xFFFFFFFF) if r else v
    while True:
        w = rng.integers(0, 256, 48, dtype=np.uint8)
        w[44:] = 0
        resid = np.uint64(target ^ o.window_hash(bytes(w)) ^ int(rot(T[0], 3) ^ rot(T[0], 2) ^ rot(T[0], 1) ^ T[0]))
        a = (rot(T, 3)[:, None] ^ rot(T, 2)[None, :]).ravel()           # bytes 44, 45
        b = (rot(T, 1)[:, None] ^ T[None, :] ^ resid).ravel()           # bytes 46, 47
        common, ia, ib = np.intersect1d(a, b, return_indices=True)
        if common.size:
            w[44], w[45] = divmod(int(ia[0]), 256)
            w[46], w[47] = divmod(int(ib[0]), 256)
            assert o.window_hash(bytes(w)) == target
            return w


@pytest.mark.parametrize("avg", [16 * 1024, 64 * 1024, 256 * 1024])
def test_scan_hash_all_ones(dctx, avg):
    """Windows whose hash is 2^32 - 1, where the boundary test's product
    (h+1)*inv is 0: the scan's hit path bounds x - qBias <= qMax as
    x <= qMax + qBias only for waves with no such product, and a wave with one
    takes the exact form.  The window is planted 200 times (next to real
    candidates too) at odd and even d; the cuts must equal the oracle's."""
    w = _window_with_hash(0xFFFFFFFF, 9)
    mn, mx = avg // 4, avg * 4
    data = o.synth_uniform(41, 0, 12 << 20).copy()
    cands = o.candidates(data, mn, avg, mx)
    rng = np.random.default_rng(2)
    spots = list(rng.integers(0, data.size - 48, 150)) + [int(c) - 60 for c in cands[:50] if c > 60]
    for s in spots:
        data[s:s + 48] = w
    assert np.array_equal(gpu_cut(dctx, data, mn, avg, mx), o.chunk_stream(data, mn, avg, mx))


def test_stitch_many_workgroups_and_repairs(monkeypatch):
    """The stitch on many walk workgroups (small segments) and on seams inside
    zero runs (suspect segments: fixup_kernel's sequential repair)."""
    from desync_amd import _lib
    monkeypatch.setenv("DSX_SEG_FLOOR", "65536")
    ctx = _lib.Context(0)
    try:
        mn, av, mx = 4096, 16384, 65536  # 256 KiB segments: 257 of them, 129 workgroups
        data = o.synth_uniform(41, 0, (64 << 20) + 4321)
        assert np.array_equal(gpu_cut(ctx, data, mn, av, mx), o.chunk_stream(data, mn, av, mx))
        rng = np.random.default_rng(11)
        null = np.zeros(4 * MAX, np.uint8)
        r1 = rng.integers(0, 256, 4 * MAX, dtype=np.uint8)
        # a random head of odd length puts the true chain inside the zero runs
        # off the segment grid: those seams do not converge (repairs)
        for parts in ([r1[:12345], null, null, null, r1, null, r1], [null] * 6 + [r1]):
            d = np.concatenate(parts)
            assert np.array_equal(gpu_cut(ctx, d), o.chunk_stream(d, MIN, AVG, MAX))
            if parts[0] is not null:
                assert ctx.stats().repaired_segments > 0
            assert np.array_equal(gpu_cut(ctx, d, mn, av, mx), o.chunk_stream(d, mn, av, mx))
        # a true chain off the max lattice through 6 segments of zeros (the
        # last cut of a random megabyte before them): every zero segment's
        # staged chain, entered from the speculative exit, misses the true
        # one, so the repair replaces its staged cuts -- the chunks make.go
        # would count as produced and dropped (ChunksProduced > ChunksAccepted)
        d = np.concatenate([rng.integers(0, 256, 1 << 20, dtype=np.uint8),
                            np.zeros(6 << 20, np.uint8), r1])
        assert np.array_equal(gpu_cut(ctx, d), o.chunk_stream(d, MIN, AVG, MAX))
        st = ctx.stats()
        assert st.repaired_segments > 0 and st.chunks_discarded > 0, (st.repaired_segments,
                                                                       st.chunks_discarded)
    finally:
        ctx.close()


# ---------------------------------------------------------------- host paths
def test_host_and_fd_paths(dctx, tmp_path):
    import desync_amd
    data = o.synth_uniform(8, 0, (600 << 20) + 777)  # > one 256 MiB pipeline chunk
    ref = o.chunk_stream(data, MIN, AVG, MAX)
    assert np.array_equal(desync_amd.cut_host(data, MIN, AVG, MAX, ctx=dctx), ref)
    f = tmp_path / "blob"
    data.tofile(str(f))
    fd = os.open(str(f), os.O_RDONLY)
    try:
        assert np.array_equal(desync_amd.cut_fd(fd, MIN, AVG, MAX, ctx=dctx), ref)
    finally:
        os.close(fd)


def test_stream_matches(dctx):
    import desync_amd
    data = o.synth_uniform(9, 0, (40 << 20) + 5)
    ref = o.chunk_stream(data, MIN, AVG, MAX)
    c = desync_amd.NewChunker(io.BytesIO(data.tobytes()), MIN, AVG, MAX, ctx=dctx)
    ends = [s + len(b) for s, b in c]
    assert ends == ref.tolist()


class _FailingReader:
    """Serves data[:E], raises OSError once, then serves data[E:] (resume) or
    nothing (EOF)."""

    def __init__(self, data, E, resume, chunk=3 << 20):
        self.b, self.E, self.resume, self.pos, self.failed, self.chunk = data, E, resume, 0, False, chunk

    def read(self, n):
        if not self.failed and self.pos >= self.E:
            self.failed = True
            raise OSError("injected read error")
        if not self.failed:
            limit = self.E
        else:
            limit = len(self.b) if self.resume else self.pos  # resume, or EOF
        end = min(self.pos + n, self.pos + self.chunk, limit)
        out = self.b[self.pos:end]
        self.pos = end
        return out


def _go_next_with_error(data, E, resume, mn, av, mx):
    """What the reference's Chunker.Next returns (chunker.go:175-277) when the
    reader fails at stream position E: chunks of the sequential chain while
    its buffer holds >= max bytes, then (cur, data[cur:E], err) at the first
    fillBuffer that would cross E, then chunking starts over at E."""
    ref = o.chunk_stream(data, mn, av, mx).tolist()
    out, cur, R, i = [], 0, 0, 0
    while True:
        if R - cur < mx:
            if cur + 10 * mx > E:
                out.append(("err", cur, E))
                break
            R = cur + 10 * mx
        while ref[i] <= cur:
            i += 1
        out.append(("chunk", cur, ref[i]))
        cur = ref[i]
    if resume:
        tail = o.chunk_stream(data[E:], mn, av, mx).tolist()
        s = E
        for e in tail:
            out.append(("chunk", s, E + e))
            s = E + e
    return out


@pytest.mark.parametrize("E,resume", [(100_000, False), ((5 << 20) + 123, False),
                                      ((5 << 20) + 123, True), ((70 << 20) + 7, True)])
def test_stream_reader_error(dctx, E, resume):
    """chunker.go:207-211: a reader error returns the buffered bytes with the
    error, where the reference's fillBuffer would hit it; then chunking
    restarts behind them (resume) or the stream ends."""
    import desync_amd
    data = o.synth_uniform(14, 0, (90 << 20) + 11)
    want = _go_next_with_error(data, E, resume, MIN, AVG, MAX)
    c = desync_amd.NewChunker(_FailingReader(data.tobytes(), E, resume), MIN, AVG, MAX)
    got = []
    while True:
        try:
            s, b = c.Next()
        except desync_amd.ChunkerReadError as e:
            assert bytes(e.chunk) == data[e.start:e.start + len(e.chunk)].tobytes()
            assert isinstance(e.__cause__, OSError)
            got.append(("err", e.start, e.start + len(e.chunk)))
            continue
        if not b:
            break
        assert bytes(b) == data[s:s + len(b)].tobytes()
        got.append(("chunk", s, s + len(b)))
    assert got == want


def test_two_chunkers_interleaved(dctx):
    """Each Chunker is independent: Next() alternated between two
    streams over different data returns each stream's own chunks; a second
    stream on a context whose stream is unfinished is refused."""
    import desync_amd
    from desync_amd import _lib
    a = o.synth_uniform(12, 0, (9 << 20) + 11)
    b = o.synth_uniform(13, 0, (7 << 20) + 5)
    ca = desync_amd.NewChunker(io.BytesIO(a.tobytes()), MIN, AVG, MAX)
    cb = desync_amd.NewChunker(io.BytesIO(b.tobytes()), 4096, 16384, 65536)
    got_a, got_b = [], []
    while True:
        sa, xa = ca.Next()
        sb, xb = cb.Next()
        if xa:
            got_a.append(sa + len(xa))
        if xb:
            got_b.append(sb + len(xb))
        if not xa and not xb:
            break
    assert got_a == o.chunk_stream(a, MIN, AVG, MAX).tolist()
    assert got_b == o.chunk_stream(b, 4096, 16384, 65536).tolist()
    ctx = _lib.Context(0)
    try:
        c1 = desync_amd.NewChunker(io.BytesIO(a.tobytes()), MIN, AVG, MAX, ctx=ctx)
        c1.Next()
        with pytest.raises(_lib.DsxError):
            desync_amd.NewChunker(io.BytesIO(b.tobytes()), MIN, AVG, MAX, ctx=ctx)
        c1.close()
        c2 = desync_amd.NewChunker(io.BytesIO(b.tobytes()), MIN, AVG, MAX, ctx=ctx)
        assert [s + len(x) for s, x in c2] == o.chunk_stream(b, MIN, AVG, MAX).tolist()
    finally:
        ctx.close()


# ---------------------------------------------------------------- BASELINE sizes
def test_config2_1gib_uniform(dctx):
    """BASELINE config 2: 1 GiB uniform bytes (seed 1), default params + sweep."""
    import desync_amd
    import torch
    n = 1 << 30
    t = torch.empty(n, dtype=torch.uint8, device="cuda")
    from desync_amd import _lib
    _lib.check(_lib.lib().dsx_gen_uniform(dctx.h, ctypes.c_void_p(t.data_ptr()), 0, n, 1), dctx.h)
    host = t.cpu().numpy()
    assert np.array_equal(host[:4096], o.synth_uniform(1, 0, 4096))
    for mn, av, mx in ((MIN, AVG, MAX), (4096, 16384, 65536), (65536, 262144, 1 << 20)):
        got = desync_amd.cut_device(t.data_ptr(), n, mn, av, mx, ctx=dctx)
        assert np.array_equal(got, o.chunk_stream(host, mn, av, mx)), (mn, av, mx)


def test_config4_zeros(dctx):
    """BASELINE config 4 (scaled to 4 GiB here): forced max-size chunks only."""
    import desync_amd
    import torch
    n = 4 << 30
    t = torch.zeros(n, dtype=torch.uint8, device="cuda")
    got = desync_amd.cut_device(t.data_ptr(), n, MIN, AVG, MAX, ctx=dctx)
    assert got.size == n // MAX
    assert np.array_equal(got, np.arange(1, n // MAX + 1, dtype=np.uint64) * MAX)
    # null chunk IDs on the GPU (nullchunk.go:17-23)
    ids = desync_amd.chunk_ids(t.data_ptr(), n, got[:64], 0, ctx=dctx)
    null_id = bytes.fromhex("1c8109946feed9f9e9fe4b5144d90f05a50fb3275e848cb72f4b9546d8c533f2")
    assert all(i == null_id for i in ids)


# ---------------------------------------------------------------- chunk IDs
def _tricky_ends(total, rng):
    """Chunk ends exercising every SHA-2 padding case: lengths around the
    block (64/128) and length-field (55/56, 111/112) boundaries, odd starts."""
    lens = [1, 2, 3, 15, 16, 17, 55, 56, 57, 63, 64, 65, 111, 112, 113, 119, 120, 127, 128, 129,
            191, 192, 255, 256, 257, 1000, 4096, 65535, 65536, 65537, 262144]
    lens += [int(x) for x in rng.integers(1, 300_000, size=200)]
    ends, e = [], 0
    for ln in lens:
        if e + ln > total:
            break
        e += ln
        ends.append(e)
    if ends[-1] != total:
        ends.append(total)
    return np.array(ends, dtype=np.uint64)


@pytest.mark.parametrize("algo", ["sha512-256", "sha256"])
def test_chunk_ids_match_hashlib(dctx, algo):
    """dsx_chunk_ids == Digest.Sum (digest.go:11-29) chunk by chunk."""
    import hashlib
    import desync_amd
    from desync_amd import _lib
    rng = np.random.default_rng(7)
    total = (31 << 20) + 13  # odd length: the last chunk ends off any alignment
    arr = rng.integers(0, 256, size=total, dtype=np.uint8)
    t = torch_dev(arr)
    ends = _tricky_ends(total, rng)
    code = _lib.DSX_DIGEST_SHA512_256 if algo == "sha512-256" else _lib.DSX_DIGEST_SHA256
    got = desync_amd.chunk_ids(t.data_ptr(), total, ends, 0, ctx=dctx, algo=code)
    starts = np.concatenate([np.zeros(1, np.uint64), ends[:-1]])
    buf = arr.tobytes()
    for i, (s, e) in enumerate(zip(starts.tolist(), ends.tolist())):
        want = hashlib.new("sha512_256" if algo == "sha512-256" else "sha256", buf[s:e]).digest()
        assert got[i] == want, (i, s, e)


@pytest.mark.parametrize("pc", ["0", "1"])
@pytest.mark.parametrize("algo", ["sha512-256", "sha256"])
def test_chunk_ids_both_kernels(monkeypatch, pc, algo):
    """Both digest kernels (DSX_DIGEST_PC=0: one wave per chunk set; 1: the
    producer/consumer split) on the padding cases and on 120 K short chunks --
    several per lane of either grid, so the queue refills lanes mid-run."""
    import hashlib
    import desync_amd
    from desync_amd import _lib
    monkeypatch.setenv("DSX_DIGEST_PC", pc)
    ctx = _lib.Context(0)
    try:
        rng = np.random.default_rng(11)
        total = (40 << 20) + 7
        arr = rng.integers(0, 256, size=total, dtype=np.uint8)
        t = torch_dev(arr)
        code = _lib.DSX_DIGEST_SHA512_256 if algo == "sha512-256" else _lib.DSX_DIGEST_SHA256
        name = "sha512_256" if algo == "sha512-256" else "sha256"
        buf = arr.tobytes()
        short = np.cumsum(rng.integers(0, 600, size=120_000)).astype(np.uint64)
        short = short[short <= total]
        for ends in (_tricky_ends(total, rng), short):
            got = desync_amd.chunk_ids(t.data_ptr(), total, ends, 0, ctx=ctx, algo=code)
            starts = np.concatenate([np.zeros(1, np.uint64), ends[:-1]])
            for i, (s0, e0) in enumerate(zip(starts.tolist(), ends.tolist())):
                assert got[i] == hashlib.new(name, buf[s0:e0]).digest(), (i, s0, e0)
    finally:
        ctx.close()


@pytest.mark.parametrize("nch", [220_000, 60_000])
@pytest.mark.parametrize("lpt", ["1", "0"])
@pytest.mark.parametrize("algo", ["sha512-256", "sha256"])
def test_chunk_ids_longest_first(monkeypatch, lpt, algo, nch):
    """~200 K chunks (more than digest_kernel's SHA-512 lanes, fewer than its
    SHA-256 lanes) and ~60 K (fewer than either: one chunk per lane), sizes
    0 .. 1000 B with a few of 100 KiB and empty ones: the chunks go out
    longest first (DSX_DIGEST_LPT=1, the default: a counting sort by size
    class) or in index order (0); every ID lands at its chunk's index either
    way."""
    import hashlib
    import desync_amd
    from desync_amd import _lib
    monkeypatch.setenv("DSX_DIGEST_PC", "0")
    monkeypatch.setenv("DSX_DIGEST_LPT", lpt)
    ctx = _lib.Context(0)
    try:
        rng = np.random.default_rng(13)
        total = (100 << 20) + 3
        arr = rng.integers(0, 256, size=total, dtype=np.uint8)
        t = torch_dev(arr)
        sizes = rng.integers(0, 1000, size=nch)
        sizes[rng.integers(0, sizes.size, 60)] = 100 << 10
        ends = np.cumsum(sizes).astype(np.uint64)
        ends = ends[ends <= total]
        assert ends.size > 0.7 * nch
        code = _lib.DSX_DIGEST_SHA512_256 if algo == "sha512-256" else _lib.DSX_DIGEST_SHA256
        name = "sha512_256" if algo == "sha512-256" else "sha256"
        got = desync_amd.chunk_ids(t.data_ptr(), total, ends, 0, ctx=ctx, algo=code)
        starts = np.concatenate([np.zeros(1, np.uint64), ends[:-1]])
        buf = arr.tobytes()
        for i, (s0, e0) in enumerate(zip(starts.tolist(), ends.tolist())):
            assert got[i] == hashlib.new(name, buf[s0:e0]).digest(), (i, s0, e0)
    finally:
        ctx.close()


def test_index_host_longest_first_range(dctx):
    """dsx_index_host with min/avg/max = 64/256/1024 over 48 MiB: ~190 K chunks
    in one window, so the window's digest takes the longest-first order of a
    device-side range (the chunk count is read on the device); cuts equal the
    oracle's chain, IDs hashlib's."""
    import hashlib
    import desync_amd
    arr = o.synth_uniform(17, 0, (48 << 20) + 5)
    ends, ids = desync_amd.index_host(arr, 64, 256, 1024, ctx=dctx)
    ref = o.chunk_stream(arr, 64, 256, 1024)
    assert np.array_equal(ends, ref) and ref.size > 150_000
    starts = np.concatenate([np.zeros(1, np.uint64), ref[:-1]])
    buf = arr.tobytes()
    for i, (s0, e0) in enumerate(zip(starts.tolist(), ref.tolist())):
        assert bytes(ids[i]) == hashlib.new("sha512_256", buf[s0:e0]).digest(), i


def test_chunk_ids_default_chunking(dctx):
    """IDs of the real chunking of a 64 MiB seeded blob (config-2 shape)."""
    import hashlib
    import desync_amd
    arr = o.synth_uniform(5, 0, 64 << 20)
    t = torch_dev(arr)
    ends = desync_amd.cut_device(t.data_ptr(), arr.size, MIN, AVG, MAX, ctx=dctx)
    got = desync_amd.chunk_ids(t.data_ptr(), arr.size, ends, 0, ctx=dctx)
    starts = np.concatenate([np.zeros(1, np.uint64), ends[:-1]])
    buf = arr.tobytes()
    want = [hashlib.new("sha512_256", buf[s:e]).digest()
            for s, e in zip(starts.tolist(), ends.tolist())]
    assert got == want


# ---------------------------------------------------------------- multi-GPU seams
def _compose_shard(kind):
    if kind == "random":
        return o.synth_uniform(21, 0, 12 << 20)
    r2 = o.synth_uniform(23, 0, 4 * MAX)
    head = o.synth_uniform(24, 0, 3 * MAX + 12345)
    # a zero run far longer than the 32*max seam window across the shard
    # boundaries, entered off the max grid: owners must re-walk (DSX_E_RESYNC)
    return np.concatenate([head, np.zeros(100 * MAX, np.uint8), r2])


@pytest.mark.parametrize("kind,world,dev", [("random", 3, False), ("random", 4, True),
                                            ("seam-zero-run", 2, False),
                                            ("seam-zero-run", 4, True)])
def test_shard_protocol_single_process(kind, world, dev):
    """dsx_shard_local / dsx_shard_resolve for `world` ranks simulated in one
    process (one context per rank, records exchanged by hand, host or device
    records): the concatenated per-rank lists equal the sequential chunker."""
    rounds = _shard_protocol(_compose_shard(kind), world, dev)
    if kind == "seam-zero-run":
        assert rounds > 1


def _shard_protocol(data, world, dev):
    import torch
    import desync_amd
    from desync_amd import _lib, shard
    L = _lib.lib()
    total = data.size
    span = total // world
    t = torch_dev(data)
    p = desync_amd.Params(MIN, AVG, MAX)
    ctxs = [_lib.Context(0) for _ in range(world)]
    geo = [(r * span, span if r < world - 1 else total - r * span) for r in range(world)]
    if dev:
        recs = [torch.empty(shard.SEAM_BYTES, dtype=torch.uint8, device="cuda") for _ in range(world)]
        ptr = [x.data_ptr() for x in recs]
    else:
        recs = [_lib.Seam() for _ in range(world)]
        ptr = [ctypes.addressof(x) for x in recs]
    sflag = _lib.DSX_SEAM_DEVICE if dev else 0
    for r, (start, length) in enumerate(geo):
        _lib.check(L.dsx_shard_local(ctxs[r].h, ctypes.c_void_p(t.data_ptr() + start),
                                     64 if r else 0, start, length, total, ctypes.byref(p.c),
                                     ctypes.c_void_p(ptr[r]), sflag), ctxs[r].h)
    outs = [np.empty(length // MIN + 4 + 1024, np.uint64) for _, length in geo]
    counts = [ctypes.c_uint64() for _ in range(world)]
    pieces = [c.stats().pieces for c in ctxs]
    rounds = 0
    while True:
        rounds += 1
        assert rounds <= world + 1
        if dev:
            allrec = torch.cat(recs)
            torch.cuda.synchronize()
            aptr = allrec.data_ptr()
        else:
            allrec = (_lib.Seam * world)(*recs)
            aptr = ctypes.addressof(allrec)
        rcs = [L.dsx_shard_resolve(ctxs[r].h, ctypes.c_void_p(aptr), world, r,
                                   ctypes.c_void_p(ptr[r]), outs[r].ctypes.data, outs[r].size,
                                   ctypes.byref(counts[r]), sflag) for r in range(world)]
        if all(rc == 0 for rc in rcs):
            break
        assert all(rc == _lib.DSX_E_RESYNC for rc in rcs), rcs
    got = np.concatenate([outs[r][:counts[r].value] for r in range(world)])
    assert np.array_equal(got, o.chunk_stream(data, MIN, AVG, MAX))
    # a re-walk re-runs only the stitch over the kept candidate lists
    assert [c.stats().pieces for c in ctxs] == pieces
    for c in ctxs:
        c.close()
    return rounds


def test_queued_no_sync_calls(dctx):
    """Up to 8 DSX_NO_SYNC dsx_cut_device calls queued on one context run in
    order; dsx_result returns them oldest first, each with its own count and
    cut list (bench.py's jobs in flight)."""
    import torch
    import desync_amd
    from desync_amd import _lib
    L = _lib.lib()
    p = desync_amd.Params(MIN, AVG, MAX)
    blobs, refs, outs = [], [], []
    for i in range(5):
        arr = o.synth_uniform(40 + i, 0, (3 << 20) + 1000 * i)
        blobs.append(torch_dev(arr))
        refs.append(o.chunk_stream(arr, MIN, AVG, MAX))
        outs.append(torch.empty(arr.size // MIN + 4, dtype=torch.int64, device="cuda"))
    cnt = ctypes.c_uint64()
    for i, (t, out) in enumerate(zip(blobs, outs)):
        timed = _lib.DSX_TIMED if i % 2 else 0  # odd calls record their events
        _lib.check(L.dsx_cut_device(dctx.h, ctypes.c_void_p(t.data_ptr()), t.numel(),
                                    ctypes.byref(p.c), ctypes.c_void_p(out.data_ptr()),
                                    out.numel(), ctypes.byref(cnt),
                                    _lib.DSX_OUT_DEVICE | _lib.DSX_NO_SYNC | timed), dctx.h)
    for i, (ref, out) in enumerate(zip(refs, outs)):
        _lib.check(L.dsx_result(dctx.h, ctypes.byref(cnt)), dctx.h)
        assert cnt.value == ref.size
        assert np.array_equal(out[:cnt.value].cpu().numpy().astype(np.uint64), ref)
        st = dctx.stats()
        if i % 2:  # DSX_TIMED: the call's own scan and stitch times
            assert 0 < st.scan_ms < 100 and 0 <= st.stitch_ms < 100  # (0: fused)
        else:
            assert st.scan_ms == 0 and st.stitch_ms == 0
    assert L.dsx_result(dctx.h, ctypes.byref(cnt)) == _lib.DSX_E_STATE
