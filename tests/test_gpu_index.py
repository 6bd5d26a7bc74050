"""dsx_index_fd / dsx_index_host: IndexFromFile's whole data path (file or
host blob -> cut list + chunk IDs) on the GPU, against the oracle.

Reference: IndexFromFile (make.go:22-163, IDs at make.go:223), flags
(make.go:35-62), GetFileSize (ioctl_linux.go:63-84), Interrupted
(make.go:201-203), TestChunkerEmptyFile (chunker_test.go:69-80) for the
empty file's 104-byte caibx.
"""
import ctypes
import hashlib
import io
import os
import subprocess
import sys

import numpy as np
import pytest

from oracle import oracle as o

pytestmark = pytest.mark.gpu

MIN, AVG, MAX = 16 * 1024, 64 * 1024, 256 * 1024
HERE = os.path.dirname(os.path.abspath(__file__))


def _ids(buf, ends, algo="sha512-256"):
    raw = buf.tobytes() if isinstance(buf, np.ndarray) else buf
    name = "sha512_256" if algo == "sha512-256" else "sha256"
    out, s = [], 0
    for e in ends.tolist():
        out.append(hashlib.new(name, raw[s:e]).digest())
        s = e
    return out


def test_abi_probe_without_torch():
    """A pure C-ABI caller (tests/abi_index_probe.py: ctypes + struct, no
    torch) reproduces the four golden caibx files byte for byte through
    dsx_index_fd."""
    r = subprocess.run([sys.executable, os.path.join(HERE, "abi_index_probe.py")],
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("ok ") == 4 and "torch imported: False" in r.stdout, r.stdout


@pytest.mark.parametrize("algo", ["sha512-256", "sha256"])
@pytest.mark.parametrize("kind", ["uniform", "nulls", "small-params"])
def test_index_fd_many_windows(tmp_path, monkeypatch, algo, kind):
    """1 MiB HBM windows and 256 KiB read slots: dozens of windows, chunks
    carried across every window boundary, zero runs across them."""
    import desync_amd
    from desync_amd import _lib
    monkeypatch.setenv("DSX_INDEX_WINDOW", str(1 << 20))
    monkeypatch.setenv("DSX_INDEX_SLOT", str(1 << 18))
    params = (MIN, AVG, MAX) if kind != "small-params" else (1024, 4096, 16384)
    if kind == "nulls":
        r = o.synth_uniform(41, 0, 4 * MAX + 999)
        data = np.concatenate([r, np.zeros(10 * MAX + 77, np.uint8), r, np.zeros(3 * MAX, np.uint8), r])
    else:
        data = o.synth_uniform(40, 0, (40 << 20) + 333)
    f = tmp_path / "blob"
    f.write_bytes(data.tobytes())
    ctx = _lib.Context(0)
    try:
        fd = os.open(str(f), os.O_RDONLY)
        try:
            ends, ids = desync_amd.index_fd(fd, *params, algo=algo, ctx=ctx)
        finally:
            os.close(fd)
    finally:
        ctx.close()
    ref = o.chunk_stream(data, *params)
    assert np.array_equal(ends, ref)
    assert [bytes(x) for x in ids] == _ids(data, ref, algo)


@pytest.mark.parametrize("readers", ["1", "7"])
def test_index_fd_reader_threads(tmp_path, monkeypatch, readers):
    """DSX_INDEX_READERS: one reader thread, and more threads than the 4
    pinned slots a 1 MiB window needs, fill the slots out of order; the cut
    list and IDs are the same."""
    import desync_amd
    from desync_amd import _lib
    monkeypatch.setenv("DSX_INDEX_READERS", readers)
    monkeypatch.setenv("DSX_INDEX_WINDOW", str(1 << 20))
    monkeypatch.setenv("DSX_INDEX_SLOT", str(1 << 18))
    data = o.synth_uniform(43, 0, (24 << 20) + 4321)
    f = tmp_path / "blob"
    f.write_bytes(data.tobytes())
    ctx = _lib.Context(0)
    try:
        fd = os.open(str(f), os.O_RDONLY)
        try:
            ends, ids = desync_amd.index_fd(fd, MIN, AVG, MAX, ctx=ctx)
        finally:
            os.close(fd)
    finally:
        ctx.close()
    ref = o.chunk_stream(data, MIN, AVG, MAX)
    assert np.array_equal(ends, ref)
    assert [bytes(x) for x in ids] == _ids(data, ref, "sha512-256")


@pytest.mark.parametrize("threads", ["1", "3"])
def test_index_host_threads(tmp_path, monkeypatch, threads):
    """DSX_HOST_THREADS caps the host threads (the tail feeder gets this less
    the readers, at least one, and a higher cut); IDs stay hashlib's over
    several windows and over one."""
    import desync_amd
    from desync_amd import _lib
    monkeypatch.setenv("DSX_HOST_THREADS", threads)
    data = o.synth_uniform(44, 0, (12 << 20) + 777)
    f = tmp_path / "blob"
    f.write_bytes(data.tobytes())
    ref = o.chunk_stream(data, MIN, AVG, MAX)
    for window in (4 << 20, 64 << 20):
        monkeypatch.setenv("DSX_INDEX_WINDOW", str(window))
        ctx = _lib.Context(0)
        try:
            fd = os.open(str(f), os.O_RDONLY)
            try:
                ends, ids = desync_amd.index_fd(fd, MIN, AVG, MAX, ctx=ctx)
            finally:
                os.close(fd)
            n_host = ctx.stats().host_tail_chunks
        finally:
            ctx.close()
        assert np.array_equal(ends, ref)
        assert [bytes(x) for x in ids] == _ids(data, ref, "sha512-256")
        avx512 = "avx512f" in open("/proc/cpuinfo").read() and "avx512bw" in open("/proc/cpuinfo").read()
        if window > data.size and avx512:
            # one window: one feeder thread (1 or 3 host threads less the 4
            # readers) and the cut 28 KiB x 28 / 1 capped at 128 KiB
            lens = np.diff(np.concatenate([[0], ref.astype(np.int64)]))
            assert n_host == int(np.sum(lens > 131072))


@pytest.mark.parametrize("mib,cut1", [(320, 81920), (640, 163840)])
def test_index_host_tail_gpu_shares(tmp_path, monkeypatch, mib, cut1):
    """One window large enough for the GPU's shares during the read (at 1/2,
    3/4, ... of the window, a digest on the digest stream of the chunks
    confirmed since the previous point up to that point's cut; the feeder
    taking each segment's chunks above its cut and the last segment's above
    the usual cut): every ID is hashlib's, and the host took between the
    chunks above the first cut and those above the usual cut.  32 host
    threads -> 28 feeders, cut 28 KiB.  The first cut is the read time after
    1/2 over the shares' 45 ns per byte, rounded down to 4 KiB: 320 MiB / 45
    B/ns -> 81920 (one point: 3/4's would be below 1.5 x 28 KiB); 640 MiB ->
    163840 (two points).  Then VerifyIndex of the same list, whose shares take
    host-known chunk ranges."""
    import concurrent.futures as cf

    import desync_amd
    from desync_amd import _lib
    monkeypatch.setenv("DSX_HOST_THREADS", "32")
    n = (mib << 20) + 4321
    data = o.synth_uniform_c(48, 0, n)
    f = tmp_path / "blob"
    data.tofile(str(f))
    ctx = _lib.Context(0)
    try:
        fd = os.open(str(f), os.O_RDONLY)
        try:
            ends, ids = desync_amd.index_fd(fd, MIN, AVG, MAX, ctx=ctx)
        finally:
            os.close(fd)
        n_host = ctx.stats().host_tail_chunks
        ends2, ids2 = desync_amd.index_host(data, MIN, AVG, MAX, ctx=ctx)
        # VerifyIndex of the same list (run_ids' shares: the chunk ranges known
        # on the host, the last segment's chunks above a budgeted cut on the
        # host from the call's start)
        fd = os.open(str(f), os.O_RDONLY)
        try:
            vids = desync_amd.ids_fd(fd, 0, ends, ctx=ctx)
        finally:
            os.close(fd)
        vids2 = desync_amd.ids_host(data, 0, ends, ctx=ctx)
    finally:
        ctx.close()
    ref = o.chunk_parallel(data, MIN, AVG, MAX, o.default_threads())
    assert np.array_equal(ends, ref) and np.array_equal(ends2, ref)
    starts = np.concatenate([[0], ref[:-1]]).astype(np.uint64)
    mv = memoryview(data)

    def h(i):
        return hashlib.new("sha512_256", mv[int(starts[i]):int(ref[i])]).digest()

    with cf.ThreadPoolExecutor(o.default_threads()) as pool:
        want = list(pool.map(h, range(ref.size), chunksize=256))
    assert [bytes(x) for x in ids] == want
    assert [bytes(x) for x in ids2] == want
    assert [bytes(x) for x in vids] == want
    assert [bytes(x) for x in vids2] == want
    avx512 = "avx512f" in open("/proc/cpuinfo").read() and "avx512bw" in open("/proc/cpuinfo").read()
    if avx512:
        lens = (ref - starts).astype(np.int64)
        assert int(np.sum(lens > cut1)) <= n_host < int(np.sum(lens > 28672)), n_host


@pytest.mark.parametrize("tail,window", [("65536", 16 << 20), ("0", 16 << 20), ("-1", 16 << 20),
                                         ("100000", None), ("-1", None)])
def test_index_host_tail(tmp_path, monkeypatch, tail, window):
    """DSX_INDEX_HOST_TAIL (make.go:223's Digest.Sum for the last window's
    longest chunks on the host, AVX-512 multi-buffer SHA-512/256, while the
    GPU digest skips them): forced for every chunk above 64 KiB, off, and the
    default (the pipeline's own cut), over several windows (only the last one
    has a tail); and in one window, where a feeder thread hashes the long
    chunks while the file is still being read (forced above 100000 bytes, and
    the default 28 KiB).  From a file and from host memory.  The cut list equals the
    oracle's and every ID hashlib's, and so are VerifyIndex's IDs of the same
    list (dsx_ids_fd / dsx_ids_host); the stats count the host's chunks."""
    import desync_amd
    from desync_amd import _lib
    monkeypatch.setenv("DSX_INDEX_HOST_TAIL", tail)
    # the default cut follows the feeder's threads (the CPU share less the 4
    # readers): 32 host threads -> 28 feeders -> 28 KiB, independent of the box
    monkeypatch.setenv("DSX_HOST_THREADS", "32")
    if window:
        monkeypatch.setenv("DSX_INDEX_WINDOW", str(window))
    data = o.synth_uniform(47, 0, (40 << 20) + 777)
    f = tmp_path / "blob"
    f.write_bytes(data.tobytes())
    ref = o.chunk_stream(data, MIN, AVG, MAX)
    want = _ids(data, ref, "sha512-256")
    long_chunks = int(np.sum(np.diff(np.concatenate([[0], ref.astype(np.int64)])) > 65536))
    ctx = _lib.Context(0)
    try:
        fd = os.open(str(f), os.O_RDONLY)
        try:
            ends, ids = desync_amd.index_fd(fd, MIN, AVG, MAX, ctx=ctx)
        finally:
            os.close(fd)
        n_host = ctx.stats().host_tail_chunks
        assert np.array_equal(ends, ref)
        assert [bytes(x) for x in ids] == want
        ends2, ids2 = desync_amd.index_host(data, MIN, AVG, MAX, ctx=ctx)
        assert np.array_equal(ends2, ref) and [bytes(x) for x in ids2] == want
        assert ctx.stats().host_tail_chunks == n_host
        # VerifyIndex's IDs of a given list (dsx_ids_fd / dsx_ids_host): the same tail
        fd = os.open(str(f), os.O_RDONLY)
        try:
            ids3 = desync_amd.make.ids_fd(fd, 0, ref, ctx=ctx)
        finally:
            os.close(fd)
        assert [bytes(x) for x in ids3] == want
        ids4 = desync_amd.make.ids_host(data, 0, ref, ctx=ctx)
        assert [bytes(x) for x in ids4] == want
        if tail == "0":
            assert ctx.stats().host_tail_chunks == 0
        elif tail != "-1":
            assert ctx.stats().host_tail_chunks > 0
    finally:
        ctx.close()
    if tail == "0":
        assert n_host == 0
    elif window is None:  # one window: the feeder takes every chunk above the cut
        cut = int(tail) if tail != "-1" else 28672
        lens = np.diff(np.concatenate([[0], ref.astype(np.int64)]))
        avx512 = "avx512f" in open("/proc/cpuinfo").read() and "avx512bw" in open("/proc/cpuinfo").read()
        if tail != "-1" or avx512:  # (auto needs AVX-512)
            assert n_host == int(np.sum(lens > cut)) > 0
    elif tail == "65536":
        assert 0 < n_host < long_chunks  # (the last window's share of them)
    else:
        assert n_host < long_chunks


def test_index_host_two_gib_windows():
    """1.5 GiB through the default 1 GiB windows (two of them): every cut
    against oracle.chunk_parallel, every ID against hashlib -- also those of
    VerifyIndex over the same list (the last window's GPU shares in both:
    snapshot ranges in dsx_index_host, host-known ranges in dsx_ids_host)."""
    import concurrent.futures as cf

    import desync_amd
    n = (3 << 29) + 777
    data = o.synth_uniform_c(17, 0, n)
    ends, ids = desync_amd.index_host(data, MIN, AVG, MAX)
    vids = desync_amd.ids_host(data, 0, ends)
    ref = o.chunk_parallel(data, MIN, AVG, MAX, o.default_threads())
    assert np.array_equal(ends, ref)
    starts = np.concatenate([[0], ref[:-1]]).astype(np.uint64)
    mv = memoryview(data)

    def h(i):
        return hashlib.new("sha512_256", mv[int(starts[i]):int(ref[i])]).digest()

    with cf.ThreadPoolExecutor(o.default_threads()) as pool:
        want = list(pool.map(h, range(ref.size), chunksize=256))
    assert [bytes(x) for x in ids] == want
    assert [bytes(x) for x in vids] == want


def test_urandom_file(tmp_path):
    """SURVEY.md 8(d) config 2's extra run: 1 GiB of real /dev/urandom bytes
    saved to a file, so the CPU oracle sees exactly the bytes the GPU chunked
    (dsx_index_fd: cuts and IDs)."""
    import concurrent.futures as cf

    import desync_amd
    n = 1 << 30
    f = tmp_path / "urandom.bin"
    with open("/dev/urandom", "rb") as src, open(f, "wb") as dst:
        left = n
        while left:
            b = src.read(min(left, 64 << 20))
            dst.write(b)
            left -= len(b)
    data = np.fromfile(str(f), dtype=np.uint8)
    fd = os.open(str(f), os.O_RDONLY)
    try:
        ends, ids = desync_amd.index_fd(fd, MIN, AVG, MAX)
    finally:
        os.close(fd)
    ref = o.chunk_parallel(data, MIN, AVG, MAX, o.default_threads())
    assert np.array_equal(ends, ref)
    starts = np.concatenate([[0], ref[:-1]]).astype(np.uint64)
    mv = memoryview(data)

    def h(i):
        z = hashlib.new("sha512_256")
        z.update(mv[int(starts[i]):int(ref[i])])
        return z.digest()

    with cf.ThreadPoolExecutor(o.default_threads()) as pool:
        want = list(pool.map(h, range(ref.size), chunksize=256))
    assert [bytes(x) for x in ids] == want


def test_empty_file_and_sha256_flags(tmp_path, golden):
    """The empty file gives the 104-byte caibx (header + table marker + tail);
    under --digest sha256 the index flags lack CaFormatSHA512256
    (make.go:35-38) and the IDs are SHA-256."""
    import desync_amd
    from desync_amd import digest
    f = tmp_path / "empty"
    f.write_bytes(b"")
    index, stats = desync_amd.IndexFromFile(None, str(f), 4, MIN, AVG, MAX)
    b = io.BytesIO()
    index.WriteTo(b)
    assert len(b.getvalue()) == 104 and stats.ChunksAccepted == 0
    assert b.getvalue() == o.encode_caibx(o.index_flags(b""), MIN, AVG, MAX, [], [])
    g = tmp_path / "blob1"
    g.write_bytes(golden("blob1"))
    ref = o.decode_caibx(golden("blob1.caibx"))
    prev = digest.Digest.Algorithm()
    desync_amd.set_digest("sha256")
    try:
        index, _ = desync_amd.IndexFromFile(None, str(g), 4, ref["min"], ref["avg"], ref["max"])
    finally:
        desync_amd.set_digest(prev)
    assert index.Index.FeatureFlags == o.CA_FORMAT_EXCLUDE_NO_DUMP
    data = np.frombuffer(golden("blob1"), np.uint8)
    assert [c.Start + c.Size for c in index.Chunks] == ref["ends"].tolist()
    assert [c.ID for c in index.Chunks] == _ids(data, ref["ends"], "sha256")


def test_index_cancel_and_io_error(tmp_path):
    """dsx_cancel before the call -> Interrupted (and the next call runs);
    a range past the end of the file -> DSX_E_IO."""
    import desync_amd
    from desync_amd import _lib
    data = o.synth_uniform(42, 0, 5 << 20)
    f = tmp_path / "blob"
    f.write_bytes(data.tobytes())
    ctx = _lib.Context(0)
    fd = os.open(str(f), os.O_RDONLY)
    try:
        _lib.lib().dsx_cancel(ctx.h)
        with pytest.raises(desync_amd.Interrupted):
            desync_amd.index_fd(fd, MIN, AVG, MAX, ctx=ctx)
        ends, _ = desync_amd.index_fd(fd, MIN, AVG, MAX, ctx=ctx)
        assert np.array_equal(ends, o.chunk_stream(data, MIN, AVG, MAX))
        with pytest.raises(_lib.DsxError) as ei:
            desync_amd.index_fd(fd, MIN, AVG, MAX, length=data.size + 4096, ctx=ctx)
        assert ei.value.code == _lib.DSX_E_IO
    finally:
        os.close(fd)
        ctx.close()


class _RecordingBar:
    """A ProgressBar (progress.go:7-15) that records its calls."""

    def __init__(self):
        self.calls = []

    def SetTotal(self, total):
        self.calls.append(("SetTotal", total))

    def Start(self):
        self.calls.append(("Start",))

    def Set(self, v):
        self.calls.append(("Set", v))

    def Finish(self):
        self.calls.append(("Finish",))

    def sets(self):
        return [c[1] for c in self.calls if c[0] == "Set"]


def test_index_progress(tmp_path, monkeypatch):
    """a14: IndexFromFile calls pb.Set while the data path runs (make.go:138,
    per assembled chunk): every value is the end of a confirmed chunk, the
    values never decrease, there is more than one before the end, and the
    last is the file size; SetTotal/Start first, Finish last."""
    import desync_amd
    monkeypatch.setenv("DSX_INDEX_WINDOW", str(4 << 20))
    monkeypatch.setenv("DSX_INDEX_SLOT", str(1 << 20))
    data = o.synth_uniform(43, 0, (192 << 20) + 12345)
    f = tmp_path / "blob"
    f.write_bytes(data.tobytes())
    pb = _RecordingBar()
    desync_amd._lib.reset_context_pool()  # (the pooled contexts read the env when created)
    try:
        index, stats = desync_amd.IndexFromFile(None, str(f), 4, MIN, AVG, MAX, pb=pb)
    finally:
        desync_amd._lib.reset_context_pool()
    ref = o.chunk_stream(data, MIN, AVG, MAX)
    assert [c.Start + c.Size for c in index.Chunks] == ref.tolist()
    sets = pb.sets()
    assert pb.calls[0] == ("SetTotal", data.size) and pb.calls[1] == ("Start",)
    assert pb.calls[-1] == ("Finish",) and sets[-1] == data.size
    assert sets == sorted(sets) and len(set(sets)) >= 2, sets[:20]
    ends = set(ref.tolist())
    assert all(v in ends for v in sets), [v for v in sets if v not in ends][:5]


def test_index_progress_granularity(tmp_path):
    """Default pipeline geometry over 1 GiB: the progress bar sees the chain
    advance in steps of the 32 MiB scan pieces -- at least 16 distinct
    confirmed-chunk ends per GiB (make.go:138 sets it per chunk)."""
    import desync_amd
    data = o.synth_uniform(45, 0, 1 << 30)
    f = tmp_path / "blob"
    f.write_bytes(data.tobytes())
    pb = _RecordingBar()
    desync_amd._lib.reset_context_pool()
    try:
        index, _ = desync_amd.IndexFromFile(None, str(f), 4, MIN, AVG, MAX, pb=pb)
    finally:
        desync_amd._lib.reset_context_pool()
    sets = pb.sets()
    ref = o.chunk_parallel(data, MIN, AVG, MAX, 8)
    assert len(index.Chunks) == ref.size
    assert sets == sorted(sets) and sets[-1] == data.size
    assert len(set(sets)) >= 16, len(set(sets))
    ends = set(ref.tolist())
    assert all(v in ends for v in sets)


@pytest.mark.parametrize("window", [1 << 20, None])
def test_index_partial_on_io_error(tmp_path, monkeypatch, window):
    """A read error mid-file (the range runs past the end of the file): the
    error carries the confirmed prefix -- IndexFromFile returns the chunks
    assembled so far with chunkErr (make.go:133-162) -- cut for cut the
    oracle's chain and ID for ID hashlib.  Over many windows, and in one (the
    tail feeder hashing beside the read when the error comes)."""
    import desync_amd
    from desync_amd import _lib
    if window:
        monkeypatch.setenv("DSX_INDEX_WINDOW", str(window))
    monkeypatch.setenv("DSX_INDEX_SLOT", str(1 << 18))
    # (one window confirms cuts every 32 MiB scan step: a file of several)
    data = o.synth_uniform(44, 0, ((24 if window else 72) << 20) + 5)
    f = tmp_path / "blob"
    f.write_bytes(data.tobytes())
    ref = o.chunk_stream(data, MIN, AVG, MAX)
    ctx = _lib.Context(0)
    fd = os.open(str(f), os.O_RDONLY)
    try:
        for algo in ("sha512-256", "sha256"):
            with pytest.raises(_lib.DsxError) as ei:
                desync_amd.index_fd(fd, MIN, AVG, MAX, length=data.size + (3 << 20), ctx=ctx,
                                    algo=algo)
            e = ei.value
            assert e.code == _lib.DSX_E_IO
            n = len(e.ends)
            assert 0 < n < ref.size and np.array_equal(e.ends, ref[:n])
            assert int(e.ends[-1]) > data.size - 4 * MAX - ((2 if window else 32) << 20)
            assert [bytes(x) for x in e.ids] == _ids(data, ref[:n], algo)
            # the next call on the context is unaffected
            ends, _ = desync_amd.index_fd(fd, MIN, AVG, MAX, ctx=ctx)
            assert np.array_equal(ends, ref)
    finally:
        os.close(fd)
        ctx.close()


@pytest.mark.parametrize("window", [8 << 20, None])
def test_index_partial_on_cancel(tmp_path, monkeypatch, window):
    """Interrupted mid-file (make.go:201-203): cancelled from the progress
    callback at the first confirmed chunk, IndexFromFile raises Interrupted
    carrying a non-empty strict prefix of the chain with its IDs (many
    windows, and one: the tail feeder running)."""
    import desync_amd
    from desync_amd import _lib
    if window:
        monkeypatch.setenv("DSX_INDEX_WINDOW", str(window))
    monkeypatch.setenv("DSX_INDEX_SLOT", str(1 << 20))
    data = o.synth_uniform(45, 0, 768 << 20)
    f = tmp_path / "blob"
    f.write_bytes(data.tobytes())
    ctx = _lib.Context(0)
    fd = os.open(str(f), os.O_RDONLY)

    def cancel_at_first(v):
        if v > 0:
            _lib.lib().dsx_cancel(ctx.h)

    try:
        with pytest.raises(desync_amd.Interrupted) as ei:
            desync_amd.index_fd(fd, MIN, AVG, MAX, ctx=ctx, progress=cancel_at_first)
    finally:
        os.close(fd)
        ctx.close()
    e = ei.value
    n = len(e.ends)
    ref = o.chunk_stream(data[:int(e.ends[-1]) + 4 * MAX] if n else data[:1], MIN, AVG, MAX)
    assert 0 < n and int(e.ends[-1]) < data.size
    assert np.array_equal(e.ends, ref[:n])
    assert [bytes(x) for x in e.ids] == _ids(data, e.ends)


def test_chunk_ids_rejects_malformed_ends(dctx):
    """host ends are validated (order, bounds) before any launch."""
    import torch
    from desync_amd import _lib
    t = torch.zeros(4096, dtype=torch.uint8, device="cuda")
    out = np.empty((3, 32), np.uint8)
    for ends, start in (([100, 50, 4096], 0), ([100, 200, 5000], 0), ([100, 200, 300], 150)):
        e = np.array(ends, np.uint64)
        rc = _lib.lib().dsx_chunk_ids(dctx.h, ctypes.c_void_p(t.data_ptr()), 4096, start,
                                      e.ctypes.data, 3, out.ctypes.data, 0, 0)
        assert rc == _lib.DSX_E_INVAL, ends


# ---------------------------------------------------------------- ChunkStream
def test_chunk_stream_golden(golden):
    """index_test.go:55-112 TestIndexChunking: ChunkStream over
    testdata/chunker.input, written with WriteTo, is chunker.index byte for
    byte, and the store holds every chunk."""
    import desync_amd
    store = desync_amd.MemoryStore()
    c = desync_amd.NewChunker(io.BytesIO(golden("chunker.input")), MIN, AVG, MAX)
    idx = desync_amd.ChunkStream(None, c, store, 10)
    b = io.BytesIO()
    idx.WriteTo(b)
    assert b.getvalue() == golden("chunker.index")
    want = o.decode_caibx(golden("chunker.index"))["ids"]
    assert len(want) == 20 and all(store.HasChunk(i) for i in want)


@pytest.mark.parametrize("algo", ["sha512-256", "sha256"])
def test_chunk_stream_large(algo):
    """300 MiB with repeated blocks through ChunkStream (128 MiB GPU batches,
    IDs on the side stream): every cut and ID against the oracle / hashlib,
    repeated chunks stored once; the index flags are the reference's fixed
    ExcludeNoDump|SHA512256 (index.go:226) whatever the digest."""
    import desync_amd
    from desync_amd import digest
    blk = o.synth_uniform(43, 0, 8 << 20)
    parts = [o.synth_uniform(44, 0, 100 << 20), blk, np.zeros(3 << 20, np.uint8), blk,
             o.synth_uniform(45, 0, 150 << 20), blk, o.synth_uniform(46, 0, (30 << 20) + 17)]
    data = np.concatenate(parts)
    store = desync_amd.MemoryStore()
    prev = digest.Digest.Algorithm()
    desync_amd.set_digest(algo)
    try:
        c = desync_amd.NewChunker(io.BytesIO(data.tobytes()), MIN, AVG, MAX)
        idx = desync_amd.ChunkStream(None, c, store, 4)
    finally:
        desync_amd.set_digest(prev)
    ref = o.chunk_stream(data, MIN, AVG, MAX)
    assert [ch.Start + ch.Size for ch in idx.Chunks] == ref.tolist()
    want = _ids(data, ref, algo)
    assert [ch.ID for ch in idx.Chunks] == want
    assert len(store.chunks) == len(set(want)) < len(want)
    assert idx.Index.FeatureFlags == o.CA_FORMAT_EXCLUDE_NO_DUMP | o.CA_FORMAT_SHA512256


def test_chunker_runs_equal_next():
    """Chunker._next_run (ChunkStream's path: the chunks Next() would return up
    to its next read, in one call) gives Next()'s (start, bytes, ID) sequence,
    with IDs on and off, across 8 MiB reads and a 10*max refill boundary."""
    import desync_amd
    data = np.concatenate([o.synth_uniform(48, 0, 40 << 20), np.zeros(2 << 20, np.uint8),
                           o.synth_uniform(49, 0, (9 << 20) + 3)]).tobytes()
    for ids in (False, True):
        a = desync_amd.NewChunker(io.BytesIO(data), MIN, AVG, MAX)
        b = desync_amd.NewChunker(io.BytesIO(data), MIN, AVG, MAX)
        if ids:
            a.EnableIDs()
            b.EnableIDs()
        want = []
        while True:
            s, chunk = a.Next()
            if not chunk:
                break
            want.append((s, bytes(chunk), a.ChunkID()))
        got, runs = [], 0
        while True:
            run = b._next_run()
            if not run:
                break
            runs += 1
            got.extend(run)
        a.close()
        b.close()
        assert got == want and runs < len(want)


def test_chunker_blocks_equal_next():
    """Chunker._next_block (ChunkStream's path: one block of ends, IDs and a
    single clone of the bytes per run) describes exactly Next()'s (start,
    bytes, ID) sequence, with IDs on and off and with the read-ahead, across
    8 MiB reads, a zero run and a 10*max refill boundary."""
    import desync_amd
    data = np.concatenate([o.synth_uniform(48, 0, 40 << 20), np.zeros(2 << 20, np.uint8),
                           o.synth_uniform(49, 0, (9 << 20) + 3)]).tobytes()
    for ids, ra in ((False, 0), (True, 0), (True, 256 << 20)):
        a = desync_amd.NewChunker(io.BytesIO(data), MIN, AVG, MAX)
        b = desync_amd.NewChunker(io.BytesIO(data), MIN, AVG, MAX)
        if ids:
            a.EnableIDs()
            b.EnableIDs()
        b._ra = ra
        want = []
        while True:
            s, chunk = a.Next()
            if not chunk:
                break
            want.append((s, bytes(chunk), a.ChunkID()))
        got, blocks = [], 0
        while True:
            blk = b._next_block()
            if blk is None:
                break
            blocks += 1
            s0, ends, idb, raw = blk
            assert len(raw) == ends[-1] - s0 and len(idb) == (32 * len(ends) if ids else 0)
            s = s0
            for i, e in enumerate(ends):
                got.append((s, raw[s - s0:e - s0], idb[32 * i:32 * i + 32] if ids else None))
                s = e
        a.close()
        b.close()
        assert got == want and blocks < len(want)


def test_chunk_stream_errors():
    """A failing store raises out of ChunkStream; a cancelled ctx stops the
    producer and returns the chunks so far (index.go:203-206)."""
    import desync_amd
    data = o.synth_uniform(47, 0, 20 << 20)

    class Bad(desync_amd.MemoryStore):
        def StoreChunk(self, chunk):
            raise IOError("disk full")

    with pytest.raises(IOError, match="disk full"):
        desync_amd.ChunkStream(None, desync_amd.NewChunker(io.BytesIO(data.tobytes()), MIN, AVG, MAX),
                               Bad(), 2)

    class After:
        def __init__(self, k):
            self.k = k

        def done(self):
            self.k -= 1
            return self.k < 0

    idx = desync_amd.ChunkStream(After(5), desync_amd.NewChunker(io.BytesIO(data.tobytes()), MIN,
                                                                 AVG, MAX), desync_amd.MemoryStore(), 2)
    ref = o.chunk_stream(data, MIN, AVG, MAX)
    assert [ch.Start + ch.Size for ch in idx.Chunks] == ref[:5].tolist()


def test_chunker_context_pool(monkeypatch):
    """A Chunker without a ctx takes an idle pooled context and returns it on
    close(), mid-stream too; the next Chunker chunks correctly on it.  A
    context made under other DSX_* settings is not handed out (and is closed
    once a context is asked for under the new ones)."""
    import desync_amd
    from desync_amd import _lib
    _lib.reset_context_pool()
    data = o.synth_uniform(48, 0, (24 << 20) + 5)
    ref = o.chunk_stream(data, MIN, AVG, MAX).tolist()

    def chunker():
        return desync_amd.NewChunker(io.BytesIO(data.tobytes()), MIN, AVG, MAX)

    try:
        c1 = chunker()
        x1 = c1.ctx
        s, b = c1.Next()
        assert s == 0 and len(b) == ref[0]
        c1.close()  # mid-stream
        c2 = chunker()
        assert c2.ctx is x1
        assert [s + len(b) for s, b in c2] == ref
        c2.close()
        monkeypatch.setenv("DSX_SCAN_NT", "0")
        c3 = chunker()
        x3 = c3.ctx
        assert x3 is not x1 and not x1.h  # (the idle one, made under other settings, closed)
        assert [s + len(b) for s, b in c3] == ref
        c3.close()
        c5 = chunker()
        assert c5.ctx is x3
        c5.close()
        monkeypatch.delenv("DSX_SCAN_NT")
        c4 = chunker()
        assert c4.ctx is not x3 and not x3.h
        assert [s + len(b) for s, b in c4] == ref
        c4.close()
    finally:
        _lib.reset_context_pool()


# ------------------------------------------------- dsx_ids_fd / dsx_ids_host
@pytest.mark.parametrize("algo", ["sha512-256", "sha256"])
def test_ids_fd_many_windows(tmp_path, monkeypatch, algo):
    """The re-hash of a given chunk list (VerifyIndex / ChopFile) through 1 MiB
    HBM windows and 256 KiB read slots: the oracle's cut list of 24 MiB from a
    non-zero start, a file range at an offset, a 3 MiB chunk (longer than a
    window: the window overlap grows to it) and zero-length chunks; every ID
    against hashlib, fd and host paths alike."""
    import desync_amd
    from desync_amd import _lib
    monkeypatch.setenv("DSX_INDEX_WINDOW", str(1 << 20))
    monkeypatch.setenv("DSX_INDEX_SLOT", str(1 << 18))
    data = o.synth_uniform(48, 0, (24 << 20) + 4321)
    ref = o.chunk_stream(data, MIN, AVG, MAX)
    f = tmp_path / "blob"
    f.write_bytes(data.tobytes())
    ctx = _lib.Context(0)
    fd = os.open(str(f), os.O_RDONLY)
    try:
        start = int(ref[3])
        ends = ref[4:]
        want = _ids(data[start:], ends - start, algo)
        got = desync_amd.ids_fd(fd, start, ends, algo=algo, ctx=ctx)
        assert [bytes(x) for x in got] == want
        got = desync_amd.ids_host(data, start, ends, algo=algo, ctx=ctx)
        assert [bytes(x) for x in got] == want
        # a range of the file at an offset: offsets relative to it
        off = 777
        sub = data[off:off + (9 << 20)]
        e2 = np.array([5, 5, 5 + (3 << 20), (3 << 20) + 70000, (3 << 20) + 70000, sub.size], np.uint64)
        got = desync_amd.ids_fd(fd, 5, e2, offset=off, length=sub.size, algo=algo, ctx=ctx)
        assert [bytes(x) for x in got] == _ids(sub[5:], e2 - 5, algo)
        # one chunk: the whole file; no chunks
        got = desync_amd.ids_fd(fd, 0, np.array([data.size], np.uint64), algo=algo, ctx=ctx)
        assert bytes(got[0]) == _ids(data, np.array([data.size], np.uint64), algo)[0]
        assert desync_amd.ids_fd(fd, 0, np.array([], np.uint64), ctx=ctx).shape == (0, 32)
    finally:
        os.close(fd)
        ctx.close()


def test_ids_fd_errors(tmp_path):
    """Malformed chunk lists are rejected before any read (DSX_E_INVAL); a
    list past the end of the file gives DSX_E_IO; the context keeps working."""
    import desync_amd
    from desync_amd import _lib
    data = o.synth_uniform(49, 0, 1 << 20)
    f = tmp_path / "blob"
    f.write_bytes(data.tobytes())
    ctx = _lib.Context(0)
    fd = os.open(str(f), os.O_RDONLY)
    try:
        for start, ends in ((0, [100, 50]), (200, [100, 300]), (0, [100, data.size + 1])):
            with pytest.raises(_lib.DsxError) as ei:
                desync_amd.ids_fd(fd, start, np.array(ends, np.uint64), length=data.size, ctx=ctx)
            assert ei.value.code == _lib.DSX_E_INVAL, (start, ends)
        with pytest.raises(_lib.DsxError) as ei:
            desync_amd.ids_fd(fd, 0, np.array([100, data.size + 4096], np.uint64),
                              length=data.size + 4096, ctx=ctx)
        assert ei.value.code == _lib.DSX_E_IO
        got = desync_amd.ids_fd(fd, 0, np.array([100, data.size], np.uint64), ctx=ctx)
        assert [bytes(x) for x in got] == _ids(data, np.array([100, data.size], np.uint64))
    finally:
        os.close(fd)
        ctx.close()


# ------------------------------------------------------------------- ChopFile
class _Count:
    def __init__(self):
        self.total, self.inc, self.finished = None, 0, False

    def SetTotal(self, n):
        self.total = n

    def Start(self):
        pass

    def Increment(self):
        self.inc += 1

    def Finish(self):
        self.finished = True


def test_chop_file_golden(tmp_path, golden):
    """chop.go:14-81 over testdata/chunker.input with its golden index: every
    chunk stored once under its ID with its exact bytes; a wrong ID raises
    ChunkInvalid with errors.go's message; a truncated file raises EOFError;
    a store error is raised."""
    import desync_amd
    f = tmp_path / "chunker.input"
    raw = golden("chunker.input")
    f.write_bytes(raw)
    idx = desync_amd.IndexFromReader(golden("chunker.index"))
    store, pb = desync_amd.MemoryStore(), _Count()
    assert desync_amd.ChopFile(None, str(f), idx.Chunks, store, 4, pb) is None
    assert pb.total == pb.inc == len(idx.Chunks) == 20 and pb.finished
    assert sorted(store.chunks) == sorted(bytes(c.ID) for c in idx.Chunks)
    for c in idx.Chunks:
        assert store.chunks[bytes(c.ID)] == raw[c.Start:c.Start + c.Size]

    bad = list(idx.Chunks)
    k = 7
    bad[k] = desync_amd.IndexChunk(bytes(32), bad[k].Start, bad[k].Size)
    with pytest.raises(desync_amd.ChunkInvalid) as ei:
        desync_amd.ChopFile(None, str(f), bad, desync_amd.MemoryStore(), 2)
    want_sum = hashlib.new("sha512_256", raw[bad[k].Start:bad[k].Start + bad[k].Size]).digest()
    assert str(ei.value) == f"chunk id {'00' * 32} does not match its hash {want_sum.hex()}"

    short = tmp_path / "short"
    short.write_bytes(raw[:idx.Chunks[-3].Start + 10])
    with pytest.raises(EOFError):
        desync_amd.ChopFile(None, str(short), idx.Chunks, desync_amd.MemoryStore(), 3)

    class Bad(desync_amd.MemoryStore):
        def StoreChunk(self, chunk):
            raise IOError("store down")

    with pytest.raises(IOError, match="store down"):
        desync_amd.ChopFile(None, str(f), idx.Chunks, Bad(), 2)


def test_chop_file_large_sha256(tmp_path):
    """IndexFromFile -> ChopFile over 64 MiB with repeated blocks, SHA-256:
    the store holds each distinct chunk once with its bytes."""
    import desync_amd
    from desync_amd import digest
    blk = o.synth_uniform(50, 0, 4 << 20)
    data = np.concatenate([o.synth_uniform(51, 0, 30 << 20), blk, o.synth_uniform(52, 0, 20 << 20),
                           blk, np.zeros(2 << 20, np.uint8), blk])
    f = tmp_path / "blob"
    f.write_bytes(data.tobytes())
    prev = digest.Digest.Algorithm()
    desync_amd.set_digest("sha256")
    try:
        idx, _ = desync_amd.IndexFromFile(None, str(f), 4, MIN, AVG, MAX)
        store = desync_amd.MemoryStore()
        desync_amd.ChopFile(None, str(f), idx.Chunks, store, 8)
    finally:
        desync_amd.set_digest(prev)
    raw = data.tobytes()
    assert len(store.chunks) == len({bytes(c.ID) for c in idx.Chunks}) < len(idx.Chunks)
    for c in idx.Chunks[::37]:
        assert store.chunks[bytes(c.ID)] == raw[c.Start:c.Start + c.Size]
        assert hashlib.sha256(raw[c.Start:c.Start + c.Size]).digest() == bytes(c.ID)
