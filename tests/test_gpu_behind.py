"""Stitch behind the scan: queued (DSX_NO_SYNC) dsx_cut_device calls whose
walk and finish run as tasks inside the next calls' scans.

The fused stitch (DSX_FUSE=1) is in the diagnostic build only (it does not
move the bench line under the board's power cap), so
its scenarios run in one child process on libdsx_diag.so
(test_fused_stitch_diag); the same scenarios without it run here on the
product library.

Every call's cut list must equal the oracle's chain (chunker.go:206-277)
whatever runs between the calls: more fused calls, calls that cannot be
fused (a pointer off the 128-B grid, a dense-candidate parameter set), a
dsx_sync, a synchronous call, collection at every queue depth.  Suspect
segments (seams inside zero runs with short segments) take the redo path.
"""
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest

from oracle import oracle as o

pytestmark = pytest.mark.gpu

MIN, AVG, MAX = 16 * 1024, 64 * 1024, 256 * 1024


def _dev(arr, pad=0):
    import torch
    t = torch.empty(arr.size + pad, dtype=torch.uint8, device="cuda")
    t[pad:].copy_(torch.from_numpy(np.ascontiguousarray(arr, dtype=np.uint8)))
    torch.cuda.synchronize()
    return t, t.data_ptr() + pad


class Queue:
    """Queued calls on one context, collected oldest first."""

    def __init__(self, ctx):
        from desync_amd import _lib
        self.ctx, self.L, self.lib = ctx, _lib.lib(), _lib
        self.pending = []  # (ref, out tensor, keepalive)

    def submit(self, arr, mn=MIN, av=AVG, mx=MAX, pad=0, flags=0):
        import torch
        import desync_amd
        t, ptr = _dev(arr, pad)
        p = desync_amd.Params(mn, av, mx)
        out = torch.empty(arr.size // mn + 4, dtype=torch.int64, device="cuda")
        cnt = ctypes.c_uint64()
        self.lib.check(self.L.dsx_cut_device(
            self.ctx.h, ctypes.c_void_p(ptr), arr.size, ctypes.byref(p.c),
            ctypes.c_void_p(out.data_ptr()), out.numel(), ctypes.byref(cnt),
            self.lib.DSX_OUT_DEVICE | self.lib.DSX_NO_SYNC | flags), self.ctx.h)
        self.pending.append((o.chunk_stream(arr, mn, av, mx), out, (t, p)))

    def collect(self):
        ref, out, _ = self.pending.pop(0)
        cnt = ctypes.c_uint64()
        self.lib.check(self.L.dsx_result(self.ctx.h, ctypes.byref(cnt)), self.ctx.h)
        assert cnt.value == ref.size
        got = out[:cnt.value].cpu().numpy().astype(np.uint64)
        assert np.array_equal(got, ref)


def _fused():
    """The child process runs on libdsx_diag.so with DSX_FUSE=1."""
    return os.environ.get("DSX_FUSE", "0") == "1"


def _blobs():
    rng = np.random.default_rng(5)
    dense_blk = None
    P = o.params(MIN, AVG, MAX)
    while dense_blk is None:  # a 48-byte period whose window hash is a candidate
        blk = rng.integers(0, 256, 48, dtype=np.uint8)
        if o.window_hash(bytes(blk)) % P.d == P.d - 1:
            dense_blk = blk
    return {
        "u1": o.synth_uniform(61, 0, (1 << 20) + 12345),
        "u40": o.synth_uniform(62, 0, (40 << 20) + 7),
        "u300": o.synth_uniform(63, 0, (300 << 20) + 4097),
        "zeros": np.zeros((24 << 20) + 5, np.uint8),
        "mixed": np.concatenate([o.synth_uniform(64, 0, 3 << 20), np.zeros(5 << 20, np.uint8),
                                 o.synth_uniform(65, 0, (7 << 20) + 3)]),
        "periodic": np.tile(dense_blk, (3 << 20) // 48),
        "tiny": o.synth_uniform(66, 0, 1000),
    }


def scenario_sequence(fctx):
    """A run of queued calls, fused and not, collected at depths 1..8."""
    from desync_amd import _lib
    b = _blobs()
    q = Queue(fctx)
    plan = ["u40", "u1", "u300", "zeros", "mixed", "u40", "tiny", "u1", "periodic",
            "u300", "mixed", "zeros"]
    for depth in (1, 2, 3, 4, 8):
        for name in plan:
            while len(q.pending) >= depth:
                q.collect()
            q.submit(b[name])
        while q.pending:
            q.collect()
    # other parameters and a pointer off the line grid (not fused: flushes)
    for depth in (3, 5):
        q.submit(b["u40"])
        q.submit(b["u40"], 4096, 8192, 65536)
        q.submit(b["u1"], pad=1)
        q.submit(b["mixed"], 64 << 10, 1 << 20, 4 << 20)
        q.submit(b["u300"])
        if depth == 5:
            _lib.check(_lib.lib().dsx_sync(fctx.h), fctx.h)  # flushes the calls behind
        q.submit(b["u40"], 1000, 8000, 64000)  # dense candidates: not fused
        q.submit(b["u1"])
        while q.pending:
            q.collect()


def scenario_interleaved_sync_calls(fctx):
    """A synchronous call, a chunk-ID call and a host-memory call between
    queued ones run after the stitches still behind (DSX_FUSE=1) and after
    the queued calls' pending publish (the next scan publishes a queued call's
    state, or flush_publish), and every result stays exact; a timed queued
    call (its own events) mixes in."""
    import desync_amd
    from desync_amd import _lib
    b = _blobs()
    q = Queue(fctx)
    q.submit(b["u40"])
    q.submit(b["mixed"])
    t, ptr = _dev(b["u300"])
    got = desync_amd.cut_device(ptr, b["u300"].size, MIN, AVG, MAX, ctx=fctx)
    assert np.array_equal(got, o.chunk_stream(b["u300"], MIN, AVG, MAX))
    q.submit(b["zeros"])
    ids = desync_amd.chunk_ids(ptr, b["u300"].size, got[:50], 0, ctx=fctx)
    assert len(ids) == 50
    q.submit(b["u1"], flags=_lib.DSX_TIMED)
    q.submit(b["u40"])
    q.collect()  # (the oldest: published by a later scan)
    assert np.array_equal(desync_amd.cut_host(b["u1"], MIN, AVG, MAX, ctx=fctx),
                          o.chunk_stream(b["u1"], MIN, AVG, MAX))
    while q.pending:
        q.collect()
    q.submit(b["u1"])  # the last queued call: collected with no scan after it
    q.collect()


def scenario_redo_on_suspect_segments():
    """Short segments (64 KiB floor, 4 x max) with the true chain inside zero
    runs off the segment grid: seams that do not converge.  The tasks publish
    kErrRedo and dsx_result redoes the call with fixup_kernel's repair."""
    from desync_amd import _lib
    os.environ["DSX_SEG_FLOOR"] = "65536"
    ctx = _lib.Context(0)
    del os.environ["DSX_SEG_FLOOR"]
    try:
        rng = np.random.default_rng(11)
        null = np.zeros(4 * MAX, np.uint8)
        r1 = rng.integers(0, 256, 4 * MAX, dtype=np.uint8)
        d = np.concatenate([r1[:12345], null, null, null, r1, null, r1])
        u = o.synth_uniform(67, 0, 9 << 20)
        q = Queue(ctx)
        for _ in range(3):
            q.submit(d)
            q.submit(u)
        while q.pending:
            q.collect()  # d: redone on the general path, which repairs
            assert ctx.stats().repaired_segments > 0
            q.collect()
    finally:
        ctx.close()


def scenario_timed_calls(fctx):
    """DSX_TIMED fused calls report the scan kernel's time (it carries the
    stitch tasks of the calls behind it) and no separate stitch time."""
    from desync_amd import _lib
    b = _blobs()
    q = Queue(fctx)
    for name in ("u40", "u40", "u40", "u40"):
        q.submit(b[name], flags=_lib.DSX_TIMED)
    while q.pending:
        q.collect()
        st = fctx.stats()
        assert 0 < st.scan_ms < 100 and st.stitch_ms == 0


def _run_queued_jobs(ctx, ptr, n, njobs, depth, ref, stamps=False):
    """bench.py's N = 1 step loop: njobs dsx_cut_device jobs over the same
    device blob, DSX_NO_SYNC, up to `depth` in flight on one context, each
    collected oldest first and compared in full with `ref`."""
    import torch
    import desync_amd
    from desync_amd import _lib
    p = desync_amd.Params(MIN, AVG, MAX)
    L = _lib.lib()
    cap = n // MIN + 4
    outs = [torch.empty(cap, dtype=torch.int64, device="cuda") for _ in range(depth)]
    cnt = ctypes.c_uint64()
    pend = []
    if stamps:
        ctx.stamps_begin(njobs * ((n + (8 << 30) - 1) >> 33) + 8)

    def collect():
        i = pend.pop(0)
        _lib.check(L.dsx_result(ctx.h, ctypes.byref(cnt)), ctx.h)
        assert cnt.value == ref.size
        assert np.array_equal(outs[i][:cnt.value].cpu().numpy().astype(np.uint64), ref)

    for s in range(njobs):
        if len(pend) == depth:
            collect()
        _lib.check(L.dsx_cut_device(ctx.h, ctypes.c_void_p(ptr), n, ctypes.byref(p.c),
                                    ctypes.c_void_p(outs[s % depth].data_ptr()), cap,
                                    ctypes.byref(cnt), _lib.DSX_OUT_DEVICE | _lib.DSX_NO_SYNC),
                   ctx.h)
        pend.append(s % depth)
    while pend:
        collect()
    return ctx.stamps_end() if stamps else []


def scenario_bench_steady_state_counts(ctx):
    """bench.py's config-2 shape: 1 GiB uniform jobs queued 4 deep on one
    context give the same cut list as the oracle."""
    import torch
    n = 1 << 30
    arr = o.synth_uniform(1, 0, n)
    ref = o.chunk_parallel(arr, MIN, AVG, MAX, 16)
    t = torch.from_numpy(arr).to("cuda")
    del arr
    _run_queued_jobs(ctx, t.data_ptr(), n, 12, 4, ref)


def scenario_bench_headline_job(ctx):
    """The job bench.py's default line is printed on (BASELINE config 5's
    per-GPU shard): 32 GiB of dsx_gen_uniform seed 3 in HBM, four 8 GiB
    pieces per job, 4 DSX_NO_SYNC jobs in flight on one context (so the
    chain state is carried across 3 piece seams while later jobs queue
    behind), in-kernel stamps on.  Every job's full cut list equals
    oracle.chunk_parallel (make.go:69-127's split-and-align, C restatement)
    over the oracle's own twin generator, and the count is the bench line's
    config.chunks."""
    import torch
    from desync_amd import _lib
    n = 32 << 30
    host = o.synth_uniform_c(3, 0, n)
    ref = o.chunk_parallel(host, MIN, AVG, MAX, o.default_threads())
    assert ref.size == 524384 and int(ref[-1]) == n
    t = torch.empty(n, dtype=torch.uint8, device="cuda")
    _lib.check(_lib.lib().dsx_gen_uniform(ctx.h, ctypes.c_void_p(t.data_ptr()), 0, n, 3), ctx.h)
    # the device generator's bytes are the oracle's at the ends of each piece
    for off in (0, (8 << 30) - (1 << 20), (16 << 30) - 4096, n - (1 << 20)):
        m = min(1 << 20, n - off)
        assert np.array_equal(t[off:off + m].cpu().numpy(), host[off:off + m]), off
    del host
    st = _run_queued_jobs(ctx, t.data_ptr(), n, 8, 4, ref, stamps=True)
    assert len(st) == 8 * 4 and all(s.bytes == 8 << 30 for s in st)
    assert all(0 < s.ms < 50 for s in st)
    del t


# ---- product library (no fused stitch) ----------------------------------------
def _ctx():
    from desync_amd import _lib
    return _lib.Context(0)


def test_interleaved_sync_calls():
    ctx = _ctx()
    try:
        scenario_interleaved_sync_calls(ctx)
    finally:
        ctx.close()


def test_bench_steady_state_counts():
    ctx = _ctx()
    try:
        scenario_bench_steady_state_counts(ctx)
    finally:
        ctx.close()


def test_bench_headline_job():
    ctx = _ctx()
    try:
        scenario_bench_headline_job(ctx)
    finally:
        ctx.close()
    import torch
    torch.cuda.empty_cache()


def test_fuse_needs_the_diagnostic_build(monkeypatch):
    """DSX_FUSE=1 against the product library is refused loudly (a fresh
    interpreter: the library is loaded once per process)."""
    env = dict(os.environ, DSX_FUSE="1")
    env.pop("DSX_LIB_PATH", None)
    r = subprocess.run([sys.executable, "-c", "from desync_amd import _lib; _lib.lib()"],
                       env=env, capture_output=True, text=True, timeout=120, cwd=REPO)
    assert r.returncode != 0 and "libdsx_diag" in r.stderr


# ---- the fused stitch: libdsx_diag.so, one child process ----------------------
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DIAG = os.path.join(REPO, "desync_amd", "libdsx_diag.so")


@pytest.mark.skipif(not os.path.exists(DIAG), reason="libdsx_diag.so not built (make -C desync_amd/csrc diag)")
def test_fused_stitch_diag():
    env = dict(os.environ, DSX_LIB_PATH=DIAG, DSX_FUSE="1", PYTHONPATH=REPO)
    r = subprocess.run([sys.executable, "-u", os.path.abspath(__file__)], env=env,
                       capture_output=True, text=True, timeout=900, cwd=REPO)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "fused stitch scenarios ok" in r.stdout


def _main():
    assert _fused() and os.path.basename(os.environ["DSX_LIB_PATH"]).startswith("libdsx_diag")
    from desync_amd import _lib
    for name, f in (("sequence", scenario_sequence),
                    ("interleaved", scenario_interleaved_sync_calls),
                    ("timed", scenario_timed_calls),
                    ("bench", scenario_bench_steady_state_counts)):
        ctx = _lib.Context(0)
        try:
            f(ctx)
        finally:
            ctx.close()
        print("ok:", name, flush=True)
    scenario_redo_on_suspect_segments()
    print("ok: redo", flush=True)
    print("fused stitch scenarios ok", flush=True)


if __name__ == "__main__":
    sys.path.insert(0, REPO)
    _main()
