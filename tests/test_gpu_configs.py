"""BASELINE.json configs 3, 4 and 5 at their stated sizes, and a > 8 GiB
uniform blob, on the device, against the CPU oracle.

* config 3: 16 GiB, 30 % repeated 1 MiB blocks (dsx_gen_dedup, seed 2): the
  device bytes equal the oracle's twin generator, and the cut list equals
  oracle.chunk_parallel (make.go's split-and-align, C restatement) on them.
* config 4: 64 GiB of zeros: 262,144 forced max-size cuts at k*max and the
  null-chunk ID (nullchunk.go:17-23) on chunks sampled in all 8 pieces.
* 9 GiB + 12,345 B uniform: crosses 2^32 and the 8 GiB piece boundary of
  dsx_cut_device (kPieceMax, dsx_api.cpp), compared cut for cut.
* config 5: 256 GiB as 8 range shards of 32 GiB (seed 3), the seam protocol
  (dsx_shard_local / dsx_shard_resolve) for 8 ranks simulated in one process;
  every rank's list must equal the sequential chain, which is recomputed per
  rank on the device from the rank's true entry cut (the chain from any true
  cut c is the chunking of blob[c:], chunker.go:206-277) and checked against
  the CPU oracle in a window at every seam; an interior rank and the last
  rank are compared in full with the oracle over their whole range.

Reference: make_test.go:16-80 (parallel == sequential at any size),
chunker_test.go:69-131 (zeros -> max-size chunks).
"""
import ctypes
import gc

import numpy as np
import pytest

from oracle import oracle as o

pytestmark = pytest.mark.gpu

MIN, AVG, MAX = 16 * 1024, 64 * 1024, 256 * 1024
GiB = 1 << 30
MiB = 1 << 20
NULL_ID = bytes.fromhex("1c8109946feed9f9e9fe4b5144d90f05a50fb3275e848cb72f4b9546d8c533f2")


def _free():
    import torch
    gc.collect()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


def _gen(ctx, t, offset, n, kind, seed):
    from desync_amd import _lib
    L = _lib.lib()
    if kind == "uniform":
        _lib.check(L.dsx_gen_uniform(ctx.h, ctypes.c_void_p(t.data_ptr()), offset, n, seed), ctx.h)
    else:
        _lib.check(L.dsx_gen_dedup(ctx.h, ctypes.c_void_p(t.data_ptr()), offset, n, seed, 0.30),
                   ctx.h)


def _check_bytes(host, offset, kind, seed):
    """Device bytes (copied to host) == the oracle's twin generator, 1 GiB at a time."""
    buf = np.empty(min(GiB, host.size), dtype=np.uint8)
    for o0 in range(0, host.size, buf.size):
        n = min(buf.size, host.size - o0)
        if kind == "uniform":
            o.synth_uniform_c(seed, offset + o0, n, out=buf)
        else:
            o.synth_dedup(seed, offset + o0, n, 0.30, out=buf)
        assert np.array_equal(host[o0:o0 + n], buf[:n]), f"generator bytes differ at {offset + o0}"


def test_dedup_generator_windows(dctx):
    """dsx_gen_dedup == oracle.synth_dedup on windows spread over 16 GiB."""
    import torch
    n = 64 * MiB + 777
    t = torch.empty(n, dtype=torch.uint8, device="cuda")
    for off in (0, 5 * GiB + 12345, 16 * GiB - n):
        _gen(dctx, t, off, n, "dedup", 2)
        _check_bytes(t.cpu().numpy(), off, "dedup", 2)


def test_config3_16gib_dedup(dctx):
    import torch
    import desync_amd
    n = 16 * GiB
    t = torch.empty(n, dtype=torch.uint8, device="cuda")
    _gen(dctx, t, 0, n, "dedup", 2)
    host = t.cpu().numpy()
    _check_bytes(host, 0, "dedup", 2)
    got = desync_amd.cut_device(t.data_ptr(), n, MIN, AVG, MAX, ctx=dctx)
    del t
    _free()
    ref = o.chunk_parallel(host, MIN, AVG, MAX, o.default_threads())
    assert got.size == ref.size and np.array_equal(got, ref)


def test_config4_64gib_zeros(dctx):
    import torch
    import desync_amd
    n = 64 * GiB
    t = torch.zeros(n, dtype=torch.uint8, device="cuda")
    got = desync_amd.cut_device(t.data_ptr(), n, MIN, AVG, MAX, ctx=dctx)
    assert got.size == n // MAX == 262144
    assert np.array_equal(got, np.arange(1, n // MAX + 1, dtype=np.uint64) * MAX)
    # null-chunk IDs for 16 chunks on both sides of each of the 8 piece starts
    per_piece = (8 * GiB) // MAX
    for k in range(8):
        i0 = max(0, k * per_piece - 16)
        ends = got[i0:i0 + 32]
        start = int(got[i0 - 1]) if i0 else 0
        ids = desync_amd.chunk_ids(t.data_ptr(), n, ends, start, ctx=dctx)
        assert all(i == NULL_ID for i in ids), k
    del t
    _free()


@pytest.mark.parametrize("params,tail", [((MIN, AVG, MAX), 0), ((4096, 16384, 65536), 0),
                                         ((MIN, AVG, MAX), 3), ((4096, 16384, 65536), 3),
                                         ((MIN, AVG, MAX), 4)])
def test_uniform_9gib_two_pieces(dctx, monkeypatch, params, tail):
    """> 2^32 bytes and two 8 GiB pieces: the carried chain state, 64-bit
    offsets and the second piece's region grid, cut for cut.  tail = 4
    (DSX_TAIL_SPLIT, the default): the 8 GiB piece's last regions have 4x
    shorter lane segments (two region sizes in the scan and the stitch);
    tail = 3: 3x; tail = 0: one region size."""
    import torch
    import desync_amd
    from desync_amd import _lib
    ctx = dctx
    if tail != 4:
        monkeypatch.setenv("DSX_TAIL_SPLIT", str(tail))
        ctx = _lib.Context(0)
    n = 9 * GiB + 12345
    t = torch.empty(n, dtype=torch.uint8, device="cuda")
    _gen(ctx, t, 0, n, "uniform", 7)
    host = t.cpu().numpy()
    if params == (MIN, AVG, MAX) and tail == 4:
        _check_bytes(host, 0, "uniform", 7)
    got = desync_amd.cut_device(t.data_ptr(), n, *params, ctx=ctx)
    if ctx is not dctx:
        ctx.close()
    del t
    _free()
    ref = o.chunk_parallel(host, *params, o.default_threads())
    assert got.size == ref.size and np.array_equal(got, ref)
    assert got[-1] == n and np.any(got > (1 << 32)) and np.any((got > 8 * GiB) & (got < 9 * GiB))


@pytest.mark.parametrize("n,params", [(int(3.25 * GiB) + 4567, (MIN, AVG, MAX)),
                                      (4 * GiB - 999, (4096, 16384, 65536))])
def test_two_region_sizes_edges(dctx, n, params):
    """One piece just above the two-region-size threshold (three big regions
    per wave slot, ~3.1 GiB on 256 CUs) and one with a partial last tail
    region, with a 3 MiB zero run where the big regions give way to the tail
    regions (~1.03 GiB before the end) and a repeated 1 MiB block inside the
    tail: cut for cut against the oracle (two region sizes)."""
    import torch
    import desync_amd
    t = torch.empty(n, dtype=torch.uint8, device="cuda")
    _gen(dctx, t, 0, n, "uniform", 11)
    z0 = n - int(1.1 * GiB)
    t[z0:z0 + 3 * MiB].zero_()
    t[n - 5 * MiB:n - 4 * MiB].copy_(t[n - 9 * MiB:n - 8 * MiB])
    host = t.cpu().numpy()
    got = desync_amd.cut_device(t.data_ptr(), n, *params, ctx=dctx)
    del t
    _free()
    ref = o.chunk_parallel(host, *params, o.default_threads())
    assert got.size == ref.size and np.array_equal(got, ref)
    if params == (MIN, AVG, MAX):
        # the zero run holds only forced max-size cuts
        inside = got[(got > z0 + MAX) & (got < z0 + 3 * MiB)]
        assert inside.size and np.all(np.diff(inside) == MAX)


@pytest.mark.parametrize("n", [4 * GiB + 3 * MiB + 123, 6 * GiB + 7])
def test_stitch_segment_doubling(dctx, n):
    """Pieces whose 1 MiB stitch segments would number more than 4097 get 2 MiB
    ones (dsx_api.cpp stitch_seg): 4 GiB + 3 MiB is 2050 of them (just past
    finish_kernel's 2048: fixup_fast_kernel<4> + gather), 6 GiB 3072; cut for
    cut against the oracle, with a zero run across a 2 MiB segment boundary."""
    import torch
    import desync_amd
    t = torch.empty(n, dtype=torch.uint8, device="cuda")
    _gen(dctx, t, 0, n, "uniform", 19)
    z0 = 3 * GiB + 2 * MiB - 300 * 1024  # (a 2 MiB boundary inside the run)
    t[z0:z0 + MiB].zero_()
    host = t.cpu().numpy()
    got = desync_amd.cut_device(t.data_ptr(), n, MIN, AVG, MAX, ctx=dctx)
    del t
    _free()
    ref = o.chunk_parallel(host, MIN, AVG, MAX, o.default_threads())
    assert got.size == ref.size and np.array_equal(got, ref)


def test_config5_8x32gib_shards(dctx):
    """256 GiB range-sharded over 8 ranks (one process, one context per rank,
    seam records exchanged by hand as the all-gather would)."""
    import torch
    import desync_amd
    from desync_amd import _lib
    L = _lib.lib()
    world, span = 8, 32 * GiB
    total = world * span
    p = desync_amd.Params(MIN, AVG, MAX)
    ctxs = [_lib.Context(0) for _ in range(world)]
    buf = torch.empty(span + 64, dtype=torch.uint8, device="cuda")
    recs = [_lib.Seam() for _ in range(world)]
    try:
        for r in range(world):
            halo = 64 if r else 0
            _gen(dctx, buf, r * span - halo, span + halo, "uniform", 3)
            _lib.check(L.dsx_shard_local(ctxs[r].h, ctypes.c_void_p(buf.data_ptr() + halo), halo,
                                         r * span, span, total, ctypes.byref(p.c),
                                         ctypes.addressof(recs[r]), 0), ctxs[r].h)
        # uniform data converges inside every seam window: one exchange round,
        # so no rank needs its shard bytes again (a re-walk would)
        allrec = (_lib.Seam * world)(*recs)
        lists = []
        for r in range(world):
            out = np.empty(span // MIN + 4 + 1024, np.uint64)
            cnt = ctypes.c_uint64()
            rc = L.dsx_shard_resolve(ctxs[r].h, ctypes.addressof(allrec), world, r,
                                     ctypes.addressof(recs[r]), out.ctypes.data, out.size,
                                     ctypes.byref(cnt), 0)
            assert rc == 0, rc
            lists.append(out[:cnt.value].copy())
    finally:
        for c in ctxs:
            c.close()
    for r in range(world):
        lo, hi = r * span, (r + 1) * span
        mine = lists[r]
        assert mine.size and np.all(mine > lo) and np.all(mine <= hi) and np.all(np.diff(mine) > 0)
        entry = int(lists[r - 1][-1]) if r else 0
        assert hi - int(mine[-1]) < MAX and (r == 0 or lo - entry < MAX)
        # the sequential chain from the true entry: device path over
        # [entry, hi + max) (cuts <= hi never depend on bytes beyond it)
        wend = min(total, hi + MAX)
        _gen(dctx, buf, entry, wend - entry, "uniform", 3)
        seq = desync_amd.cut_device(buf.data_ptr(), wend - entry, MIN, AVG, MAX, ctx=dctx) + entry
        assert np.array_equal(mine, seq[seq <= hi]), r
        # and the CPU oracle on the seam window [entry, entry + 64 MiB)
        win = o.synth_uniform_c(3, entry, 64 * MiB)
        ref = o.chunk_stream(win, MIN, AVG, MAX) + np.uint64(entry)
        ref = ref[ref <= entry + 64 * MiB - MAX]
        assert np.array_equal(mine[:ref.size], ref), r
    del buf
    _free()
    # an interior rank and the last rank in full against the CPU oracle over
    # their whole range [entry, hi + max): the chain from the true entry cut
    for r in (3, world - 1):
        lo, hi = r * span, (r + 1) * span
        entry = int(lists[r - 1][-1])
        wend = min(total, hi + MAX)
        host = o.synth_uniform_c(3, entry, wend - entry)
        ref = o.chunk_parallel(host, MIN, AVG, MAX, o.default_threads()) + np.uint64(entry)
        del host
        ref = ref[ref <= hi]
        assert lists[r].size == ref.size and np.array_equal(lists[r], ref), r
