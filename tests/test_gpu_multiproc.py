"""The N>1 path as shipped, on one MI355X: 2 processes share the GPU and talk
over "gloo" (RCCL needs one GPU per rank; the seam protocol is the same).

* desync_amd.shard.shard_chunk (dsx_shard_local / dsx_shard_resolve through
  seam_protocol) and shard_chunk_ids (the seam tails all-gathered, IDs on the
  GPU) in every rank: the concatenated cut lists and IDs equal the oracle's
  sequential chunking and hashlib (make_test.go:16-80's property), including a
  zero run across the seam that forces the O(candidates) re-walk.
* bench.py's DeviceShard path (records in HBM) under torch.distributed.run
  with --check, as the driver launches it for N > 1.
* DeviceShard over RCCL (the driver's N > 1 backend) in a one-rank "nccl"
  group -- RCCL needs one GPU per rank, so this is the only RCCL shape a
  one-GPU box can run: the asynchronous step with the all-gather and the
  agreement all-reduce on the library stream, pipelined over two lanes.
"""
import ctypes
import hashlib
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

MIN, AVG, MAX = 16 * 1024, 64 * 1024, 256 * 1024
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _compose(kind):
    from oracle import oracle as o
    if kind == "random":
        return o.synth_uniform(51, 0, (24 << 20) + 999)
    head = o.synth_uniform(52, 0, 3 * MAX + 12345)
    return np.concatenate([head, np.zeros(100 * MAX, np.uint8), o.synth_uniform(53, 0, 5 * MAX)])


def _worker(rank, world, port, data, q):
    sys.path.insert(0, REPO)
    import torch
    import torch.distributed as dist

    import desync_amd
    from desync_amd import _lib, shard
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        total = data.size
        span = total // world
        start = rank * span
        length = span if rank < world - 1 else total - start
        halo = 64 if rank else 0
        t = torch.from_numpy(data[start - halo:start + length].copy()).to("cuda:0")
        torch.cuda.synchronize()
        p = desync_amd.Params(MIN, AVG, MAX)
        ctx = _lib.Context(0)
        cuts = shard.shard_chunk(t.data_ptr() + halo, halo, start, length, total, p, ctx=ctx)
        pieces = ctx.stats().pieces
        ids = shard.shard_chunk_ids(t.data_ptr() + halo, start, length, cuts, p, ctx=ctx)
        out = [None] * world
        dist.all_gather_object(out, (cuts.tolist(), [i.hex() for i in ids], pieces))
        if rank == 0:
            q.put(out)
        ctx.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("kind", ["random", "seam-zero-run"])
def test_shard_chunk_two_processes(kind):
    import torch.multiprocessing as mp

    from oracle import oracle as o
    data = _compose(kind)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, data, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    cuts = sum((x[0] for x in out), [])
    ids = sum((x[1] for x in out), [])
    ref = o.chunk_stream(data, MIN, AVG, MAX)
    assert cuts == ref.tolist()
    raw, s, want = data.tobytes(), 0, []
    for e in ref.tolist():
        want.append(hashlib.new("sha512_256", raw[s:e]).hexdigest())
        s = e
    assert ids == want
    # one scan per piece per rank: the re-walk of the zero-run seam re-ran
    # only the stitch over the kept candidate lists
    assert all(x[2] == 1 for x in out)


def test_bench_two_ranks_gloo_check():
    """bench.py --gpus 2 --check through torch.distributed.run (DeviceShard,
    HBM seam records, gloo staging): the sharded cut list equals one
    dsx_cut_device over the whole blob."""
    env = dict(os.environ, DSX_DIST_BACKEND="gloo")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(REPO, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--gib", "0.25", "--check", "--no-cpu"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=REPO)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "check ok" in r.stderr, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2
    # the N > 1 line validates itself: what torch.distributed reports, every
    # rank's in-kernel scan stamps, every rank's HBM footprint
    assert line["dist"]["backend"] == "gloo" and line["dist"]["world_size"] == 2
    assert line["dist"]["ranks_reporting"] == 2
    assert line["dist"]["ranks_counted_by_backend"] == 2
    rl = line["roofline"]
    assert len(rl["per_rank"]) == 2 and all(x["launches"] >= 3 for x in rl["per_rank"])
    assert rl["frac"] == min(x["frac"] for x in rl["per_rank"]) > 0
    hbm = line["hbm"]
    assert len(hbm["per_rank_bytes"]) == 2 and 0 < hbm["max_frac"] < 1
    r0 = hbm["rank0"]
    assert len(r0["context_bytes"]) == 3 and all(b > 0 for b in r0["context_bytes"])
    assert r0["blob_bytes"] == int(0.25 * (1 << 30))


def test_context_device_bytes_accounts_for_its_hbm():
    """dsx_stats_t.device_bytes (bench.py's per-rank HBM footprint) covers
    what the device lost to the context: hipMemGetInfo's drop across
    creating a context and running a 1 GiB job, with the blob and the cut
    list allocated before, is close to device_bytes.

    hipMemGetInfo moves in 2 MiB reservations, and the runtime may place a
    buffer below 2 MiB in memory it reserved earlier in this process (the
    round-5 driver box: device_bytes 23,722,712 against a drop of exactly
    22 MiB), so the sound bounds are: the drop is at most device_bytes plus
    the runtime's own stream / code-object memory, and at least device_bytes
    less what the context's small buffers (< 2 MiB each, about 40 of them)
    could have taken from earlier reservations."""
    import torch

    import desync_amd
    from desync_amd import _lib
    n = 1 << 30
    t = torch.empty(n, dtype=torch.uint8, device="cuda")
    out = torch.empty(n // MIN + 4, dtype=torch.int64, device="cuda")
    torch.cuda.synchronize()
    free0, _ = torch.cuda.mem_get_info()
    ctx = _lib.Context(0)
    try:
        _lib.check(_lib.lib().dsx_gen_uniform(ctx.h, ctypes.c_void_p(t.data_ptr()), 0, n, 5), ctx.h)
        got = desync_amd.cut_device(t.data_ptr(), n, MIN, AVG, MAX, ctx=ctx)
        assert got.size > 0
        torch.cuda.synchronize()
        free1, _ = torch.cuda.mem_get_info()
        dev = ctx.stats().device_bytes
    finally:
        ctx.close()
    drop = free0 - free1
    assert dev > (n // (8 * 1024))  # at least the region lists of a 1 GiB piece
    small_slack = 48 * (2 << 20)
    assert dev - small_slack <= drop <= dev + (256 << 20), (dev, drop)


def _nccl_worker(port, q):
    sys.path.insert(0, REPO)
    import torch
    import torch.distributed as dist

    import desync_amd
    from desync_amd import _lib
    from desync_amd.shard import DeviceShard
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        from oracle import oracle as o
        n = (64 << 20) + 4321
        host = o.synth_uniform(61, 0, n)
        t = torch.from_numpy(host).to("cuda:0")
        p = desync_amd.Params(MIN, AVG, MAX)
        ctxs = [_lib.Context(0), _lib.Context(0)]
        lanes = [DeviceShard(ctxs[0], t.data_ptr(), 0, 0, n, n, p),
                 DeviceShard(ctxs[1], t.data_ptr(), 0, 0, n, n, p, group=dist.new_group())]
        assert all(ln.device_agree for ln in lanes)
        counts = []
        for s in range(6):  # step s on lane s % 2, one step queued ahead
            lanes[s % 2].begin()
            if s:
                counts.append(lanes[(s - 1) % 2].finish())
        counts.append(lanes[1].finish())
        ref = o.chunk_stream(host, MIN, AVG, MAX)
        q.put((counts, [ln.cuts().tolist() == ref.tolist() for ln in lanes], int(ref.size)))
        for c in ctxs:
            c.close()
    finally:
        dist.destroy_process_group()


def test_device_shard_rccl_one_rank():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    proc = ctx.Process(target=_nccl_worker, args=(_free_port(), q))
    proc.start()
    counts, same, nref = q.get(timeout=240)
    proc.join(timeout=60)
    assert proc.exitcode == 0
    assert counts == [nref] * 6 and all(same)
