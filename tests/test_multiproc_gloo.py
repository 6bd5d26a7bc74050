"""N>1 path on CPU: world_size-2 "gloo" processes run the seam protocol of
desync_amd.shard (fixed-size dsx_seam_t records, all-gathered) with the CPU
restatement of dsx_shard_local / dsx_shard_resolve (oracle/seam.py), and the
concatenated per-rank cut lists must equal the sequential chunker
(make_test.go:16-80's property, across processes)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

MIN, AVG, MAX = 16 * 1024, 64 * 1024, 256 * 1024


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _to_struct(seam):
    from desync_amd import _lib
    S = _lib.Seam()
    S.shard_start, S.shard_len, S.total = seam["shard_start"], seam["shard_len"], seam["total"]
    S.exit_cut, S.window_end, S.flags = seam["exit_cut"], seam["window_end"], seam["flags"]
    S.entry = seam["entry"]
    S.first_cand_beyond = 2**64 - 1
    S.ncands, S.ncuts = len(seam["cands"]), len(seam["cuts"])
    for i, x in enumerate(seam["cands"]):
        S.cands[i] = x
    for i, x in enumerate(seam["cuts"]):
        S.cuts[i] = x
    return S


def _from_struct(S):
    return dict(shard_start=S.shard_start, shard_len=S.shard_len, total=S.total,
                exit_cut=S.exit_cut, window_end=S.window_end, flags=S.flags, entry=S.entry,
                cands=[S.cands[i] for i in range(S.ncands)],
                cuts=[S.cuts[i] for i in range(S.ncuts)])


def _worker(rank, world, port, data, result_q):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch.distributed as dist
    from desync_amd import shard
    from oracle import seam as oseam
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    total = data.size
    span = total // world
    start = rank * span
    length = span if rank < world - 1 else total - start
    rec, spec, cands = oseam.shard_local(data, start, length, total, MIN, AVG, MAX)
    rounds = 0
    while True:  # the DSX_E_RESYNC protocol of desync_amd.shard.shard_chunk
        rounds += 1
        assert rounds <= world + 1
        allb = shard.exchange_seams(shard.seam_to_bytes(_to_struct(rec)))
        seams = [_from_struct(s) for s in shard.seams_from_bytes(allb, world)]
        assert seams[rank]["exit_cut"] == rec["exit_cut"]
        st, a, b = oseam.resolve(seams, rank, MIN, MAX)
        if st == "ok":
            mine = oseam.rank_cuts(a, b, spec)
            break
        if a == rank:  # this rank's seam did not converge: re-walk from the true entry
            rec, spec = oseam.rewalk(cands, b, start, length, total, MIN, MAX)
    out = [None] * world
    dist.all_gather_object(out, mine.tolist())
    if rank == 0:
        result_q.put((sum(out, []), rounds))
    dist.destroy_process_group()


def _compose(kind):
    from oracle import oracle as o
    if kind == "random":
        return o.synth_uniform(21, 0, 12 << 20)
    null = np.zeros(4 * MAX, np.uint8)
    r1 = o.synth_uniform(22, 0, 4 * MAX)
    r2 = o.synth_uniform(23, 0, 4 * MAX)
    if kind == "seam-zero-run":
        # a zero run far longer than the 32*max seam window across every shard
        # boundary, entered off the max grid: seams cannot converge in their
        # window, so the owners re-walk (README.md:114-119's worst case)
        head = o.synth_uniform(24, 0, 3 * MAX + 12345)
        return np.concatenate([head, np.zeros(100 * MAX, np.uint8), r2])
    return np.concatenate([r1, null, null, null, r1, null, null, null, r2])


@pytest.mark.parametrize("kind", ["random", "spread-null", "seam-zero-run"])
@pytest.mark.parametrize("world", [2, 3])
def test_seam_protocol_gloo(kind, world):
    from oracle import oracle as o
    data = _compose(kind)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, data, q)) for r in range(world)]
    for p in procs:
        p.start()
    got, rounds = q.get(timeout=300)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got == o.chunk_stream(data, MIN, AVG, MAX).tolist()
    if kind == "seam-zero-run":
        assert rounds > 1  # the re-walk path ran
