"""N>1 path on CPU: world_size 2 and 3 "gloo" processes run desync_amd.shard's
seam_protocol -- the exchange / resolve / re-walk loop every transport of
the product shares -- with an engine that restates the two library calls on
the CPU (oracle/seam.py).  The concatenated per-rank cut lists must equal the
sequential chunker (make_test.go:16-80's property, across processes), and a
rank that fails mid-protocol must make every rank fail instead of hanging
(ADVICE r1).  The same loop over libdsx runs on the GPU in
tests/test_gpu_multiproc.py."""
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


class OracleEngine:
    """seam_protocol's engine interface with dsx_shard_local / resolve
    restated on the CPU (oracle/seam.py); records are the dsx_seam_t bytes
    the library exchanges."""

    def __init__(self, data, rank, world, fail_at=None):
        from desync_amd import shard
        self.sh = shard
        self.data, self.rank, self.world = data, rank, world
        total = data.size
        span = total // world
        self.start = rank * span
        self.length = span if rank < world - 1 else total - self.start
        self.fail_at = fail_at
        self.rounds = 0

    def local(self):
        from oracle import seam as oseam
        self.rec, self.spec, self.cands = oseam.shard_local(self.data, self.start, self.length,
                                                            self.data.size, MIN, AVG, MAX)
        return self.sh.seam_to_bytes(_to_struct(self.rec))

    def exchange(self, rec):
        return self.sh.exchange_seams(rec)

    def failed(self, allb):
        return self.sh.failed_ranks(allb, self.world)

    def resolve(self, allb):
        from oracle import seam as oseam
        self.rounds += 1
        if self.fail_at == self.rounds:
            raise IOError("injected failure")
        seams = [_from_struct(s) for s in self.sh.seams_from_bytes(allb, self.world)]
        st, a, b = oseam.resolve(seams, self.rank, MIN, MAX)
        if st == "ok":
            self.mine = oseam.rank_cuts(a, b, self.spec)
            return "ok"
        if a == self.rank:  # this rank's seam did not converge: re-walk from the true entry
            self.rec, self.spec = oseam.rewalk(self.cands, b, self.start, self.length,
                                               self.data.size, MIN, MAX)
        return "resync"

    def record(self):
        return self.sh.seam_to_bytes(_to_struct(self.rec))

    def agree(self, code):
        return self.sh.agree_max(code)

    def result(self):
        return self.mine


class OracleDeviceEngine(OracleEngine):
    """device_protocol's engine interface over the same CPU restatement, with
    the library's asynchronous semantics: resolve() only computes the round
    code (the device word), reduce() is the ranks' MAX agreement on it (RCCL
    on the GPU; gloo here), and collect() applies the outcome afterwards
    (the owner's re-walk).  With device_agree False the agreement comes after
    collect, as over host-staged records.  ``fail`` injects a failure in
    start, resolve or the re-walk."""

    def __init__(self, data, rank, world, fail=None, device_agree=True):
        super().__init__(data, rank, world)
        self.fail, self.device_agree = fail, device_agree
        self.recb = None

    def local_async(self):
        if self.fail == "start":
            raise IOError("injected failure")
        self.recb = self.local()

    def mark_error(self):
        from desync_amd import _lib
        S = _lib.Seam()
        S.flags = _lib.DSX_SEAM_ERROR
        self.recb = self.sh.seam_to_bytes(S)

    def gather(self):
        self.allb = self.sh.exchange_seams(self.recb)

    def resolve(self):
        from oracle import seam as oseam
        self.rounds += 1
        if self.fail == "resolve":
            raise IOError("injected failure")
        if self.sh.failed_ranks(self.allb, self.world):
            self.pend, self.code = ("peer",), 2
            return
        if self.fail == "capacity":  # the device resolve's own FAIL code (cut list too long)
            self.pend, self.code = ("capacity",), 2
            return
        seams = [_from_struct(s) for s in self.sh.seams_from_bytes(self.allb, self.world)]
        self.pend = oseam.resolve(seams, self.rank, MIN, MAX)
        self.code = 0 if self.pend[0] == "ok" else 1

    def fail_code(self):
        self.code = 2

    def reduce(self):
        self.agreed = self.sh.agree_max(self.code)

    def collect(self):
        from oracle import seam as oseam
        agreed = self.agreed if self.device_agree else None
        self.last_agreed = agreed
        if self.pend[0] == "capacity":  # dsx_shard_collect: this rank's own failure
            raise IOError("injected capacity failure")
        if agreed == 2 or self.pend[0] == "peer":
            return "peer", agreed
        st, a, b = self.pend
        if st == "ok":
            self.mine = oseam.rank_cuts(a, b, self.spec)
            return "ok", agreed
        if a == self.rank:
            if self.fail == "rewalk":
                self.mark_error()  # as dsx_shard_collect marks my_seam
                raise IOError("injected failure")
            self.rec, self.spec = oseam.rewalk(self.cands, b, self.start, self.length,
                                               self.data.size, MIN, MAX)
            self.recb = self.record()
        return "resync", agreed


def _worker(rank, world, port, data, result_q, fail_rank):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch.distributed as dist
    from desync_amd import shard
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    eng = OracleEngine(data, rank, world, fail_at=1 if rank == fail_rank else None)
    try:
        mine = shard.seam_protocol(eng, world)
        out = [None] * world
        dist.all_gather_object(out, mine.tolist())
        if rank == 0:
            result_q.put(("ok", sum(out, []), eng.rounds))
    except shard.PeerFailed:
        result_q.put(("peer", rank, None))
    except IOError:
        result_q.put(("own", rank, None))
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


def _run(data, world, fail_rank=None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, data, q, fail_rank))
             for r in range(world)]
    for p in procs:
        p.start()
    msgs = [q.get(timeout=300) for _ in range(1 if fail_rank is None else world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return msgs


@pytest.mark.parametrize("kind", ["random", "spread-null", "seam-zero-run"])
@pytest.mark.parametrize("world", [2, 3])
def test_seam_protocol_gloo(kind, world):
    from oracle import oracle as o
    data = _compose(kind)
    (st, got, rounds), = _run(data, world)
    assert st == "ok"
    assert got == o.chunk_stream(data, MIN, AVG, MAX).tolist()
    if kind == "seam-zero-run":
        assert rounds > 1  # the re-walk path ran


@pytest.mark.parametrize("kind", ["seam-zero-run", "random"])
@pytest.mark.parametrize("world,fail_rank", [(2, 1), (3, 0), (3, 2)])
def test_seam_protocol_failure_propagates(world, fail_rank, kind):
    """One rank's resolve fails: the round's agreement tells every other rank,
    which raises PeerFailed; nobody hangs.  "random" data settles in round 1
    (the peers' own resolves say "ok"), "seam-zero-run" needs re-walks."""
    msgs = _run(_compose(kind), world, fail_rank)
    kinds = sorted((m[1], m[0]) for m in msgs)
    assert kinds == [(r, "own" if r == fail_rank else "peer") for r in range(world)]


def _dworker(rank, world, port, data, result_q, fail_rank, fail, device_agree):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import torch.distributed as dist
    from desync_amd import shard
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    eng = OracleDeviceEngine(data, rank, world, fail if rank == fail_rank else None, device_agree)
    try:
        mine = shard.run_device_protocol(eng, world)
        out = [None] * world
        dist.all_gather_object(out, mine.tolist())
        if rank == 0:
            result_q.put(("ok", sum(out, []), eng.rounds))
    except shard.PeerFailed:
        result_q.put(("peer", rank, None))
    except IOError:
        result_q.put(("own", rank, None))
    dist.destroy_process_group()


def _drun(data, world, fail_rank=None, fail=None, device_agree=True):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dworker,
                         args=(r, world, port, data, q, fail_rank, fail, device_agree))
             for r in range(world)]
    for p in procs:
        p.start()
    msgs = [q.get(timeout=300) for _ in range(1 if fail_rank is None else world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return msgs


@pytest.mark.parametrize("device_agree", [True, False])
@pytest.mark.parametrize("kind,world", [("random", 2), ("seam-zero-run", 2), ("seam-zero-run", 3),
                                        ("spread-null", 3)])
def test_device_protocol_gloo(kind, world, device_agree):
    """DeviceShard's asynchronous loop (one host wait per converged step)
    gives the sequential chunker's cut list, re-walks included."""
    from oracle import oracle as o
    data = _compose(kind)
    (st, got, rounds), = _drun(data, world, device_agree=device_agree)
    assert st == "ok"
    assert got == o.chunk_stream(data, MIN, AVG, MAX).tolist()
    if kind == "seam-zero-run":
        assert rounds > 1


@pytest.mark.parametrize("device_agree", [True, False])
@pytest.mark.parametrize("fail,world,fail_rank", [("start", 2, 0), ("start", 3, 2),
                                                  ("resolve", 3, 1), ("rewalk", 2, 1),
                                                  ("rewalk", 3, 1), ("capacity", 2, 1),
                                                  ("capacity", 3, 0)])
def test_device_protocol_failure_propagates(fail, world, fail_rank, device_agree):
    """A rank failing before its round code is known (start, resolve) or after
    the device agreement (its re-walk, on a zero run across every seam), or
    its collect raising its own error after the ranks agreed FAIL (a cut list
    that does not fit: the peers already raise in that round): the failing
    rank raises its own error, every other rank PeerFailed, nobody hangs."""
    kind = "seam-zero-run" if fail == "rewalk" else "random"
    msgs = _drun(_compose(kind), world, fail_rank, fail, device_agree)
    kinds = sorted((m[1], m[0]) for m in msgs)
    assert kinds == [(r, "own" if r == fail_rank else "peer") for r in range(world)]
