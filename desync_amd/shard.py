"""Multi-GPU range sharding (one process per GPU) -- make.go's split-and-align
across ranks.

Reference: IndexFromFile starts n workers span*i apart (make.go:69-116); each
chunks speculatively from its start and the main routine aligns it with its
predecessor when both produce the same chunk (syncWith, make.go:277-298).
Here rank r chunks [r*span, (r+1)*span) on its own GPU (dsx_shard_local),
the ranks all-gather fixed-size seam records (16 KiB: the first candidates
and speculative cuts of each shard; RCCL over xGMI when the group uses the
"nccl" backend, the records never leave HBM), and every rank aligns all seams
(dsx_shard_resolve) to get its exact slice of the sequential cut list.  A
seam that does not converge inside its window (a zero run across a shard
boundary -- README.md:114-119) makes its owner re-walk its shard from the
true entry cut over its kept candidate lists (no byte is scanned again); the
ranks then exchange the records again (DSX_E_RESYNC; at most nranks rounds).
Every round ends with a one-integer all-reduce of the ranks' outcomes, so a
rank whose resolve fails makes every peer fail in the same round instead of
leaving one rank waiting in a collective (PeerFailed).

Chunk IDs across seams (shard_chunk_ids): the chunk that ends at a rank's
first cut starts in an earlier shard, at most max bytes back; the ranks
all-gather the tails behind their last cut (the "overlap bytes" of the seams,
<= max each), and each rank hashes its chunks on its own GPU.

Two forms of the protocol loop, each shared by its transports and driven on
the CPU by the gloo tests with the oracle's restatement of the library calls:
seam_protocol (synchronous calls, host records over any torch.distributed
backend: shard_chunk) and device_protocol (dsx_shard_resolve_async /
dsx_shard_collect, records in HBM: DeviceShard, bench.py), which over RCCL
keeps the whole step on the library stream -- one host wait per converged
step.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib
from ._lib import DSX_E_PEER, DSX_E_RESYNC, DSX_NO_SYNC, DSX_SEAM_DEVICE, check, lib

SEAM_BYTES = ctypes.sizeof(_lib.Seam)
FLAGS_OFF = _lib.Seam.flags.offset


class PeerFailed(RuntimeError):
    """Another rank's seam record carries DSX_SEAM_ERROR."""


def seam_to_bytes(seam: "_lib.Seam") -> bytes:
    return ctypes.string_at(ctypes.addressof(seam), SEAM_BYTES)


def seams_from_bytes(blob: bytes, nranks: int):
    return (_lib.Seam * nranks).from_buffer_copy(blob)


def exchange_seams(seam_bytes: bytes, group=None, device=None) -> bytes:
    """All-gather one fixed-size seam record per rank (rank order), host bytes."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    mine = torch.frombuffer(bytearray(seam_bytes), dtype=torch.uint8)
    if device is not None:
        mine = mine.to(device)
    bufs = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(bufs, mine, group=group)
    return b"".join(b.cpu().numpy().tobytes() for b in bufs)


def failed_ranks(all_bytes: bytes, world: int):
    """Ranks whose record in the gathered bytes carries DSX_SEAM_ERROR."""
    return [r for r in range(world)
            if int.from_bytes(all_bytes[r * SEAM_BYTES + FLAGS_OFF:r * SEAM_BYTES + FLAGS_OFF + 4],
                              "little") & _lib.DSX_SEAM_ERROR]


# round outcomes, agreed as their maximum over the ranks
AGREE_OK, AGREE_RESYNC, AGREE_FAIL = 0, 1, 2


def agree_max(code, group=None, device=None):
    """max(code) over the ranks of ``group`` (one tiny all-reduce)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor([int(code)], dtype=torch.int32, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return int(t.item())


def seam_protocol(engine, world, rec=None):
    """The exchange / resolve loop (dsx.h, multi-GPU shards).  ``engine``:
    local() -> record; exchange(record) -> all records; failed(all) -> ranks
    with DSX_SEAM_ERROR; resolve(all) -> "ok" | "resync" (raises on a local
    failure); agree(code) -> the maximum of the ranks' AGREE_* codes;
    record() -> the (re-walked) record; result() -> this rank's cut list.

    Every round ends with agree(): a rank whose resolve fails (or that sees a
    DSX_SEAM_ERROR record) contributes AGREE_FAIL, so every rank learns of the
    failure in the same round and raises -- nobody returns while a peer waits
    in a collective that will never be joined.  Resolve outcomes
    are a function of the gathered records, so the ranks agree on "ok" /
    "resync" unless one of them failed."""
    rec = engine.local() if rec is None else rec
    for _ in range(world + 1):
        allrec = engine.exchange(rec)
        bad = engine.failed(allrec)
        err = None
        if bad:
            code, err = AGREE_FAIL, PeerFailed(f"rank(s) {bad} failed during seam resolution")
        else:
            try:
                code = AGREE_RESYNC if engine.resolve(allrec) == "resync" else AGREE_OK
            except BaseException as e:  # noqa: BLE001 -- re-raised after the agreement
                code, err = AGREE_FAIL, e
        agreed = engine.agree(code)
        if err is not None:
            raise err
        if agreed == AGREE_FAIL:
            raise PeerFailed("a peer rank failed during seam resolution")
        if agreed == AGREE_OK:
            return engine.result()
        rec = engine.record()
    raise RuntimeError("seam resolution did not settle within nranks rounds")


def _resolve_rc(rc, h):
    if rc == DSX_E_RESYNC:
        return "resync"
    if rc == DSX_E_PEER:
        raise PeerFailed("a peer rank failed during seam resolution")
    check(rc, h)
    return "ok"


class _HostEngine:
    """Library calls with host-memory seam records, any torch.distributed
    backend (records through host memory)."""

    def __init__(self, ctx, d_ptr, halo, shard_start, shard_len, total, params, group, device):
        import torch.distributed as dist
        self.ctx, self.d_ptr, self.halo = ctx, d_ptr, halo
        self.start, self.len, self.total, self.params = shard_start, shard_len, total, params
        self.group, self.device = group, device
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.seam = _lib.Seam()
        self.cap = shard_len // params.min + 4 + _lib.DSX_SEAM_MAX_CUTS
        self.out = np.empty(self.cap, dtype=np.uint64)
        self.n = ctypes.c_uint64()

    def local(self):
        L, h = lib(), self.ctx.h
        check(L.dsx_shard_local(h, ctypes.c_void_p(self.d_ptr), self.halo, self.start, self.len,
                                self.total, ctypes.byref(self.params.c),
                                ctypes.addressof(self.seam), 0), h)
        return seam_to_bytes(self.seam)

    def exchange(self, rec):
        return exchange_seams(rec, self.group, self.device)

    def failed(self, allrec):
        return failed_ranks(allrec, self.world)

    def agree(self, code):
        return agree_max(code, self.group, self.device)

    def resolve(self, allrec):
        arr = seams_from_bytes(allrec, self.world)
        rc = lib().dsx_shard_resolve(self.ctx.h, ctypes.addressof(arr), self.world, self.rank,
                                     ctypes.addressof(self.seam), self.out.ctypes.data, self.cap,
                                     ctypes.byref(self.n), 0)
        return _resolve_rc(rc, self.ctx.h)

    def record(self):
        return seam_to_bytes(self.seam)

    def mark_error(self, rec):
        b = bytearray(rec)
        fl = int.from_bytes(b[FLAGS_OFF:FLAGS_OFF + 4], "little") | _lib.DSX_SEAM_ERROR
        b[FLAGS_OFF:FLAGS_OFF + 4] = fl.to_bytes(4, "little")
        return bytes(b)

    def result(self):
        return self.out[:self.n.value].copy()


def shard_chunk(d_ptr, halo, shard_start, shard_len, total, params, ctx=None, group=None,
                device=None):
    """This rank's exact cut list (np.uint64 chunk end offsets c with
    shard_start < c <= shard_start + shard_len).  The seam records go through
    host memory and ``torch.distributed`` (any backend)."""
    ctx = ctx or _lib.default_context()
    eng = _HostEngine(ctx, d_ptr, halo, shard_start, shard_len, total, params, group, device)
    return seam_protocol(eng, eng.world)


def device_protocol(engine, world):
    """The asynchronous form of seam_protocol (dsx_shard_resolve_async /
    dsx_shard_collect), as a generator: it yields once, when the step's work
    is enqueued and the next thing would be the host's wait, and returns this
    rank's result (StopIteration.value; see run_device_protocol).  A
    pipelined caller starts step k+1 between the two.

    engine: local_async() enqueues the shard's scan + stitch + seam record;
    mark_error() replaces the record with a DSX_SEAM_ERROR one; gather()
    all-gathers the records; resolve() enqueues the resolve, whose round
    outcome (AGREE_*) lands in a device word; collect() waits and returns
    ("ok" | "resync" | "peer", agreed) or raises this rank's failure (leaving the
    round's agreed code in engine.last_agreed); result().
    With engine.device_agree (RCCL) the ranks agree on the device before the
    wait: fail_code() overwrites the word with AGREE_FAIL and reduce() enqueues
    its MAX all-reduce, so a converged step waits on the host exactly once
    (in collect).  Without it (records staged through host memory, e.g. gloo)
    the agreement is agree() after collect, as in seam_protocol.

    A failure before this rank's code is known (local_async / resolve) is published
    in the same round (its record or its code says FAIL); one found by collect
    after a device agreement (a failed re-walk, which marks the record
    DSX_SEAM_ERROR) is published by one more exchange round.  Either way every
    rank raises in the same round: nobody waits in a collective a peer left."""
    err = None
    try:
        engine.local_async()
    except BaseException as e:  # noqa: BLE001 -- raised once the peers know
        err = e
        engine.mark_error()
    if not engine.device_agree:
        yield
    for rnd in range(world + 1):
        engine.gather()
        if err is None:
            try:
                engine.resolve()
            except BaseException as e:  # noqa: BLE001
                err = e
        if engine.device_agree:
            if err is not None:
                engine.fail_code()
            engine.reduce()
            if err is not None:
                raise err
            if rnd == 0:
                yield
            try:
                out, agreed = engine.collect()
            except BaseException as e:  # noqa: BLE001
                # Agreed FAIL: every peer saw it and is raising PeerFailed in
                # this round, so this rank's own failure (e.g. its cut list
                # did not fit) is raised now -- another exchange round would
                # wait in a collective nobody joins.  Below FAIL (a re-walk
                # that failed after an OK/RESYNC agreement, the record marked
                # DSX_SEAM_ERROR): published by one more exchange round.
                if (getattr(engine, "last_agreed", None) or 0) >= AGREE_FAIL:
                    raise
                err = e
                continue
        else:
            out = None
            if err is None:
                try:
                    out, _ = engine.collect()
                except BaseException as e:  # noqa: BLE001
                    err = e
            code = (AGREE_FAIL if err is not None or out == "peer" else
                    AGREE_RESYNC if out == "resync" else AGREE_OK)
            agreed = engine.agree(code)
            if err is not None:
                raise err
        if agreed == AGREE_FAIL or out == "peer":
            raise PeerFailed("a peer rank failed during seam resolution")
        if agreed == AGREE_OK:
            return engine.result()
    if err is not None:
        raise err
    raise RuntimeError("seam resolution did not settle within nranks rounds")


def _drive(g):
    """Runs a device_protocol generator to its end; returns its result."""
    while True:
        try:
            next(g)
        except StopIteration as stop:
            return stop.value


def run_device_protocol(engine, world):
    return _drive(device_protocol(engine, world))


_COLLECT_RC = {0: "ok", DSX_E_RESYNC: "resync", DSX_E_PEER: "peer"}


class DeviceShard:
    """The N>1 path with the seam records in HBM (bench.py's step).

    ``run()`` chunks this rank's shard and returns its exact cut count; the
    cuts stay in ``self.out`` (an int64 device tensor).  Everything is
    ordered on the library context's stream (``dsx_ctx_stream``, wrapped as a
    torch ExternalStream): the asynchronous dsx_shard_local, the RCCL
    all-gather of the 16 KiB records, dsx_shard_resolve_async and the RCCL
    MAX all-reduce of the round code -- one host wait per converged step
    (dsx_shard_collect).  ``begin()`` / ``finish()`` split a step at that wait
    for a pipelined caller.  Over gloo (CPU tensors) the records are staged
    through host memory and the ranks agree on the host: two waits.
    """

    def __init__(self, ctx, d_ptr, halo, shard_start, shard_len, total, params, group=None):
        import torch
        import torch.distributed as dist
        self.ctx, self.d_ptr, self.halo = ctx, d_ptr, halo
        self.start, self.len, self.total, self.params = shard_start, shard_len, total, params
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.device_agree = dist.get_backend(group) == "nccl"
        dev = torch.device("cuda", ctx.device)
        self.seam = torch.empty(SEAM_BYTES, dtype=torch.uint8, device=dev)
        self.all = torch.empty(self.world * SEAM_BYTES, dtype=torch.uint8, device=dev)
        self.cap = shard_len // params.min + 4 + _lib.DSX_SEAM_MAX_CUTS
        self.out = torch.empty(self.cap, dtype=torch.int64, device=dev)
        self.code = torch.zeros(1, dtype=torch.int32, device=dev)
        self.n = ctypes.c_uint64()
        self.agreed = ctypes.c_int32()
        sp = ctypes.c_void_p()
        check(lib().dsx_ctx_stream(ctx.h, ctypes.byref(sp)), ctx.h)
        self.stream = torch.cuda.ExternalStream(sp.value, device=dev)
        self._g = None

    # -- engine interface (device_protocol) ------------------------------------
    def local_async(self):
        L, h = lib(), self.ctx.h
        check(L.dsx_shard_local(h, ctypes.c_void_p(self.d_ptr), self.halo, self.start, self.len,
                                self.total, ctypes.byref(self.params.c),
                                ctypes.c_void_p(self.seam.data_ptr()),
                                DSX_SEAM_DEVICE | DSX_NO_SYNC), h)

    def mark_error(self):
        import torch
        with torch.cuda.stream(self.stream):
            self.seam.zero_()
            self.seam[FLAGS_OFF] = _lib.DSX_SEAM_ERROR

    def gather(self):
        import torch
        import torch.distributed as dist
        with torch.cuda.stream(self.stream):
            if self.device_agree:
                dist.all_gather_into_tensor(self.all, self.seam, group=self.group)
            else:  # e.g. gloo (CPU tensors only): stage through host memory
                mine = self.seam.cpu()
                bufs = [torch.empty_like(mine) for _ in range(self.world)]
                dist.all_gather(bufs, mine, group=self.group)
                self.all.copy_(torch.cat(bufs))

    def resolve(self):
        check(lib().dsx_shard_resolve_async(self.ctx.h, ctypes.c_void_p(self.all.data_ptr()),
                                            self.world, self.rank,
                                            ctypes.c_void_p(self.out.data_ptr()), self.cap,
                                            ctypes.c_void_p(self.code.data_ptr())), self.ctx.h)

    def fail_code(self):
        import torch
        with torch.cuda.stream(self.stream):
            self.code.fill_(AGREE_FAIL)

    def reduce(self):
        import torch
        import torch.distributed as dist
        with torch.cuda.stream(self.stream):
            dist.all_reduce(self.code, op=dist.ReduceOp.MAX, group=self.group)

    def collect(self):
        d_agreed = ctypes.c_void_p(self.code.data_ptr()) if self.device_agree else None
        self.agreed.value = 0
        rc = lib().dsx_shard_collect(self.ctx.h, ctypes.c_void_p(self.seam.data_ptr()), d_agreed,
                                     ctypes.byref(self.agreed), ctypes.byref(self.n))
        # the round's agreed code, also when rc is this rank's own failure
        self.last_agreed = self.agreed.value if self.device_agree else None
        if rc not in _COLLECT_RC:
            check(rc, self.ctx.h)
        return _COLLECT_RC[rc], (self.agreed.value if self.device_agree else None)

    def agree(self, code):
        return agree_max(code, self.group)

    def result(self):
        return self.n.value

    # -- bench step ------------------------------------------------------------
    def begin(self):
        """Enqueue a step (up to the host wait)."""
        self._g = device_protocol(self, self.world)
        next(self._g)

    def finish(self):
        """Complete the step begun last; returns the exact cut count."""
        g, self._g = self._g, None
        return _drive(g)

    def run(self):
        self.begin()
        return self.finish()

    def cuts(self):
        return self.out[:self.n.value].cpu().numpy().astype(np.uint64)


# ---------------------------------------------------------------------------
# chunk IDs across shards
# ---------------------------------------------------------------------------
def tail_record(ctx, d_ptr, shard_start, shard_len, cuts, max_size):
    """This rank's seam tail: {has_cut, length} + the bytes behind its last
    cut (or, without a cut, its whole shard, < max bytes: a shard of max
    bytes or more always holds a cut), padded to 16 + max bytes -- the
    overlap bytes the next rank's first chunk needs."""
    end = shard_start + shard_len
    has_cut = len(cuts) > 0
    t0 = int(cuts[-1]) if has_cut else shard_start
    n = end - t0
    if n > max_size:
        raise ValueError(f"tail of {n} bytes behind the last cut exceeds max")
    rec = np.zeros(16 + max_size, dtype=np.uint8)
    rec[:16] = np.frombuffer(np.array([1 if has_cut else 0, n], np.uint64).tobytes(), np.uint8)
    if n:
        check(lib().dsx_copy(ctx.h, rec[16:].ctypes.data, ctypes.c_void_p(d_ptr + (t0 - shard_start)),
                             n), ctx.h)
    return rec.tobytes()


def rank_chunk_ids(ctx, d_ptr, shard_start, shard_len, cuts, tails, rank, algo=None):
    """IDs of this rank's chunks (those ending at its cuts), given every
    rank's tail_record (rank order).  The first chunk starts in an earlier
    shard (at most max bytes back): its prefix is the concatenated tails back
    to the first rank that has a cut; it is assembled in HBM and hashed with
    the rest of the shard's chunks by dsx_chunk_ids."""
    import torch

    from .make import chunk_ids
    cuts = np.asarray(cuts, dtype=np.uint64)
    if cuts.size == 0:
        return []
    prefix = b""
    for q in range(rank - 1, -1, -1):
        head = np.frombuffer(tails[q][:16], np.uint64)
        n = int(head[1])
        prefix = tails[q][16:16 + n] + prefix
        if head[0]:
            break
    first = int(cuts[0])
    head_len = first - shard_start
    buf = torch.empty(len(prefix) + head_len, dtype=torch.uint8, device=f"cuda:{ctx.device}")
    if prefix:
        buf[:len(prefix)].copy_(torch.frombuffer(bytearray(prefix), dtype=torch.uint8))
        torch.cuda.synchronize()
    if head_len:
        check(lib().dsx_copy(ctx.h, ctypes.c_void_p(buf.data_ptr() + len(prefix)),
                             ctypes.c_void_p(d_ptr), head_len), ctx.h)
    ids = chunk_ids(buf.data_ptr(), buf.numel(), np.array([buf.numel()], np.uint64), 0, ctx=ctx,
                    algo=algo)
    if cuts.size > 1:
        ids += chunk_ids(d_ptr, shard_len, cuts[1:] - np.uint64(shard_start), head_len, ctx=ctx,
                         algo=algo)
    return ids


def shard_chunk_ids(d_ptr, shard_start, shard_len, cuts, params, ctx=None, group=None,
                    device=None, algo=None):
    """Chunk IDs of this rank's cuts (shard_chunk's result), the seam-straddling
    chunk included: one all-gather of the <= max-byte tails (the overlap
    bytes), then dsx_chunk_ids on this rank's GPU."""
    import torch
    import torch.distributed as dist
    ctx = ctx or _lib.default_context()
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    rec = tail_record(ctx, d_ptr, shard_start, shard_len, cuts, params.max)
    mine = torch.frombuffer(bytearray(rec), dtype=torch.uint8)
    if device is not None:
        mine = mine.to(device)
    bufs = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(bufs, mine, group=group)
    tails = [b.cpu().numpy().tobytes() for b in bufs]
    return rank_chunk_ids(ctx, d_ptr, shard_start, shard_len, cuts, tails, rank, algo)
