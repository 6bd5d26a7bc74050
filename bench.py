#!/usr/bin/env python3
"""Benchmark: GiB/s chunked (device-resident blob -> cut list), BASELINE.json.

Workload (default): BASELINE config 5's per-GPU shard -- 32 GiB of the seed-3
splitmix64 uniform blob per GPU (256 GiB over 8 GPUs), generated on device and
chunked with desync's default min/avg/max = 16/64/256 KiB.  The blob is in HBM
when the timed region starts and one step produces the complete cut list of
the shard in HBM (scan + stitch of four 8 GiB pieces, libdsx.so).  The same
per-GPU shape runs at every N (weak scaling), so the N = 1 line and the
1/2/4/8-GPU curve are one configuration.  --config2 runs BASELINE config 2's
shape instead (1 GiB, seed 1).

N > 1 (one process per GPU, torch.distributed over RCCL): rank r holds bytes
[r*n, (r+1)*n) of the N*n-byte blob (+64 B halo, regenerated locally), chunks
it speculatively (dsx_shard_local), all-gathers the small seam records (RCCL,
in place in HBM), and resolves its final cut list in HBM
(dsx_shard_resolve_async).  The whole step is ordered on the library stream;
the host waits once per step (dsx_shard_collect).

roofline.kernel_ms is the mean duration of the scan launches of exactly the
timed jobs, stamped from inside the kernel (dsx_stamps_begin/end:
s_memrealtime at the first wave's first and the last wave's last
instruction), with nothing added between the launches.

Prints ONE JSON line on rank 0 (contract in the task statement).
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

GiB = 1 << 30
MIN, AVG, MAX = 16 * 1024, 64 * 1024, 256 * 1024
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table: 8.0 TB/s spec
PIECE = 8 * GiB          # bytes per scan launch (the engine's piece, kPieceMax)
CPU_SAMPLE = GiB         # cpu_baseline: the first GiB of the shard
METRIC = "GiB/s chunked (device-resident blob→cut list), 16/64/256KiB, 1/2/4/8 MI355X"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--gib", type=float, default=None,
                    help="GiB per GPU (default: the workload's BASELINE config: 32 uniform "
                         "(config 5 shard), 16 dedup (config 3), 64 zeros (config 4))")
    ap.add_argument("--workload", default="uniform", choices=["uniform", "dedup", "zeros"])
    ap.add_argument("--seed", type=int, default=0,
                    help="generator seed (0: 3 for uniform -- config 5 --, 2 for dedup)")
    ap.add_argument("--config5", action="store_true",
                    help="BASELINE config 5's shard shape (the default): 32 GiB of the seed-3 "
                         "uniform blob per GPU (256 GiB over 8 GPUs)")
    ap.add_argument("--config2", action="store_true",
                    help="BASELINE config 2's shape: 1 GiB of the seed-1 uniform blob per GPU")
    ap.add_argument("--avg", type=int, default=64,
                    help="average chunk size in KiB, min = avg/4, max = 4*avg (SURVEY.md 8(d)'s "
                         "sweep 16/64/256, chunker_test.go:191's set); default 64 = desync make's "
                         "16/64/256 KiB")
    ap.add_argument("--no-cpu", action="store_true", help="skip the cpu_baseline leg")
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="threads of the cpu_baseline leg (0: the job's CPU share)")
    ap.add_argument("--inflight", type=int, default=0,
                    help="chunking jobs kept in flight (0: 4 at N = 1, queued on one library "
                         "context; N > 1: 3 pipeline lanes, one library context and process "
                         "group each)")
    ap.add_argument("--check", action="store_true",
                    help="N>1: compare the concatenated per-rank cut lists with one "
                         "dsx_cut_device over the whole blob on rank 0 (small sizes)")
    ap.add_argument("--marks", default=None,
                    help="write {t0, t1, bytes} (unix time around the timed steps) to this "
                         "file, for tools/smu_summary.py's energy window")
    args = ap.parse_args()
    if args.config2:
        args.workload, args.gib, args.seed = "uniform", args.gib or 1.0, args.seed or 1
    elif args.config5:
        args.workload = "uniform"
    if args.gib is None:
        args.gib = {"uniform": 32.0, "dedup": 16.0, "zeros": 64.0}[args.workload]
    if not args.seed:
        args.seed = 2 if args.workload == "dedup" else 3
    args.config = ("config 5 shard" if (args.workload, args.gib, args.seed) == ("uniform", 32.0, 3)
                   else "config 2" if (args.workload, args.gib, args.seed) == ("uniform", 1.0, 1)
                   else "config 3" if (args.workload, args.gib) == ("dedup", 16.0)
                   else "config 4" if (args.workload, args.gib) == ("zeros", 64.0) else None)
    if args.avg != 64:
        args.config = None
    if args.inflight <= 0:
        args.inflight = 4 if int(os.environ.get("WORLD_SIZE", "1")) == 1 else 3
    return args


DATA_LABEL = {"uniform": "uniform, splitmix64 seed {seed} (dsx_gen_uniform)",
              "dedup": "dedup, seed {seed}, 30 % of 1 MiB blocks copy earlier ones (dsx_gen_dedup)",
              "zeros": "zeros"}


def make_blob(ctx, t, offset, n, workload, seed):
    from desync_amd import _lib
    L = _lib.lib()
    if workload == "uniform":
        _lib.check(L.dsx_gen_uniform(ctx.h, ctypes.c_void_p(t.data_ptr()), offset, n, seed), ctx.h)
    elif workload == "dedup":
        _lib.check(L.dsx_gen_dedup(ctx.h, ctypes.c_void_p(t.data_ptr()), offset, n, seed, 0.30),
                   ctx.h)
    else:
        t.zero_()


def load_traffic(workload, nbytes):
    """HBM bytes per scan launch of `nbytes` from the committed rocprofv3 PMC
    pass (profiles/traffic_<workload>_<nbytes>.json, or the older
    profiles/traffic_<workload>.json: L2 -> fabric read requests x their
    sizes, tools/traffic_json.py)."""
    for name in (f"traffic_{workload}_{int(nbytes)}.json", f"traffic_{workload}.json"):
        try:
            with open(os.path.join(REPO, "profiles", name)) as f:
                d = json.load(f)
            if int(d.get("bytes", -1)) == int(nbytes):
                return float(d["hbm_bytes_per_launch"])
        except (OSError, ValueError, KeyError):
            pass
    return None


def cpu_share():
    """Host threads this job may use: the GPU box exports OMP_NUM_THREADS (16,
    its CPU share for one GPU); nproc / os.cpu_count() there report the whole
    machine, which a one-GPU job must not take."""
    try:
        return max(1, int(os.environ["OMP_NUM_THREADS"]))
    except (KeyError, ValueError):
        return max(1, min(os.cpu_count() or 1, 16))


def _cpu_leg(sample, threads, budget_s):
    """Repeat oracle.chunk_parallel over the sample until ~budget_s core-seconds."""
    from oracle import oracle as o
    o.chunk_parallel(sample[:64 << 20], MIN, AVG, MAX, threads)  # threads + pages warm
    reps, t_total = 0, 0.0
    while True:
        t0 = time.perf_counter()
        o.chunk_parallel(sample, MIN, AVG, MAX, threads)
        t_total += time.perf_counter() - t0
        reps += 1
        if t_total * threads >= budget_s or reps >= 20:
            break
    return reps, reps * sample.size / t_total / GiB


def _ids_rate(sample, threads):
    """SHA-512/256 chunk IDs on the host (hashlib releases the GIL), reported
    separately as BASELINE.md's plan asks."""
    import concurrent.futures as cf
    import hashlib
    from oracle import oracle as o
    ends = o.chunk_parallel(sample, MIN, AVG, MAX, threads).tolist()
    starts = [0] + ends[:-1]
    mv = memoryview(sample)

    def h(i):
        z = hashlib.new("sha512_256")
        z.update(mv[starts[i]:ends[i]])
        return z.digest()

    t0 = time.perf_counter()
    with cf.ThreadPoolExecutor(threads) as pool:
        for _ in pool.map(h, range(len(ends)), chunksize=64):
            pass
    return sample.size / (time.perf_counter() - t0) / GiB


def cpu_baseline(host_blob, threads=None):
    """make.go-style split-and-align (C restatement, oracle/) on the host:
    at the job's CPU share and at n = 10 (desync make's default -n), plus one
    thread and the SHA-512/256 ID rate."""
    from oracle import oracle as o
    threads = threads or cpu_share()
    sample = host_blob
    n = sample.size
    pre = sample[:128 << 20]
    t0 = time.perf_counter()
    o.chunk_stream(pre, MIN, AVG, MAX)
    single = pre.size / (time.perf_counter() - t0) / GiB
    reps, rate = _cpu_leg(sample, threads, 10.0)
    reps10, rate10 = _cpu_leg(sample, 10, 8.0)
    ids = _ids_rate(sample[:256 << 20], threads)
    return {
        "value": round(rate, 3),
        "unit": "GiB/s",
        "cores": threads,
        "kind": "port",
        "sample": (f"{reps}x the same {n / GiB:.2f} GiB blob, C restatement of desync's "
                   f"Chunker.Next loop with make.go split-and-align over {threads} threads "
                   f"(the job's CPU share; oracle/dsx_oracle.c, in memory, no chunk IDs); "
                   f"n=10 (desync make default): {rate10:.3f} GiB/s over {reps10}x; "
                   f"single thread {single:.3f} GiB/s on 128 MiB; SHA-512/256 IDs "
                   f"{ids:.3f} GiB/s over {threads} threads on 256 MiB"),
        "bytes": int(n),
        "gpu_bytes_per_step": None,
        "n10_gibs": round(rate10, 3),
        "single_thread_gibs": round(single, 3),
        "ids_sha512_256_gibs": round(ids, 3),
    }


def roofline_of(stamps, dt, workload):
    """The roofline object of one rank from its scan launches' in-kernel
    stamps (None without stamps)."""
    if not stamps:
        return None
    dur = np.array([st.ms for st in stamps])
    nb = np.array([st.bytes for st in stamps], dtype=np.float64)
    cyc = sum(st.wave_cycles for st in stamps)
    tick = sum(st.wave_ticks for st in stamps)
    per_launch = int(np.median(nb))
    achieved = float(nb.sum() / (dur.sum() / 1e3) / 1e9)
    return {
        "bound": "hbm",
        "achieved": round(achieved, 1),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        "traffic": load_traffic(workload, per_launch),
        "kernel": "dsx::scanl_kernel",
        "bytes_per_launch": per_launch,
        "launches": len(stamps),
        "kernel_ms": round(float(dur.mean()), 4),
        "kernel_ms_min_max": [round(float(dur.min()), 4), round(float(dur.max()), 4)],
        "clock_mhz": round(100.0 * cyc / tick, 1) if tick else None,
        "wave_busy": round(float(np.mean([st.busy for st in stamps])), 4),
        "scan_share_of_step": round(float(dur.sum()) / (dt * 1e3), 4),
        "timing": "in-kernel s_memrealtime stamps of the timed jobs' scan launches",
    }


def hbm_footprint(torch, blob, outs, ctxs):
    """This rank's HBM: the blob, the cut-list buffers, and every library
    context's pipeline buffers (dsx_stats_t.device_bytes), against the
    device's capacity.  Raises if they would not fit (a config the GPU
    cannot hold must fail here, not in a kernel)."""
    free, total = torch.cuda.mem_get_info()
    lib_bytes = [int(c.stats().device_bytes) for c in ctxs]
    out_bytes = sum(o.numel() * o.element_size() for o in outs)
    used = blob.numel() + out_bytes + sum(lib_bytes)
    if used > total:
        raise RuntimeError(f"HBM footprint {used} B exceeds the device's {total} B")
    return {"blob_bytes": blob.numel(), "cut_list_bytes": out_bytes,
            "context_bytes": lib_bytes, "total_bytes": used, "device_bytes": total,
            "device_free_bytes": free, "frac_of_device": round(used / total, 4)}


def dist_info(dist, backend, per_rank):
    """What torch.distributed reports for the job: the backend of the
    default group, its world size and, over RCCL, the library version."""
    info = {"backend": dist.get_backend(), "requested": backend,
            "world_size": dist.get_world_size(), "ranks_reporting": len(per_rank)}
    if info["backend"] == "nccl":
        try:
            import torch
            v = torch.cuda.nccl.version()
            info["rccl_version"] = ".".join(map(str, v)) if isinstance(v, tuple) else str(v)
        except Exception as e:  # noqa: BLE001 -- reported, not fatal
            info["rccl_version"] = f"unknown ({e})"
    return info


def main():
    args = parse()
    global MIN, AVG, MAX
    AVG = args.avg * 1024
    MIN, MAX = AVG // 4, AVG * 4
    import torch
    from desync_amd import _lib
    import desync_amd

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        # a line for N GPUs must come from N ranks (the driver launches N > 1
        # through torch.distributed.run with --nproc-per-node N)
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE {world}: launch N > 1 "
                         f"through torch.distributed.run --nproc-per-node {args.gpus}")
    # one GPU per rank; DSX_DIST_BACKEND=gloo with more ranks than GPUs is a
    # functional rehearsal of the N>1 path on a one-GPU box (not a measurement)
    backend = os.environ.get("DSX_DIST_BACKEND", "nccl")
    gpu = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(gpu)
    dist = None
    ranks_counted = 1
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
        else:
            dist.init_process_group(backend)
        # the ranks the collective backend itself sees (RCCL over xGMI for
        # "nccl"): a sum of ones over the default group, before anything is
        # timed, so that no curve point comes from fewer ranks than it claims
        one = torch.ones(1, dtype=torch.int64, device="cuda" if backend == "nccl" else "cpu")
        dist.all_reduce(one)
        ranks_counted = int(one.item())
        if int(one.item()) != world or dist.get_world_size() != world:
            raise SystemExit(f"bench.py: {backend} group has {int(one.item())} ranks "
                             f"(world_size {dist.get_world_size()}), expected {world}")
    ctx = _lib.Context(gpu)
    n = int(args.gib * GiB)
    p = desync_amd.Params(MIN, AVG, MAX)
    L = _lib.lib()

    # ---------------- inputs (outside the timed region) ----------------
    halo = 64 if rank > 0 else 0
    blob = torch.empty(n + halo, dtype=torch.uint8, device="cuda")
    make_blob(ctx, blob, rank * n - halo, n + halo, args.workload, args.seed)
    d_ptr = blob.data_ptr() + halo
    cap = n // MIN + 4
    shard = None
    lanes = []
    if world > 1:
        # N > 1: `inflight` pipeline lanes, each with its own library context
        # and process group; step s runs on lane s mod L.  A step is enqueued
        # whole on its lane's stream (scan, stitch, seam record, RCCL
        # all-gather, resolve, RCCL agreement) before the host waits for step
        # s - L, the step's one host wait
        from desync_amd.shard import DeviceShard
        for i in range(max(1, args.inflight)):
            c_i = ctx if i == 0 else _lib.Context(gpu)
            g_i = None if i == 0 else dist.new_group()
            lanes.append(DeviceShard(c_i, d_ptr, halo, rank * n, n, n * world, p, group=g_i))
        shard = lanes[0]

    # N = 1: every step is one complete dsx_cut_device job (scan + stitch, cut
    # list in HBM) whose count the host collects.  Up to `inflight` jobs are
    # queued on the context (DSX_NO_SYNC): job s is enqueued before the host
    # waits for job s - inflight, so the GPU is not idle while the host wakes
    # up.  Each job's stitch follows its scan on the library stream; the host
    # polls the state the stitch publishes (no event between jobs).
    depth = min(8, max(1, args.inflight)) if world == 1 else 1
    outs = [torch.empty(cap, dtype=torch.int64, device="cuda") for _ in range(depth)]
    queued = []
    cnt = ctypes.c_uint64()

    def collect():
        _lib.check(L.dsx_result(ctx.h, ctypes.byref(cnt)), ctx.h)
        queued.pop(0)
        return cnt.value

    def step(s):
        if world == 1:
            got = collect() if len(queued) == depth else None
            _lib.check(L.dsx_cut_device(ctx.h, ctypes.c_void_p(d_ptr), n, ctypes.byref(p.c),
                                        ctypes.c_void_p(outs[s % depth].data_ptr()), cap,
                                        ctypes.byref(cnt), _lib.DSX_OUT_DEVICE | _lib.DSX_NO_SYNC),
                       ctx.h)
            queued.append(s)
            return got
        # N > 1: chunk this rank's shard, RCCL all-gather of the 16 KiB seam
        # records in HBM, resolve the seams (desync_amd/shard.py)
        return shard.run()

    def drain():
        last = None
        while queued:
            last = collect()
        return last

    def run_lanes(nsteps):
        """N > 1: step s on lane s mod L, from one host thread: every rank
        issues the same collectives in the same order (no cross-communicator
        deadlock), and up to L steps are queued on the GPU."""
        from collections import deque
        pending, last = deque(), None
        for s in range(nsteps):
            if len(pending) == len(lanes):
                last = pending.popleft().finish()
            ln = lanes[s % len(lanes)]
            ln.begin()
            pending.append(ln)
        while pending:
            last = pending.popleft().finish()
        return last

    if world == 1:
        for s in range(args.warmup):
            step(s)
        drain()
    else:
        for ln in lanes:  # every lane once, in order on every rank
            ln.run()
        run_lanes(args.warmup)
    torch.cuda.synchronize()
    stamping = os.environ.get("DSX_BENCH_STAMPS", "1") != "0"  # (0: A/B of their cost)
    # in-kernel stamps of exactly the timed jobs' scan launches, on every
    # library context of this rank (N > 1: one per pipeline lane)
    stamp_ctxs = [ln.ctx for ln in lanes] if world > 1 else [ctx]
    if stamping:
        for c in stamp_ctxs:
            c.stamps_begin(args.steps * ((n + PIECE - 1) // PIECE) + 8)
    if dist:
        dist.barrier()
    t0 = time.perf_counter()
    wall0 = time.time()
    chunks = 0
    if world == 1:
        for s in range(args.steps):
            r = step(s)
            chunks = r if r is not None else chunks
        chunks = drain()
    else:
        chunks = run_lanes(args.steps)
    torch.cuda.synchronize()
    if dist:
        dist.barrier()
    dt = time.perf_counter() - t0
    wall1 = time.time()
    if args.marks:
        with open(args.marks, "w") as f:
            json.dump({"t0": wall0, "t1": wall1, "bytes": n * args.steps, "rank": rank}, f)
    stamps = [st for c in stamp_ctxs for st in c.stamps_end()] if stamping else []
    mine = {"rank": rank, "roofline": roofline_of(stamps, dt, args.workload), "hbm": hbm_footprint(
        torch, blob, outs + ([sh.out for sh in lanes] if lanes else []), stamp_ctxs)}
    per_rank = [mine]
    if dist:
        per_rank = [None] * world
        dist.all_gather_object(per_rank, mine)
        tdev = "cuda" if backend == "nccl" else "cpu"
        tt = torch.tensor([dt], dtype=torch.float64, device=tdev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        dt = float(tt.item())
        tc = torch.tensor([chunks], dtype=torch.int64, device=tdev)
        dist.all_reduce(tc)
        chunks = int(tc.item())
    ms_per_step = dt / args.steps * 1000.0
    value = (n * world * args.steps) / dt / GiB

    if args.check and world > 1:
        mine = torch.from_numpy(shard.cuts().astype(np.int64))
        lists = [None] * world
        dist.all_gather_object(lists, mine.tolist())
        if rank == 0:
            whole = torch.empty(n * world, dtype=torch.uint8, device="cuda")
            make_blob(ctx, whole, 0, n * world, args.workload, args.seed)
            ref = desync_amd.cut_device(whole.data_ptr(), n * world, MIN, AVG, MAX, ctx=ctx)
            got = np.array(sum(lists, []), dtype=np.uint64)
            assert np.array_equal(got, ref), "sharded cut list differs from the single-GPU one"
            print(f"check ok: {got.size} cuts across {world} shards", file=sys.stderr)
    if rank == 0:
        res = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": f"synthetic ({DATA_LABEL[args.workload].format(seed=args.seed)}, generated on device)",
            "config": {
                "workload": (f"{args.gib:g} GiB {args.workload} blob per GPU"
                             f"{' (BASELINE ' + args.config + ' shape)' if args.config else ''}, "
                             f"desync make min/avg/max {MIN >> 10}/{AVG >> 10}/{MAX >> 10} KiB, device-resident blob -> "
                             f"cut list in HBM"),
                "bytes_per_gpu": n,
                "chunks": int(chunks),
                "parallelism": f"range-shard x{world}" if world > 1 else "single GPU",
                "jobs_in_flight": depth if world == 1 else len(lanes),
            },
        }
        rl = [r["roofline"] for r in per_rank]
        if all(rl):
            # N = 1: this rank's scan; N > 1: the slowest rank's (min frac),
            # with every rank's own figures beside it
            worst = min(rl, key=lambda x: x["frac"])
            res["roofline"] = dict(worst)
            if world > 1:
                res["roofline"]["rank"] = rl.index(worst)
                res["roofline"]["per_rank"] = [
                    {k: x[k] for k in ("achieved", "frac", "kernel_ms", "clock_mhz", "launches")}
                    for x in rl]
                res["roofline"]["frac_min_max"] = [min(x["frac"] for x in rl),
                                                   max(x["frac"] for x in rl)]
        res["hbm"] = per_rank[0]["hbm"] if world == 1 else {
            "per_rank_bytes": [r["hbm"]["total_bytes"] for r in per_rank],
            "device_bytes": per_rank[0]["hbm"]["device_bytes"],
            "max_frac": max(r["hbm"]["frac_of_device"] for r in per_rank),
            "rank0": per_rank[0]["hbm"]}
        if dist:
            res["dist"] = dist_info(dist, backend, per_rank)
            res["dist"]["ranks_counted_by_backend"] = ranks_counted
        if world == 1 and not args.no_cpu:
            # a bounded sample: the shard's first GiB (the leg is ~10-30 s of CPU work)
            host = blob[halo:halo + min(n, CPU_SAMPLE)].cpu().numpy()
            res["cpu_baseline"] = cpu_baseline(host, args.cpu_threads or None)
            res["cpu_baseline"]["gpu_bytes_per_step"] = n  # (the sample is the shard's first GiB)
        print(json.dumps(res), flush=True)
    if dist:
        dist.destroy_process_group()
    ctx.close()


if __name__ == "__main__":
    main()
