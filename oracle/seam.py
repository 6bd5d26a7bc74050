"""CPU restatement of the multi-GPU seam protocol -- TEST INFRASTRUCTURE ONLY.

Mirrors dsx_shard_local / dsx_shard_resolve (include/dsx.h) on top of the
oracle's candidate predicate and chain rule, so the N>1 exchange (seam record
packing + all-gather + alignment) can be tested with torch.distributed "gloo"
on CPU.  The alignment is make.go's syncWith (make.go:277-298): the chain that
enters a shard is walked until it lands on a cut of the shard's speculative
chain.
"""
from __future__ import annotations

import numpy as np

from . import oracle as o

UNDET = None


def _next(s, cands, j, mn, mx, L, PE, is_last):
    """Chain rule step; returns (next, j) or (None, j) if undetermined."""
    if is_last:
        if L - s <= mn:
            return L, j
        lim = min(s + mx, L)
    else:
        lim = s + mx
    while j < len(cands) and cands[j] <= s + mn:
        j += 1
    if j < len(cands) and cands[j] <= lim:
        return int(cands[j]), j
    if not is_last and lim > PE:
        return UNDET, j
    return lim, j


def spec_chain(cands, start, mn, mx, L, PE, is_last):
    """Cuts of the chain started at `start`, until undetermined or L."""
    cuts, s, j = [], start, 0
    while True:
        if is_last and s >= L:
            break
        nx, j = _next(s, cands, j, mn, mx, L, PE, is_last)
        if nx is UNDET:
            break
        cuts.append(nx)
        s = nx
    return cuts


def shard_local(full, start, length, total, mn, av, mx, max_cands=1024, max_cuts=1024):
    """Seam record + speculative cut list of one shard (positions absolute)."""
    is_last = start + length == total
    lo = max(0, start - 64)
    c = o.candidates(full[lo:start + length], mn, av, mx) + lo  # halo for windows
    c = c[(c > start) & (c >= 48)]
    cuts = spec_chain(c, start, mn, mx, total, start + length, is_last)
    wend = start + min(length, 32 * mx)
    wc = [int(x) for x in c if x <= wend]
    if len(wc) > max_cands:
        wend = wc[max_cands - 1]
        wc = wc[:max_cands]
    wcuts = []
    for x in cuts:
        if x > wend:
            break
        if len(wcuts) == max_cuts:
            wend = wcuts[-1]
            break
        wcuts.append(x)
    wc = [x for x in wc if x <= wend]
    exit_cut = cuts[-1] if cuts else start
    seam = dict(shard_start=start, shard_len=length, total=total, exit_cut=exit_cut,
                window_end=wend, cands=wc, cuts=wcuts, flags=1 if is_last else 0)
    return seam, cuts


def resolve(seams, rank, mn, mx):
    """(ext cuts, c_rank): the true cuts of `rank` before its convergence point."""
    if rank == 0:
        return [], seams[0]["shard_start"]
    entry = seams[0]["exit_cut"]
    for r in range(1, rank + 1):
        s = seams[r]
        L, PE = s["total"], s["window_end"]
        is_last = PE == L
        x, j, ext, c = entry, 0, [], None
        cutset = set(s["cuts"])
        if x == s["shard_start"] or s["shard_len"] == 0:
            c = s["shard_start"]
        else:
            while True:
                if is_last and x >= L:
                    c = x
                    break
                nx, j = _next(x, s["cands"], j, mn, mx, L, PE, is_last)
                if nx is UNDET:
                    break
                if nx in cutset:
                    c = nx
                    break
                if r == rank:
                    ext.append(nx)
                x = nx
        if c is None:
            raise RuntimeError(f"seam {r} did not converge inside its window")
        if r == rank:
            return ext, c
        entry = s["exit_cut"] if s["shard_len"] else entry
    raise AssertionError


def rank_cuts(seams, rank, spec_cuts, mn, mx):
    ext, c = resolve(seams, rank, mn, mx)
    return np.array(ext + [x for x in spec_cuts if x >= c], dtype=np.uint64)
