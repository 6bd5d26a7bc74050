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


SEAM_LAST = 1
SEAM_REWALKED = 2


def shard_local(full, start, length, total, mn, av, mx, max_cands=1024, max_cuts=1024):
    """Seam record + speculative cut list + candidates of one shard (absolute
    positions).  Mirrors dsx_shard_local (seam_cands_kernel /
    seam_finalize_kernel)."""
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
                window_end=wend, entry=start, cands=wc, cuts=wcuts,
                flags=SEAM_LAST if is_last else 0)
    return seam, cuts, c


def rewalk(cands, entry, start, length, total, mn, mx):
    """The shard's chain re-walked from its true entry cut (dsx_shard_resolve's
    DSX_E_RESYNC path): every cut of it is true."""
    is_last = start + length == total
    cuts = spec_chain(cands, entry, mn, mx, total, start + length, is_last)
    seam = dict(shard_start=start, shard_len=length, total=total,
                exit_cut=cuts[-1] if cuts else entry, window_end=start, entry=entry, cands=[],
                cuts=[], flags=(SEAM_LAST if is_last else 0) | SEAM_REWALKED)
    return seam, cuts


def resolve(seams, rank, mn, mx):
    """seam_resolve_kernel: ("ok", ext cuts, c_rank) where the rank's true cuts
    are ext + [spec cuts >= c_rank], or ("resync", failing rank, its true entry
    cut) when some seam did not converge inside its window (every rank checks
    every seam, so all ranks agree on another exchange round)."""
    mine = ([], seams[rank]["shard_start"])
    entry = seams[0]["exit_cut"]
    for r in range(1, len(seams)):
        s = seams[r]
        ext, c = [], None
        if s["flags"] & SEAM_REWALKED:
            if entry == s["entry"]:
                c = 0
        elif entry == s["shard_start"] or s["shard_len"] == 0:
            c = s["shard_start"]
        else:
            L, PE = s["total"], s["window_end"]
            is_last = PE == L
            x, j = entry, 0
            cutset = set(s["cuts"])
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
            return "resync", r, entry
        if r == rank:
            mine = (ext, c)
        entry = s["exit_cut"] if s["shard_len"] else entry
    return ("ok",) + mine


def rank_cuts(ext, c, spec_cuts):
    return np.array(list(ext) + [x for x in spec_cuts if x >= c], dtype=np.uint64)
