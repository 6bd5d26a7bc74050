#!/usr/bin/env python3
"""Price the reference's min-skip for the GPU scan.

chunker.go:225-237 hashes a chunk only from start+min-48 and tests only from
start+min+1, so ~25 % of the bytes (16,336 of a 65.5 KiB mean chunk) are
never read by the sequential path.  The exhaustive scan (scanl_kernel) stages,
hashes and tests all of them.  This model takes the candidate list of real
random data and counts, per design, the bytes a skipping GPU scan must stage
and the hash steps it must run, per input byte, and what the speculative
chains' merges and the work distribution cost.

Design WC(G): a wave's 64 lanes split into G groups of 64/G lanes; each group
follows ONE chain (make.go's worker, chunker.go:206-277) over a span of the
blob: after a cut c it jumps to the line of c+min-47 and scans windows of
(64/G) lines, lane j hashing line j (48 warm-up steps from the line before,
then 128 tested positions) until a window holds the next cut.  The next
window's DMA is issued before the current one is hashed (else its HBM
latency is exposed once per window), so at every cut one window is staged
for nothing.  A span's chain starts at a virtual cut (the span start) and
runs past the span end until it meets the next span's chain (make.go's
syncWith, :277-327); the merge overrun is counted as work.

Design L (lane chains): one lane per chain, lanes of a wave in lockstep; a
lane's work is its own bytes; the wave lasts as long as its busiest lane.

Energy per byte (profiles/r05b, r05c at the 1400 W cap): staging 0.145 J/GiB
(line DMA + LDS round trip, per staged byte), hashing 0.097 J/GiB (per tested
position; a warm-up step has no boundary test: ~0.6 of a tested step by the
VALU count, 3 of 4.9 instructions).  The scan is held at the package power
cap, so its rate is ~ (P_cap - P_idle) / energy per byte; the exhaustive scan
measures 0.245 J/GiB above idle at frac 0.637.

Usage: python tools/skip_model.py [MiB]   (prints one JSON line)
"""
import json
import os
import re
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MIN, AVG, MAX = 16 << 10, 64 << 10, 256 << 10
LINE = 128
E_STAGE, E_HASH, E_EXH, FRAC_EXH = 0.145, 0.097, 0.245, 0.637
WARM_COST = 3.0 / 4.9


def table():
    txt = open(os.path.join(REPO, "include", "dsx_buzhash_table.h")).read()
    body = txt[txt.index("DSX_BUZHASH_TABLE_INIT"):]
    vals = [int(x, 16) for x in re.findall(r"0x([0-9A-Fa-f]{8})u", body)[:256]]
    assert len(vals) == 256
    return np.array(vals, dtype=np.uint32)


def discriminator(avg):
    return int(avg / (-1.42888852e-7 * avg + 1.33237515))


def candidates(b):
    """Positions p (cut after byte p-1) whose 48-byte window [p-48, p) hashes
    to h % d == d-1 (chunker.go:259-271's test, position form)."""
    T = table()
    n = b.size
    h = np.zeros(n - 47, dtype=np.uint32)
    for j in range(48):
        r = (47 - j) % 32
        t = T[b[j:n - 47 + j]]
        if r:
            t = (t << np.uint32(r)) | (t >> np.uint32(32 - r))
        h ^= t
    d = discriminator(AVG)
    hit = np.nonzero(h % np.uint32(d) == np.uint32(d - 1))[0]
    return hit.astype(np.int64) + 48  # window [i, i+48) -> cut position i + 48


class Cands:
    def __init__(self, pos, n):
        self.pos, self.n = pos, n

    def next_cut(self, s):
        """chunker.go:206-277: the chunk after a cut at s (None at the end)."""
        if s >= self.n:
            return None
        if self.n - s <= MIN:
            return self.n
        hi = s + min(MAX, self.n - s)
        i = np.searchsorted(self.pos, s + MIN + 1)
        if i < self.pos.size and self.pos[i] <= hi:
            return int(self.pos[i])
        return hi

    def chain(self, s, stop):
        out = []
        while s is not None and s < stop:
            s = self.next_cut(s)
            if s is not None:
                out.append(s)
        return out


def wc_chunk_cost(c, c2, group_lines):
    """Staged bytes and hash steps of one chunk (c, c2] in WC with windows of
    `group_lines` lines."""
    a0 = (c + MIN - 47) // LINE * LINE
    wb = group_lines * LINE
    k = max(0, (c2 - a0 - 1) // wb)  # window index holding c2 (tests (a, a + wb])
    windows = k + 1
    staged = (windows + 1) * wb      # + the speculatively issued next window
    tested = windows * wb
    warm = windows * group_lines * 48
    return staged, tested, warm


def span_work(C, v, v_next, group_lines):
    """One span's chain from the virtual cut v until it meets the chain of
    the span starting at v_next (or the blob end); returns (staged, tested,
    warm, overrun chunks)."""
    nxt = set(C.chain(v_next, v_next + 8 * MAX)) if v_next < C.n else set()
    staged = tested = warm = 0
    s, over = v, 0
    while True:
        s2 = C.next_cut(s)
        if s2 is None:
            break
        st, te, wa = wc_chunk_cost(s, s2, group_lines)
        staged, tested, warm = staged + st, tested + te, warm + wa
        if s2 >= v_next:
            over += 1
            if s2 in nxt or s2 >= C.n or over > 64:
                break
        s = s2
    return staged, tested, warm, over


def energy(staged, tested, warm, n):
    return (E_STAGE * staged + E_HASH * (tested + WARM_COST * warm)) / n


def main():
    mib = float(sys.argv[1]) if len(sys.argv) > 1 else 96
    n = int(mib * (1 << 20))
    b = np.random.default_rng(3).integers(0, 256, n, dtype=np.uint8)
    C = Cands(candidates(b), n)
    true = C.chain(0, n)
    sizes = np.diff([0] + true)
    skip_ideal = float(np.sum(np.minimum(sizes, MIN - 48)) / n)
    res = {"tool": "skip_model", "bytes": n, "chunks": len(true),
           "mean_chunk": float(sizes.mean()),
           "ideal_skip_fraction": round(skip_ideal, 4),
           "exhaustive": {"j_per_gib": E_EXH, "frac": FRAC_EXH}, "designs": []}
    # the driver's shape: 32 GiB per GPU, 2048 waves (8 per CU) -> per-GPU
    # chains = 2048 * G, 32 GiB / chains per chain
    for G in (1, 2, 4, 8):
        glines = 64 // G
        for span_mib in (0.25, 0.5, 1, 2, 4):
            span = int(span_mib * (1 << 20))
            if span > n // 4:
                continue
            tot = np.zeros(3)
            overs, works = [], []
            for v in range(0, n - span, span):
                st, te, wa, ov = span_work(C, v, v + span, glines)
                tot += (st, te, wa)
                overs.append(ov)
                works.append(E_STAGE * st + E_HASH * (te + WARM_COST * wa))
            covered = (n - span) // span * span
            e = energy(*tot, covered) * E_EXH / (E_STAGE + E_HASH)
            works = np.array(works)
            # list scheduling of 32 GiB worth of spans over 2048 * G groups:
            # the tail is ~ the mean remaining of a group's last span
            groups = 2048 * G
            per_group = (32 << 30) / span / groups
            tail = 0.5 / per_group if per_group >= 1 else None
            frac = FRAC_EXH * E_EXH / e
            res["designs"].append({
                "design": f"WC(G={G})", "lanes_per_chain": glines, "span_mib": span_mib,
                "staged_per_byte": round(tot[0] / covered, 4),
                "tested_per_byte": round(tot[1] / covered, 4),
                "warm_steps_per_byte": round(tot[2] / covered, 4),
                "merge_overrun_chunks_mean": round(float(np.mean(overs)), 3),
                "span_work_cv": round(float(works.std() / works.mean()), 4),
                "j_per_gib": round(e, 4),
                "frac_energy_bound": round(frac, 4),
                "spans_per_group_at_32gib": round(per_group, 2),
                "frac_with_tail": round(frac * (1 - tail), 4) if tail is not None else None})
    print(json.dumps(res))


if __name__ == "__main__":
    main()
