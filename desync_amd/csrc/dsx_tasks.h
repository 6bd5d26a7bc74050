// dsx_tasks.h -- the stitch as one-wave tasks ("stitch behind
// the scan"): walk tasks (walk_kernel's two phases for a few segments) and
// finish tasks (finish_kernel's rule, offsets and copy for a few segments).
// They run on scan wave slots that have no region to hash (scanl_kernel's
// FUSE variant) or in stitch_task_kernel, and never wait for each other: a
// walk task reads the region lists of an earlier scan, a finish task the
// SegInfo of an earlier walk.  Reference: make.go:277-327 (syncWith), the
// chain rule chunker.go:206-277.
#pragma once
#include <hip/hip_runtime.h>

#include "dsx_chain.h"
#include "dsx_common.h"
#include "dsx_stitch.h"

namespace dsx {

static_assert(sizeof(TaskSeg) == 32 && sizeof(SegInfo) == 32, "finish_task reads TaskSeg as 8 words");

__device__ __forceinline__ uint64_t wjob_seg_end(const WalkJob& j, uint32_t k) {
  return k + 1 >= j.nseg ? j.L : (uint64_t)(k + 1) * j.seg;
}

// Walk task t: segments kA..kB (kA-1's speculative chain redundantly, for its
// exit).  One wave; `cand` is the wave's own LDS (kTaskCand words).  Its global
// reads are few and issued together: under the scan's full HBM load every
// dependent round trip costs microseconds.
__device__ __attribute__((noinline)) void walk_task(const WalkJob& jr, uint32_t t, uint32_t wseg,
                                                   uint32_t* cand, uint32_t lane,
                                                   uint64_t* tm = nullptr) {
  const uint64_t tm0 = tm ? __builtin_amdgcn_s_memrealtime() : 0;
  // (a local copy: through the reference every field would be re-read from
  // memory after each store, the compiler cannot rule out aliasing)
  const WalkJob j = jr;
  const uint32_t kA = t * wseg;
  if (kA >= j.nseg) return;
  const uint32_t kB = (kA + wseg < j.nseg ? kA + wseg : j.nseg) - 1;
  const uint32_t kFirst = kA > 0 ? kA - 1 : 0;
  const uint64_t lo = (uint64_t)kFirst * j.seg;  // seg_start(kFirst): the chain starts at 0
  const uint64_t hi = wjob_seg_end(j, kB);
  const PieceCands& pc = j.pc;
  const uint32_t ovf = *(volatile const uint32_t*)pc.overflow;

  // ---- the candidates in (lo, hi], sorted, into LDS: per batch of 16
  // regions one round of loads (counts and the first 64 entries of each) ----
  const uint64_t r0 = lo <= pc.P ? 0 : pc_region_of(pc, lo - pc.P);
  uint64_t r1 = hi <= pc.P ? 0 : pc_region_of(pc, hi - pc.P - 1) + 1;  // exclusive
  if (r1 > pc.nregions) r1 = pc.nregions;
  const uint32_t nreg = r1 > r0 ? (uint32_t)(r1 - r0) : 0u;
  uint32_t total = 0;
  bool dense = false;
  constexpr int RBATCH = 16;
  for (uint32_t rb = 0; rb < nreg && !dense; rb += RBATCH) {
    const uint32_t nr = nreg - rb < (uint32_t)RBATCH ? nreg - rb : (uint32_t)RBATCH;
    const uint64_t rbase = r0 + rb;
    uint32_t cl = 0;
    if (lane < nr) cl = pc.region_cnt[rbase + lane];
    uint32_t e[RBATCH];
#pragma unroll
    for (int i = 0; i < RBATCH; ++i)  // (lists hold region_cap >= 64 entries)
      e[i] = (uint32_t)i < nr ? pc.region_list[(rbase + i) * pc.region_cap + lane] : 0u;
    if (ovf) return;  // finish publishes kErrDense
    cl = cl < pc.region_cap ? cl : pc.region_cap;
    uint32_t incl = cl;
#pragma unroll
    for (int d = 1; d < RBATCH; d <<= 1) {
      const uint32_t v = __shfl_up(incl, d, 64);
      if (lane >= (uint32_t)d) incl += v;
    }
    const uint32_t bt = (uint32_t)__builtin_amdgcn_readlane((int)incl, RBATCH - 1);
    if (total + bt > kTaskCand) {
      dense = true;
      break;
    }
    const uint32_t excl = incl - cl;
#pragma unroll
    for (int i = 0; i < RBATCH; ++i) {
      if ((uint32_t)i >= nr) continue;  // (not break: the loop stays unrolled)
      const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)cl, i);
      const uint32_t o = total + (uint32_t)__builtin_amdgcn_readlane((int)excl, i);
      const uint64_t rp = pc.P + pc_region_base(pc, rbase + i);
      auto put = [&](uint32_t idx, uint32_t ent) {
        const uint64_t p = rp + ent;
        cand[o + idx] = p <= lo ? 0u : (p > hi ? 0xFFFFFFFFu : (uint32_t)(p - lo));
      };
      if (lane < c) put(lane, e[i]);
      for (uint32_t g = 64 + lane; g < c; g += 64)  // (regions of more than 64: rare)
        put(g, pc.region_list[(rbase + i) * pc.region_cap + g]);
    }
    total += bt;
  }
  // (one wave: its LDS writes land before its reads below)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
  const uint64_t tm1 = tm ? __builtin_amdgcn_s_memrealtime() : 0;

  ChainParams cp;
  cp.min = j.min;
  cp.max = j.max;
  cp.L = j.L;
  cp.PE = j.L;
  cp.is_last = 1;
  cp.pad = 0;
  const RelChain rc = rel_chain(cp, lo);

  // ---- one chain per lane: lane i walks segment kFirst + i ----
  // (a wave walking one chain at a time spends ~300 ns per cut; the lanes of
  // one wave walk up to 64 segments' chains in about the time of one)
  const uint32_t nwalk = kB - kFirst + 1;  // <= 64 (wseg <= 63)
  const uint32_t i0 = kA - kFirst;         // lane 0 is kA-1's redundant walk when kA > 0
  const uint32_t k = kFirst + lane;
  const bool act = lane < nwalk;
  const bool own = act && lane >= i0;
  TaskSeg* ts = reinterpret_cast<TaskSeg*>(j.seg_info);
  if (dense) {
    if (own) {
      ts[k].X = kUndet;
      ts[k].Z = kUndet;
      ts[k].cnt = 0;
      ts[k].flags = kSegDense;  // forces the redo path
      ts[k].n2 = 0;
      ts[k].f1 = 0;
    }
    return;
  }
  // first candidate index > a (binary search over the staged list)
  auto lower = [&](uint32_t a) {
    uint32_t l = 0, h = total;
    while (l < h) {
      const uint32_t m = (l + h) >> 1;
      if (cand[m] <= a) l = m + 1; else h = m;
    }
    return l;
  };
  // next(s) of chunker.go:206-277 with a per-lane cursor into the list (the
  // chain only moves forward; this is the final piece: never undetermined)
  auto step = [&](uint32_t s, uint32_t& cur) -> uint32_t {
    if (s >= rc.tail_at) return rc.L;                  // chunker.go:215-217
    const uint32_t lim = min(s + rc.max, rc.lim_cap);  // chunker.go:221
    const uint32_t a = s + rc.min;
    while (cur < total && cand[cur] <= a) ++cur;       // chunker.go:259-271
    const uint32_t c = cur < total ? cand[cur] : 0xFFFFFFFFu;
    return c <= lim ? c : lim;                         // chunker.go:276
  };
  const uint64_t v = (uint64_t)k * j.seg;
  const uint32_t er = act ? rel_clamp(wjob_seg_end(j, k), lo) : 0u;
  const uint32_t sr = act ? rel_clamp(v, lo) : 0u;
  // ---- phase 1: the speculative chain from seg_start(k) -> S1 (spec), X_k ----
  uint64_t* s1 = j.spec + (uint64_t)k * j.scap;
  uint32_t ns = 0, why = 0, x1 = sr;
  if (act) {
    uint32_t cur = lower(sr);
    while (true) {
      if (x1 >= rc.end_at) { why = 1; break; }
      const uint32_t nx = step(x1, cur);
      if (nx > er) break;
      if (own && ns < j.scap) s1[ns] = lo + nx;
      ++ns;
      x1 = nx;
    }
  }
  const uint64_t X = lo + x1;
  // ---- phase 2: the chain entering from X_{k-1} -> P2 (stage), merged
  // with S1 where the two meet (two cursors: the one behind moves) ----
  const uint64_t xm1 = __shfl_up(X, 1, 64);
  if (own) {
  const uint64_t E = k == 0 ? 0ull : xm1;
  uint64_t* p2 = j.stage + (uint64_t)k * j.scap;
  uint32_t x = rel_clamp(E, lo), cx = lower(x);
  uint32_t y = sr, cy = lower(sr), fy = 0;  // y = S1[fy-1] (sr before any)
  uint32_t n2 = 0, flags = 0;
  bool merged = false;
  while (true) {
    if (x == y) { merged = true; break; }
    if (x < y || fy >= ns) {  // the P2 chain moves
      if (x >= rc.end_at) { flags |= kSegEnd; break; }
      const uint32_t nx = step(x, cx);
      if (nx > er) break;
      if (nx > sr) {
        if (n2 < j.scap) p2[n2] = lo + nx;
        ++n2;
      }
      x = nx;
    } else {                  // the S1 chain moves (its cuts are recomputed)
      y = step(y, cy);
      ++fy;
    }
  }
  const uint32_t f1 = merged ? fy : ns;  // S1[f1..ns) follows P2
  if (merged && why == 1) flags |= kSegEnd;
  if (ns > j.scap || n2 > j.scap || n2 + (ns - f1) > j.scap) flags |= kSegOverflow;
  ts[k].X = X;
  ts[k].Z = ns > f1 ? X : lo + x;
  ts[k].cnt = n2 + (ns - f1);
  ts[k].flags = flags;
  ts[k].n2 = n2;
  ts[k].f1 = f1;
  }
  if (tm) {
    tm[0] += tm1 - tm0;
    tm[1] += __builtin_amdgcn_s_memrealtime() - tm1;
  }
}

// Finish task t: segments kb..ke-1 (fseg <= 32).  Every task checks the rule
// over all the segments (no suspect segment: flagged, or X_k != Z_k before
// the last), sums the counts before kb and copies its segments' lists (P2
// from stage, then S1's tail from spec) to the cut list; the last task to
// arrive publishes the call's state.  Two rounds of loads (the TaskSeg words,
// then the lists), then the stores.  A suspect segment or an overflowed scan
// publishes kErrRedo / kErrDense: the host redoes the call on the general
// path (fixup_kernel's repair), as rare as fixup's repairs.
__device__ __attribute__((noinline)) void finish_task(const FinishJob& fr, uint32_t t, uint32_t fseg,
                                                     uint32_t nf, uint32_t* farrive, uint32_t lane) {
  const FinishJob f = fr;  // (local copy, as in walk_task)
  constexpr uint32_t kBad = kSegDense | kSegOverflow;
  constexpr int QS = 16;  // SegInfo per lane per round (T <= 1024: one round)
  constexpr int QF = 32;  // segments per task, at most
  const uint32_t T = f.nseg;
  const uint32_t kb = t * fseg;
  const uint32_t ke = kb + fseg < T ? kb + fseg : T;
  const uint32_t nown = ke - kb;
  const uint32_t* sw = reinterpret_cast<const uint32_t*>(f.seg_info);  // 8 words per TaskSeg
  // round 1: this task's segments' {cnt, n2, f1} (lane q), every segment's rule words
  uint32_t myc = 0, myn = 0, myf = 0;
  if (lane < nown) {
    myc = sw[8 * (kb + lane) + 4];
    myn = sw[8 * (kb + lane) + 6];
    myf = sw[8 * (kb + lane) + 7];
  }
  const uint32_t ovf = *(volatile const uint32_t*)f.overflow;
  uint64_t before = 0, total = 0;
  int lastk = -1;
  bool bad = false;
  for (uint32_t k0 = 0; k0 < T; k0 += 64u * QS) {
    uint32_t xl[QS], zl[QS], cn[QS], fl[QS];
#pragma unroll
    for (int i = 0; i < QS; ++i) {
      const uint32_t k = k0 + 64u * i + lane;
      xl[i] = zl[i] = cn[i] = fl[i] = 0;
      if (k < T) {  // low words of X and Z (both in segment k: equal iff the low words are)
        xl[i] = sw[8 * k + 0];
        zl[i] = sw[8 * k + 2];
        cn[i] = sw[8 * k + 4];
        fl[i] = sw[8 * k + 5];
      }
    }
#pragma unroll
    for (int i = 0; i < QS; ++i) {
      const uint32_t k = k0 + 64u * i + lane;
      if (k < T) {
        bad = bad || (fl[i] & kBad) != 0 || (k + 1 < T && xl[i] != zl[i]);
        total += cn[i];
        before += k < kb ? cn[i] : 0u;
        if (cn[i]) lastk = (int)k;
      }
    }
  }
  // round 2: each own segment's list, lane t = cut t: P2 (stage) then S1's
  // tail from f1 (spec), the first 64 cuts at once
  uint64_t v[QF];
#pragma unroll
  for (int q = 0; q < QF; ++q) {
    v[q] = 0;
    if ((uint32_t)q < nown) {
      const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)myc, q);
      const uint32_t n2 = (uint32_t)__builtin_amdgcn_readlane((int)myn, q);
      const uint32_t f1 = (uint32_t)__builtin_amdgcn_readlane((int)myf, q);
      const uint64_t base = (uint64_t)(kb + q) * f.scap;
      // (indices below scap even for a flagged segment, whose lists are not copied)
      const uint32_t si = f1 + (lane - n2);
      if (lane < c && lane < f.scap && (lane < n2 || si < f.scap))
        v[q] = lane < n2 ? f.stage[base + lane] : f.spec[base + si];
    }
  }
  const bool any_bad = __ballot(bad) != 0;
  int mk = lastk;
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    total += __shfl_xor(total, d, 64);
    before += __shfl_xor(before, d, 64);
    const int o = __shfl_xor(mk, d, 64);
    mk = o > mk ? o : mk;
  }
  const bool fits = total <= f.out_cap;
  if (!ovf && !any_bad && fits) {
    uint32_t incl = myc;  // offsets of this task's segments
#pragma unroll
    for (int d = 1; d < QF; d <<= 1) {
      const uint32_t o = __shfl_up(incl, d, 64);
      if (lane >= (uint32_t)d) incl += o;
    }
    const uint32_t excl = incl - myc;
#pragma unroll
    for (int q = 0; q < QF; ++q) {
      if ((uint32_t)q >= nown) continue;  // (not break: the loop stays unrolled)
      const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)myc, q);
      const uint64_t off = before + (uint32_t)__builtin_amdgcn_readlane((int)excl, q);
      if (lane < c) f.out[off + lane] = v[q];
      if (c > 64) {  // (more than 64 cuts: rare)
        const uint32_t n2 = (uint32_t)__builtin_amdgcn_readlane((int)myn, q);
        const uint32_t f1 = (uint32_t)__builtin_amdgcn_readlane((int)myf, q);
        const uint64_t base = (uint64_t)(kb + q) * f.scap;
        for (uint32_t i = 64 + lane; i < c; i += 64)
          f.out[off + i] = i < n2 ? f.stage[base + i] : f.spec[base + f1 + (i - n2)];
      }
    }
  }
  __threadfence();  // this task's cuts before its arrival
  uint32_t n = 0;
  if (lane == 0) n = atomicAdd(farrive, 1u);
  n = __builtin_amdgcn_readfirstlane(n);
  if (n + 1 == nf && lane == 0) {
    atomicExch(farrive, 0u);
    __threadfence();  // every task's cuts are written
    volatile HostState* h = f.host_state;
    h->carry = mk >= 0 ? reinterpret_cast<const TaskSeg*>(f.seg_info)[mk].Z : 0ull;  // the last cut
    h->total = (!ovf && !any_bad) ? total : 0ull;
    h->repaired = 0;
    h->discarded = 0;
    h->done = 1;
    h->err = (ovf ? kErrDense : 0u) | (!ovf && any_bad ? kErrRedo : 0u) |
             (!ovf && !any_bad && !fits ? kErrCapacity : 0u);
    __threadfence_system();
    h->seq = f.seq;
  }
}

// A wave's share of the tasks: tickets from the counter until none is left.
// (walk_task / finish_task are calls: inlined, their registers would count
// against the scan's allocation and spill in its loop)
// trace (DSX_SCAN_TRACE, may be null): {first ticket, last task end,
// tasks run | finish tasks << 16} of this wave, s_memrealtime ticks
__device__ __forceinline__ void run_tasks(const TaskArgs* bp, uint32_t* cand, uint32_t lane,
                                          uint64_t* trace = nullptr) {
  // The arguments are copied from the pinned ring once: read in place, every
  // field a task uses would be a dependent round trip to host memory.
  if (bp->nf + bp->nw == 0) return;
  TaskArgs b;
  {
    constexpr int NW = (int)(sizeof(TaskArgs) / 8);
    static_assert(sizeof(TaskArgs) % 8 == 0, "TaskArgs copy");
    const uint64_t* src = reinterpret_cast<const uint64_t*>(bp);
    uint64_t* dst = reinterpret_cast<uint64_t*>(&b);
    uint64_t tmp[NW];
#pragma unroll
    for (int i = 0; i < NW; ++i) tmp[i] = src[i];  // one round of loads
#pragma unroll
    for (int i = 0; i < NW; ++i) dst[i] = tmp[i];
  }
  const uint32_t ntask = b.nf + b.nw;
  const uint64_t t0 = trace ? __builtin_amdgcn_s_memrealtime() : 0;
  uint32_t nrun = 0, nfin = 0;
  uint64_t tm[3] = {0, 0, 0};  // trace: staging, walking, finishing ticks
  // the tasks are latency-bound chains: issue them first whenever they are
  // ready (priority 0 measured the same)
  __builtin_amdgcn_s_setprio(3);
  while (true) {
    uint32_t t = 0;
    if (lane == 0) t = atomicAdd(b.counter, 1u);
    t = __builtin_amdgcn_readfirstlane(t);
    if (t >= ntask) break;
    if (t < b.nf) {
      const uint64_t f0 = trace ? __builtin_amdgcn_s_memrealtime() : 0;
      finish_task(b.f, t, b.fseg, b.nf, b.farrive, lane);
      if (trace) tm[2] += __builtin_amdgcn_s_memrealtime() - f0;
    } else {
      walk_task(b.w, t - b.nf, b.wseg, cand, lane, trace ? tm : nullptr);
    }
    ++nrun;
    nfin += t < b.nf ? 1u : 0u;
  }
  if (trace && lane == 0) {
    trace[0] = t0;
    trace[1] = __builtin_amdgcn_s_memrealtime();
    trace[2] = nrun | (nfin << 16);
    trace[3] = tm[0];
    trace[4] = tm[1];
    trace[5] = tm[2];
  }
}

}  // namespace dsx
