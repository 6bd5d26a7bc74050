// dsx_stitch.hip -- candidates -> cut chain, on the GPU.
//
// Reference semantics: the sequential chain of Chunker.Next()
// (chunker.go:206-277): from a cut s the next cut is the tail end if
// len-s <= min, else the first candidate in (s+min, s+min(len-s,max)], else
// s+min(len-s,max).  make.go:22-163 parallelises this by starting workers at
// span*i and aligning each with its successor (syncWith, make.go:277-327);
// the result equals the sequential chain (make_test.go:16-80).
//
// GPU form of that split-and-align (DESIGN.md "Stitch"):
//   segments  [seg_start(k), seg_end(k)) of SEG bytes; segment 0 starts at the
//             true carried cut s0, segment k>0 at a virtual cut (make.go's
//             worker start).
//   K2 walk   per segment k (one lane each, candidates staged in LDS):
//             X_k  = exit of the speculative chain started at seg_start(k)
//                    (the last cut <= seg_end(k));
//             staged(k) = cuts in (seg_start(k), seg_end(k)] of the chain that
//                    enters from X_{k-1} (spec chain of the previous segment);
//             Z_k  = last cut of staged(k).
//             staged(k+1) is the true chain iff staged(k) is and X_k == Z_k
//             (the two chains met inside segment k -- syncWith's test).
//   K3 fixup  one workgroup: repairs the rare segments where X_k != Z_k by a
//             sequential walk over global candidates until it rejoins the
//             staged chain, then an exclusive scan of per-segment counts.
//   K4 gather contiguous cut list.
#include <hip/hip_runtime.h>

#include "dsx_chain.h"
#include "dsx_common.h"
#include "dsx_stitch.h"
#if DSX_DIAG  // the stitch behind the scan (DSX_FUSE): libdsx_diag.so only
#include "dsx_tasks.h"
#endif

namespace dsx {

// ---- candidate sources -----------------------------------------------------
// Sorted candidates in LDS, positions lo + c[i].  first_in(a, b) returns the
// first candidate in (a, b] or kNone; `a` must be non-decreasing across calls.
struct LdsSrc {
  const uint32_t* c;
  uint32_t n;
  uint32_t j;
  uint64_t lo;
  __device__ uint64_t first_in(uint64_t a, uint64_t b) {
    const uint64_t ar = a - lo;  // a >= lo always (a = s+min, s >= lo)
    while (j < n && (uint64_t)c[j] <= ar) ++j;
    if (j < n) {
      // (the builtin returns int: keep the u32 offset from sign-extending)
      const uint64_t p = lo + (uint32_t)__builtin_amdgcn_readfirstlane(c[j]);
      if (p <= b) return p;
    }
    return kNone;
  }
  // reset j to the first candidate > a (binary search)
  __device__ void seek(uint64_t a) {
    const uint64_t ar = a < lo ? 0 : a - lo;
    uint32_t l = 0, h = n;
    while (l < h) {
      const uint32_t m = (l + h) >> 1;
      if ((uint64_t)c[m] <= ar) l = m + 1; else h = m;
    }
    j = l;
  }
};

// Candidates straight from the scan's per-region sorted lists (global
// memory); used by the sequential repair only.
struct GlobalSrc {
  const PieceCands* pc;
  __device__ uint64_t first_in(uint64_t a, uint64_t b) const {
    if (b <= pc->P) return kNone;
    const uint64_t pos = a < pc->P ? pc->P : a;
    for (uint64_t r = pc_region_of(*pc, pos - pc->P); r < pc->nregions; ++r) {
      const uint64_t base = pc->P + pc_region_base(*pc, r);  // region covers (base, base + bytes]
      if (base >= b) break;
      const uint32_t cnt = pc->region_cnt[r];
      const uint32_t n = cnt < pc->region_cap ? cnt : pc->region_cap;
      const uint32_t* l = pc->region_list + r * (uint64_t)pc->region_cap;
      const uint64_t ar = a > base ? a - base : 0;  // want entry > ar
      uint32_t lo = 0, hi = n;
      while (lo < hi) {
        const uint32_t m = (lo + hi) >> 1;
        if ((uint64_t)l[m] <= ar) lo = m + 1; else hi = m;
      }
      if (lo < n) {
        const uint64_t p = base + l[lo];
        return p <= b ? p : kNone;
      }
    }
    return kNone;
  }
};

// One step of the chain rule.  Returns the next cut, or kUndet if it depends
// on bytes beyond the piece end (non-final piece).
template <class Src>
__device__ __forceinline__ uint64_t next_cut(uint64_t s, Src& src, const ChainParams& w) {
  uint64_t lim;
  if (w.is_last) {
    if (w.L - s <= w.min) return w.L;  // chunker.go:215-217
    lim = s + w.max < w.L ? s + w.max : w.L;  // chunker.go:221
  } else {
    lim = s + w.max;
  }
  const uint64_t c = src.first_in(s + w.min, lim);  // chunker.go:259-271
  if (c != kNone) return c;
  if (!w.is_last && lim > w.PE) return kUndet;
  return lim;  // chunker.go:276
}

// ---- K2: per-segment speculative walks ------------------------------------
constexpr uint32_t kWalkMaxRegions = 4096;  // regions a walk workgroup can stage

// Block-wide exclusive scan of one value per thread (NT threads); returns the
// exclusive prefix, *total gets the block sum.
template <int NT>
__device__ uint32_t walk_block_scan(uint32_t v, uint32_t* s_wave, uint32_t* total) {
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t incl = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t t = __shfl_up(incl, d, 64);
    if (lane >= (uint32_t)d) incl += t;
  }
  if (lane == 63) s_wave[wv] = incl;
  __syncthreads();
  uint32_t before = 0, all = 0;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) {
    const uint32_t t = s_wave[i];
    before += (i < (int)wv) ? t : 0u;
    all += t;
  }
  __syncthreads();
  *total = all;
  return before + incl - v;
}

// NT = 576 threads for 8 segments per workgroup (an 8 GiB piece: every chain
// its own wave, so phase 1 is one chain long), 256 otherwise, or 1024 (split
// streams: a few workgroups beside the next piece's scan, on the CUs it leaves
// free, each wave walking several segments)
template <int NT>
__global__ __launch_bounds__(NT) void walk_kernel(StitchArgs a) {
  constexpr int kWalkThreads = NT;
  extern __shared__ __attribute__((aligned(16))) uint32_t smem[];
  uint32_t* cand = smem;                         // [a.lds_cap]
  uint64_t* xs = (uint64_t*)(smem + a.lds_cap);  // [kMaxSpg + 1] spec exits
  __shared__ uint32_t s_off[kWalkMaxRegions + 1];
  __shared__ uint32_t s_wave[kWalkThreads / 64];
  // phase 1's speculative chains (relative cuts), so phase 2 can stop as soon
  // as its chain meets them: the rest of the staged chain is the same cuts
  constexpr uint32_t kSpecLds = 4096;
  __shared__ uint32_t s_spec[kSpecLds];
  __shared__ uint32_t s_spec_n[kMaxSpg + 1];    // cuts recorded (capped at scap)
  __shared__ uint32_t s_spec_end[kMaxSpg + 1];  // 0: left the segment, 1: reached L, 2: undetermined

  uint64_t* tr = (a.trace && threadIdx.x == 0) ? a.trace + 10ull * blockIdx.x : nullptr;
  if (tr) tr[0] = __builtin_amdgcn_s_memrealtime();
  DevState* st = a.state;
  // the first piece of a call starts the chain at init_carry: the state is
  // reset here (block 0) and every workgroup uses the initial values, so no
  // kernel of another stream (the next piece's scan) touches the state
  const bool init = a.init != 0;
  const uint32_t done0 = init ? 0u : st->done;
  if (blockIdx.x == 0 && threadIdx.x == 0) {  // for finish_kernel
    if (init) {
      st->carry = a.init_carry;
      st->total = 0;
      st->piece_cuts = 0;
      st->repaired = 0;
      st->discarded = 0;
      st->done = 0;
      st->err = 0;
      st->active = 0;
    }
    st->base = init ? 0ull : st->total;
    st->skip = (done0 || *a.pc.overflow) ? 1u : 0u;
  }
  if (done0 || *a.pc.overflow) return;  // finished, or scan lists overflowed
  const uint64_t s0 = init ? a.init_carry : uniform64(st->carry);  // scalar: wave-uniform walks
  const uint32_t kA = blockIdx.x * a.spg;
  if (kA >= a.nseg) return;
  const uint32_t kB = (kA + a.spg < a.nseg ? kA + a.spg : a.nseg) - 1;  // inclusive
  const uint32_t kFirst = kA > 0 ? kA - 1 : 0;                             // redundant walk
  const uint64_t lo = seg_start(a, s0, kFirst);
  const uint64_t hi = seg_end(a, kB);
  const PieceCands& pc = a.pc;

  // ---- gather candidates in (lo, hi] into LDS, sorted (region order) ----
  const uint64_t r0 = lo <= pc.P ? 0 : pc_region_of(pc, lo - pc.P);
  uint64_t r1 = hi <= pc.P ? 0 : pc_region_of(pc, hi - pc.P - 1) + 1;  // exclusive
  if (r1 > pc.nregions) r1 = pc.nregions;
  const uint32_t nreg = r1 > r0 ? (uint32_t)(r1 - r0) : 0u;
  bool dense = nreg > kWalkMaxRegions;
  uint32_t total = 0;
  if (!dense) {
    // region counts -> exclusive offsets s_off[0..nreg]
    for (uint32_t b = 0; b < nreg; b += kWalkThreads) {
      const uint32_t i = b + threadIdx.x;
      uint32_t c = 0;
      if (i < nreg) {
        c = pc.region_cnt[r0 + i];
        c = c < pc.region_cap ? c : pc.region_cap;
      }
      uint32_t part;
      const uint32_t ex = walk_block_scan<NT>(c, s_wave, &part);
      if (i < nreg) s_off[i] = total + ex;
      total += part;
    }
    if (threadIdx.x == 0) s_off[nreg] = total;
    __syncthreads();
    dense = total > a.lds_cap;
  }
  if (tr) tr[1] = __builtin_amdgcn_s_memrealtime();
  if (!dense) {
    // one candidate per thread: find its region by binary search over s_off
    for (uint32_t g = threadIdx.x; g < total; g += kWalkThreads) {
      uint32_t l = 0, h = nreg;  // last r with s_off[r] <= g
      while (h - l > 1) {
        const uint32_t m = (l + h) >> 1;
        if (s_off[m] <= g) l = m; else h = m;
      }
      const uint64_t r = r0 + l;
      const uint64_t p = pc.P + pc_region_base(pc, r) +
                         pc.region_list[r * (uint64_t)pc.region_cap + (g - s_off[l])];
      // keep the array sorted: below-range -> 0, above-range -> UINT32_MAX
      cand[g] = p <= lo ? 0u : (p > hi ? 0xFFFFFFFFu : (uint32_t)(p - lo));
    }
  }
  __syncthreads();
  if (tr) {
    tr[2] = __builtin_amdgcn_s_memrealtime();
    tr[5] = __builtin_amdgcn_s_memtime();
  }

  const uint32_t nwalk = kB - kFirst + 1;
  const RelChain rc = rel_chain(a.chain, lo);
  // LDS slots per recorded speculative chain (a chain longer than that is not
  // recorded: phase 2 then walks its segment in full)
  const uint32_t stride = min(a.scap, kSpecLds / nwalk);
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), ln = threadIdx.x & 63;
  constexpr uint32_t kWaves = kWalkThreads / 64;
  // ---- phase 1: speculative chain of each segment -> exit X_k (one wave each) ----
  // A chain step is a ballot over the 64 candidates the wave holds in a
  // register, s_ff1 and a readlane; the chain's cuts are bits of a scalar
  // mask over the window's lanes and go to LDS once per window, so no step
  // waits on LDS (each step's LDS store used to cost an lgkmcnt(0) wait).
  // Chains of any length up to the LDS slots are recorded (avg 16 KiB: ~128
  // cuts per 2 MiB segment).
  // (One lane per chain, a cursor into the LDS candidates, was slower: 37.1
  // against 31.4 us per 8 GiB piece, its steps wait on dependent LDS reads;
  // profiles/r04r.)
  if (!dense) {
    for (uint32_t t = wv; t < nwalk; t += kWaves) {
      const uint32_t k = kFirst + t;
      const uint64_t v = seg_start(a, s0, k);
      const uint64_t e = seg_end(a, k);
      WaveLdsSrc src{cand, total, 0, lo, ln, 0};
      src.seek(v);
      if (tr && t == wv) tr[7] = __builtin_amdgcn_s_memrealtime();
      const uint32_t er = rel_clamp(e, lo);
      uint32_t x = rel_clamp(v, lo);
      uint32_t ns = 0, why = 0;
      uint32_t* spec_t = s_spec + t * stride;
      // The common step's bound: chunker.go:221's limit, the segment end, and
      // below the last piece's tail (chunker.go:215-217), so a common step
      // never needs the tail test.
      const uint32_t cap = __builtin_amdgcn_readfirstlane(rc.tail_at ? min(min(rc.lim_cap, er), rc.tail_at - 1u) : 0u);
      // window lanes cut since the last flush: a common step records its cut
      // with one scalar bit-set; the cuts reach LDS once per window, in order
      uint64_t cm = 0;
      auto flush = [&]() __attribute__((always_inline)) {
        if (cm) {
          const uint32_t idx = ns + __builtin_amdgcn_mbcnt_hi((uint32_t)(cm >> 32),
                                                             __builtin_amdgcn_mbcnt_lo((uint32_t)cm, 0u));
          if (((cm >> ln) & 1u) && idx < stride) spec_t[idx] = src.v;
          ns += (uint32_t)__builtin_popcountll(cm);
          cm = 0;
        }
      };
      while (true) {
        // The common step, with one exit for everything else: the next
        // candidate in the register window past x + min is the next cut
        // (chunker.go:259-271) when it lies within x + max and below `cap`
        // (round 5: ballot, s_ff1, readlane, one compare and a bit-set;
        // DESIGN.md 4.2)
        if (x < rc.tail_at) {
          uint64_t m = __ballot(src.v > x + rc.min);
          // while (m != 0) {  (m == 0: window exhausted, rel_step refills)
          //   l = ctz(m); c = v[l]; if (c > min(x + max, cap)) break;
          //   cm |= 1 << l; x = c; m = ballot(v > x + min); }
          // by hand: the compiler's form of this loop takes 18 instructions
          // a step (a select and a vcc copy per exit test), these 13; the
          // steps of all the CU's walking waves share its scalar unit
          uint32_t l, c, lim, xm;
          asm volatile(
              "L_walk_step_%=:\n\t"
              "s_cmp_eq_u64 %[m], 0\n\t"
              "s_cbranch_scc1 L_walk_out_%=\n\t"
              "s_ff1_i32_b64 %[l], %[m]\n\t"
              "s_add_u32 %[lim], %[x], %[mx]\n\t"
              "v_readlane_b32 %[c], %[v], %[l]\n\t"
              "s_min_u32 %[lim], %[lim], %[cap]\n\t"
              "s_cmp_gt_u32 %[c], %[lim]\n\t"
              "s_cbranch_scc1 L_walk_out_%=\n\t"
              "s_bitset1_b64 %[cm], %[l]\n\t"
              "s_add_u32 %[xm], %[c], %[mn]\n\t"
              "s_mov_b32 %[x], %[c]\n\t"
              "v_cmp_lt_u32_e64 %[m], %[xm], %[v]\n\t"
              "s_branch L_walk_step_%=\n"
              "L_walk_out_%=:"
              : [m] "+s"(m), [x] "+s"(x), [cm] "+s"(cm), [l] "=&s"(l), [c] "=&s"(c),
                [lim] "=&s"(lim), [xm] "=&s"(xm)
              : [v] "v"(src.v), [mx] "s"(rc.max), [mn] "s"(rc.min), [cap] "s"(cap)
              : "scc");
        }
        flush();  // (before rel_step moves the window)
        uint32_t nx;
        if (__builtin_expect(x >= rc.tail_at, 0)) {  // (tail_at <= end_at)
          if (x >= rc.end_at) { why = 1; break; }
          nx = rc.L;                                   // chunker.go:215-217
        } else {
          nx = rel_step(x, src, rc);
        }
        if (__builtin_expect(nx > er, 0)) {  // (kRelUndet > er)
          if (nx == kRelUndet) why = 2;
          break;
        }
        if (ln == 0 && ns < stride) spec_t[ns] = nx;  // a rare step's cut
        ++ns;
        x = nx;
      }
      if (tr && t == wv) tr[9] = __builtin_amdgcn_s_memrealtime();
      // (more cuts than the chain's LDS slots: no phase-2 shortcut)
      const bool keep = ns <= stride;
      if (ln == 0) {
        xs[t] = lo + x;
        s_spec_n[t] = keep ? ns : 0xFFFFFFFFu;
        s_spec_end[t] = why;
        if (k >= kA) a.seg_info[k].X = lo + x;  // kA-1 belongs to the previous workgroup
      }
    }
  }
  __syncthreads();
  if (tr) {
    tr[3] = __builtin_amdgcn_s_memrealtime();
    uint32_t xcc, hwid;  // where this workgroup ran (XCC, SE/SH/CU)
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
    tr[6] = ((uint64_t)xcc << 32) | hwid;
  }

  // ---- phase 2: staged chain entering from X_{k-1} (one wave each) ----
  for (uint32_t i = wv; i < kB - kA + 1; i += kWaves) {
    const uint32_t k = kA + i;
    const uint32_t t = i + (kA - kFirst);
    SegInfo& si = a.seg_info[k];
    if (dense) {
      if (ln == 0) {
        si.E = kUndet;
        si.Z = kUndet;
        si.X = kUndet;  // forces the repair of this and the next segment
        si.cnt = 0;
        si.flags = kSegDense;
      }
      continue;
    }
    const uint64_t E = (k == 0) ? s0 : uniform64(xs[t - 1]);
    const uint64_t sst = seg_start(a, s0, k);
    const uint64_t e = seg_end(a, k);
    WaveLdsSrc src{cand, total, 0, lo, ln, 0};
    src.seek(E);
    uint64_t* out = a.stage + (uint64_t)k * a.scap;
    uint32_t n = 0, flags = 0;
    const uint32_t er = rel_clamp(e, lo), sr = rel_clamp(sst, lo);
    uint32_t x = rel_clamp(E, lo), last = x;
    // the speculative chain of this segment (phase 1): its first 64 cuts, one
    // per lane (the chains meet within the first few cuts, or not at all)
    const uint32_t sn = s_spec_n[t];
    const bool have_spec = sn != 0xFFFFFFFFu;
    const uint32_t* spec = s_spec + t * stride;
    const uint32_t specv = have_spec && ln < sn ? spec[ln] : 0xFFFFFFFFu;
    while (true) {
      uint32_t nx;
      if (__builtin_expect(x >= rc.tail_at, 0)) {  // (tail_at <= end_at)
        if (x >= rc.end_at) { flags |= kSegEnd; break; }
        nx = rc.L;                                   // chunker.go:215-217
      } else {
        nx = rel_step(x, src, rc);
      }
      if (__builtin_expect(nx > er, 0)) {  // (kRelUndet > er)
        if (nx == kRelUndet) flags |= kSegUndet;
        break;
      }
      if (nx > sr) {
        if (ln == (n & 63u) && n < a.scap) out[n] = lo + nx;  // spread the stores over lanes
        ++n;
      }
      last = nx;
      x = nx;
      if (have_spec) {
        const uint64_t hit = __ballot(specv == nx);
        if (hit) {
          // met the speculative chain (all its cuts are > sst): the staged
          // chain continues with its cuts and ends the way it ended
          const uint32_t f = (uint32_t)__builtin_ctzll(hit);
          const uint32_t rest = sn - f - 1;
          for (uint32_t j = f + 1u + ln; j < sn; j += 64u)
            if (n + (j - f - 1u) < a.scap) out[n + (j - f - 1u)] = lo + spec[j];
          n += rest;
          if (rest) last = spec[sn - 1u];
          if (s_spec_end[t] == 1) flags |= kSegEnd;
          if (s_spec_end[t] == 2) flags |= kSegUndet;
          break;
        }
      }
    }
    if (n > a.scap) flags |= kSegOverflow;
    if (ln == 0) {
      si.E = E;
      si.Z = lo + last;
      si.cnt = n;
      si.flags = flags;
    }
  }
  if (a.trace) {
    __syncthreads();
    if (tr) tr[4] = __builtin_amdgcn_s_memrealtime();
  }
}

template __global__ void walk_kernel<256>(StitchArgs);
template __global__ void walk_kernel<1024>(StitchArgs);
template __global__ void walk_kernel<576>(StitchArgs);

// ---- K3: validity propagation, sequential repair, scan of counts ----------
constexpr int kFixThreads = 1024;

// Mirror the chain state into pinned host memory (the host reads it after the
// stream synchronises, no D2H copy needed).
__device__ void publish(const StitchArgs& a, const DevState* st) {
  if (!a.host_state) return;
  publish_state(a.host_state, st, a.seq);
}

// The piece's chain state into the pinned host slot, after the stitch's last
// kernel (a kernel boundary: every cut is written).  Cheaper than a
// last-arriving workgroup in finish_kernel, whose 64 device-scope releases
// cost 4 us (13.0 against 8.8 us, rocprofv3), and than an event record
// (~6 us of idle stream).
__global__ void publish_kernel(StitchArgs a) {
  if (threadIdx.x == 0 && blockIdx.x == 0) publish(a, a.state);
}

// (diagnostic: an empty kernel, to locate launch gaps in a kernel trace)
__global__ void noop_kernel() {}

__device__ uint32_t bsearch_u64(const uint64_t* v, uint32_t n, uint64_t x) {
  uint32_t l = 0, h = n;
  while (l < h) {
    const uint32_t m = (l + h) >> 1;
    if (v[m] < x) l = m + 1; else h = m;
  }
  return l;
}

// K3's body for a workgroup of NT threads (fixup_kernel, and the repair path
// of fixup_fast_kernel).
template <int NT>
__device__ void fixup_body(const StitchArgs& a, bool do_publish = true) {
  __shared__ uint32_t s_flag_cnt;
  __shared__ uint64_t s_part[NT / 64];
  __shared__ int s_last_seg;
  __shared__ uint64_t s_carry, s_total0;
  DevState* st = a.state;
  if (threadIdx.x == 0) s_total0 = st->total;
  if (st->done || *a.pc.overflow) {
    if (threadIdx.x == 0) {
      st->active = 0;
      st->piece_cuts = 0;
      if (*a.pc.overflow) st->err |= kErrDense;
      if (do_publish) publish(a, st);
    }
    return;
  }
  const uint32_t T = a.nseg;
  const uint32_t kBad = kSegDense | kSegOverflow;

  // (1) suspect segments: staged(k) was built from X_{k-1}; it is the true
  //     chain iff staged(k-1) is and ended on X_{k-1} (Z_{k-1} == X_{k-1}).
  if (threadIdx.x == 0) s_flag_cnt = 0;
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < T; k += NT) {
    const SegInfo& si = a.seg_info[k];
    bool bad = (si.flags & kBad) != 0;
    if (k > 0) {
      const SegInfo& sp = a.seg_info[k - 1];
      bad = bad || (sp.X != sp.Z) || (sp.flags & kBad);
    }
    a.rep_cnt[k] = 0;
    a.rep_from[k] = 0;
    if (bad) a.flag_list[atomicAdd(&s_flag_cnt, 1u)] = k;
  }
  __syncthreads();
  const uint32_t nflag = s_flag_cnt;

  // (2) sequential repair, visiting only suspect segments and the segments a
  //     repair runs into, until the true chain rejoins a staged chain.
  if (nflag > 0 && threadIdx.x == 0) {
    for (uint32_t i = 1; i < nflag; ++i) {  // insertion sort: the list is small
      const uint32_t v = a.flag_list[i];
      uint32_t j = i;
      while (j > 0 && a.flag_list[j - 1] > v) { a.flag_list[j] = a.flag_list[j - 1]; --j; }
      a.flag_list[j] = v;
    }
    GlobalSrc src{&a.pc};
    const uint64_t s0 = st->carry;
    uint32_t fi = 0, repaired = 0;
    uint64_t discarded = 0;  // staged cuts the repairs replaced
    uint32_t k = a.flag_list[0];
    bool rp = false;  // was segment k-1 repaired?
    uint64_t rex = 0; // its repaired exit
    while (k < T) {
      const SegInfo& si = a.seg_info[k];
      const uint64_t te = (k == 0) ? s0 : (rp ? rex : a.seg_info[k - 1].Z);
      if ((si.flags & kBad) == 0 && si.E == te) {
        // staged(k) entered from the true exit: valid; jump to next suspect
        rp = false;
        while (fi < nflag && a.flag_list[fi] <= k) ++fi;
        if (fi >= nflag) break;
        k = a.flag_list[fi];
        continue;
      }
      // repair segment k from te until it lands on a staged cut
      const uint64_t sst = (k == 0) ? s0 : a.anchor + (uint64_t)k * a.seg;
      const uint64_t e = seg_end(a, k);
      const uint64_t* stg = a.stage + (uint64_t)k * a.scap;
      const uint32_t scnt = (si.flags & kBad) ? 0u : si.cnt;
      uint64_t* rep = a.rep + (uint64_t)k * a.scap;
      uint32_t n = 0;
      uint64_t x = te, last = te;
      bool joined = false;
      while (true) {
        if (a.chain.is_last && x >= a.chain.L) break;
        const uint64_t nx = next_cut(x, src, a.chain);
        if (nx == kUndet || nx > e) break;
        if (nx > sst) {
          const uint32_t idx = bsearch_u64(stg, scnt, nx);
          if (idx < scnt && stg[idx] == nx) {
            joined = true;
            a.rep_from[k] = idx;
            break;
          }
          if (n < a.scap) rep[n] = nx;
          ++n;
        }
        last = nx;
        x = nx;
      }
      if (n > a.scap) st->err |= kErrCapacity;
      a.rep_cnt[k] = n;
      if (!joined) a.rep_from[k] = scnt;
      discarded += a.rep_from[k];
      ++repaired;
      rp = true;
      rex = joined ? si.Z : last;
      ++k;
    }
    st->repaired += repaired;
    st->discarded += discarded;
  }
  __syncthreads();

  // (3) per-segment final counts -> exclusive block scan -> output offsets
  const uint32_t per = (T + NT - 1) / NT;
  const uint32_t k0 = threadIdx.x * per < T ? threadIdx.x * per : T;
  const uint32_t k1 = (k0 + per < T) ? k0 + per : T;
  uint64_t mine = 0;
  int last_nonempty = -1;
  uint64_t my_last = 0;  // last cut of this thread's last non-empty segment
  for (uint32_t k = k0; k < k1; ++k) {
    const SegInfo& si = a.seg_info[k];
    const uint32_t scnt = (si.flags & kBad) ? 0u : si.cnt;
    const uint32_t rc = a.rep_cnt[k], rf = a.rep_from[k];
    const uint64_t c = (uint64_t)rc + (scnt - rf);
    mine += c;
    if (c > 0) {
      last_nonempty = (int)k;
      my_last = scnt > rf ? a.stage[(uint64_t)k * a.scap + scnt - 1]
                          : a.rep[(uint64_t)k * a.scap + rc - 1];
    }
  }
  if (threadIdx.x == 0) s_last_seg = -1;
  // wave-level inclusive scan, then a scan over the 16 wave totals
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint64_t incl = mine;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t v = __shfl_up(incl, d, 64);
    if (lane >= (uint32_t)d) incl += v;
  }
  if (lane == 63) s_part[wv] = incl;
  __syncthreads();
  atomicMax(&s_last_seg, last_nonempty);
  if (threadIdx.x == 0) {
    uint64_t acc = 0;
    for (int i = 0; i < NT / 64; ++i) {
      const uint64_t v = s_part[i];
      s_part[i] = acc;
      acc += v;
    }
    st->piece_cuts = acc;
  }
  __syncthreads();
  uint64_t off = s_total0 + s_part[wv] + (incl - mine);
  for (uint32_t k = k0; k < k1; ++k) {
    const SegInfo& si = a.seg_info[k];
    const uint32_t scnt = (si.flags & kBad) ? 0u : si.cnt;
    a.out_off[k] = off;
    off += (uint64_t)a.rep_cnt[k] + (scnt - a.rep_from[k]);
  }
  // the owner of the last non-empty segment hands its last cut to thread 0
  if (last_nonempty >= 0 && last_nonempty == s_last_seg) s_carry = my_last;
  __syncthreads();
  if (threadIdx.x == 0) {
    const int ls = s_last_seg;
    if (ls >= 0) st->carry = s_carry;
    if (a.chain.is_last && st->carry >= a.chain.L) st->done = 1;
    const uint64_t tot = s_total0 + st->piece_cuts;
    if (tot > a.out_cap) st->err |= kErrCapacity;
    st->total = tot;
    st->active = 1;
    if (do_publish) publish(a, st);
  }
}

__global__ __launch_bounds__(kFixThreads) void fixup_kernel(StitchArgs a) {
  fixup_body<kFixThreads>(a, false);  // (publish_kernel follows the gather)
}

// K3 for pieces of at most 1024 * PER segments (thread t owns segments
// t*PER .. t*PER + PER-1), with one round of global loads (the chain state and
// every segment's SegInfo) instead of fixup_kernel's chain of dependent round
// trips: when no segment is suspect (fixup_kernel's rule: flagged, or the
// previous segment's X != Z or flagged) the staged lists are the true chain,
// the counts are scanned in LDS, the gather's offsets written and the chain
// state published (the carry is the last non-empty segment's Z, its last
// staged cut).  Otherwise it runs fixup_kernel's body.  9.3 us per GiB against
// fixup_kernel's 13.6 (rocprofv3).  Folding the gather in as
// well was slower (34 us): one CU keeps too few misses in flight to move the
// 128 KiB cut list from memory written by other XCDs.
template <int PER>
__global__ __launch_bounds__(kFixThreads) void fixup_fast_kernel(StitchArgs a) {
  constexpr int NT = kFixThreads;
  constexpr uint32_t kBad = kSegDense | kSegOverflow;
  __shared__ uint64_t s_lx[NT], s_lz[NT];  // X, Z of each thread's last segment
  __shared__ uint32_t s_lf[NT];            // and its flags
  __shared__ uint64_t s_part[NT / 64];
  __shared__ int s_last_seg;
  __shared__ uint64_t s_carry, s_piece;
  DevState* st = a.state;
  const uint32_t T = a.nseg;
  const uint32_t tid = threadIdx.x;
  const uint32_t k0 = tid * PER;
  const uint64_t total0 = st->total;
  const uint32_t done = st->done, ovf = *a.pc.overflow;
  uint64_t X[PER], Z[PER];
  uint32_t cnt[PER], fl[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    X[j] = Z[j] = 0;
    cnt[j] = 0;
    fl[j] = 0;
    if (k0 + j < T) {
      const SegInfo& si = a.seg_info[k0 + j];
      X[j] = si.X;
      Z[j] = si.Z;
      cnt[j] = si.cnt;
      fl[j] = si.flags;
    }
  }
  if (done || ovf) {
    if (tid == 0) {
      st->active = 0;
      st->piece_cuts = 0;
      if (ovf) st->err |= kErrDense;
    }
    return;
  }
  s_lx[tid] = X[PER - 1];
  s_lz[tid] = Z[PER - 1];
  s_lf[tid] = fl[PER - 1];
  if (tid == 0) s_last_seg = -1;
  __syncthreads();
  bool bad = false;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const uint32_t k = k0 + j;
    if (k >= T) break;
    bad = bad || (fl[j] & kBad) != 0;
    if (k > 0) {
      const uint64_t px = j ? X[j - 1] : s_lx[tid - 1];
      const uint64_t pz = j ? Z[j - 1] : s_lz[tid - 1];
      const uint32_t pf = j ? fl[j - 1] : s_lf[tid - 1];
      bad = bad || px != pz || (pf & kBad) != 0;
    }
  }
  if (__syncthreads_count(bad) != 0) {  // a suspect segment: fixup_kernel's general path
    fixup_body<NT>(a, false);
    return;
  }
  // every staged list is the true chain
  uint64_t mine = 0, my_last = 0;
  int last_nonempty = -1;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    mine += cnt[j];
    if (cnt[j]) {
      last_nonempty = (int)(k0 + j);
      my_last = Z[j];
    }
  }
  const uint32_t lane = tid & 63, wv = tid >> 6;
  uint64_t incl = mine;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t v = __shfl_up(incl, d, 64);
    if (lane >= (uint32_t)d) incl += v;
  }
  if (lane == 63) s_part[wv] = incl;
  atomicMax(&s_last_seg, last_nonempty);
  __syncthreads();
  if (tid == 0) {
    uint64_t acc = 0;
    for (int i = 0; i < NT / 64; ++i) {
      const uint64_t v = s_part[i];
      s_part[i] = acc;
      acc += v;
    }
    s_piece = acc;
  }
  __syncthreads();
  if (last_nonempty >= 0 && last_nonempty == s_last_seg) s_carry = my_last;
  const uint64_t piece = s_piece;
  const bool fits = total0 + piece <= a.out_cap;
  {  // what the gather kernel reads: output offsets, no repaired cuts
    uint64_t off = total0 + s_part[wv] + (incl - mine);
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      if (k0 + j < T) {
        a.out_off[k0 + j] = off;
        a.rep_cnt[k0 + j] = 0;
        a.rep_from[k0 + j] = 0;
      }
      off += cnt[j];
    }
  }
  __syncthreads();
  if (tid == 0) {
    if (s_last_seg >= 0) st->carry = s_carry;
    if (a.chain.is_last && st->carry >= a.chain.L) st->done = 1;
    st->piece_cuts = piece;
    if (!fits) st->err |= kErrCapacity;
    st->total = total0 + piece;
    st->active = 1;
  }
}
template __global__ void fixup_fast_kernel<1>(StitchArgs);
template __global__ void fixup_fast_kernel<2>(StitchArgs);
template __global__ void fixup_fast_kernel<4>(StitchArgs);
// (an 8 GiB piece after the first in 2 MiB segments: 4097 of them)
template __global__ void fixup_fast_kernel<5>(StitchArgs);
template __global__ void fixup_fast_kernel<8>(StitchArgs);
// (an 8 GiB piece after the first: its stitch anchors max bytes before the
// piece, so 8193 one-MiB segments)
template __global__ void fixup_fast_kernel<9>(StitchArgs);

// K3 + K4 over many workgroups, for pieces of at most kFinMaxSeg segments:
// every workgroup loads all the SegInfo (40 B per segment, one round of global
// loads), checks fixup_kernel's rule (no suspect segment: flagged, or the
// previous segment's X != Z or flagged) and scans the counts in LDS; then it
// copies its own 16 segments' staged lists to the output, one wave per
// segment and one lane per cut (coalesced).  The last workgroup publishes the
// chain state.  It reads only walk_kernel's snapshots (DevState.base/skip),
// never a field the last workgroup writes.  With a suspect segment, workgroup
// 0 runs fixup_kernel's body and the gather alone (rare: a seam that did not
// converge, dense candidates).  Replaces fixup_fast_kernel + gather_kernel
// (one launch and a single-workgroup round trip less).
constexpr int kFinThreads = 256;
constexpr uint32_t kFinMaxSeg = 2048;  // 8 per thread
constexpr uint32_t kFinSegPerWg = 16;  // 4 per wave

template <int PER>
__global__ __launch_bounds__(kFinThreads) void finish_kernel(StitchArgs a) {
  constexpr int NT = kFinThreads;
  constexpr uint32_t kBad = kSegDense | kSegOverflow;
  __shared__ uint64_t s_lx[NT], s_lz[NT];  // X, Z of each thread's last segment
  __shared__ uint32_t s_lf[NT];            // and its flags
  __shared__ uint64_t s_off[kFinMaxSeg];   // output offset of every segment
  __shared__ uint32_t s_cnt[kFinMaxSeg];
  __shared__ uint64_t s_part[NT / 64];
  __shared__ int s_last_seg;
  __shared__ uint64_t s_carry, s_piece;
  DevState* st = a.state;
  const uint32_t T = a.nseg;
  const uint32_t tid = threadIdx.x;
  const uint32_t k0 = tid * PER;
  const uint32_t skip = st->skip;
  const uint64_t base = st->base;
  uint64_t X[PER], Z[PER];
  uint32_t cnt[PER], fl[PER];
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    X[j] = Z[j] = 0;
    cnt[j] = 0;
    fl[j] = 0;
    if (k0 + j < T) {
      const SegInfo& si = a.seg_info[k0 + j];
      X[j] = si.X;
      Z[j] = si.Z;
      cnt[j] = si.cnt;
      fl[j] = si.flags;
    }
  }
  // this workgroup's segments' staged lists (wave wv takes kb + wv + 4q), loaded
  // now so that their round trip overlaps the SegInfo loads instead of
  // following the count scan (the stage buffer holds nseg * scap entries)
  constexpr int QW = (int)kFinSegPerWg / (NT / 64);
  const uint32_t lane = tid & 63, wv = tid >> 6;
  const uint32_t kb = blockIdx.x * kFinSegPerWg;
  const uint32_t ke = kb + kFinSegPerWg < T ? kb + kFinSegPerWg : T;
  uint64_t v[QW];
  {
    const uint32_t sc1 = a.scap - 1;
#pragma unroll
    for (int q = 0; q < QW; ++q) {
      uint32_t k = kb + wv + (uint32_t)q * (NT / 64);
      k = k < T ? k : T - 1;
      v[q] = a.stage[(uint64_t)k * a.scap + (lane < sc1 ? lane : sc1)];
    }
  }
  const bool last_wg = blockIdx.x == gridDim.x - 1;
  if (skip) {  // what fixup_kernel leaves when the piece was not walked
    if (last_wg && tid == 0) {
      st->active = 0;
      st->piece_cuts = 0;
      if (*a.pc.overflow) st->err |= kErrDense;
    }
    return;
  }
  s_lx[tid] = X[PER - 1];
  s_lz[tid] = Z[PER - 1];
  s_lf[tid] = fl[PER - 1];
  if (tid == 0) s_last_seg = -1;
  __syncthreads();
  bool bad = false;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const uint32_t k = k0 + j;
    if (k >= T) break;
    bad = bad || (fl[j] & kBad) != 0;
    if (k > 0) {
      const uint64_t px = j ? X[j - 1] : s_lx[tid - 1];
      const uint64_t pz = j ? Z[j - 1] : s_lz[tid - 1];
      const uint32_t pf = j ? fl[j - 1] : s_lf[tid - 1];
      bad = bad || px != pz || (pf & kBad) != 0;
    }
  }
  if (__syncthreads_or(bad)) {  // a suspect segment: workgroup 0 does it all
    if (blockIdx.x == 0) {
      fixup_body<NT>(a, false);
      __threadfence_block();
      __syncthreads();
      if (st->active && !(st->err & kErrCapacity)) {
        for (uint32_t k = tid; k < T; k += NT) {
          const uint32_t scnt = (a.seg_info[k].flags & kBad) ? 0u : a.seg_info[k].cnt;
          const uint32_t rc = a.rep_cnt[k], rf = a.rep_from[k];
          const uint64_t off = a.out_off[k];
          const uint64_t* rep = a.rep + (uint64_t)k * a.scap;
          const uint64_t* stg = a.stage + (uint64_t)k * a.scap;
          for (uint32_t i = 0; i < rc; ++i) a.out[off + i] = rep[i];
          for (uint32_t i = rf; i < scnt; ++i) a.out[off + rc + (i - rf)] = stg[i];
        }
      }
    }
    return;
  }
  // every staged list is the true chain: counts -> offsets
  uint64_t mine = 0, my_last = 0;
  int last_nonempty = -1;
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    mine += cnt[j];
    if (cnt[j]) {
      last_nonempty = (int)(k0 + j);
      my_last = Z[j];
    }
  }
  uint64_t incl = mine;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint64_t v = __shfl_up(incl, d, 64);
    if (lane >= (uint32_t)d) incl += v;
  }
  if (lane == 63) s_part[wv] = incl;
  atomicMax(&s_last_seg, last_nonempty);
  __syncthreads();
  if (tid == 0) {
    uint64_t acc = 0;
    for (int i = 0; i < NT / 64; ++i) {
      const uint64_t v = s_part[i];
      s_part[i] = acc;
      acc += v;
    }
    s_piece = acc;
  }
  __syncthreads();
  {
    uint64_t off = base + s_part[wv] + (incl - mine);
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      if (k0 + j < T) {
        s_off[k0 + j] = off;
        s_cnt[k0 + j] = cnt[j];
      }
      off += cnt[j];
    }
  }
  if (last_nonempty >= 0 && last_nonempty == s_last_seg) s_carry = my_last;
  __syncthreads();
  const uint64_t piece = s_piece;
  const bool fits = base + piece <= a.out_cap;
  if (fits) {
#pragma unroll
    for (int q = 0; q < QW; ++q) {
      const uint32_t k = kb + wv + (uint32_t)q * (NT / 64);
      if (k < ke && lane < s_cnt[k]) a.out[s_off[k] + lane] = v[q];
    }
#pragma unroll 1
    for (int q = 0; q < QW; ++q) {  // lists of more than 64 cuts
      const uint32_t k = kb + wv + (uint32_t)q * (NT / 64);
      if (k >= ke) break;
      for (uint32_t i = 64 + lane; i < s_cnt[k]; i += 64)
        a.out[s_off[k] + i] = a.stage[(uint64_t)k * a.scap + i];
    }
  }
  if (last_wg && tid == 0) {
    if (s_last_seg >= 0) st->carry = s_carry;
    if (a.chain.is_last && st->carry >= a.chain.L) st->done = 1;
    st->piece_cuts = piece;
    if (!fits) st->err |= kErrCapacity;
    st->total = base + piece;
    st->active = 1;
  }
}
template __global__ void finish_kernel<1>(StitchArgs);
template __global__ void finish_kernel<2>(StitchArgs);
template __global__ void finish_kernel<4>(StitchArgs);
template __global__ void finish_kernel<8>(StitchArgs);

#if DSX_DIAG
// The stitch tasks of queued calls that no later scan carried (flush_behind):
// one task per wave, finish tasks first.
__global__ __launch_bounds__(256) void stitch_task_kernel(TaskArgs b) {
  __shared__ __attribute__((aligned(16))) uint32_t cand[4 * kTaskCand];
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t t = blockIdx.x * 4u + wave;
  if (t < b.nf) finish_task(b.f, t, b.fseg, b.nf, b.farrive, lane);
  else if (t - b.nf < b.nw) walk_task(b.w, t - b.nf, b.wseg, cand + wave * kTaskCand, lane);
}
#endif

// The chain state of a stitch-only pass (a shard re-walked from its true
// entry over kept candidate lists; normally the scan initialises it).
__global__ void state_init_kernel(DevState* st, uint64_t carry) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    st->carry = carry;
    st->total = 0;
    st->piece_cuts = 0;
    st->repaired = 0;
    st->discarded = 0;
    st->done = 0;
    st->err = 0;
    st->active = 0;
  }
}

// ---- K4: gather the per-segment lists into the contiguous output ---------
__global__ __launch_bounds__(256) void gather_kernel(StitchArgs a) {
  const uint32_t k = blockIdx.x;
  if (k >= a.nseg) return;
  if (!a.state->active || (a.state->err & kErrCapacity)) return;
  const SegInfo& si = a.seg_info[k];
  const uint32_t scnt = (si.flags & (kSegDense | kSegOverflow)) ? 0u : si.cnt;
  const uint32_t rc = a.rep_cnt[k], rf = a.rep_from[k];
  const uint64_t off = a.out_off[k];
  const uint64_t* rep = a.rep + (uint64_t)k * a.scap;
  const uint64_t* stg = a.stage + (uint64_t)k * a.scap;
  for (uint32_t i = threadIdx.x; i < rc; i += blockDim.x) a.out[off + i] = rep[i];
  for (uint32_t i = rf + threadIdx.x; i < scnt; i += blockDim.x) a.out[off + rc + (i - rf)] = stg[i];
}

}  // namespace dsx

// ---- multi-GPU seam alignment (syncWith across ranks, make.go:277-298) ----
#include "../../include/dsx.h"

namespace dsx {

// Candidates of a piece in (lo, wend], in order, from the scan's region lists:
// the first DSX_SEAM_MAX_CANDS go to seam->cands, the next one (if any) to
// seam->first_cand_beyond.  One wavefront; runs after the piece's scan and
// before the next piece's scan overwrites the lists.
__global__ __launch_bounds__(64) void seam_cands_kernel(PieceCands pc, uint64_t lo, uint64_t wend,
                                                        dsx_seam_t* seam) {
  const uint32_t lane = threadIdx.x;
  constexpr uint32_t kMax = DSX_SEAM_MAX_CANDS;
  uint32_t n = 0;  // wave-uniform
  const uint64_t r0 = lo > pc.P ? pc_region_of(pc, lo - pc.P) : 0;
  for (uint64_t r = r0; r < pc.nregions && n <= kMax; ++r) {
    const uint64_t base = pc.P + pc_region_base(pc, r);  // region covers (base, base + bytes]
    if (base >= wend) break;
    const uint32_t cnt0 = pc.region_cnt[r];
    const uint32_t cnt = cnt0 < pc.region_cap ? cnt0 : pc.region_cap;
    const uint32_t* l = pc.region_list + r * (uint64_t)pc.region_cap;
    for (uint32_t i0 = 0; i0 < cnt && n <= kMax; i0 += 64) {
      const uint32_t i = i0 + lane;
      const uint64_t p = i < cnt ? base + l[i] : 0;
      const bool ok = i < cnt && p > lo && p <= wend;
      const uint64_t m = __ballot(ok);
      const uint32_t idx = n + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
      if (ok) {
        if (idx < kMax) seam->cands[idx] = p;
        else if (idx == kMax) seam->first_cand_beyond = p;
      }
      n += (uint32_t)__popcll(m);
    }
  }
  if (lane == 0) {
    seam->ncands = n < kMax ? n : kMax;
    if (n <= kMax) seam->first_cand_beyond = ~0ull;
  }
}

// Completes a seam record once the shard's chain is known: truncates the
// window to the candidate and cut capacities (as the CPU restatement
// oracle/seam.py does), copies the speculative cuts of the window and the
// exit cut.  One thread.
__global__ void seam_finalize_kernel(dsx_seam_t* seam, const uint64_t* cuts, const DevState* st,
                                     uint64_t shard_start, uint64_t shard_len, uint64_t total,
                                     uint64_t wend0, uint64_t entry, uint32_t flags) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  uint64_t wend = wend0;
  if (seam->first_cand_beyond != ~0ull) wend = seam->cands[DSX_SEAM_MAX_CANDS - 1];
  const uint64_t n = st->total;
  uint32_t nc = 0;
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t x = cuts[i];
    if (x > wend) break;
    if (nc == DSX_SEAM_MAX_CUTS) {
      wend = seam->cuts[nc - 1];
      break;
    }
    seam->cuts[nc++] = x;
  }
  uint32_t ncand = 0;
  while (ncand < seam->ncands && seam->cands[ncand] <= wend) ++ncand;
  seam->shard_start = shard_start;
  seam->shard_len = shard_len;
  seam->total = total;
  seam->exit_cut = st->carry;
  seam->window_end = wend;
  seam->entry = entry;
  seam->ncands = ncand;
  seam->ncuts = nc;
  // an asynchronous dsx_shard_local does not read the chain state back: a
  // stitch error (e.g. a lane that overflowed its candidate slots, which the
  // synchronous path retries on the dense path) is published in the record,
  // and every rank's resolve asks the owner to redo its shard synchronously
  seam->flags = flags | (st->err ? (uint32_t)DSX_SEAM_REDO : 0u);
  seam->pad = 0;
}

struct SeamSrc {
  const uint64_t* c;
  uint32_t n;
  uint32_t j;
  __device__ uint64_t first_in(uint64_t a, uint64_t b) {
    while (j < n && c[j] <= a) ++j;
    if (j < n && c[j] <= b) return c[j];
    return kNone;
  }
};

// One lane walks the true chain across ALL seams in rank order: the chain
// entering rank r (the exit of rank r-1's chain, true by induction) is walked
// over rank r's seam window until it lands on a cut of rank r's speculative
// chain (convergence c_r).  A re-walked shard (DSX_SEAM_REWALKED) is true from
// its recorded entry on.  Every rank checks every seam, so all ranks agree on
// whether another exchange round is needed.
// info: [0] 0, or 1 + the first rank whose seam did not converge; [1] c_rank
// (keep the speculative cuts >= c_rank), or on failure the true entry cut of
// the failing rank; [2] number of cuts written to ext (the true cuts of
// `rank` before c_rank).  A record flagged DSX_SEAM_ERROR gives
// [0] = kSeamPeerFailed, one flagged DSX_SEAM_REDO [0] = kSeamRedo, [1] = its
// rank.
__global__ void seam_resolve_kernel(const dsx_seam_t* all, int nranks, int rank, uint64_t min,
                                    uint64_t max, uint64_t* ext, uint64_t* info) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  for (int r = 0; r < nranks; ++r) {
    if (all[r].flags & DSX_SEAM_ERROR) {  // a peer failed: every rank stops
      info[0] = kSeamPeerFailed;
      info[1] = (uint64_t)r;
      info[2] = 0;
      return;
    }
  }
  for (int r = 0; r < nranks; ++r) {
    if (all[r].flags & DSX_SEAM_REDO) {  // rank r redoes its shard, then everyone resyncs
      info[0] = kSeamRedo;
      info[1] = (uint64_t)r;
      info[2] = 0;
      return;
    }
  }
  uint64_t mine_c = all[rank].shard_start, mine_n = 0;
  uint64_t entry = all[0].exit_cut;
  for (int r = 1; r < nranks; ++r) {
    const dsx_seam_t& s = all[r];
    uint64_t c = kNone;
    uint32_t n = 0;
    if (s.flags & DSX_SEAM_REWALKED) {
      if (entry == s.entry) c = 0;  // the whole re-walked chain is true
    } else if (entry == s.shard_start || s.shard_len == 0) {
      c = s.shard_start;
    } else {
      ChainParams w;
      w.min = min;
      w.max = max;
      w.L = s.total;
      w.PE = s.window_end;
      w.is_last = s.window_end == s.total ? 1u : 0u;
      w.pad = 0;
      SeamSrc src{s.cands, s.ncands, 0};
      uint64_t x = entry;
      while (true) {
        if (w.is_last && x >= w.L) { c = x; break; }
        const uint64_t nx = next_cut(x, src, w);
        if (nx == kUndet) break;
        const uint32_t idx = bsearch_u64(s.cuts, s.ncuts, nx);
        if (idx < s.ncuts && s.cuts[idx] == nx) { c = nx; break; }
        if (r == rank && n < DSX_SEAM_MAX_CUTS) ext[n++] = nx;
        x = nx;
      }
    }
    if (c == kNone) {
      info[0] = (uint64_t)r + 1;
      info[1] = entry;
      info[2] = 0;
      return;
    }
    if (r == rank) {
      mine_c = c;
      mine_n = n;
    }
    entry = s.shard_len == 0 ? entry : s.exit_cut;
  }
  info[0] = 0;
  info[1] = mine_c;
  info[2] = mine_n;
}

// This rank's final cut list = ext cuts, then the speculative cuts >= c_rank
// (the st->total cuts the shard's chain left in `spec`); the count and status
// go to pinned host memory (res[0] status, [1] count, [2] entry of the failing
// rank), and the round's outcome to `code` (device, may be null) for the
// ranks' device-side agreement: 0 done, 1 exchange again, 2 failed.
__global__ __launch_bounds__(256) void shard_emit_kernel(const uint64_t* info, const uint64_t* ext,
                                                         const uint64_t* spec, const DevState* st,
                                                         uint64_t* out, uint64_t cap,
                                                         volatile uint64_t* res, int32_t* code) {
  const uint64_t status = info[0];
  if (status != 0) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      res[0] = status;
      res[1] = 0;
      res[2] = info[1];
      if (code) *code = status == kSeamPeerFailed ? 2 : 1;
      __threadfence_system();
    }
    return;
  }
  const uint64_t nspec = st->total;
  const uint64_t cr = info[1], next = info[2];
  uint64_t lo = 0, hi = nspec;  // first spec cut >= cr
  while (lo < hi) {
    const uint64_t m = (lo + hi) >> 1;
    if (spec[m] < cr) lo = m + 1; else hi = m;
  }
  const uint64_t n = next + (nspec - lo);
  if (n <= cap) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x)
      out[i] = i < next ? ext[i] : spec[lo + (i - next)];
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    res[0] = 0;
    res[1] = n;
    res[2] = 0;
    if (code) *code = n <= cap ? 0 : 2;
    __threadfence_system();
  }
}

}  // namespace dsx
