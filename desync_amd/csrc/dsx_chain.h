// dsx_chain.h -- the chain rule (chunker.go:206-277) as wave-level device
// code, shared by the stitch kernels (dsx_stitch.hip) and the stitch tasks
// that run inside the scan (dsx_scan.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "dsx_common.h"
#include "dsx_stitch.h"

namespace dsx {

constexpr uint64_t kNone = ~0ull;

// A piece's chain state into its pinned host slot, seq last once the field
// stores are complete (the slot is uncached host memory: a store completes
// when it is performed there), so a host that polls seq (queued calls,
// dsx_result) reads this piece's fields.  Called after the piece's stitch
// has ended (publish_kernel, or the next scan's block 0), so its cut list
// is complete too.  (A system-scope fence here also wrote back and
// invalidated the L2: 4.3 us per piece.)
__device__ __forceinline__ void publish_state(volatile HostState* h, const DevState* st,
                                              uint64_t seq) {
  h->carry = st->carry;
  h->total = st->total;
  h->repaired = st->repaired;
  h->discarded = st->discarded;
  h->done = st->done;
  h->err = st->err;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  h->seq = seq;
}

// The same source searched by a whole wavefront: 64 candidates per LDS read
// and a ballot, so a chain step costs one LDS round trip instead of one per
// candidate passed (the walks are latency-bound: one chain per wave).
struct WaveLdsSrc {
  const uint32_t* c;
  uint32_t n;
  uint32_t base;  // window start: lane l holds c[base + l] in v
  uint64_t lo;
  uint32_t lane;
  uint32_t v;
  __device__ void load() { v = base + lane < n ? c[base + lane] : 0xFFFFFFFFu; }
  // first candidate > a (relative ar), searching forward from the window;
  // returns its relative offset or 0xFFFFFFFF.  Steps of a chain advance by
  // about one candidate, so most calls hit the window already in registers.
  __device__ uint32_t next_after(uint64_t ar) {
    const uint32_t ar32 = ar > 0xFFFFFFFEull ? 0xFFFFFFFEu : (uint32_t)ar;
    while (true) {
      const uint64_t m = __ballot(v > ar32);
      if (m) {
        const uint32_t f = (uint32_t)__builtin_ctzll(m);
        if (base + f >= n) return 0xFFFFFFFFu;
        return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)f);
      }
      if (base + 64u >= n) return 0xFFFFFFFFu;
      base += 64u;
      load();
    }
  }
  // (lanes past n hold 0xFFFFFFFF, which is also "none": the first lane
  // above ar32 needs no range check, and a window with no such lane is full)
  __device__ uint32_t next_after32(uint32_t ar32) {
    uint64_t m = __ballot(v > ar32);
    while (__builtin_expect(m == 0, 0)) {
      if (base + 64u >= n) return 0xFFFFFFFFu;
      base += 64u;
      load();
      m = __ballot(v > ar32);
    }
    return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)__builtin_ctzll(m));
  }
  __device__ uint64_t first_in(uint64_t a, uint64_t b) {
    const uint32_t r = next_after(a - lo);  // a >= lo always (a = s+min, s >= lo)
    if (r != 0xFFFFFFFFu) {
      const uint64_t p = lo + r;
      if (p <= b) return p;
    }
    return kNone;
  }
  // position the window at the first candidate > a
  __device__ void seek(uint64_t a) {
    base = 0;
    load();
    const uint64_t ar = a < lo ? 0 : a - lo;
    const uint32_t ar32 = ar > 0xFFFFFFFEull ? 0xFFFFFFFEu : (uint32_t)ar;
    while (base + 64u < n && __ballot(v > ar32) == 0) {
      base += 64u;
      load();
    }
  }
};

// wave-uniform 64-bit value (scalar registers, scalar control flow)
__device__ __forceinline__ uint64_t uniform64(uint64_t v) {
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return ((uint64_t)hi << 32) | lo;
}

// The chain rule in 32-bit coordinates relative to a walk workgroup's `lo`
// (its candidates and segments span far less than 4 GiB): every chain step is
// a handful of scalar 32-bit operations instead of 64-bit vector compares.
constexpr uint32_t kRelUndet = 0xFFFFFFFFu;
constexpr uint32_t kRelClamp = 0xFFFFFFF0u;
struct RelChain {
  uint32_t min, max, L, PE;  // L, PE relative to lo, clamped to kRelClamp
  bool is_last;
  // the same bounds folded for branch-free steps: a chain at s >= tail_at
  // ends at L (chunker.go:215-217: len - s <= min); steps are capped at
  // lim_cap (L: chunker.go:221); a bound beyond undet_at is undetermined
  // (non-final piece).  Unused bounds are 0xFFFFFFFF.
  uint32_t tail_at, lim_cap, undet_at, end_at;
};
__device__ __forceinline__ uint32_t rel_clamp(uint64_t v, uint64_t lo) {
  return v <= lo ? 0u : (v - lo >= kRelClamp ? kRelClamp : (uint32_t)(v - lo));
}
__device__ __forceinline__ RelChain rel_chain(const ChainParams& w, uint64_t lo) {
  // min/max clamped to 2^30: a walk workgroup spans far less, so a bound
  // beyond 2^30 decides exactly like the real one (the chain leaves the
  // segment either way), and s + max never overflows 32 bits
  RelChain r;
  r.min = w.min < (1ull << 30) ? (uint32_t)w.min : (1u << 30);
  r.max = w.max < (1ull << 30) ? (uint32_t)w.max : (1u << 30);
  r.L = rel_clamp(w.L, lo);
  r.PE = rel_clamp(w.PE, lo);
  r.is_last = w.is_last != 0;
  r.tail_at = r.is_last ? (r.L > r.min ? r.L - r.min : 0u) : 0xFFFFFFFFu;
  r.lim_cap = r.is_last ? r.L : 0xFFFFFFFFu;
  r.undet_at = r.is_last ? 0xFFFFFFFFu : r.PE;
  r.end_at = r.is_last ? r.L : 0xFFFFFFFFu;
  return r;
}
// next(s) of chunker.go:206-277 for a relative chain position s < tail_at
// (the walks test s >= tail_at, which is <= end_at, once per step and sort
// out the chain's end on that rare branch: next = L, chunker.go:215-217);
// kRelUndet if the successor depends on bytes beyond the piece.  kRelUndet is
// above every relative position, so the walks test only nx > er on the way
// out: two scalar compares a step fewer (the steps are bound by the CU's one
// scalar unit).
__device__ __forceinline__ uint32_t rel_step(uint32_t s, WaveLdsSrc& src, const RelChain& w) {
  const uint32_t lim = min(s + w.max, w.lim_cap);  // chunker.go:221
  const uint32_t c = src.next_after32(s + w.min);  // chunker.go:259-271
  if (c <= lim) return c;                          // (none = 0xFFFFFFFF > lim)
  return lim > w.undet_at ? kRelUndet : lim;       // chunker.go:276
}
static_assert(kRelUndet > kRelClamp, "kRelUndet must exceed every relative position");



__device__ __forceinline__ uint64_t seg_start(const StitchArgs& a, uint64_t s0, uint32_t k) {
  return k == 0 ? s0 : a.anchor + (uint64_t)k * a.seg;
}
__device__ __forceinline__ uint64_t seg_end(const StitchArgs& a, uint32_t k) {
  if (k + 1 >= a.nseg) return a.chain.is_last ? a.chain.L : a.chain.PE;
  return a.anchor + (uint64_t)(k + 1) * a.seg;
}


}  // namespace dsx
