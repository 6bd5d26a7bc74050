// skipscan.hip -- DIAGNOSTIC (tools/, never loaded by the package): the
// reference's min-skip priced on the GPU.
//
// chunker.go:225-237 hashes a chunk only from start+min-48 and tests only
// from start+min+1: after every cut the sequential path never reads the next
// min-48 bytes (~25 % of the input at 16/64/256 KiB).  The product scan
// (scanl_kernel) stages, hashes and tests every byte.  This kernel skips like
// the reference and is built to be measured against it at the bench's shape:
//
//   * Chains.  A wave's 64 lanes are G groups of L = 64/G lanes; a group
//     follows ONE chain (Chunker.Next, chunker.go:206-277) over a span of the
//     blob from a virtual cut at the span start, as make.go's worker at
//     span*i does (make.go:167-258).  Spans come from a queue.
//   * Windows.  After a cut s the group jumps to the line of s+min-47 and
//     scans windows of L lines (lane j: line j; the 48 bytes before the line
//     from the lane before, lane 0 from the group's carry), until a window
//     holds the next cut: the first candidate in (s+min, s+max], else the
//     forced cut s+min(max, len-s); a tail of <= min bytes is one chunk.
//   * Staging.  One 128-B line per lane per window by LDS-DMA (8 wave
//     instructions, one descriptor per group); the next window's DMA is
//     issued before the current one is hashed, and after a cut a corrective
//     DMA for that group's jump target follows it (loads retire in order, so
//     the corrective line lands last).
//   * Merge.  Past its span's end a group keeps chunking until one of its
//     cuts is a cut the next span's chain published (syncWith,
//     make.go:277-327); from there the chains agree.  merge[k] = that cut
//     (len at the end, ~0 when no merge within kMaxOverrun chunks).
//
// The boundary test is chunker.go:265's for odd d with qBias 1 (the default
// 16/64/256 KiB, d = 49535): t = (h+1)*inv, candidate iff 1 <= t <= qMax+1;
// the hash is kept inverted, so t = (~h)*(2^32-inv) is one multiply
// (scanl_kernel's MODE 2).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>

#include "../include/dsx_buzhash_table.h"

namespace {

constexpr int kWave = 64;
constexpr int kLine = 128;
constexpr int kWaves = 8;                  // waves per workgroup (one workgroup per CU)
constexpr int kTableBytes = 256 * 256;     // {T, rotl16 T} x 32 lane slots per byte value
constexpr int kMaxOverrun = 32;            // chunks past the span end before giving up
constexpr uint64_t kNone = ~0ull;

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void_t;

__constant__ uint32_t kT[256] = DSX_BUZHASH_TABLE_INIT;

struct SkipArgs {
  const uint8_t* blob;
  uint64_t len, min, max;
  uint32_t ninv;   // 2^32 - inverse_odd: (~h) * ninv = (h+1) * inv
  uint32_t qlim;   // qMax + 1
  uint64_t span;   // bytes per span
  uint32_t nspans;
  uint32_t cap;    // cut slots per span
  uint32_t* queue;                 // [0]: next span
  uint64_t* cuts;                  // nspans x cap
  uint32_t* ncut;                  // per span: cuts published (release)
  uint64_t* merge;                 // per span: the first cut shared with the next span's chain
  unsigned long long* stats;       // see kStat*
  uint64_t* stamps;                // per wave {start, end} (s_memrealtime)
};
enum { kStatLines, kStatWindows, kStatJumps, kStatOverrun, kStatFailed, kStatCuts, kStatSpans,
       kStatIdleLaneWindows, kStatN };

template <class F, int... I>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}

__device__ __forceinline__ void dma16(const u32x4& rsrc, uint32_t voff, uint32_t lds_addr) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %1, %3, 0 offen nt lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(lds_addr), "s"(rsrc)
      : "memory");
}

__device__ __forceinline__ uint32_t lookup_addr(uint32_t w, uint32_t slot8, int k) {
  if (k == 1) return __builtin_amdgcn_bitop3_b32(w, 0xFF00u, slot8, 0xEA);
  const uint32_t sel = 0x0C0C0000u | ((4u + (uint32_t)k) << 8);
  return __builtin_amdgcn_perm(w, slot8, sel);
}

__device__ __forceinline__ uint64_t rl64(uint64_t v, int lane) {
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)v, lane);
  const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(v >> 32), lane);
  return ((uint64_t)hi << 32) | lo;
}

template <int G>
__global__ __launch_bounds__(kWaves * kWave, 2) void skip_kernel(SkipArgs a) {
  constexpr int L = kWave / G;               // lanes (lines) per group
  constexpr uint64_t WB = (uint64_t)L * kLine;  // window bytes
  static_assert(L >= 8, "a DMA instruction covers 8 rows of one group");
  __shared__ __attribute__((aligned(16))) uint8_t lds[kTableBytes + kWaves * kWave * kLine];
  __shared__ __attribute__((aligned(16))) uint8_t s_carry[kWaves * G * 48];
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t g = lane / L, li = lane % L;
  const uint32_t slot8 = (lane & 31u) * 8u;
  uint8_t* const stage = lds + kTableBytes + wave * kWave * kLine;
  const uint32_t stage_lds = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_void_t*)stage);
  uint64_t t_start = 0;
  if (lane == 0) t_start = __builtin_amdgcn_s_memrealtime();

  {  // the replicated table
    const uint32_t v = threadIdx.x & 255u;
    const uint32_t tv = kT[v];
    uint2 t;
    t.x = tv;
    t.y = __builtin_amdgcn_alignbit(tv, tv, 16);
    for (uint32_t slot = threadIdx.x >> 8; slot < 32u; slot += (kWaves * kWave) / 256)
      *reinterpret_cast<uint2*>(lds + v * 256u + slot * 8u) = t;
  }
  __syncthreads();

  // group-uniform chain state (every lane of a group holds the same values)
  uint32_t sp = 0xFFFFFFFFu;  // span (0xFFFFFFFF: idle)
  uint64_t s = 0, E = 0, lo = 0, hi = 0, wa = 0;  // last cut, span end, test range (lo, hi], window
  uint32_t n = 0, j = 0, over = 0;                // cuts published, merge pointer, overrun chunks
  unsigned long long st_lines = 0, st_windows = 0, st_jumps = 0, st_over = 0, st_failed = 0,
                     st_cuts = 0, st_spans = 0, st_idle = 0;

  // per-lane DMA geometry: instruction i, DMA lane l -> row 8i + l/8, physical
  // 16-B chunk l%8 holding logical chunk (l%8 - rot(row)) % 8, rot(row) =
  // (row >> 1) % 8 (conflict-free ds_read_b128 of the rows, as scanl_kernel)
  auto voff_of = [&](int i) -> uint32_t {
    const uint32_t row = 8u * (uint32_t)i + (lane >> 3);
    const uint32_t rot = (row >> 1) & 7u;
    return (row % (uint32_t)L) * (uint32_t)kLine + 16u * (((lane & 7u) - rot) & 7u);
  };
  // DMA of the windows of the groups in `gm` (bit per group) at their `wa`
  auto issue = [&](uint32_t gm) {
    static_for<8>([&](auto ic) {
      constexpr int i = decltype(ic)::value;
      constexpr int gi = (8 * i) / L;
      if (!((gm >> gi) & 1u)) return;
      const uint64_t base = rl64(wa, gi * L);
      if (base >= a.len) return;
      const uint64_t nrec64 = a.len - base;
      const uint64_t rp = (uint64_t)(uintptr_t)(a.blob + base);
      u32x4 rsrc;
      rsrc.x = __builtin_amdgcn_readfirstlane((uint32_t)rp);
      rsrc.y = __builtin_amdgcn_readfirstlane((uint32_t)(rp >> 32) & 0xFFFFu);
      rsrc.z = __builtin_amdgcn_readfirstlane(nrec64 > 0xFFFFFFF0ull ? 0xFFFFFFF0u : (uint32_t)nrec64);
      rsrc.w = 0x00020000u;
      dma16(rsrc, voff_of(i), stage_lds + 1024u * (uint32_t)i);
      st_lines += 8;
    });
  };
  // publish this group's cut c (lane li == 0): a relaxed device-scope store
  // (written through to memory, visible to every XCD) into a slot the host
  // zeroed, so a slot is its own valid flag -- no release fence, whose L2
  // write-back per cut stalled the wave (the first version, profiles/r06g)
  auto publish = [&](uint64_t c) {
    if (li == 0 && n < a.cap)
      __hip_atomic_store(a.cuts + (uint64_t)sp * a.cap + n, c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    ++n;
  };
  auto close_span = [&](uint64_t m) {  // (the host reads these after the launch)
    if (li == 0) {
      a.merge[sp] = m;
      a.ncut[sp] = n;
    }
  };
  // take the next span (the group's lane 0 draws, the group follows)
  auto take_span = [&]() {
    uint32_t t = 0;
    if (li == 0) t = atomicAdd(a.queue, 1u);
    t = __shfl(t, (int)(g * L), kWave);
    if (t < a.nspans) {
      sp = t;
      s = (uint64_t)t * a.span;
      E = s + a.span < a.len ? s + a.span : a.len;
      n = j = over = 0;
      st_spans += li == 0;
    } else {
      sp = 0xFFFFFFFFu;
    }
  };
  // set up the chain after the cut / virtual cut s: the window of s+min-47,
  // or, for a tail of <= min bytes, the final chunk right away (loops until
  // the group has a window to scan or is idle)
  auto setup = [&]() {
    while (sp != 0xFFFFFFFFu) {
      if (a.len - s <= a.min) {  // chunker.go:215-217: the rest is one chunk
        publish(a.len);
        close_span(a.len);
        take_span();
        continue;
      }
      lo = s + a.min;
      hi = s + (a.len - s < a.max ? a.len - s : a.max);
      wa = (s + a.min - 47u) & ~(uint64_t)(kLine - 1);
      return;
    }
  };

  take_span();
  setup();
  // (bit g of `gbits`: group g active; from the ballot of the groups' lane 0)
  auto gbits_of = [&](uint64_t bal) -> uint32_t {
    uint32_t m = 0;
    static_for<G>([&](auto gc) {
      constexpr int gg = decltype(gc)::value;
      m |= ((bal >> (gg * L)) & 1ull) ? (1u << gg) : 0u;
    });
    return m;
  };
  uint32_t active = gbits_of(__ballot(sp != 0xFFFFFFFFu && li == 0));
  issue(active);

  uint32_t ring[48];
  uint32_t w[44];  // 12 warm-up words, then the line's 32
  uint64_t guard = 0;
  while (active) {
    if (++guard > (1ull << 26)) break;  // (never: every window moves a chain forward)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    // this lane's warm-up (the line before: lane li-1's last 48 bytes, lane 0
    // the group's carry) and its line
    {
      const uint32_t prow = lane - 1u;
      const uint32_t prot = (prow >> 1) & 7u;
      const uint8_t* warm_base = stage + prow * kLine;
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const uint8_t* src = li == 0 ? s_carry + (wave * G + g) * 48u + 16u * c
                                     : warm_base + 16u * (((uint32_t)(c + 5) + prot) & 7u);
        const uint4 q = *reinterpret_cast<const uint4*>(src);
        w[4 * c] = q.x, w[4 * c + 1] = q.y, w[4 * c + 2] = q.z, w[4 * c + 3] = q.w;
      }
      const uint32_t rot = (lane >> 1) & 7u;
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const uint4 q = *reinterpret_cast<const uint4*>(stage + lane * kLine + 16u * (((uint32_t)c + rot) & 7u));
        w[12 + 4 * c] = q.x, w[13 + 4 * c] = q.y, w[14 + 4 * c] = q.z, w[15 + 4 * c] = q.w;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (li == (uint32_t)L - 1u) {  // the next window's lane-0 warm-up
#pragma unroll
        for (int c = 0; c < 3; ++c)
          *reinterpret_cast<uint4*>(s_carry + (wave * G + g) * 48u + 16u * c) =
              make_uint4(w[32 + 4 * c], w[33 + 4 * c], w[34 + 4 * c], w[35 + 4 * c]);
      }
    }
    // speculative: every active group's next contiguous window
    const uint64_t x = wa + (uint64_t)li * kLine;  // this lane's line
    const bool mine = sp != 0xFFFFFFFFu;
    wa += WB;
    issue(active);
    wa -= WB;
    ++st_windows;
    st_idle += __builtin_popcountll(__ballot(!mine));

    // hash: 48 warm-up steps (no test), then the line's 128 positions
    uint32_t h = ~0u;  // ~hash (MODE 2 of scanl_kernel)
    uint64_t first = kNone;
    uint64_t L8[2][8];
    auto issue_sub = [&](auto sc) {
      constexpr int sg = decltype(sc)::value;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int k = sg * 8 + q;
        L8[sg & 1][q] = *reinterpret_cast<const uint64_t*>(lds + lookup_addr(w[k >> 2], slot8, k & 3));
      }
    };
    issue_sub(std::integral_constant<int, 0>{});
    static_for<22>([&](auto sc) {
      constexpr int sg = decltype(sc)::value;
      if constexpr (sg + 1 < 22) issue_sub(std::integral_constant<int, sg + 1>{});
      uint32_t t[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int k = sg * 8 + q;
        const int rk = k % 48;
        const uint32_t outv = k < 48 ? 0u : ring[rk];
        h = __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_alignbit(h, h, 31), (uint32_t)L8[sg & 1][q],
                                        outv, 0x96);
        ring[rk] = (uint32_t)(L8[sg & 1][q] >> 32);
        t[q] = h * a.ninv;
      }
      if constexpr (sg >= 6) {  // (subgroups 0..5: the warm-up)
        uint32_t mn = t[0];
#pragma unroll
        for (int q = 1; q < 8; ++q) mn = __builtin_elementwise_min(mn, t[q]);
        // candidate: 1 <= t <= qlim (t = 0 wraps under Go's t - qBias)
        if (__builtin_expect(__ballot(mn <= a.qlim) != 0, 0)) {
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const uint64_t p = x + (uint64_t)((sg - 6) * 8 + q) + 1u;  // the cut after this byte
            if (t[q] - 1u <= a.qlim - 1u && mine && p > lo && p <= hi && p < first) first = p;
          }
        }
      }
    });

    // window end: each group's first candidate (lanes hold their lines in
    // order, so the lowest lane with one has it), or the forced cut
    const uint64_t has = __ballot(first != kNone);
    uint64_t cut = kNone;
    static_for<G>([&](auto gc) {
      constexpr int gg = decltype(gc)::value;
      constexpr uint64_t kGroupMask = L == 64 ? ~0ull : ((1ull << (L % 64)) - 1ull);
      const uint64_t m = (has >> (gg * L)) & kGroupMask;
      if (m) {
        const uint64_t c = rl64(first, gg * L + __builtin_ctzll(m));
        if (g == (uint32_t)gg) cut = c;
      }
    });
    if (mine && cut == kNone && wa + WB >= hi) cut = hi;  // chunker.go:276
    const uint32_t cut_groups = gbits_of(__ballot(cut != kNone && li == 0));
    if (__builtin_expect(cut_groups == 0, 1)) {
      wa += WB;
      continue;
    }
    // rare: the groups with a cut publish it, check the merge, set up the next chunk
    uint32_t jumped = 0;
    if (cut != kNone) {
      publish(cut);
      ++st_cuts;
      s = cut;
      bool done = false;
      if (cut >= a.len) {
        close_span(a.len);
        done = true;
      } else if (cut >= E) {  // past the span end: meet the next span's chain
        ++over;
        ++st_over;
        uint32_t merged = 0;
        if (li == 0) {
          const uint32_t nx = sp + 1u;
          uint64_t* c1 = a.cuts + (uint64_t)nx * a.cap;
          uint32_t jj = j;
          uint64_t v = 0;
          while (jj < a.cap &&
                 (v = __hip_atomic_load(c1 + jj, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) != 0 &&
                 v < cut)
            ++jj;
          j = jj;
          if (v == cut) {
            merged = 1;
          } else if (over > (uint32_t)kMaxOverrun || n >= a.cap) {
            merged = 2;
          }
        }
        merged = __shfl(merged, (int)(g * L), kWave);
        j = __shfl(j, (int)(g * L), kWave);
        if (merged) {
          close_span(merged == 1 ? cut : kNone);
          done = true;
          st_failed += merged == 2 && li == 0;
        }
      }
      if (done) take_span();
      setup();
      jumped = 1;
    }
    const uint32_t jgroups = gbits_of(__ballot(jumped && sp != 0xFFFFFFFFu && li == 0));
    // the groups without a cut move on to their next window (already issued)
    if (!(jumped)) wa += WB;
    st_jumps += __builtin_popcount(jgroups);
    active = gbits_of(__ballot(sp != 0xFFFFFFFFu && li == 0));
    issue(jgroups);  // (lands after the speculative lines of those groups)
  }
  if (lane == 0) {
    atomicAdd(a.stats + kStatLines, st_lines);
    atomicAdd(a.stats + kStatWindows, st_windows);
    atomicAdd(a.stats + kStatIdleLaneWindows, st_idle);
  }
  // (per-group counters live in the groups' lane 0)
  unsigned long long sj = 0, so = 0, sf = 0, sc = 0, ss = 0;
  if (lane == 0) sj = st_jumps;
  if (li == 0) so = st_over, sf = st_failed, sc = st_cuts, ss = st_spans;
  if (li == 0) {
    if (sj) atomicAdd(a.stats + kStatJumps, sj);
    atomicAdd(a.stats + kStatOverrun, so);
    atomicAdd(a.stats + kStatFailed, sf);
    atomicAdd(a.stats + kStatCuts, sc);
    atomicAdd(a.stats + kStatSpans, ss);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (lane == 0) {
    const uint64_t t_end = __builtin_amdgcn_s_memrealtime();
    uint64_t* r = a.stamps + 2ull * (blockIdx.x * kWaves + wave);
    r[0] = t_start;
    r[1] = t_end;
  }
}

}  // namespace

// Runs `iters` launches over the blob (queue and counts reset before each)
// and returns the mean launch time in ms from HIP events (stream 0).
extern "C" int skipscan_run(const void* blob, uint64_t len, uint64_t min, uint64_t max,
                            uint32_t inverse_odd, uint32_t qmax, uint64_t span, int groups,
                            uint64_t* cuts, uint32_t* ncut, uint64_t* merge, uint32_t* queue,
                            unsigned long long* stats, uint64_t* stamps, uint32_t cap, int iters,
                            float* ms_out) {
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, 0) != hipSuccess) return -1;
  if (min < 48 || span < min || (groups != 1 && groups != 2 && groups != 4 && groups != 8)) return -2;
  SkipArgs a{};
  a.blob = (const uint8_t*)blob;
  a.len = len;
  a.min = min;
  a.max = max;
  a.ninv = 0u - inverse_odd;
  a.qlim = qmax + 1u;
  a.span = span;
  a.nspans = (uint32_t)((len + span - 1) / span);
  a.cap = cap;
  a.queue = queue;
  a.cuts = cuts;
  a.ncut = ncut;
  a.merge = merge;
  a.stats = stats;
  a.stamps = stamps;
  const dim3 grid((uint32_t)prop.multiProcessorCount), block(kWaves * kWave);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float total = 0.f;
  for (int it = 0; it < iters; ++it) {
    // (inside the timed region: the zeroed cut slots are part of the method)
    (void)hipEventRecord(e0, 0);
    (void)hipMemsetAsync(queue, 0, 4, 0);
    (void)hipMemsetAsync(ncut, 0, 4ull * a.nspans, 0);
    (void)hipMemsetAsync(cuts, 0, 8ull * a.nspans * cap, 0);
    (void)hipMemsetAsync(stats, 0, 8ull * kStatN, 0);
    switch (groups) {
      case 1: hipLaunchKernelGGL(skip_kernel<1>, grid, block, 0, 0, a); break;
      case 2: hipLaunchKernelGGL(skip_kernel<2>, grid, block, 0, 0, a); break;
      case 4: hipLaunchKernelGGL(skip_kernel<4>, grid, block, 0, 0, a); break;
      default: hipLaunchKernelGGL(skip_kernel<8>, grid, block, 0, 0, a); break;
    }
    (void)hipEventRecord(e1, 0);
    if (hipEventSynchronize(e1) != hipSuccess) return -3;
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    total += ms;
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  if (hipGetLastError() != hipSuccess) return -4;
  *ms_out = total / (float)(iters > 0 ? iters : 1);
  return 0;
}
