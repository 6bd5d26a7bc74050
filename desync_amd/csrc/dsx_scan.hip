// dsx_scan.hip -- boundary-candidate scan over a device-resident piece.
//
// Reference semantics: the rolling Buzhash of chunker.go:225-271 evaluated at
// EVERY byte position instead of only inside (s+min, s+max] of the current
// chunk.  Because the hash at a tested cut p only depends on the 48 bytes
// [p-48, p) (SURVEY.md sec.0 finding 1), the per-position candidate set is the
// same for every possible chunk start; dsx_stitch.hip turns it into the cut
// chain.
//
// MI355X mapping (DESIGN.md "Scan kernel"):
//   * one workgroup = 8 waves (2 per SIMD), 1 per CU (160 KiB LDS), persistent
//     over regions; a wave owns a region of 64 lane segments of S bytes and
//     lane l rolls the hash through its own segment;
//   * HBM -> LDS by LDS-DMA (buffer_load_dwordx4 ... lds) in batches of 4
//     rounds = 192 B per lane (12 KiB per wave): long per-lane runs keep DRAM
//     and the texture path efficient (tools/ubench_staging.hip: 48 B rows
//     4.0 TB/s, 192 B rows 6.3 TB/s); the batch is copied to registers at
//     once so the next batch's DMA overlaps the hashing of this one;
//   * the substitution table lives in LDS replicated over 32 lane slots
//     (byte v, slot s at v*256 + s*8 = {T[v], rotl16(T[v])}) so each lookup is
//     ONE v_perm_b32 (address = byte<<8 | slot) + ONE conflict-free
//     ds_read_b64; the outgoing byte's rotated term comes from a 48-entry
//     register ring;
//   * the boundary test is ONE cvt + ONE fma + ONE 24-bit mad + ONE compare
//     (magic-number rounding, exact for 1024 < d < 2^22), a wave ballot per
//     byte, and one scalar branch per 16 bytes for the rare hits;
//   * at the end of a region the wave compacts its lanes' hits into one
//     sorted per-region list for the stitch.
#include <hip/hip_runtime.h>

#include "../../include/dsx_buzhash_table.h"
#include "dsx_common.h"

namespace dsx {

typedef __attribute__((address_space(3))) void lds_void_t;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__constant__ uint32_t kT[256] = DSX_BUZHASH_TABLE_INIT;

// One 1 KiB LDS-DMA wave instruction (buffer_load_dwordx4 ... lds): lane j's
// 16 bytes from rsrc+voff land at LDS byte lds_addr + 16*j.  Inline asm so
// hipcc does not treat later ds_reads as aliasing a pending DMA (it would
// drain vmcnt(0) in front of unrelated LDS reads); completion is tracked by
// the explicit s_waitcnt vmcnt(0) before a batch is read.
__device__ __forceinline__ void dma16(const u32x4& rsrc, uint32_t voff, uint32_t lds_addr) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "buffer_load_dwordx4 %1, %3, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(lds_addr), "s"(rsrc)
      : "memory");
}

// h % d == d-1 on the GPU.
//   MODE 0: exactly Go's multiply-inverse form (chunker.go:265): v_mul_lo_u32.
//   MODE 1: one fma lands h/d - (d-1)/d in [2^23, 2^24) where float spacing
//           is 1, so the mantissa bits ARE round(q) (magic-number rounding);
//           then the exact check h == q*d + d-1 with a 24-bit mad on those
//           bits (the constant float offset is folded into tc.madc).
//           Exact for 1024 < d < 2^22 (DESIGN.md "Boundary test").
template <int MODE>
__device__ __forceinline__ bool is_cand(uint32_t h, const TestConsts& tc) {
  if constexpr (MODE == 0) {
    uint32_t v = (h + 1u) * tc.inv;
    v = __builtin_amdgcn_alignbit(v, v, tc.rot);
    return v - tc.qbias <= tc.qmax;
  } else {
    const float f = __builtin_fmaf((float)h, tc.rcp, tc.c0);
    const uint32_t bits = __builtin_bit_cast(uint32_t, f);
    return __umul24(bits, tc.d) + tc.madc == h;
  }
}

// Process one 48-byte round of one lane.  `w` holds the round's bytes,
// `ring[k]` the rotated table value of the byte 48 positions earlier.
// The 48 bytes run as 6 subgroups of 8; the table lookups of subgroup j+1 are
// issued before subgroup j is hashed (explicit software pipeline: the LDS
// latency hides under the previous subgroup's hashing, and at most 16 LDS
// reads are in flight, within the 4-bit lgkmcnt).
// VARIANT (diagnostic ablations; results are wrong for VARIANT != 0):
// 1 = no boundary test, 3 = staging only (no hashing).
template <bool TEST, int MODE, int VARIANT>
__device__ __forceinline__ void round48(const uint32_t* w, uint32_t& h, uint32_t (&ring)[48],
                                        const uint8_t* __restrict__ tbl, uint32_t slot8,
                                        const TestConsts& tc, uint32_t lane, uint32_t obase,
                                        uint32_t seg_valid, uint32_t& cnt,
                                        uint16_t* __restrict__ myslots, uint32_t lane_slots) {
  if constexpr (VARIANT == 3) {
#pragma unroll
    for (int k = 0; k < 12; ++k) h ^= w[k];
    asm volatile("" ::"v"(h));
    return;
  }
  constexpr int SUB = 8;
  uint2 LA[SUB], LB[SUB];
  auto issue = [&](int j, uint2 (&L)[SUB]) {
#pragma unroll
    for (int i = 0; i < SUB; ++i) {
      const int k = j * SUB + i;
      const uint32_t sel = 0x0C0C0000u | ((4u + (uint32_t)(k & 3)) << 8);
      const uint32_t addr = __builtin_amdgcn_perm(w[k >> 2], slot8, sel);
      L[i] = *reinterpret_cast<const uint2*>(tbl + addr);
    }
  };
  uint64_t m[16];
  auto compute = [&](int j, uint2 (&L)[SUB]) {
#pragma unroll
    for (int i = 0; i < SUB; ++i) {
      const int k = j * SUB + i;
      // rotl1(h) ^ (T[in] ^ Trot[out]); the asm fence keeps the compiler from
      // re-associating the second xor back onto the h chain
      uint32_t x = L[i].x ^ ring[k];
      asm("" : "+v"(x));
      h = __builtin_amdgcn_alignbit(h, h, 31) ^ x;
      ring[k] = L[i].y;
      if constexpr (TEST && VARIANT == 0) m[k & 15] = __ballot(is_cand<MODE>(h, tc));
    }
    if constexpr (TEST && VARIANT != 0) {
      asm volatile("" ::"v"(h));  // keep the ablated chain live (no DCE)
    } else if constexpr (TEST) {
      if ((j & 1) == 1) {  // rare-hit check once per 16 bytes
        const int g = j >> 1;
        uint64_t any = 0;
#pragma unroll
        for (int i = 0; i < 16; ++i) any |= m[i];
        if (__builtin_expect(any != 0, 0)) {
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            if ((m[i] >> lane) & 1ull) {
              const uint32_t o = obase + (uint32_t)(g * 16 + i) + 1u;  // offset in lane seg
              if (o <= seg_valid) {
                if (cnt < lane_slots) myslots[cnt] = (uint16_t)o;
                ++cnt;
              }
            }
          }
        }
      }
    }
  };
  issue(0, LA);
  __builtin_amdgcn_sched_barrier(0);
  issue(1, LB);
  __builtin_amdgcn_sched_barrier(0);
  compute(0, LA);
  __builtin_amdgcn_sched_barrier(0);
  issue(2, LA);
  __builtin_amdgcn_sched_barrier(0);
  compute(1, LB);
  __builtin_amdgcn_sched_barrier(0);
  issue(3, LB);
  __builtin_amdgcn_sched_barrier(0);
  compute(2, LA);
  __builtin_amdgcn_sched_barrier(0);
  issue(4, LA);
  __builtin_amdgcn_sched_barrier(0);
  compute(3, LB);
  __builtin_amdgcn_sched_barrier(0);
  issue(5, LB);
  __builtin_amdgcn_sched_barrier(0);
  compute(4, LA);
  __builtin_amdgcn_sched_barrier(0);
  compute(5, LB);
  __builtin_amdgcn_sched_barrier(0);
}

// BR rounds per LDS-DMA batch (rows of BR*48 B per lane), NBUF LDS buffers per
// wave: (4,1) = 192 B rows copied to registers at once; (2,2) = 96 B rows,
// double-buffered in LDS.  Both use 96 KiB of staging.
template <int MODE, int VARIANT, int BR, int NBUF>
__global__ __launch_bounds__(kScanThreads, 2) void scan_kernel(ScanArgs a) {
  constexpr int BB = BR * kRound;        // batch bytes per lane
  constexpr int NC = BB / 16;            // 16 B chunks per lane row
  constexpr int NI = kWave * BB / 1024;  // DMA wave instructions per batch
  constexpr int STG = kWave * BB;        // staging bytes per buffer
  static_assert(kTableBytes + kScanWaves * NBUF * STG <= kScanLds, "LDS budget");
  __shared__ __attribute__((aligned(16))) uint8_t lds[kScanLds];

  if (blockIdx.x == 0 && threadIdx.x == 0) {
    *a.overflow_next = 0u;  // parity buffer of the next piece (no reader now)
    if (a.state_init) {     // first piece of a call: reset the chain state
      uint64_t* st = (uint64_t*)a.state_init;
      st[0] = a.init_carry;  // DevState.carry
      st[1] = 0;             // total
      st[2] = 0;             // piece_cuts
      st[3] = 0;             // repaired
      st[4] = 0;             // done, err
      st[5] = 0;             // active, pad
    }
  }
  // ---- replicate {T, rotl16(T)} over 32 lane slots (64 KiB) ----
  for (int e = threadIdx.x; e < 256 * 32; e += kScanThreads) {
    const uint32_t v = kT[e >> 5];
    uint2 t;
    t.x = v;
    t.y = __builtin_amdgcn_alignbit(v, v, 16);  // rotl32(v, 48) == rotl32(v, 16)
    *reinterpret_cast<uint2*>(lds + (e >> 5) * 256 + (e & 31) * 8) = t;
  }
  __syncthreads();

  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t slot8 = (lane & 31u) * 8u;
  uint8_t* stage = lds + kTableBytes + wave * (NBUF * STG);
  const uint32_t stage_lds =
      __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_void_t*)stage);
  const uint32_t S = a.lane_bytes;
  const uint32_t NB = a.batches;  // batches of BR rounds, warm-up round included

  // DMA geometry: instruction i (0..NI-1), lane j -> 16 B unit u = 64i + j of
  // the 64 x BB batch image: row u/NC, physical chunk u%NC.  Rows are stored
  // rotated so that the ds_read_b128 row reads are bank-conflict free: chunk c
  // of lane l lives at l*BB + ((c + rot(l)) % NC)*16 with rot(l) = (l>>2)%12
  // for 12-chunk rows and (l>>4)%6 for 6-chunk rows (exhaustive search over
  // the ds_read_b128 lane groups, DESIGN.md "Scan kernel").
  auto rot_of = [](uint32_t l) -> uint32_t {
    return NC == 12 ? (l >> 2) % 12u : (NC == 6 ? (l >> 4) % 6u : 0u);
  };
  uint32_t dma_off[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const uint32_t u = (uint32_t)i * 64u + lane;
    const uint32_t row = u / (uint32_t)NC, phys = u % (uint32_t)NC;
    const uint32_t c = (phys + (uint32_t)NC - rot_of(row)) % (uint32_t)NC;
    dma_off[i] = row * S + c * 16u;
  }
  const uint32_t rot = rot_of(lane);

  for (uint32_t region = blockIdx.x * kScanWaves + wave; region < a.nregions;
       region += gridDim.x * kScanWaves) {
    const uint64_t rbase = (uint64_t)region * 64u * S;  // piece-relative
    // readable bytes before the region (fewer than 48 only at the chain origin,
    // where the missing window bytes are virtual zeros: those loads fall out of
    // the buffer range and return 0)
    const uint32_t H = (rbase + a.halo >= (uint64_t)kRound) ? (uint32_t)kRound
                                                             : (uint32_t)(rbase + a.halo);
    const uint8_t* rptr = a.base + rbase - H;
    const uint64_t nrec64 = a.len - rbase + H;
    const uint32_t nrec = nrec64 > 0xFFFFFFF0ull ? 0xFFFFFFF0u : (uint32_t)nrec64;
    const uint64_t rp = (uint64_t)(uintptr_t)rptr;
    u32x4 rsrc;
    rsrc.x = __builtin_amdgcn_readfirstlane((uint32_t)rp);
    rsrc.y = __builtin_amdgcn_readfirstlane((uint32_t)(rp >> 32) & 0xFFFFu);  // stride 0
    rsrc.z = __builtin_amdgcn_readfirstlane(nrec);
    rsrc.w = 0x00020000u;
    // batch b covers lane bytes [b*BB - 48, b*BB + BB - 48): buffer offset
    // row*S + b*BB + chunk*16 + (H - 48) (negative wraps -> out of range -> 0)
    const uint32_t hfix = H - (uint32_t)kRound;
    auto issue = [&](uint32_t b) {
      const uint32_t dst = stage_lds + (b % NBUF) * (uint32_t)STG;
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        const uint32_t vo = (b < NB) ? dma_off[i] + b * (uint32_t)BB + hfix : 0xFFFFFFF0u;
        dma16(rsrc, vo, dst + (uint32_t)i * 1024u);
      }
    };

    // lane state
    const uint64_t lane_rel = rbase + (uint64_t)lane * S;  // piece-relative lane base
    uint32_t seg_valid = 0;  // offsets o (p = lane base + o) must stay in the piece
    if (lane_rel < a.len) {
      const uint64_t rem = a.len - lane_rel;
      seg_valid = rem < S ? (uint32_t)rem : S;
    }
    uint32_t cnt = 0;
    const uint64_t gl = (uint64_t)region * 64u + lane;
    uint16_t* myslots = a.lane_slot + gl * a.lane_slots;

    uint32_t h = 0;
    uint32_t ring[48];
#pragma unroll
    for (int k = 0; k < 48; ++k) ring[k] = 0;

#pragma unroll
    for (int q = 0; q < NBUF; ++q) issue((uint32_t)q);
    for (uint32_t b = 0; b < NB; ++b) {
      // batch b has landed once at most NBUF-1 younger batches are pending
      if constexpr (NBUF == 1) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NI * (NBUF - 1)) : "memory");
      }
      const uint8_t* my_row = stage + (b % NBUF) * STG + lane * (uint32_t)BB;
      uint32_t w[BR * 12];  // BR rounds x 12 dwords
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const uint32_t pc = (uint32_t)c + rot < (uint32_t)NC ? (uint32_t)c + rot
                                                              : (uint32_t)c + rot - (uint32_t)NC;
        const uint4 q = *reinterpret_cast<const uint4*>(my_row + pc * 16u);
        w[4 * c] = q.x;
        w[4 * c + 1] = q.y;
        w[4 * c + 2] = q.z;
        w[4 * c + 3] = q.w;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      issue(b + NBUF);  // refill the buffer just copied; lands during hashing
#pragma unroll
      for (int r = 0; r < BR; ++r) {
        const int ri = (int)(b * BR) + r - 1;  // round index, -1 = warm-up
        if (ri < 0) {
          round48<false, MODE, VARIANT>(w + 12 * r, h, ring, lds, slot8, a.tc, lane, 0u, 0u, cnt,
                                        myslots, 0u);
        } else {
          round48<true, MODE, VARIANT>(w + 12 * r, h, ring, lds, slot8, a.tc, lane,
                                       (uint32_t)ri * 48u, seg_valid, cnt, myslots,
                                       a.lane_slots);
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

    // ---- region end: compact the lanes' hits into one sorted region list ----
    // (slots were written by this lane in the rare path; candidates before
    // min_pos -- windows reaching before the chain origin -- are dropped)
    const uint64_t lane_abs = a.piece_abs + lane_rel;
    const uint32_t o_min = lane_abs >= a.min_pos ? 0u : (uint32_t)(a.min_pos - lane_abs);
    const uint32_t n = cnt < a.lane_slots ? cnt : a.lane_slots;
    uint32_t keep = 0;
    for (uint32_t i = 0; i < n; ++i) keep += myslots[i] >= o_min ? 1u : 0u;
    uint32_t incl = keep;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t v = __shfl_up(incl, d, 64);
      if (lane >= (uint32_t)d) incl += v;
    }
    const uint32_t excl = incl - keep;
    uint32_t exact = cnt - (n - keep);
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) exact += __shfl_xor(exact, d, 64);
    uint32_t* rl = a.region_list + (uint64_t)region * a.region_cap;
    for (uint32_t i = 0, j = 0; i < n; ++i) {
      const uint16_t o = myslots[i];
      if (o >= o_min) {
        if (excl + j < a.region_cap) rl[excl + j] = lane * S + o;
        ++j;
      }
    }
    const bool lane_ovf = __ballot(cnt > a.lane_slots) != 0;
    if (lane == 0) {
      a.region_cnt[region] = exact;
      if (lane_ovf || exact > a.region_cap) atomicAdd(a.overflow, 1u);
    }
  }
}

#define DSX_SCAN_INST(BR, NBUF)                                   \
  template __global__ void scan_kernel<0, 0, BR, NBUF>(ScanArgs); \
  template __global__ void scan_kernel<1, 0, BR, NBUF>(ScanArgs); \
  template __global__ void scan_kernel<1, 1, BR, NBUF>(ScanArgs); \
  template __global__ void scan_kernel<1, 3, BR, NBUF>(ScanArgs);
DSX_SCAN_INST(4, 1)
DSX_SCAN_INST(2, 2)

// Exhaustive/ranged check of the GPU boundary predicate against h % d == d-1
// (the plain form of chunker_test.go:190-213).  Diagnostic entry point.
__global__ void boundary_selftest_kernel(TestConsts tc, int mode, uint64_t h0, uint64_t n,
                                         unsigned long long* mismatches) {
  unsigned long long bad = 0;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint32_t h = (uint32_t)(h0 + i);
    const bool want = (h % tc.d) == tc.dm1;
    const bool got = mode == 1 ? is_cand<1>(h, tc) : is_cand<0>(h, tc);
    bad += (want != got);
  }
  if (bad) atomicAdd(mismatches, bad);
}

}  // namespace dsx
