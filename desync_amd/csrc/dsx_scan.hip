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
#include <type_traits>
#include <utility>
#include "dsx_chain.h"
#include "dsx_common.h"
#include "dsx_stitch.h"
#if DSX_DIAG  // the stitch behind the scan (DSX_FUSE): libdsx_diag.so only
#include "dsx_tasks.h"
#endif

namespace dsx {

typedef __attribute__((address_space(3))) void lds_void_t;

// f(integral_constant<int, G>) for G = 0..N-1, unrolled at compile time
template <class F, int... G>
__device__ __forceinline__ void static_for_impl(F&& f, std::integer_sequence<int, G...>) {
  (f(std::integral_constant<int, G>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(f, std::make_integer_sequence<int, N>{});
}
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

// One line batch of scanl_kernel: 8 LDS-DMA wave instructions into 8
// consecutive 1 KiB LDS blocks from lds_base, M0 saved once and stepped by
// 1 KiB (per-instruction dma16 calls saved and restored M0 around each one:
// 8 issue slots per instruction instead of 4).  POL selects the cache policy
// of the loads: 0 default, 1 nt (streamed), 2 sc1, 3 sc0 sc1 nt (DSX_SCAN_NT).
#define DSX_DMA8(POLSTR)                                                              \
  asm volatile("s_mov_b32 %0, m0\n\t"                                                 \
               "s_mov_b32 m0, %9\n\t"                                                 \
               "s_nop 0\n\t"                                                          \
               "buffer_load_dwordx4 %1, %10, 0 offen " POLSTR "lds\n\t"               \
               "s_add_u32 m0, m0, 0x400\n\t"                                          \
               "s_nop 0\n\t"                                                          \
               "buffer_load_dwordx4 %2, %10, 0 offen " POLSTR "lds\n\t"               \
               "s_add_u32 m0, m0, 0x400\n\t"                                          \
               "s_nop 0\n\t"                                                          \
               "buffer_load_dwordx4 %3, %10, 0 offen " POLSTR "lds\n\t"               \
               "s_add_u32 m0, m0, 0x400\n\t"                                          \
               "s_nop 0\n\t"                                                          \
               "buffer_load_dwordx4 %4, %10, 0 offen " POLSTR "lds\n\t"               \
               "s_add_u32 m0, m0, 0x400\n\t"                                          \
               "s_nop 0\n\t"                                                          \
               "buffer_load_dwordx4 %5, %10, 0 offen " POLSTR "lds\n\t"               \
               "s_add_u32 m0, m0, 0x400\n\t"                                          \
               "s_nop 0\n\t"                                                          \
               "buffer_load_dwordx4 %6, %10, 0 offen " POLSTR "lds\n\t"               \
               "s_add_u32 m0, m0, 0x400\n\t"                                          \
               "s_nop 0\n\t"                                                          \
               "buffer_load_dwordx4 %7, %10, 0 offen " POLSTR "lds\n\t"               \
               "s_add_u32 m0, m0, 0x400\n\t"                                          \
               "s_nop 0\n\t"                                                          \
               "buffer_load_dwordx4 %8, %10, 0 offen " POLSTR "lds\n\t"               \
               "s_mov_b32 m0, %0"                                                       \
               : "=&s"(keep)                                                            \
               : "v"(vo[0]), "v"(vo[1]), "v"(vo[2]), "v"(vo[3]), "v"(vo[4]), "v"(vo[5]), \
                 "v"(vo[6]), "v"(vo[7]), "s"(lds_base), "s"(rsrc)                       \
               : "memory", "scc")

template <int POL = 0>
__device__ __forceinline__ void dma16x8(const u32x4& rsrc, const uint32_t (&vo)[8],
                                        uint32_t lds_base) {
  uint32_t keep;
  if constexpr (POL == 1) {
    DSX_DMA8("nt ");
  } else if constexpr (POL == 2) {
    DSX_DMA8("sc1 ");
  } else if constexpr (POL == 3) {
    DSX_DMA8("sc0 sc1 nt ");
  } else {
    DSX_DMA8("");
  }
}
#undef DSX_DMA8

// L2 prefetch: one dword per lane (buffer_load_dword ... lds) into the first
// 256 B of a staging slot that the next DMA overwrites (loads retire in issue
// order, so the real data lands last); the line it touches is in L2/MALL when
// that lane's real DMA reaches it a few batches later.
__device__ __forceinline__ void prefetch4(const u32x4& rsrc, uint32_t voff, uint32_t lds_addr) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "buffer_load_dword %1, %3, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(voff), "s"(lds_addr), "s"(rsrc)
      : "memory");
}

// Realtime (100 MHz) and shader-clock counters, read together; the wait sits
// inside the statement so no counted lgkmcnt of the kernel is disturbed.
__device__ __forceinline__ void stamp_now(uint64_t& rt, uint64_t& cy) {
  asm volatile("s_memrealtime %0\n\ts_memtime %1\n\ts_waitcnt lgkmcnt(0)"
               : "=s"(rt), "=s"(cy)
               :
               : "memory");
}

// A wave's stamp record {start realtime, end realtime, start cycles, end
// cycles} (lane 0, plain stores into the wave slot's own record: a shared
// record updated by atomics from every wave at the launch start serialised
// in the L2 and delayed each wave's first line by ~100 us).  The start pair
// waits in LDS meanwhile, so no register stays live across the scan.
__device__ __forceinline__ void stamp_begin(uint64_t* s_stamp, uint32_t wave) {
  uint64_t rt, cy;
  stamp_now(rt, cy);
  if ((threadIdx.x & 63) == 0) {
    s_stamp[2 * wave] = rt;
    s_stamp[2 * wave + 1] = cy;
  }
}
__device__ __forceinline__ void stamp_end(uint64_t* rec, const uint64_t* s_stamp, uint32_t wave) {
  uint64_t rt, cy;
  stamp_now(rt, cy);
  if ((threadIdx.x & 63) == 0) {
    uint64_t* r = rec + (uint64_t)kStampWords * (blockIdx.x * (blockDim.x >> 6) + wave);
    r[0] = s_stamp[2 * wave];
    r[1] = rt;
    r[2] = s_stamp[2 * wave + 1];
    r[3] = cy;
  }
}

// h % d == d-1 on the GPU.
//   MODE 0: exactly Go's multiply-inverse form (chunker.go:265): v_mul_lo_u32.
//   MODE 1: one fma lands h/d - (d-1)/d in [2^23, 2^24) where float spacing
//           is 1, so the mantissa bits ARE round(q) (magic-number rounding);
//           then the exact check h == q*d + d-1 with a 24-bit mad on those
//           bits (the constant float offset is folded into tc.madc).
//           Exact for 1024 < d < 2^22 (DESIGN.md "Boundary test").
//   MODE 2: t = h*inv + (inv-1) = (h+1)*inv - 1 (mod 2^32); with d = 2^k*dodd
//           a candidate has h+1 = d*m, so t = 2^k*m - 1 < vmax = 2^k*floor(2^32/d).
//           For odd d that is exact (multiply back by d); for even d it is a
//           prefilter with ~2^k/d false positives that mode2_exact re-checks.
//           The scan accumulates min(t) over 8 bytes and tests once: all
//           full- or half-rate VALU, no per-byte compare.
__device__ __forceinline__ uint32_t mode2_t(uint32_t h, const TestConsts& tc) {
  return h * tc.inv + tc.tadd;
}
// The same t with ONE v_mad_u64_u32 (h * inv + tadd as a 64-bit value, low
// half used): 5.0 cycles per wave64 on gfx950 against 4.6 + 2.7 for
// v_mul_lo_u32 + v_add_u32 (tools/ubench_valu.hip).  inv must be in a VGPR
// (one scalar operand per VALU instruction: the addend pair is the SGPR one).
__device__ __forceinline__ uint32_t mode2_t_mad(uint32_t h, uint32_t inv_v, uint64_t tadd64) {
  uint64_t m, carry;
  asm("v_mad_u64_u32 %0, %1, %2, %3, %4" : "=v"(m), "=s"(carry) : "v"(h), "v"(inv_v), "s"(tadd64));
  return (uint32_t)m;
}
__device__ __forceinline__ bool mode2_exact(uint32_t t, const TestConsts& tc) {
  const uint32_t h = (t - tc.tadd) * tc.dodd;  // inv * dodd == 1 (mod 2^32)
  // chunker.go:265's multiply-inverse form (no division: a `%` here costs a
  // magic-number register that spills on the rare path of the scan)
  uint32_t v = (h + 1u) * tc.inv;
  v = __builtin_amdgcn_alignbit(v, v, tc.rot);
  return t < tc.vmax && v - tc.qbias <= tc.qmax;
}

// Bit q of the result = (x[q] <= lim), x[0] in bit 0: a compare into a mask
// and one v_addc (bits = 2 bits + carry, the carry-out back into that mask)
// per value, last value first.  VCC and one SGPR pair in turn, each read at
// least two instructions after its write (a VALU write of an SGPR read by a
// VOP3 needs two wait states on gfx950); lim in a VGPR, so the scan's scarce
// SGPRs are not spilled for it.  The compiler's select + or form costs a
// v_cndmask, half a v_or3 and the same nops per value.
__device__ __forceinline__ uint32_t le_bits8(const uint32_t (&x)[8], uint32_t lim_v) {
  uint32_t b;
  uint64_t m;
  asm volatile(
      "v_cmp_ge_u32_e64 vcc, %[lim], %[x7]\n\t"
      "v_cmp_ge_u32_e64 %[m], %[lim], %[x6]\n\t"
      "s_nop 0\n\t"
      "v_addc_co_u32_e64 %[b], vcc, 0, 0, vcc\n\t"
      "v_cmp_ge_u32_e64 vcc, %[lim], %[x5]\n\t"
      "v_addc_co_u32_e64 %[b], %[m], %[b], %[b], %[m]\n\t"
      "v_cmp_ge_u32_e64 %[m], %[lim], %[x4]\n\t"
      "s_nop 0\n\t"
      "v_addc_co_u32_e64 %[b], vcc, %[b], %[b], vcc\n\t"
      "v_cmp_ge_u32_e64 vcc, %[lim], %[x3]\n\t"
      "v_addc_co_u32_e64 %[b], %[m], %[b], %[b], %[m]\n\t"
      "v_cmp_ge_u32_e64 %[m], %[lim], %[x2]\n\t"
      "s_nop 0\n\t"
      "v_addc_co_u32_e64 %[b], vcc, %[b], %[b], vcc\n\t"
      "v_cmp_ge_u32_e64 vcc, %[lim], %[x1]\n\t"
      "v_addc_co_u32_e64 %[b], %[m], %[b], %[b], %[m]\n\t"
      "v_cmp_ge_u32_e64 %[m], %[lim], %[x0]\n\t"
      "s_nop 0\n\t"
      "v_addc_co_u32_e64 %[b], vcc, %[b], %[b], vcc\n\t"
      "s_nop 0\n\t"
      "v_addc_co_u32_e64 %[b], %[m], %[b], %[b], %[m]"
      : [b] "=&v"(b), [m] "=&s"(m)
      : [lim] "v"(lim_v), [x0] "v"(x[0]), [x1] "v"(x[1]), [x2] "v"(x[2]), [x3] "v"(x[3]),
        [x4] "v"(x[4]), [x5] "v"(x[5]), [x6] "v"(x[6]), [x7] "v"(x[7])
      : "vcc");
  return b;
}

template <int MODE>
__device__ __forceinline__ bool is_cand(uint32_t h, const TestConsts& tc) {
  if constexpr (MODE == 2) {
    return mode2_exact(mode2_t(h, tc), tc);
  } else if constexpr (MODE == 0) {
    uint32_t v = (h + 1u) * tc.inv;
    v = __builtin_amdgcn_alignbit(v, v, tc.rot);
    return v - tc.qbias <= tc.qmax;
  } else {
    const float f = __builtin_fmaf((float)h, tc.rcp, tc.c0);
    const uint32_t bits = __builtin_bit_cast(uint32_t, f);
    return __umul24(bits, tc.d) + tc.madc == h;
  }
}

// LDS address of byte k (0..3) of w in the replicated table: byte << 8 |
// slot8.  Byte 1 already sits at bits 8..15, so (w & 0xFF00) | slot8 is one
// v_bitop3_b32, which gfx950 issues at the full VALU rate (2.7 cycles per wave64
// instruction at 4 waves per SIMD, tools/ubench_valu.hip); v_perm_b32, needed
// to move the other bytes, takes 4.3.
__device__ __forceinline__ uint32_t lookup_addr(uint32_t w, uint32_t slot8, int k) {
  if (k == 1) return __builtin_amdgcn_bitop3_b32(w, 0xFF00u, slot8, 0xEA);  // (a & b) | c
  const uint32_t sel = 0x0C0C0000u | ((4u + (uint32_t)k) << 8);
  return __builtin_amdgcn_perm(w, slot8, sel);
}

// Process one 48-byte round of one lane.  `w` holds the round's bytes,
// `ring[k]` the rotated table value of the byte 48 positions earlier.
// The 48 bytes run as 48/SUB subgroups; the table lookups of subgroup j+1 are
// issued before subgroup j is hashed (explicit software pipeline: the LDS
// latency hides under the previous subgroup's hashing; at most 2*SUB LDS
// reads are in flight, within the 4-bit lgkmcnt).
// VARIANT (diagnostic ablations; results are wrong for VARIANT != 0):
// 1 = no boundary test, 3 = staging only (no hashing), 4 = no staging (the
// kernel hashes zeroed LDS staging: compute ceiling).
// hit entries a lane keeps in registers before spilling to its global slots
// (a lane segment sees ~S/d hits: 0.2 at 8 KiB and d(64K))
constexpr int kHitRegs = 4;

template <int SUB>
__device__ __forceinline__ void lookups_landed(uint64_t (&L)[SUB]) {
  // the empty asm consumes all lookups of a subgroup, so the compiler emits a
  // single s_waitcnt in front of it instead of one per use
  if constexpr (SUB == 8) {
    asm volatile("" : "+v"(L[0]), "+v"(L[1]), "+v"(L[2]), "+v"(L[3]), "+v"(L[4]), "+v"(L[5]),
                 "+v"(L[6]), "+v"(L[7]));
  } else {
    static_assert(SUB == 4, "SUB is 4 or 8");
    asm volatile("" : "+v"(L[0]), "+v"(L[1]), "+v"(L[2]), "+v"(L[3]));
  }
}

// Hash bytes [0, NB) of w (byte i is byte i&3 of w[i>>2]); byte i uses ring
// slot (PH + i) % 48, so spans of any length keep the ring static.
template <int NB, int PH, bool TEST, int MODE, int VARIANT, int SUB>
__device__ __forceinline__ void hash_span(const uint32_t* w, uint32_t& h, uint32_t (&ring)[48],
                                          const uint8_t* __restrict__ tbl, uint32_t slot8,
                                          const TestConsts& tc, uint32_t lane, uint32_t obase,
                                          uint32_t& cnt, uint32_t (&ereg)[kHitRegs],
                                          uint32_t* __restrict__ myslots, uint32_t lane_slots) {
  static_assert(NB % SUB == 0 && NB % 4 == 0, "span shape");
  if constexpr (VARIANT == 3) {
#pragma unroll
    for (int k = 0; k < NB / 4; ++k) h ^= w[k];
    asm volatile("" ::"v"(h));
    return;
  }
  constexpr int NSG = NB / SUB;
  uint64_t L[2][SUB];  // {T[in], rotl16(T[in])} lookups, double-buffered
  auto issue = [&](int j) {
#pragma unroll
    for (int i = 0; i < SUB; ++i) {
      const int k = j * SUB + i;
      const uint32_t sel = 0x0C0C0000u | ((4u + (uint32_t)(k & 3)) << 8);
      const uint32_t addr = __builtin_amdgcn_perm(w[k >> 2], slot8, sel);
      if constexpr (VARIANT == 7)
        L[j & 1][i] = *reinterpret_cast<const uint32_t*>(tbl + addr);
      else
        L[j & 1][i] = *reinterpret_cast<const uint64_t*>(tbl + addr);
    }
  };
  auto compute = [&](int j) {
    lookups_landed<SUB>(L[j & 1]);
    constexpr bool kTest = TEST && (VARIANT == 0 || VARIANT == 4 || VARIANT == 7);
    uint64_t m[SUB];   // MODE 0/1: per-byte ballots
    uint32_t t[SUB];   // MODE 2: prefilter values
#pragma unroll
    for (int i = 0; i < SUB; ++i) {
      const int k = j * SUB + i;
      // rotl1(h) ^ T[in] ^ Trot[out]: one v_alignbit + one three-input
      // v_bitop3_b32 (xor3, gfx950)
      const int rk = (PH + k) % 48;
      // (VARIANT 7: 4-byte table entries, the ring holds T and the outgoing
      // term is rotated here)
      const uint32_t outv = VARIANT == 7 ? __builtin_amdgcn_alignbit(ring[rk], ring[rk], 16) : ring[rk];
      h = __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_alignbit(h, h, 31),
                                      (uint32_t)L[j & 1][i], outv, 0x96);
      ring[rk] = VARIANT == 7 ? (uint32_t)L[j & 1][i] : (uint32_t)(L[j & 1][i] >> 32);
      if constexpr (kTest && MODE == 2) t[i] = mode2_t_mad(h, tc.inv, (uint64_t)tc.tadd);
      else if constexpr (kTest) m[i] = __ballot(is_cand<MODE>(h, tc));
    }
    if constexpr (TEST && !kTest) {
      asm volatile("" ::"v"(h));  // keep the ablated chain live (no DCE)
    } else if constexpr (TEST) {
      // rare path, once per subgroup: a lane with hits appends one entry
      // {hit bits << 16 | offset of the subgroup} (region end expands them)
      bool any;
      if constexpr (MODE == 2) {
        uint32_t mn = t[0];
#pragma unroll
        for (int i = 1; i < SUB; ++i) mn = __builtin_elementwise_min(mn, t[i]);
        any = __ballot(mn < tc.vmax) != 0;
      } else {
        uint64_t a = 0;
#pragma unroll
        for (int i = 0; i < SUB; ++i) a |= m[i];
        any = a != 0;
      }
      if (__builtin_expect(any, 0)) {
        uint32_t bits = 0;
#pragma unroll
        for (int i = 0; i < SUB; ++i) {
          if constexpr (MODE == 2) bits |= (mode2_exact(t[i], tc) ? 1u : 0u) << i;
          else bits |= (uint32_t)((m[i] >> lane) & 1ull) << i;
        }
        if (bits) {
          const uint32_t e = (bits << 16) | (obase + (uint32_t)(j * SUB));
#pragma unroll
          for (int q = 0; q < kHitRegs; ++q) ereg[q] = cnt == (uint32_t)q ? e : ereg[q];
          if (cnt >= (uint32_t)kHitRegs && cnt - kHitRegs < lane_slots) myslots[cnt - kHitRegs] = e;
          ++cnt;
        }
      }
    }
  };
  issue(0);
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int j = 0; j < NSG; ++j) {
    if (j + 1 < NSG) issue(j + 1);
    __builtin_amdgcn_sched_barrier(0);
    compute(j);
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <bool TEST, int MODE, int VARIANT, int SUB>
__device__ __forceinline__ void round48(const uint32_t* w, uint32_t& h, uint32_t (&ring)[48],
                                        const uint8_t* __restrict__ tbl, uint32_t slot8,
                                        const TestConsts& tc, uint32_t lane, uint32_t obase,
                                        uint32_t& cnt, uint32_t (&ereg)[kHitRegs],
                                        uint32_t* __restrict__ myslots, uint32_t lane_slots) {
  hash_span<kRound, 0, TEST, MODE, VARIANT, SUB>(w, h, ring, tbl, slot8, tc, lane, obase, cnt,
                                                 ereg, myslots, lane_slots);
}

// BR rounds per LDS-DMA batch (rows of BR*48 B per lane), NBUF LDS buffers per
// wave, W waves per workgroup (one workgroup per CU: the 64 KiB table is
// per workgroup).  With NBUF == 1 the row is copied to registers before the
// refill is issued, so LDS + registers still double-buffer.
template <int MODE, int VARIANT, int BR, int NBUF, int W, int SUB, bool PF>
__global__ __launch_bounds__(W * kWave, W / 4) void scan_kernel(ScanArgs a) {
  constexpr int BB = BR * kRound;        // batch bytes per lane
  constexpr int NC = BB / 16;            // 16 B chunks per lane row
  constexpr int NI = kWave * BB / 1024;  // DMA wave instructions per batch
  constexpr int STG = kWave * BB;        // staging bytes per buffer
  constexpr int LDSB = kTableBytes + W * NBUF * STG;
  constexpr int NT = W * kWave;
  static_assert(LDSB <= kScanLds, "LDS budget");
  __shared__ __attribute__((aligned(16))) uint8_t lds[LDSB];

  if (blockIdx.x == 0 && threadIdx.x < 8) a.queue_next[32 * threadIdx.x] = 0u;
  if (blockIdx.x == 0 && threadIdx.x == 0 && a.pub_host)  // the previous piece's state
    publish_state(a.pub_host, a.pub_state, a.pub_seq);
  if (blockIdx.x == 0 && threadIdx.x == 8) {  // the task counters of the next slot
    a.queue_next[1] = 0u;
    a.queue_next[2] = 0u;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) *a.overflow_next = 0u;  // (the next piece's slot)
  if constexpr (VARIANT == 4) {  // ablation: staging never filled -> zero bytes
    for (int e = threadIdx.x; e < W * NBUF * STG / 4; e += NT)
      reinterpret_cast<uint32_t*>(lds + kTableBytes)[e] = 0u;
  }
  // ---- replicate {T, rotl16(T)} over 32 lane slots (64 KiB) ----
  for (int e = threadIdx.x; e < 256 * 32; e += NT) {
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
  // test constants: c0 and madc live in VGPRs for the whole kernel (each VALU
  // instruction reads at most one SGPR; otherwise the compiler re-moves them
  // into VGPRs before every use)
  TestConsts tcv = a.tc;
  asm volatile("" : "+v"(tcv.c0));
  asm volatile("" : "+v"(tcv.madc));
  if constexpr (MODE == 2) asm volatile("" : "+v"(tcv.inv));  // v_mad_u64_u32 operand

  // Regions: the first one per wave statically, then from a work queue (the
  // two waves sharing a SIMD progress at different rates: VALU arbitration
  // favours the older one, so static equal shares leave a one-wave tail).
  // The DMA pipeline runs across regions: the last batches of a region issue
  // the first batches of the next one, so a region start pays no HBM latency.
  auto desc_of = [&](uint32_t region, u32x4& rsrc, uint32_t& hfix) {
    const uint64_t rbase = (uint64_t)region * 64u * S;  // piece-relative
    // readable bytes before the region (fewer than 48 only at the chain
    // origin, where the missing window bytes are virtual zeros: those loads
    // fall out of the buffer range and return 0)
    const uint32_t H = (rbase + a.halo >= (uint64_t)kRound) ? (uint32_t)kRound
                                                             : (uint32_t)(rbase + a.halo);
    const uint8_t* rptr = a.base + rbase - H;
    const uint64_t nrec64 = a.len - rbase + H;
    const uint32_t nrec = nrec64 > 0xFFFFFFF0ull ? 0xFFFFFFF0u : (uint32_t)nrec64;
    const uint64_t rp = (uint64_t)(uintptr_t)rptr;
    rsrc.x = __builtin_amdgcn_readfirstlane((uint32_t)rp);
    rsrc.y = __builtin_amdgcn_readfirstlane((uint32_t)(rp >> 32) & 0xFFFFu);  // stride 0
    rsrc.z = __builtin_amdgcn_readfirstlane(nrec);
    rsrc.w = 0x00020000u;
    // batch b covers lane bytes [b*BB - 48, b*BB + BB - 48): buffer offset
    // row*S + b*BB + chunk*16 + (H - 48) (negative wraps -> out of range -> 0)
    hfix = H - (uint32_t)kRound;
  };
  // one batch of DMA into staging slot `slot`; b >= NB issues out-of-range
  // (zero) loads so that every batch is NI instructions for vmcnt counting
  auto issue = [&](const u32x4& rsrc, uint32_t hfix, uint32_t b, uint32_t slot) {
    if constexpr (VARIANT == 4) return;  // ablation: hash stale LDS, no HBM traffic
    const uint32_t dst = stage_lds + slot * (uint32_t)STG;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const uint32_t vo = (b < NB) ? dma_off[i] + b * (uint32_t)BB + hfix : 0xFFFFFFF0u;
      dma16(rsrc, vo, dst + (uint32_t)i * 1024u);
    }
  };

  uint32_t region = blockIdx.x * W + wave;
  if (region >= a.nregions) return;
  u32x4 rsrc;
  uint32_t hfix;
  desc_of(region, rsrc, hfix);
  uint32_t gb = 0;  // batches consumed by this wave (staging slot = gb % NBUF)
  // queue tickets run one region ahead: the ticket naming the successor of
  // region R is drawn when R-1 starts and read when R starts, where the
  // implied vmcnt(0) only waits for R's first batches, issued a batch or two
  // of hashing earlier
  uint32_t ticket = 0;
  if (lane == 0) ticket = atomicAdd(a.queue, 1u);
#pragma unroll
  for (int q = 0; q < NBUF; ++q) issue(rsrc, hfix, (uint32_t)q, (uint32_t)q);

  while (true) {
    const uint32_t next = gridDim.x * W + __builtin_amdgcn_readfirstlane(ticket);
    u32x4 nrsrc = rsrc;
    uint32_t nhfix = 0;
    if (next < a.nregions) {
      if (lane == 0) ticket = atomicAdd(a.queue, 1u);
      desc_of(next, nrsrc, nhfix);
    }

    // lane state
    const uint64_t lane_rel = (uint64_t)region * 64u * S + (uint64_t)lane * S;
    uint32_t seg_valid = 0;  // offsets o (p = lane base + o) must stay in the piece
    if (lane_rel < a.len) {
      const uint64_t rem = a.len - lane_rel;
      seg_valid = rem < S ? (uint32_t)rem : S;
    }
    uint32_t cnt = 0;
    uint32_t ereg[kHitRegs] = {};
    const uint64_t gl = (uint64_t)region * 64u + lane;
    uint32_t* myslots = a.lane_slot + gl * a.lane_slots;

    uint32_t h = 0;
    uint32_t ring[48];
#pragma unroll
    for (int k = 0; k < 48; ++k) ring[k] = 0;

    // one batch; the warm-up round (window fill, no test) is peeled into the
    // first batch so the steady-state loop has no branch around the rounds
    // (a branch lets the compiler hoist all of a round's table addresses)
    auto batch = [&](uint32_t b, auto first) {
      // batch b has landed once at most NBUF-1 younger batches (and the one
      // prefetch issued after b's DMA) are pending
      static_assert(!PF || NBUF > 1, "prefetch needs double buffering");
      if constexpr (NBUF == 1) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      } else {
        asm volatile("s_waitcnt vmcnt(%0)" ::"n"(NI * (NBUF - 1) + (PF ? 1 : 0)) : "memory");
      }
      const uint32_t slot = NBUF == 1 ? 0u : gb % NBUF;
      const uint8_t* my_row = stage + slot * STG + lane * (uint32_t)BB;
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
      if constexpr (PF && VARIANT != 4) {  // always one op per batch (vmcnt counting)
        const uint32_t pb = b + NBUF + a.pf_batches;
        const uint32_t vo = pb < NB ? lane * S + pb * (uint32_t)BB + hfix : 0xFFFFFFF0u;
        prefetch4(rsrc, vo, stage_lds + slot * (uint32_t)STG);
      }
      // refill the slot just copied (lands during hashing): this region's
      // batch b+NBUF, or the next region's first batches
      if (b + NBUF < NB)
        issue(rsrc, hfix, b + NBUF, slot);
      else
        issue(nrsrc, nhfix, next < a.nregions ? b + NBUF - NB : NB, slot);
      ++gb;
#pragma unroll
      for (int r = 0; r < BR; ++r) {
        if (decltype(first)::value && r == 0) {
          round48<false, MODE, VARIANT, SUB>(w, h, ring, lds, slot8, tcv, lane, 0u, cnt, ereg,
                                             myslots, 0u);
        } else {
          const uint32_t ri = b * (uint32_t)BR + (uint32_t)r - 1u;  // round index
          round48<true, MODE, VARIANT, SUB>(w + 12 * r, h, ring, lds, slot8, tcv, lane, ri * 48u,
                                            cnt, ereg, myslots, a.lane_slots);
        }
      }
    };
    batch(0u, std::true_type{});
    for (uint32_t b = 1; b < NB; ++b) batch(b, std::false_type{});

    // ---- region end: compact the lanes' hits into one sorted region list ----
    // (entries were written by this lane in the rare path; candidates before
    // min_pos -- windows reaching before the chain origin -- are dropped)
    const uint64_t lane_abs = a.piece_abs + lane_rel;
    const uint32_t o_min = lane_abs >= a.min_pos ? 0u : (uint32_t)(a.min_pos - lane_abs);
    const uint32_t n = cnt < a.lane_slots + kHitRegs ? cnt : a.lane_slots + kHitRegs;
    const bool spilled = __ballot(cnt > (uint32_t)kHitRegs) != 0;  // rare: global reads
    auto for_each_hit = [&](auto&& f) {
      auto expand = [&](uint32_t e) {
        const uint32_t base = e & 0xFFFFu;
        for (uint32_t bits = e >> 16; bits; bits &= bits - 1u) {
          const uint32_t o = base + (uint32_t)__builtin_ctz(bits) + 1u;  // offset in lane seg
          if (o >= o_min && o <= seg_valid) f(o);
        }
      };
#pragma unroll
      for (int q = 0; q < kHitRegs; ++q)
        if ((uint32_t)q < n) expand(ereg[q]);
      if (spilled)
        for (uint32_t i = kHitRegs; i < n; ++i) expand(myslots[i - kHitRegs]);
    };
    uint32_t keep = 0;
    for_each_hit([&](uint32_t) { ++keep; });
    uint32_t incl = keep;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t v = __shfl_up(incl, d, 64);
      if (lane >= (uint32_t)d) incl += v;
    }
    const uint32_t excl = incl - keep;
    uint32_t exact = keep;  // (a lane overflow below sends the piece to the dense path)
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) exact += __shfl_xor(exact, d, 64);
    uint32_t* rl = a.region_list + (uint64_t)region * a.region_cap;
    uint32_t j = 0;
    for_each_hit([&](uint32_t o) {
      if (excl + j < a.region_cap) rl[excl + j] = lane * S + o;
      ++j;
    });
    const bool lane_ovf = __ballot(cnt > a.lane_slots + kHitRegs) != 0;
    if (lane == 0) {
      a.region_cnt[region] = exact;
      if (lane_ovf || exact > a.region_cap) atomicAdd(a.overflow, 1u);
    }
    if (next >= a.nregions) break;
    region = next;
    rsrc = nrsrc;
    hfix = nhfix;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // retire the trailing zero loads
}

// The product library holds the results-exact kernels (VARIANT 0) of the
// default configurations; the diagnostic build (make diag -> libdsx_diag.so,
// -DDSX_DIAG=1, loaded through DSX_LIB_PATH by tools/) adds the ablations and
// the other geometries.
#define DSX_SCAN_INST(BR, NBUF, W, SUB, PF)                                   \
  template __global__ void scan_kernel<0, 0, BR, NBUF, W, SUB, PF>(ScanArgs); \
  template __global__ void scan_kernel<1, 0, BR, NBUF, W, SUB, PF>(ScanArgs); \
  template __global__ void scan_kernel<2, 0, BR, NBUF, W, SUB, PF>(ScanArgs);
#define DSX_SCAN_INST_DIAG(BR, NBUF, W, SUB, PF)                              \
  template __global__ void scan_kernel<2, 1, BR, NBUF, W, SUB, PF>(ScanArgs); \
  template __global__ void scan_kernel<2, 3, BR, NBUF, W, SUB, PF>(ScanArgs); \
  template __global__ void scan_kernel<2, 4, BR, NBUF, W, SUB, PF>(ScanArgs);
DSX_SCAN_INST(2, 2, 8, 8, false)
#if DSX_DIAG
DSX_SCAN_INST(2, 2, 8, 8, true)  // DSX_PREFETCH (L2 prefetch: measured slower)
DSX_SCAN_INST_DIAG(2, 2, 8, 8, false)
DSX_SCAN_INST_DIAG(2, 2, 8, 8, true)
#define DSX_SCAN_INST_ALL(BR, NBUF, W, SUB, PF) \
  DSX_SCAN_INST(BR, NBUF, W, SUB, PF) DSX_SCAN_INST_DIAG(BR, NBUF, W, SUB, PF)
DSX_SCAN_INST_ALL(1, 2, 12, 4, false)
DSX_SCAN_INST_ALL(1, 2, 16, 4, false)
DSX_SCAN_INST_ALL(2, 1, 12, 8, false)
DSX_SCAN_INST_ALL(2, 1, 8, 8, false)
DSX_SCAN_INST_ALL(2, 1, 16, 4, false)
#endif

// ---------------------------------------------------------------------------
// scanl_kernel -- the line-aligned scan (default path).
//
// Same per-byte work as scan_kernel, but every HBM request is a whole 128-B
// line fetched once: lane segments of S = 384*m bytes start on line
// boundaries of the grid base - delta, and each DMA batch is ONE line per
// lane (8 wave instructions, each 8 lanes x 128 B = 8 whole lines).
// scan_kernel's 96-B rows straddle lines, and 18 % of those lines were
// fetched twice from HBM (TCC_EA0_RDREQ_128B = 1.18 x the input bytes,
// tools/pmc_tcc.sh): the L2 dropped a half-used line before the row next to
// it arrived.  The warm-up is the last 48 bytes of the line before the
// segment -- for lane 0 of a region only: lanes 1..63 hash their first 48
// positions from a zero window and drop them, and the lane before tests them
// at the end of its own segment from 48 bytes they leave in LDS (the
// handoff; HBM reads 1.018 -> 1.0004 x the input, profiles/r04z, r04ab).
// One LDS staging line per lane (8 KiB per
// wave): a batch is copied to registers, then the next batch's DMA is issued
// at once, so it lands while this one is hashed.  A batch of 128 B is three
// ring phases apart from the next (128 = 2*48 + 32), so the steady-state loop
// runs three batches with phases 0, 32, 16.
// ---------------------------------------------------------------------------
//
// FUSE: the kernel also runs the stitch tasks of earlier queued calls
// (*a.tasks, dsx_tasks.h) on wave slots with no region to hash: the waves
// the grid has beyond the regions at once, the others once the regions run
// out ("stitch behind the scan").
// ---------------------------------------------------------------------------
template <int MODE, int VARIANT, int W, int SUB, int D, bool FUSE, bool TWO>
__global__ __launch_bounds__(W * kWave, W / 4) void scanl_kernel(ScanArgs a) {
  constexpr int NC = kLine / 16;             // 16-B chunks per lane row
  constexpr int NI = kWave * kLine / 1024;   // DMA wave instructions per batch
  constexpr int STG = kWave * kLine;         // staging bytes per wave
  constexpr int LDSB = kTableBytes + W * STG;
  constexpr int NT = W * kWave;
  // with 12 waves the table and the staging lines fill the LDS: no room for
  // the SIMD-partner balancing counters (three waves per SIMD need it less)
  constexpr bool kBal = LDSB + 4 * W <= kScanLds;
  static_assert(LDSB <= kScanLds, "LDS budget");
  __shared__ __attribute__((aligned(16))) uint8_t lds[LDSB];
  __shared__ uint32_t s_prog[kBal ? W : 1];  // batches hashed per wave (SIMD partner balancing)
  // warm-up handoff: each lane's first 48 segment bytes, which the lane before
  // it hashes and tests at the end of its own segment (lanes 1..63 read no
  // warm-up line: 128 B of HBM read per lane segment saved)
  constexpr int kHandoff = 48;
  static_assert(LDSB + (int)sizeof(uint32_t) * (W + 256) + W * kWave * kHandoff + 16 * W <= kScanLds,
                "LDS budget with the handoff");
  __shared__ __attribute__((aligned(16))) uint8_t s_hand[W * kWave * kHandoff];
  __shared__ __attribute__((aligned(16))) uint32_t s_tab[256];  // the table, landed by LDS-DMA
  // trace: the wave's first instruction (before the table fill)
  const uint64_t t_entry = VARIANT == 5 ? __builtin_amdgcn_s_memtime()
                                        : (a.trace ? __builtin_amdgcn_s_memrealtime() : 0);
  // in-kernel stamps of the launch (dsx_stamps_begin): every wave's first
  // instruction here, its last one at the end of its regions
  __shared__ uint64_t s_stamp[2 * W];
  if (a.stamp) stamp_begin(s_stamp, __builtin_amdgcn_readfirstlane(threadIdx.x >> 6));

  if (blockIdx.x == 0 && threadIdx.x < 8) a.queue_next[32 * threadIdx.x] = 0u;
  if (blockIdx.x == 0 && threadIdx.x == 0 && a.pub_host)  // the previous piece's state
    publish_state(a.pub_host, a.pub_state, a.pub_seq);
  if (blockIdx.x == 0 && threadIdx.x == 8) {  // the task counters of the next slot
    a.queue_next[1] = 0u;
    a.queue_next[2] = 0u;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) *a.overflow_next = 0u;  // (the next piece's slot)
  if constexpr (VARIANT == 4) {
    for (int e = threadIdx.x; e < W * STG / 4; e += NT)
      reinterpret_cast<uint32_t*>(lds + kTableBytes)[e] = 0u;
  }

  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t lane = threadIdx.x & 63;
  // (VARIANT 7: 64 slots of 4 B per byte value instead of 32 of 8 B)
  const uint32_t slot8 = (VARIANT == 7 || VARIANT == 10) ? lane * 4u : (lane & 31u) * 8u;
  uint8_t* stage = lds + kTableBytes + wave * STG;
  // Waves w and w + W/2 share a SIMD (waves are placed on the SIMDs
  // cyclically).  VALU issue favours the older wave, so left alone the
  // younger one finishes ~25 % later and the SIMD ends the scan with one wave
  // (tools/scan_trace.py).  Each batch, the wave that has hashed fewer
  // batches than its partner takes issue priority.
  const uint32_t partner = (wave + (uint32_t)W / 2u) % (uint32_t)W;
  uint32_t my_prog = 0;
  const uint32_t stage_lds =
      __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_void_t*)stage);
  // Two region sizes (a.lane_bytes2 != 0): regions [0, nbig) have lane
  // segments of S1 bytes, the tail regions after them S2 < S1, so the waves
  // that drain the work queue last hold small regions (a shorter tail).
  // (TWO: a separate instantiation, since the second size's state costs the
  // one-size loop SGPR spills)
  auto region_base = [&](uint32_t r) -> uint64_t {  // grid-relative start of region r
    if constexpr (TWO) {
      return r <= a.nbig
                 ? (uint64_t)r * 64u * a.lane_bytes
                 : ((uint64_t)a.nbig * a.lane_bytes + (uint64_t)(r - a.nbig) * a.lane_bytes2) * 64u;
    } else {
      return (uint64_t)r * 64u * a.lane_bytes;
    }
  };
  auto is_tail = [&](uint32_t r) -> bool {
    if constexpr (TWO) return r >= a.nbig;
    else return false;
  };

  // DMA geometry: instruction i, lane j -> 16-B unit u = 64i + j of the wave's
  // 64 x 128 B image: row u/8, physical chunk u%8.  Row r stores logical
  // chunk c at physical (c + rot(r)) % 8 with rot(r) = (r >> 1) % 8, which
  // makes the ds_read_b128 row reads conflict-free (each 16-lane group covers
  // the 16 distinct {row parity, chunk} bank quads).
  // row = 8i + (lane >> 3) and rot(row) = (4i + (lane >> 4)) % 8 depends on
  // i only through its parity: two per-lane bases, the rest is scalar
  static_assert(NC == 8 && NI == 8, "line DMA geometry");
  auto dbase_of = [&](uint32_t S, uint32_t parity) -> uint32_t {
    const uint32_t dphys = lane & 7u;
    return (lane >> 3) * S + ((dphys + 8u - ((4u * parity + (lane >> 4)) & 7u)) & 7u) * 16u;
  };
  // the current region's geometry (wave-uniform; changes at most once, when
  // the wave moves on to the tail regions)
  // S = 3*128*M; 3M+1 lines per lane (warm-up line).  Constant in the one-size
  // instantiation (left mutable there the allocator spilled 10 more SGPRs)
  using mut_u32 = std::conditional_t<TWO, uint32_t, const uint32_t>;
  mut_u32 S = a.lane_bytes, M = a.batches;
  mut_u32 dbase0 = dbase_of(a.lane_bytes, 0u), dbase1 = dbase_of(a.lane_bytes, 1u);
  const uint32_t rot = (lane >> 1) % (uint32_t)NC;
  TestConsts tcv = a.tc;
  asm volatile("" : "+v"(tcv.c0));
  asm volatile("" : "+v"(tcv.madc));
  // the rare path's constants (le_bits8), in VGPRs: the kernel has no SGPRs
  // to spare and spills whatever it keeps in them across the loop
  uint32_t qlim_v = tcv.qmax + tcv.qbias, rot_v = tcv.rot;
  asm volatile("" : "+v"(qlim_v));
  asm volatile("" : "+v"(rot_v));

  // Region r's descriptor starts at its warm-up line (grid-relative
  // r*RB - 128), shifted by shift0 for region 0 so it never precedes the
  // readable bytes; offsets below the base wrap out of range and read 0.
  auto desc_of = [&](uint32_t region, u32x4& rsrc, uint32_t& sh) {
    sh = region == 0 ? a.shift0 : 0u;
    const int64_t rel = (int64_t)region_base(region) - (int64_t)a.delta - kLine + (int64_t)sh;
    const uint64_t rp = (uint64_t)(uintptr_t)(a.base + rel);
    const uint64_t nrec64 = (uint64_t)((int64_t)a.len - rel);
    const uint32_t nrec = nrec64 > 0xFFFFFFF0ull ? 0xFFFFFFF0u : (uint32_t)nrec64;
    rsrc.x = __builtin_amdgcn_readfirstlane((uint32_t)rp);
    rsrc.y = __builtin_amdgcn_readfirstlane((uint32_t)(rp >> 32) & 0xFFFFu);
    rsrc.z = __builtin_amdgcn_readfirstlane(nrec);
    rsrc.w = 0x00020000u;
  };
  // batch b of every lane (b = 0: warm-up line); b >= NB: out-of-range loads
  // (zeros) so every batch is NI instructions
  // (issue_in: a line of a region with lane segments rS and DMA bases d0/d1,
  // or zero loads if !ok -- the first line of the first tail region, TWO)
  auto issue_in = [&](const u32x4& rsrc, uint32_t sh, uint32_t b, bool ok, uint32_t rS,
                      uint32_t d0, uint32_t d1) {
    if constexpr (VARIANT == 4) return;
    const uint32_t sb = b * (uint32_t)kLine - sh;  // scalar part
    uint32_t vo[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      uint32_t ssum = (uint32_t)i * 8u * rS + sb;
      asm volatile("" : "+s"(ssum));
      // (a warm-up line, b = 0: row 0 only = instruction 0, DMA lanes 0-7)
      vo[i] = ok && (b != 0u || (i == 0 && lane < 8u)) ? ((i & 1) ? d1 : d0) + ssum : 0xFFFFFFF0u;
    }
    switch (a.nt_loads) {
      case 1: dma16x8<1>(rsrc, vo, stage_lds); break;
      case 2: dma16x8<2>(rsrc, vo, stage_lds); break;
      case 3: dma16x8<3>(rsrc, vo, stage_lds); break;
      default: dma16x8<0>(rsrc, vo, stage_lds); break;
    }
  };
  auto issue = [&](const u32x4& rsrc, uint32_t sh, uint32_t b) {
    if constexpr (VARIANT == 4) return;
    const uint32_t sb = b * (uint32_t)kLine - sh;  // scalar part
    uint32_t vo[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      // the opaque scalar sum keeps LICM from hoisting 8 per-lane offsets
      uint32_t ssum = (uint32_t)i * 8u * S + sb;
      asm volatile("" : "+s"(ssum));
      vo[i] = (b < 3u * M + 1u) ? ((i & 1) ? dbase1 : dbase0) + ssum : 0xFFFFFFF0u;
    }
    switch (a.nt_loads) {
      case 1: dma16x8<1>(rsrc, vo, stage_lds); break;
      case 2: dma16x8<2>(rsrc, vo, stage_lds); break;
      case 3: dma16x8<3>(rsrc, vo, stage_lds); break;
      default: dma16x8<0>(rsrc, vo, stage_lds); break;
    }
  };

  // a region's warm-up line (batch 0) for row 0 only; the other lanes take
  // their window from the lane before (the handoff).  Kept apart from issue(),
  // which runs at every line of the trip loop.
  auto issue_warm = [&](const u32x4& rsrc, uint32_t sh, bool ok) {
    if constexpr (VARIANT == 4) return;
    uint32_t vo[NI];
#pragma unroll
    for (int i = 0; i < NI; ++i) vo[i] = 0xFFFFFFF0u;
    vo[0] = ok && lane < 8u ? dbase0 - sh : 0xFFFFFFF0u;
    switch (a.nt_loads) {
      case 1: dma16x8<1>(rsrc, vo, stage_lds); break;
      case 2: dma16x8<2>(rsrc, vo, stage_lds); break;
      case 3: dma16x8<3>(rsrc, vo, stage_lds); break;
      default: dma16x8<0>(rsrc, vo, stage_lds); break;
    }
  };

  // wave-major first regions: when regions do not fill every wave slot, the
  // idle slots are single waves spread over many CUs (whose partner wave then
  // runs alone, faster) instead of whole CUs at the end of the grid
  // wave_major 2 (stitch behind): the waves of SIMD 3 (3 and W/2+3) come last,
  // in pairs, so the slots without a region are whole SIMDs at the end of
  // the grid and the stitch tasks run there beside no scan wave
  uint32_t region;
  if (a.wave_major == 2 && W == 8) {
    region = (wave & 3u) == 3u ? 6u * gridDim.x + 2u * blockIdx.x + (wave >> 2)
                               : (wave - (wave > 3u ? 1u : 0u)) * gridDim.x + blockIdx.x;
  } else {
    region = a.wave_major ? wave * gridDim.x + blockIdx.x : blockIdx.x * W + wave;
  }
  const bool live = region < a.nregions;
  // The first line's DMA is issued before the table fill, so its HBM latency
  // overlaps the fill instead of following it.
  // The 1 KiB table reaches LDS by one LDS-DMA instruction of wave 0, issued
  // before the first line's DMA, so waiting for it (vmcnt(8)) does not wait
  // for the line: the fill overlaps the line's HBM latency.  (A plain load's
  // use gets a vmcnt(0) from the compiler, which also waits for the line; a
  // load in inline asm returns into a register the compiler may copy before
  // the wait -- it did, and the copy read a stale value.)
  static_assert(NT % 256 == 0, "table fill shape");
  if (wave == 0) {
    const uint64_t tp = (uint64_t)(uintptr_t)&kT[0];
    u32x4 trs;
    trs.x = __builtin_amdgcn_readfirstlane((uint32_t)tp);
    trs.y = __builtin_amdgcn_readfirstlane((uint32_t)(tp >> 32) & 0xFFFFu);
    trs.z = 1024u;
    trs.w = 0x00020000u;
    dma16(trs, lane * 16u,
          __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)(lds_void_t*)s_tab));
  }
  u32x4 rsrc = {0u, 0u, 0u, 0u};
  uint32_t sh = 0;
  if (live) {
    if constexpr (TWO) {
      if (is_tail(region)) {  // (a grid with more wave slots than big regions)
        S = a.lane_bytes2;
        M = a.batches2;
        dbase0 = dbase_of(S, 0u);
        dbase1 = dbase_of(S, 1u);
      }
    }
    desc_of(region, rsrc, sh);
    issue_warm(rsrc, sh, true);
  }
  if (wave == 0) {
    if (live && VARIANT != 4)
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  __syncthreads();
  {
    constexpr int TPV = NT / 256;  // threads per byte value
    const uint32_t v = threadIdx.x & 255u;
    const uint32_t tv = s_tab[v];
    uint2 t;
    t.x = tv;
    t.y = __builtin_amdgcn_alignbit(tv, tv, 16);
    if constexpr (VARIANT == 7 || VARIANT == 10) {
#pragma unroll
      for (int k = 0; k < (64 + TPV - 1) / TPV; ++k) {
        const uint32_t slot = (threadIdx.x >> 8) + (uint32_t)(k * TPV);
        if (slot < 64u) *reinterpret_cast<uint32_t*>(lds + v * 256u + slot * 4u) = tv;
      }
    } else {
#pragma unroll
      for (int k = 0; k < (32 + TPV - 1) / TPV; ++k) {
        const uint32_t slot = (threadIdx.x >> 8) + (uint32_t)(k * TPV);
        if (slot < 32u) *reinterpret_cast<uint2*>(lds + v * 256u + slot * 8u) = t;
      }
    }
  }
  if (kBal && threadIdx.x < W) s_prog[threadIdx.x] = 0u;
  __syncthreads();
  // (trace: 6 words per wave slot after the scan's records)
  [[maybe_unused]] uint64_t* const task_tr =
      a.trace ? a.trace + (uint64_t)kScanTraceWords * gridDim.x * W + 6ull * (blockIdx.x * W + wave)
              : nullptr;
  if (!live) {
    if (a.stamp) stamp_end(a.stamp, s_stamp, wave);
#if DSX_DIAG
    if constexpr (FUSE) run_tasks(a.tasks, reinterpret_cast<uint32_t*>(stage), lane, task_tr);
#endif
    return;
  }
  // VARIANT 5 (diagnostic, same results): the trace records shader-clock
  // cycles from start to end and those spent waiting for the line DMA
  const uint64_t t_start = VARIANT == 5 ? __builtin_amdgcn_s_memtime()
                                        : (a.trace ? __builtin_amdgcn_s_memrealtime() : 0);
  uint64_t vm_wait = 0, copy_wait = 0, dma_issue = 0;
  uint32_t nreg_done = 0;
  // trace: shader-clock cycles from the end of a region's hashing to the
  // start of the next region, and waited at the first two fetches of a
  // region other than the first
  uint64_t re_cyc = 0, rs_wait = 0;

  // Work queue for the regions beyond the first pass (region nstatic + 8t + x
  // is ticket t of counter x).  Each wave draws from its XCD's counter and
  // moves on to the next counter once one runs dry; it draws its successor's
  // ticket in the middle of a region and decodes it at the region's last
  // line, so the atomic's latency is hidden.  2048 waves drawing from ONE counter at
  // the launch serialised for ~20 us (profiles/r03/trace_prologue.txt); a
  // piece with no more regions than wave slots draws nothing.
  const uint32_t nstatic = gridDim.x * W;
  bool draw = a.nregions > nstatic;
  uint32_t qx = 0, qdry = 0;  // current counter, counters found empty
  if (draw) {
    uint32_t xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc));
    qx = xcc & 7u;
  }
  uint32_t ticket = 0;

  while (true) {
    uint32_t next = a.nregions;
    u32x4 nrsrc = rsrc;
    uint32_t nsh = 0;
    // the successor region (called once, at the region's last line)
    auto resolve_next = [&]() __attribute__((always_inline)) {
      if (!draw) return;
      uint32_t rq = 0;  // lane 0: counter | dry counters << 8
      uint32_t rr = a.nregions, qq = qx, dry = qdry;
      if (lane == 0) {  // (lane 0 holds the tickets)
        uint64_t r = nstatic + 8ull * ticket + qq;
        while (r >= a.nregions && ++dry < 8u) {  // this counter ran dry: the next one
          qq = (qq + 1u) & 7u;
          r = nstatic + 8ull * atomicAdd(a.queue + 32u * qq, 1u) + qq;
        }
        rr = r < a.nregions ? (uint32_t)r : a.nregions;
        rq = qq | (dry << 8);
      }
      next = __builtin_amdgcn_readfirstlane(rr);
      rq = __builtin_amdgcn_readfirstlane(rq);
      qx = rq & 0xFFu;
      qdry = rq >> 8;
      if (next >= a.nregions) {
        draw = false;
        return;
      }
      desc_of(next, nrsrc, nsh);
    };

    uint32_t cnt = 0;
    uint32_t ereg[kHitRegs] = {};
    const uint64_t gl = (uint64_t)region * 64u + lane;
    uint32_t* myslots = a.lane_slot + gl * a.lane_slots;
    // MODE 2 keeps ~h: rotl1(~x) == ~rotl1(x), so ~h follows the same
    // recurrence from ~0, and t + 1 = (h+1)*inv = (~h)*ninv (make_tc)
    uint32_t h = MODE == 2 ? ~0u : 0u;
    uint32_t ring[48];
#pragma unroll
    for (int k = 0; k < 48; ++k) ring[k] = 0;
    uint32_t w[NC * 4];

    // wait for batch b, copy this lane's row to registers, issue batch b+1
    // (or the next region's warm-up line) into the freed staging line
    auto fetch = [&](uint32_t b) __attribute__((always_inline)) {
      ++my_prog;
      uint32_t their = my_prog;
      if constexpr (kBal) {
        s_prog[wave] = my_prog;
        their = s_prog[partner];
      }
      uint64_t tw = 0;
      const bool rs = a.trace && b <= 1u && nreg_done > 0;
      if (VARIANT == 5 || rs) tw = __builtin_amdgcn_s_memtime();
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      uint64_t tw1 = 0;
      if constexpr (VARIANT == 5) {
        tw1 = __builtin_amdgcn_s_memtime();
        vm_wait += tw1 - tw;
      }
      if (rs) rs_wait += __builtin_amdgcn_s_memtime() - tw;
      const uint8_t* my_row = stage + lane * (uint32_t)kLine;
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const uint32_t pc = ((uint32_t)c + rot) % (uint32_t)NC;
        const uint4 q = *reinterpret_cast<const uint4*>(my_row + pc * 16u);
        w[4 * c] = q.x;
        w[4 * c + 1] = q.y;
        w[4 * c + 2] = q.z;
        w[4 * c + 3] = q.w;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      uint64_t tw2 = 0;
      if constexpr (VARIANT == 5) {
        tw2 = __builtin_amdgcn_s_memtime();
        copy_wait += tw2 - tw1;
      }
      if (__builtin_amdgcn_readfirstlane(their) < my_prog)
        __builtin_amdgcn_s_setprio(0);
      else
        __builtin_amdgcn_s_setprio(1);
      if (b + 1u < 3u * M + 1u) {
        issue(rsrc, sh, b + 1u);
      } else {
        resolve_next();
        const uint32_t nS = (TWO && next < a.nregions)
                                ? (is_tail(next) ? a.lane_bytes2 : a.lane_bytes) : S;
        if (TWO && nS != S) {
          // the next region has the other lane geometry (the first tail region,
          // or a big one stolen from a slower XCD's counter after it)
          issue_in(nrsrc, nsh, 0u, true, nS, dbase_of(nS, 0u), dbase_of(nS, 1u));
        } else {
          issue_warm(nrsrc, nsh, next < a.nregions);
        }
      }
      if constexpr (VARIANT == 5) dma_issue += __builtin_amdgcn_s_memtime() - tw2;
    };
    fetch(0u);
    // warm-up: the last 48 bytes before the segment fill the window (no test)
    hash_span<kRound, 0, false, MODE, VARIANT, SUB>(w + 20, h, ring, lds, slot8, tcv, lane, 0u,
                                                    cnt, ereg, myslots, 0u);
    // Steady state: trips of 3 lines (384 B = 8 windows, so ring slots are
    // static) as 48 subgroups of 8 bytes.  The table lookups run one subgroup
    // ahead, ACROSS line boundaries: once the last subgroup of a line has
    // issued its lookups, w is free, so the next line is copied in and its
    // first lookups are issued before that last subgroup is hashed.
    // D = lookup distance in subgroups (D + 1 lookup buffers; 48 % (D+1) == 0
    // keeps the buffer index static across trips)
    static_assert(SUB == 8, "trip pipeline is written for 8-byte subgroups");
    static_assert(D >= 1 && D <= 15 && 48 % (D + 1) == 0, "lookup distance");
    constexpr int NL = D + 1;
    uint64_t L[NL][8];
    auto issue_sub = [&](auto gc) __attribute__((always_inline)) {
      constexpr int g = decltype(gc)::value;
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int k = (g % 16) * 8 + q;  // byte within the line
        if constexpr (VARIANT == 7 || VARIANT == 10)
          L[g % NL][q] = *reinterpret_cast<const uint32_t*>(lds + lookup_addr(w[k >> 2], slot8, k & 3));
        else
          L[g % NL][q] = *reinterpret_cast<const uint64_t*>(lds + lookup_addr(w[k >> 2], slot8, k & 3));
      }
    };
    auto compute_sub = [&](auto gc, uint32_t o0) __attribute__((always_inline)) {
      constexpr int g = decltype(gc)::value;
      if constexpr (VARIANT == 3) {  // staging-only ablation: keep the data live
        h ^= w[(g % 16) * 2] ^ w[(g % 16) * 2 + 1];
        asm volatile("" ::"v"(h));
        return;
      }
      lookups_landed<8>(L[g % NL]);
      // (energy ablations, wrong results: 8 = no multiply (t = h), 9 = the 8 t
      // values OR-ed with full-rate v_bitop3 instead of the v_min3 tree, 10 =
      // 4-byte lookups, the ring takes T itself)
      // (VARIANT 6 hashes its trips in compute_il, but the handoff extension
      // after them runs here and must test too: tests/test_gpu_variants.py)
      constexpr bool kTest = VARIANT == 0 || VARIANT == 4 || VARIANT == 5 || VARIANT == 6 ||
                             VARIANT == 7 || VARIANT == 8 || VARIANT == 9 || VARIANT == 10;
      uint32_t t[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int rk = (g * 8 + q) % 48;
        const uint32_t outv =
            VARIANT == 7 ? __builtin_amdgcn_alignbit(ring[rk], ring[rk], 16) : ring[rk];
        h = __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_alignbit(h, h, 31),
                                        (uint32_t)L[g % NL][q], outv, 0x96);
        ring[rk] = (VARIANT == 7 || VARIANT == 10) ? (uint32_t)L[g % NL][q]
                                                   : (uint32_t)(L[g % NL][q] >> 32);
        if constexpr (kTest) {
          if constexpr (VARIANT == 8) t[q] = h;
          else if constexpr (MODE == 2) t[q] = h * tcv.ninv;  // t + 1: one v_mul_lo_u32
          else t[q] = is_cand<MODE>(h, tcv) ? 0u : 0xFFFFFFFFu;
        }
      }
      if constexpr (!kTest) {
        asm volatile("" ::"v"(h));
      } else {
        const uint32_t thr = MODE == 2 ? tcv.vmax1 : 1u;
        uint32_t mn = t[0];
        if constexpr (VARIANT == 9) {
          mn = __builtin_amdgcn_bitop3_b32(t[0], t[1], t[2], 0xFE);  // a | b | c
          const uint32_t m2 = __builtin_amdgcn_bitop3_b32(t[3], t[4], t[5], 0xFE);
          mn = __builtin_amdgcn_bitop3_b32(mn, m2, t[6], 0xFE) | t[7];
        } else {
#pragma unroll
          for (int q = 1; q < 8; ++q) mn = __builtin_elementwise_min(mn, t[q]);
        }
        if (__builtin_expect(__ballot(mn < thr) != 0, 0)) {
          uint32_t bits = 0;
          if (MODE == 2 && VARIANT == 0 && __builtin_expect(__ballot(mn == 0u) == 0, 1)) {
            // no t == 0 in the wave (t = 0 is h = 2^32 - 1, 2^-32 a byte):
            // then x - qBias <= qMax is x <= qMax + qBias, with x = t (odd d)
            // or rotl(t, -k) (even d), both >= 1, so qBias in {0, 1} cannot
            // wrap -- one compare and one add-carry per byte
            if (tcv.rot == 0) {
              bits = le_bits8(t, qlim_v);
            } else {
              uint32_t x[8];
#pragma unroll
              for (int q = 0; q < 8; ++q) x[q] = __builtin_amdgcn_alignbit(t[q], t[q], rot_v);
              bits = le_bits8(x, qlim_v);
            }
          } else if (MODE == 2 && tcv.rot == 0) {
            // odd d (k = 0, the default parameters): t = (h+1)*inv here, and
            // chunker.go:265's test is t - qBias <= qMax with no rotate
#pragma unroll
            for (int q = 0; q < 8; ++q) bits |= (t[q] - tcv.qbias <= tcv.qmax ? 1u : 0u) << q;
          } else if (MODE == 2) {
            // even d = 2^k * dodd: chunker.go:265's test on the same product,
            // rotl((h+1)*inv, -k) - qBias <= qMax -- one v_alignbit more
            // per byte instead of mode2_exact's two multiplies (the prefilter
            // passes 2^k times the candidates: this path runs 2^k times as
            // often as for an odd d of the same size)
#pragma unroll
            for (int q = 0; q < 8; ++q)
              bits |= (__builtin_amdgcn_alignbit(t[q], t[q], tcv.rot) - tcv.qbias <= tcv.qmax ? 1u : 0u)
                      << q;
          } else {
#pragma unroll
            for (int q = 0; q < 8; ++q) {
              if constexpr (MODE == 2) bits |= (mode2_exact(t[q] - 1u, tcv) ? 1u : 0u) << q;
              else bits |= (t[q] == 0u ? 1u : 0u) << q;
            }
          }
          if (bits) {
            const uint32_t e = (bits << 16) | (o0 + (uint32_t)(g * 8));
#pragma unroll
            for (int q = 0; q < kHitRegs; ++q) ereg[q] = cnt == (uint32_t)q ? e : ereg[q];
            if (cnt >= (uint32_t)kHitRegs && cnt - kHitRegs < a.lane_slots)
              myslots[cnt - kHitRegs] = e;
            ++cnt;
          }
        }
      }
    };
    // VARIANT 6 (same results): the lookups of subgroup g+D are issued one
    // byte at a time between the hash steps of subgroup g, so the perm /
    // ds_read of the next subgroup fill the dependency gaps of this one's
    // alignbit -> bitop3 chain instead of running as a separate phase
    auto compute_il = [&](auto gc, auto gic, uint32_t o0) __attribute__((always_inline)) {
      constexpr int g = decltype(gc)::value;
      constexpr int gi = decltype(gic)::value;
      uint32_t t[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        {  // lookup q of subgroup gi (the next trip's first ones on the last
           // subgroups: harmless reads if that trip does not come)
          const int k = (gi % 16) * 8 + q;
          const uint32_t sel = 0x0C0C0000u | ((4u + (uint32_t)(k & 3)) << 8);
          const uint32_t addr = __builtin_amdgcn_perm(w[k >> 2], slot8, sel);
          L[gi % NL][q] = *reinterpret_cast<const uint64_t*>(lds + addr);
        }
        const int rk = (g * 8 + q) % 48;
        h = __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_alignbit(h, h, 31),
                                        (uint32_t)L[g % NL][q], ring[rk], 0x96);
        ring[rk] = (uint32_t)(L[g % NL][q] >> 32);
        if constexpr (MODE == 2) t[q] = h * tcv.ninv;
        else t[q] = is_cand<MODE>(h, tcv) ? 0u : 0xFFFFFFFFu;
      }
      const uint32_t thr = MODE == 2 ? tcv.vmax1 : 1u;
      uint32_t mn = t[0];
#pragma unroll
      for (int q = 1; q < 8; ++q) mn = __builtin_elementwise_min(mn, t[q]);
      if (__builtin_expect(__ballot(mn < thr) != 0, 0)) {
        uint32_t bits = 0;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          if constexpr (MODE == 2) bits |= (mode2_exact(t[q] - 1u, tcv) ? 1u : 0u) << q;
          else bits |= (t[q] == 0u ? 1u : 0u) << q;
        }
        if (bits) {
          const uint32_t e = (bits << 16) | (o0 + (uint32_t)(g * 8));
#pragma unroll
          for (int q = 0; q < kHitRegs; ++q) ereg[q] = cnt == (uint32_t)q ? e : ereg[q];
          if (cnt >= (uint32_t)kHitRegs && cnt - kHitRegs < a.lane_slots)
            myslots[cnt - kHitRegs] = e;
          ++cnt;
        }
      }
    };
    fetch(1u);
    {  // this segment's first 48 bytes, for the lane before (the handoff)
      uint8_t* const my_hand = s_hand + (wave * kWave + lane) * kHandoff;
#pragma unroll
      for (int c = 0; c < kHandoff / 16; ++c)
        *reinterpret_cast<uint4*>(my_hand + 16 * c) =
            make_uint4(w[4 * c], w[4 * c + 1], w[4 * c + 2], w[4 * c + 3]);
    }
    static_for<D>([&](auto gc) __attribute__((always_inline)) { issue_sub(gc); });
    for (uint32_t t = 0; t < M; ++t) {
      // the successor's ticket, drawn mid-region: waves that started
      // together reach this point spread out, so the draws do not queue
      if (t == M / 2u && draw && lane == 0) ticket = atomicAdd(a.queue + 32u * qx, 1u);
      const uint32_t o0 = t * 3u * (uint32_t)kLine;
      static_for<48>([&](auto gc) __attribute__((always_inline)) {
        constexpr int g = decltype(gc)::value;
        constexpr int gi = g + D;  // subgroup whose lookups are issued now
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (VARIANT == 6) {
          if constexpr (gi < 48) {
            if constexpr (gi % 16 == 0) fetch(3u * t + 1u + (uint32_t)(gi / 16));
          } else if constexpr (gi == 48) {
            if (t + 1 < M) fetch(3u * t + 4u);
          }
          __builtin_amdgcn_sched_barrier(0);
          compute_il(gc, std::integral_constant<int, gi % 48>{}, o0);
        } else {
          if constexpr (gi < 48) {
            if constexpr (gi % 16 == 0) fetch(3u * t + 1u + (uint32_t)(gi / 16));
            issue_sub(std::integral_constant<int, gi>{});
          } else {
            if (t + 1 < M) {  // the next trip's first subgroups
              if constexpr (gi == 48) fetch(3u * t + 4u);
              issue_sub(std::integral_constant<int, gi - 48>{});
            }
          }
          __builtin_amdgcn_sched_barrier(0);
          compute_sub(gc, o0);
        }
      });
    }

    {
      // the first 48 positions of the next lane's segment, whose window reaches
      // back into this one (that lane hashed them from a zero window and drops
      // them): 6 more subgroups from the bytes it left in LDS, with this
      // segment's ring and hash, hits at offsets S + 1 .. S + 48.  (Lane 63's
      // next segment is the next region's, whose lane 0 reads its warm-up line;
      // its extension hits are dropped below.)
      const uint8_t* nb = s_hand + (wave * kWave + (lane < 63u ? lane + 1u : lane)) * kHandoff;
#pragma unroll
      for (int c = 0; c < kHandoff / 16; ++c) {
        const uint4 q = *reinterpret_cast<const uint4*>(nb + 16 * c);
        w[4 * c] = q.x;
        w[4 * c + 1] = q.y;
        w[4 * c + 2] = q.z;
        w[4 * c + 3] = q.w;
      }
      static_for<6>([&](auto gc) __attribute__((always_inline)) {
        constexpr int g = decltype(gc)::value;
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (g == 0) issue_sub(std::integral_constant<int, 0>{});
        if constexpr (g + 1 < 6) issue_sub(std::integral_constant<int, g + 1>{});
        __builtin_amdgcn_sched_barrier(0);
        compute_sub(gc, S);
      });
    }
    const uint64_t t_hash_end = a.trace ? __builtin_amdgcn_s_memtime() : 0;
    // ---- region end: compact the lanes' hits into one sorted region list ----
    // valid cut offsets o: piece-relative p = lane_p + o in [1, len] and
    // absolute p >= min_pos (windows reaching before the chain origin)
    const int64_t lane_p = (int64_t)region_base(region) + (int64_t)lane * S - (int64_t)a.delta;
    int64_t lo = 1 - lane_p;
    const int64_t lo2 = (int64_t)a.min_pos - (int64_t)a.piece_abs - lane_p;
    lo = lo > lo2 ? lo : lo2;
    // (the handoff: lanes 1..63 drop offsets 1..48, hashed from a zero window;
    // the lane before reports them as S + 1 .. S + 48, lane 63 excepted)
    const uint32_t ext = lane < 63u ? (uint32_t)kHandoff : 0u;
    if (lane > 0u && lo < (int64_t)kHandoff + 1) lo = (int64_t)kHandoff + 1;
    // (clamped past the extension too: a lane wholly before min_pos reports
    // none of the handoff positions S + 1 .. S + ext either)
    const uint32_t o_min = lo <= 1 ? 1u : (lo > (int64_t)(S + ext) ? S + ext + 1u : (uint32_t)lo);
    const int64_t hi = (int64_t)a.len - lane_p;
    const uint32_t o_max = hi <= 0 ? 0u : (hi >= (int64_t)(S + ext) ? S + ext : (uint32_t)hi);
    const uint32_t n = cnt < a.lane_slots + kHitRegs ? cnt : a.lane_slots + kHitRegs;
    const bool spilled = __ballot(cnt > (uint32_t)kHitRegs) != 0;
    auto for_each_hit = [&](auto&& f) {
      auto expand = [&](uint32_t e) {
        const uint32_t base = e & 0xFFFFu;
        for (uint32_t bits = e >> 16; bits; bits &= bits - 1u) {
          const uint32_t o = base + (uint32_t)__builtin_ctz(bits) + 1u;
          if (o >= o_min && o <= o_max) f(o);
        }
      };
#pragma unroll
      for (int q = 0; q < kHitRegs; ++q)
        if ((uint32_t)q < n) expand(ereg[q]);
      if (spilled)
        for (uint32_t i = kHitRegs; i < n; ++i) expand(myslots[i - kHitRegs]);
    };
    uint32_t keep = 0;
    for_each_hit([&](uint32_t) { ++keep; });
    uint32_t incl = keep;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t v = __shfl_up(incl, d, 64);
      if (lane >= (uint32_t)d) incl += v;
    }
    const uint32_t excl = incl - keep;
    uint32_t exact = keep;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) exact += __shfl_xor(exact, d, 64);
    uint32_t* rl = a.region_list + (uint64_t)region * a.region_cap;
    uint32_t j = 0;
    for_each_hit([&](uint32_t o) {
      if (excl + j < a.region_cap) rl[excl + j] = lane * S + o;
      ++j;
    });
    const bool lane_ovf = __ballot(cnt > a.lane_slots + kHitRegs) != 0;
    if (lane == 0) {
      a.region_cnt[region] = exact;
      if (lane_ovf || exact > a.region_cap) atomicAdd(a.overflow, 1u);
    }
    ++nreg_done;
    if (next >= a.nregions) break;
    if (a.trace) re_cyc += __builtin_amdgcn_s_memtime() - t_hash_end;
    region = next;
    rsrc = nrsrc;
    sh = nsh;
    if constexpr (TWO) {
      // the region's lane geometry (tail or big: a wave whose XCD counter ran
      // dry can steal a big region after tail ones)
      const bool tl = is_tail(region);
      const uint32_t nS = tl ? a.lane_bytes2 : a.lane_bytes;
      if (nS != S) {
        S = nS;
        M = tl ? a.batches2 : a.batches;
        dbase0 = dbase_of(S, 0u);
        dbase1 = dbase_of(S, 1u);
      }
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (a.stamp) stamp_end(a.stamp, s_stamp, wave);
  if (a.trace && lane == 0) {
    uint64_t* tr = a.trace + (uint64_t)kScanTraceWords * (blockIdx.x * W + wave);
    tr[4] = re_cyc;
    tr[5] = rs_wait;
    tr[3] = t_entry;
    tr[0] = t_start;
    tr[1] = VARIANT == 5 ? __builtin_amdgcn_s_memtime() : __builtin_amdgcn_s_memrealtime();
    // VARIANT 5: {vmcnt wait, line copy + lgkmcnt(0), DMA issue} cycles, 21 bits each
    uint32_t xcc_id, hw_id;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID, 0, 4)" : "=s"(xcc_id));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw_id));
    tr[2] = VARIANT == 5 ? (vm_wait | (copy_wait << 21) | (dma_issue << 42))
                         : (nreg_done | ((uint64_t)xcc_id << 32) | ((uint64_t)((hw_id >> 8) & 0xFF) << 40));
  }
  // the staging line is free (the last DMA landed at vmcnt(0) above)
#if DSX_DIAG
  if constexpr (FUSE) run_tasks(a.tasks, reinterpret_cast<uint32_t*>(stage), lane, task_tr);
#endif
}

#define DSX_SCANL_INST(W, SUB, D)                                          \
  template __global__ void scanl_kernel<0, 0, W, SUB, D, false, false>(ScanArgs); \
  template __global__ void scanl_kernel<1, 0, W, SUB, D, false, false>(ScanArgs); \
  template __global__ void scanl_kernel<2, 0, W, SUB, D, false, false>(ScanArgs); \
  template __global__ void scanl_kernel<0, 0, W, SUB, D, false, true>(ScanArgs);  \
  template __global__ void scanl_kernel<1, 0, W, SUB, D, false, true>(ScanArgs);  \
  template __global__ void scanl_kernel<2, 0, W, SUB, D, false, true>(ScanArgs);
#if DSX_DIAG
// the stitch behind the scan (DSX_FUSE=1): diagnostic build only
template __global__ void scanl_kernel<0, 0, 8, 8, 1, true, false>(ScanArgs);
template __global__ void scanl_kernel<1, 0, 8, 8, 1, true, false>(ScanArgs);
template __global__ void scanl_kernel<2, 0, 8, 8, 1, true, false>(ScanArgs);
template __global__ void scanl_kernel<2, 1, 8, 8, 1, false, false>(ScanArgs);
template __global__ void scanl_kernel<2, 3, 8, 8, 1, false, false>(ScanArgs);
template __global__ void scanl_kernel<2, 4, 8, 8, 1, false, false>(ScanArgs);
template __global__ void scanl_kernel<2, 5, 8, 8, 1, false, false>(ScanArgs);
template __global__ void scanl_kernel<2, 6, 8, 8, 1, false, false>(ScanArgs);
template __global__ void scanl_kernel<2, 7, 8, 8, 1, false, false>(ScanArgs);
// (the same variants over a piece with two region sizes)
template __global__ void scanl_kernel<2, 1, 8, 8, 1, false, true>(ScanArgs);
template __global__ void scanl_kernel<2, 3, 8, 8, 1, false, true>(ScanArgs);
template __global__ void scanl_kernel<2, 4, 8, 8, 1, false, true>(ScanArgs);
template __global__ void scanl_kernel<2, 5, 8, 8, 1, false, true>(ScanArgs);
template __global__ void scanl_kernel<2, 6, 8, 8, 1, false, true>(ScanArgs);
template __global__ void scanl_kernel<2, 7, 8, 8, 1, false, true>(ScanArgs);
template __global__ void scanl_kernel<2, 8, 8, 8, 1, false, true>(ScanArgs);
template __global__ void scanl_kernel<2, 9, 8, 8, 1, false, true>(ScanArgs);
template __global__ void scanl_kernel<2, 10, 8, 8, 1, false, true>(ScanArgs);
template __global__ void scanl_kernel<2, 8, 8, 8, 1, false, false>(ScanArgs);
template __global__ void scanl_kernel<2, 9, 8, 8, 1, false, false>(ScanArgs);
template __global__ void scanl_kernel<2, 10, 8, 8, 1, false, false>(ScanArgs);
#endif
DSX_SCANL_INST(8, 8, 1)  // D = 2 needs 16 more VGPRs than the 256 of two waves per SIMD

// Exhaustive/ranged check of the GPU boundary predicate against h % d == d-1
// (the plain form of chunker_test.go:190-213).  Diagnostic entry point.
__global__ void boundary_selftest_kernel(TestConsts tc, int mode, uint64_t h0, uint64_t n,
                                         unsigned long long* mismatches) {
  unsigned long long bad = 0;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    const uint32_t h = (uint32_t)(h0 + i);
    const bool want = (h % tc.d) == tc.dm1;
    const bool got = mode == 2 ? is_cand<2>(h, tc) : (mode == 1 ? is_cand<1>(h, tc) : is_cand<0>(h, tc));
    bad += (want != got);
  }
  if (bad) atomicAdd(mismatches, bad);
}

}  // namespace dsx
