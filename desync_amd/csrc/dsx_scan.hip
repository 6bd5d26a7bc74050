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
//   * one workgroup = 8 waves, 1 per CU (160 KiB LDS), persistent over regions;
//   * a wave owns a region of 64 lane segments of S bytes; lane l rolls the
//     hash through its own segment, 48 bytes per round (one ring period);
//   * HBM -> LDS with buffer_load_dwordx4 ... lds (LDS-DMA): each 1 KiB wave
//     instruction fetches 21.3 lanes x 48 B, so every 128 B line is read once,
//     4-deep ring per wave, no workgroup barrier in the loop;
//   * the substitution table lives in LDS replicated over 32 lane slots
//     (byte v, slot s at v*256 + s*8 = {T[v], rotl16(T[v])}) so the per-byte
//     lookup is ONE v_perm_b32 (address = byte<<8 | slot) + ONE conflict-free
//     ds_read_b64; the outgoing byte's rotated term comes from a 48-entry
//     register ring (no second lookup);
//   * the boundary test is a wave ballot per byte; rare hits leave the hot
//     loop through one scalar branch per 16 bytes.
#include <hip/hip_runtime.h>

#include "../../include/dsx_buzhash_table.h"
#include "dsx_common.h"

namespace dsx {

typedef __attribute__((address_space(3))) void lds_void_t;
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// One 1 KiB LDS-DMA wave instruction (buffer_load_dwordx4 ... lds): lane j's
// 16 bytes from rsrc+voff land at LDS byte lds_addr + 16*j.  Written as inline
// asm so that hipcc does not treat every later ds_read as aliasing a pending
// DMA (it would emit s_waitcnt vmcnt(0) before each round and drain the
// ring); completion is tracked by the explicit s_waitcnt vmcnt(N) in the loop.
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

__constant__ uint32_t kT[256] = DSX_BUZHASH_TABLE_INIT;

// h % d == d-1, evaluated on the GPU.
//   MODE 0: exactly Go's multiply-inverse form (chunker.go:265): v_mul_lo_u32.
//   MODE 1: float-reciprocal quotient + exact 24-bit multiply check, valid for
//           2048 < d < 2^24 (host chooses; see DESIGN.md "Boundary test").
template <int MODE>
__device__ __forceinline__ bool is_cand(uint32_t h, const TestConsts& tc) {
  if constexpr (MODE == 0) {
    uint32_t v = (h + 1u) * tc.inv;
    v = __builtin_amdgcn_alignbit(v, v, tc.rot);
    return v - tc.qbias <= tc.qmax;
  } else {
    float f = __builtin_fmaf((float)h, tc.rcp, tc.c0);
    uint32_t q = (uint32_t)f;
    return __umul24(q, tc.d) + tc.dm1 == h;
  }
}

// Process one 48-byte round of one lane.  `w` holds the round's bytes,
// `ring[k]` the rotated table value of the byte 48 positions earlier.
template <bool TEST, int MODE>
__device__ __forceinline__ void round48(const uint32_t (&w)[12], uint32_t& h, uint32_t (&ring)[48],
                                        const uint8_t* __restrict__ tbl, uint32_t slot8,
                                        const TestConsts& tc, uint32_t lane, uint32_t obase,
                                        uint32_t seg_valid, uint32_t& cnt,
                                        uint16_t* __restrict__ myslots, uint32_t lane_slots) {
#pragma unroll
  for (int g = 0; g < 3; ++g) {
    uint64_t m[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int k = g * 16 + i;
      const uint32_t sel = 0x0C0C0000u | ((4u + (uint32_t)(k & 3)) << 8);
      const uint32_t addr = __builtin_amdgcn_perm(w[k >> 2], slot8, sel);
      const uint2 e = *reinterpret_cast<const uint2*>(tbl + addr);
      h = __builtin_amdgcn_alignbit(h, h, 31) ^ e.x ^ ring[k];
      ring[k] = e.y;
      if constexpr (TEST) m[i] = __ballot(is_cand<MODE>(h, tc));
    }
    if constexpr (TEST) {
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
}

template <int MODE>
__global__ __launch_bounds__(kScanThreads, 2) void scan_kernel(ScanArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kScanLds];

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
  uint8_t* stage = lds + kTableBytes + wave * (kNBuf * kStageBytes);
  const uint32_t stage_lds = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(lds_void_t*)stage);
  const uint32_t S = a.lane_bytes;
  const uint32_t R = a.rounds;

  // DMA geometry: instruction i (0..2), lane j -> 16 B unit u = 64i + j of the
  // 64 x 48 B round image: row u/3, chunk u%3.
  uint32_t dma_row_off[3];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    const uint32_t u = (uint32_t)i * 64u + lane;
    dma_row_off[i] = (u / 3u) * S + (u % 3u) * 16u;
  }

  for (uint32_t region = blockIdx.x * kScanWaves + wave; region < a.nregions;
       region += gridDim.x * kScanWaves) {
    const uint64_t rbase = (uint64_t)region * 64u * S;  // piece-relative
    // readable bytes before the region (fewer than 48 only at the chain origin,
    // where the missing window bytes are virtual zeros: those loads fall out of
    // the buffer range and return 0)
    const uint32_t H = (rbase + a.halo >= (uint64_t)kRound) ? (uint32_t)kRound
                                                             : (uint32_t)(rbase + a.halo);
    const uint8_t* rptr = a.base + rbase - H;
    uint64_t nrec64 = a.len - rbase + H;
    const uint32_t nrec = nrec64 > 0xFFFFFFF0ull ? 0xFFFFFFF0u : (uint32_t)nrec64;
    const uint64_t rp = (uint64_t)(uintptr_t)rptr;
    u32x4 rsrc;
    rsrc.x = __builtin_amdgcn_readfirstlane((uint32_t)rp);
    rsrc.y = __builtin_amdgcn_readfirstlane((uint32_t)(rp >> 32) & 0xFFFFu);  // stride 0
    rsrc.z = __builtin_amdgcn_readfirstlane(nrec);
    rsrc.w = 0x00020000u;
    // offset of round ri's chunk: row*S + chunk*16 + (ri+1)*48 + H - 48
    const uint32_t hfix = H - (uint32_t)kRound;  // 0, or negative (wraps -> out of range)

    auto issue = [&](int ri) {  // ri in [-1, R)
      const uint32_t dst = stage_lds + ((uint32_t)(ri + 1) % kNBuf) * kStageBytes;
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        uint32_t vo = (ri < (int)R) ? dma_row_off[i] + (uint32_t)(ri + 1) * 48u + hfix
                                    : 0xFFFFFFF0u;
        dma16(rsrc, vo, dst + (uint32_t)i * 1024u);
      }
    };

    // lane state
    const uint64_t lane_rel = rbase + (uint64_t)lane * S;  // piece-relative lane base
    // valid offsets o (position = lane base + o) must stay inside the piece and
    // beyond absolute position 48 (no full window before that).
    uint32_t seg_valid = 0;
    if (lane_rel < a.len) {
      const uint64_t rem = a.len - lane_rel;
      seg_valid = rem < S ? (uint32_t)rem : S;
    }
    uint32_t cnt = 0;
    const uint64_t gl = (uint64_t)region * 64u + lane;
    uint16_t* myslots = a.lane_slot + gl * a.lane_slots;
    const uint64_t lane_abs = a.piece_abs + lane_rel;
    // p = lane_abs + o must be >= min_pos: windows before the chain origin are
    // not real (virtual zero bytes at the blob/stream start)
    const uint32_t o_min = lane_abs >= a.min_pos ? 0u : (uint32_t)(a.min_pos - lane_abs);

    uint32_t h = 0;
    uint32_t ring[48];
#pragma unroll
    for (int k = 0; k < 48; ++k) ring[k] = 0;

    issue(-1);
    issue(0);
    issue(1);
    issue(2);
    for (int ri = -1; ri < (int)R; ++ri) {
      asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
      const uint8_t* src = stage + ((uint32_t)(ri + 1) % kNBuf) * kStageBytes + lane * 48u;
      uint32_t w[12];
      {
        const uint4 q0 = *reinterpret_cast<const uint4*>(src);
        const uint4 q1 = *reinterpret_cast<const uint4*>(src + 16);
        const uint4 q2 = *reinterpret_cast<const uint4*>(src + 32);
        w[0] = q0.x; w[1] = q0.y; w[2] = q0.z; w[3] = q0.w;
        w[4] = q1.x; w[5] = q1.y; w[6] = q1.z; w[7] = q1.w;
        w[8] = q2.x; w[9] = q2.y; w[10] = q2.z; w[11] = q2.w;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      issue(ri + 4);  // refill the buffer just read
      if (ri < 0) {
        round48<false, MODE>(w, h, ring, lds, slot8, a.tc, lane, 0u, 0u, cnt, myslots, 0u);
      } else {
        const uint32_t obase = (uint32_t)ri * 48u;
        // positions <= 48 (absolute) are not real windows: clamp via seg_valid lower bound
        round48<true, MODE>(w, h, ring, lds, slot8, a.tc, lane, obase, seg_valid, cnt, myslots,
                           a.lane_slots);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (o_min > 0) {  // drop candidates before min_pos (chain origin only)
      uint32_t keep = 0;
      const uint32_t n = cnt < a.lane_slots ? cnt : a.lane_slots;
      for (uint32_t i = 0; i < n; ++i) {
        const uint16_t o = myslots[i];
        if (o >= o_min) myslots[keep++] = o;
      }
      cnt = cnt - (n - keep);
    }
    a.lane_cnt[gl] = cnt;
    if (cnt > a.lane_slots) atomicAdd(a.overflow, 1u);
  }
}

template __global__ void scan_kernel<0>(ScanArgs);
template __global__ void scan_kernel<1>(ScanArgs);

}  // namespace dsx

namespace dsx {
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
