// dsx_digest.hip -- chunk IDs on the GPU: SHA-512/256 (desync's default
// Digest, digest.go:11-22, crypto/sha512.Sum512_256) and SHA-256 (the
// --digest sha256 alternative, digest.go:24-29), one digest per chunk
// [ends[i-1], ends[i]) of a device-resident blob (IndexChunk.ID, make.go:223).
//
// SHA-2 over one chunk is a sequential chain of block compressions, so the
// parallelism is one chunk per lane.  Chunk sizes vary 16x (min..max), so a
// static chunk-per-lane split would leave most lanes of a wave idle behind its
// longest chunk: lanes instead pull chunks from a global queue the moment they
// finish one (one atomic per wave per refill, prefix by mbcnt), and every
// loop iteration compresses one block on every live lane.  A chunk's last one
// or two blocks (the padded tail, FIPS 180-4 sec.5.1) are assembled byte-wise
// with explicit bounds; full blocks come from aligned 16-byte loads
// re-aligned with v_alignbyte.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>
#include <utility>

#include "dsx_digest.h"
#include "dsx_stitch.h"

namespace dsx {

// ---- SHA-512 constants (FIPS 180-4 sec.4.2.3, sec.5.3.6.2 for the /256 IV) --
__constant__ uint64_t kK512[80] = {
    0x428a2f98d728ae22ull, 0x7137449123ef65cdull, 0xb5c0fbcfec4d3b2full, 0xe9b5dba58189dbbcull,
    0x3956c25bf348b538ull, 0x59f111f1b605d019ull, 0x923f82a4af194f9bull, 0xab1c5ed5da6d8118ull,
    0xd807aa98a3030242ull, 0x12835b0145706fbeull, 0x243185be4ee4b28cull, 0x550c7dc3d5ffb4e2ull,
    0x72be5d74f27b896full, 0x80deb1fe3b1696b1ull, 0x9bdc06a725c71235ull, 0xc19bf174cf692694ull,
    0xe49b69c19ef14ad2ull, 0xefbe4786384f25e3ull, 0x0fc19dc68b8cd5b5ull, 0x240ca1cc77ac9c65ull,
    0x2de92c6f592b0275ull, 0x4a7484aa6ea6e483ull, 0x5cb0a9dcbd41fbd4ull, 0x76f988da831153b5ull,
    0x983e5152ee66dfabull, 0xa831c66d2db43210ull, 0xb00327c898fb213full, 0xbf597fc7beef0ee4ull,
    0xc6e00bf33da88fc2ull, 0xd5a79147930aa725ull, 0x06ca6351e003826full, 0x142929670a0e6e70ull,
    0x27b70a8546d22ffcull, 0x2e1b21385c26c926ull, 0x4d2c6dfc5ac42aedull, 0x53380d139d95b3dfull,
    0x650a73548baf63deull, 0x766a0abb3c77b2a8ull, 0x81c2c92e47edaee6ull, 0x92722c851482353bull,
    0xa2bfe8a14cf10364ull, 0xa81a664bbc423001ull, 0xc24b8b70d0f89791ull, 0xc76c51a30654be30ull,
    0xd192e819d6ef5218ull, 0xd69906245565a910ull, 0xf40e35855771202aull, 0x106aa07032bbd1b8ull,
    0x19a4c116b8d2d0c8ull, 0x1e376c085141ab53ull, 0x2748774cdf8eeb99ull, 0x34b0bcb5e19b48a8ull,
    0x391c0cb3c5c95a63ull, 0x4ed8aa4ae3418acbull, 0x5b9cca4f7763e373ull, 0x682e6ff3d6b2b8a3ull,
    0x748f82ee5defb2fcull, 0x78a5636f43172f60ull, 0x84c87814a1f0ab72ull, 0x8cc702081a6439ecull,
    0x90befffa23631e28ull, 0xa4506cebde82bde9ull, 0xbef9a3f7b2c67915ull, 0xc67178f2e372532bull,
    0xca273eceea26619cull, 0xd186b8c721c0c207ull, 0xeada7dd6cde0eb1eull, 0xf57d4f7fee6ed178ull,
    0x06f067aa72176fbaull, 0x0a637dc5a2c898a6ull, 0x113f9804bef90daeull, 0x1b710b35131c471bull,
    0x28db77f523047d84ull, 0x32caab7b40c72493ull, 0x3c9ebe0a15c9bebcull, 0x431d67c49c100d4cull,
    0x4cc5d4becb3e42b6ull, 0x597f299cfc657e2aull, 0x5fcb6fab3ad6faecull, 0x6c44198c4a475817ull};
__constant__ uint64_t kIV512_256[8] = {
    0x22312194fc2bf72cull, 0x9f555fa3c84c64c2ull, 0x2393b86b6f53b151ull, 0x963877195940eabdull,
    0x96283ee2a88effe3ull, 0xbe5e1e2553863992ull, 0x2b0199fc2c85b8aaull, 0x0eb72ddc81c52ca2ull};

// ---- SHA-256 constants (FIPS 180-4 sec.4.2.2, sec.5.3.3) --------------------
__constant__ uint32_t kK256[64] = {
    0x428a2f98u, 0x71374491u, 0xb5c0fbcfu, 0xe9b5dba5u, 0x3956c25bu, 0x59f111f1u, 0x923f82a4u,
    0xab1c5ed5u, 0xd807aa98u, 0x12835b01u, 0x243185beu, 0x550c7dc3u, 0x72be5d74u, 0x80deb1feu,
    0x9bdc06a7u, 0xc19bf174u, 0xe49b69c1u, 0xefbe4786u, 0x0fc19dc6u, 0x240ca1ccu, 0x2de92c6fu,
    0x4a7484aau, 0x5cb0a9dcu, 0x76f988dau, 0x983e5152u, 0xa831c66du, 0xb00327c8u, 0xbf597fc7u,
    0xc6e00bf3u, 0xd5a79147u, 0x06ca6351u, 0x14292967u, 0x27b70a85u, 0x2e1b2138u, 0x4d2c6dfcu,
    0x53380d13u, 0x650a7354u, 0x766a0abbu, 0x81c2c92eu, 0x92722c85u, 0xa2bfe8a1u, 0xa81a664bu,
    0xc24b8b70u, 0xc76c51a3u, 0xd192e819u, 0xd6990624u, 0xf40e3585u, 0x106aa070u, 0x19a4c116u,
    0x1e376c08u, 0x2748774cu, 0x34b0bcb5u, 0x391c0cb3u, 0x4ed8aa4au, 0x5b9cca4fu, 0x682e6ff3u,
    0x748f82eeu, 0x78a5636fu, 0x84c87814u, 0x8cc70208u, 0x90befffau, 0xa4506cebu, 0xbef9a3f7u,
    0xc67178f2u};
__constant__ uint32_t kIV256[8] = {0x6a09e667u, 0xbb67ae85u, 0x3c6ef372u, 0xa54ff53au,
                                   0x510e527fu, 0x9b05688cu, 0x1f83d9abu, 0x5be0cd19u};

// 64-bit rotate / shift as two v_alignbit_b32 on the register halves (the
// generic form costs two 64-bit shifts and two ORs).  n is a compile-time
// constant after unrolling, so the n < 32 branch folds away.
__device__ __forceinline__ uint64_t rotr64(uint64_t x, int n) {
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  uint32_t rlo, rhi;
  if (n < 32) {
    rlo = __builtin_amdgcn_alignbit(hi, lo, n);
    rhi = __builtin_amdgcn_alignbit(lo, hi, n);
  } else {
    rlo = __builtin_amdgcn_alignbit(lo, hi, n - 32);
    rhi = __builtin_amdgcn_alignbit(hi, lo, n - 32);
  }
  return ((uint64_t)rhi << 32) | rlo;
}
__device__ __forceinline__ uint64_t shr64(uint64_t x, int n) {  // 0 < n < 32
  const uint32_t lo = (uint32_t)x, hi = (uint32_t)(x >> 32);
  return ((uint64_t)(hi >> n) << 32) | __builtin_amdgcn_alignbit(hi, lo, n);
}
// three-input bit functions as one v_bitop3_b32 per dword (gfx950): 0x96 =
// a^b^c, 0xE8 = majority(a,b,c) (both symmetric in their inputs)
__device__ __forceinline__ uint32_t xor3_32(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}
__device__ __forceinline__ uint32_t maj32(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0xE8);
}
// A 64-bit value from its halves, opaque to the optimizer: left visible, the
// (hi << 32) | lo feeding a 64-bit add is split into two adds (zero-extended
// lo, then hi << 32) with a v_mov for each zero half -- 3 extra instructions
// per SHA-512 round.  The empty asm makes it one register pair.
__device__ __forceinline__ uint64_t pair64(uint32_t lo, uint32_t hi) {
  uint64_t v = ((uint64_t)hi << 32) | lo;
  asm("" : "+v"(v));  // (not volatile: no scheduling barrier)
  return v;
}
__device__ __forceinline__ uint64_t xor3_64(uint64_t a, uint64_t b, uint64_t c) {
  return pair64(xor3_32((uint32_t)a, (uint32_t)b, (uint32_t)c),
                xor3_32((uint32_t)(a >> 32), (uint32_t)(b >> 32), (uint32_t)(c >> 32)));
}
__device__ __forceinline__ uint64_t maj64(uint64_t a, uint64_t b, uint64_t c) {
  return pair64(maj32((uint32_t)a, (uint32_t)b, (uint32_t)c),
                maj32((uint32_t)(a >> 32), (uint32_t)(b >> 32), (uint32_t)(c >> 32)));
}
// SHA's Ch(e, f, g) = (e & f) ^ (~e & g): one v_bfi_b32 per dword
__device__ __forceinline__ uint64_t ch64(uint64_t e, uint64_t f, uint64_t g) {
  return pair64(((uint32_t)e & (uint32_t)f) ^ (~(uint32_t)e & (uint32_t)g),
                ((uint32_t)(e >> 32) & (uint32_t)(f >> 32)) ^ (~(uint32_t)(e >> 32) & (uint32_t)(g >> 32)));
}
__device__ __forceinline__ uint32_t rotr32(uint32_t x, int n) {
  return __builtin_amdgcn_alignbit(x, x, n);
}
__device__ __forceinline__ uint32_t bswap32(uint32_t x) {
  return __builtin_amdgcn_perm(x, x, 0x00010203u);
}

template <class F, int... I>
__device__ __forceinline__ void sfor_impl(F& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void sfor(F&& f) {
  sfor_impl(f, std::make_integer_sequence<int, N>{});
}

// Hand-issued LDS reads for digest_pc_kernel's consumer (see compress_kw).
typedef __attribute__((address_space(3))) const void lds_cvoid_t;
template <int OFF>
__device__ __forceinline__ void lds_read64(uint64_t& v, uint32_t addr) {
  asm volatile("ds_read_b64 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF) : "memory");
}
template <int OFF>
__device__ __forceinline__ void lds_read32(uint32_t& v, uint32_t addr) {
  asm volatile("ds_read_b32 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "i"(OFF) : "memory");
}
// wait until at most n LDS reads are outstanding (n: compile-time after unrolling)
template <class T>
__device__ __forceinline__ void lds_wait_for(T& v, int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(v)); break;
    case 1: asm volatile("s_waitcnt lgkmcnt(1)" : "+v"(v)); break;
    case 2: asm volatile("s_waitcnt lgkmcnt(2)" : "+v"(v)); break;
    case 3: asm volatile("s_waitcnt lgkmcnt(3)" : "+v"(v)); break;
    case 4: asm volatile("s_waitcnt lgkmcnt(4)" : "+v"(v)); break;
    case 5: asm volatile("s_waitcnt lgkmcnt(5)" : "+v"(v)); break;
    case 6: asm volatile("s_waitcnt lgkmcnt(6)" : "+v"(v)); break;
    default: asm volatile("s_waitcnt lgkmcnt(7)" : "+v"(v)); break;
  }
}

// A block as 32 big-endian-assembled dwords (SHA-512: 16 words = 32 dwords,
// SHA-256: 16 words = 16 dwords; the first BLK/4 entries are used).
struct Sha512 {
  static constexpr int BLK = 128;
  static constexpr int LENB = 16;  // length field bytes
  uint64_t H[8];
  __device__ void init() {
#pragma unroll
    for (int i = 0; i < 8; ++i) H[i] = kIV512_256[i];
  }
  // d[] holds the block's 32 dwords in big-endian order (d[2i] = high half)
  __device__ void compress(const uint32_t (&d)[32]) {
    uint64_t W[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) W[i] = ((uint64_t)d[2 * i] << 32) | d[2 * i + 1];
    uint64_t a = H[0], b = H[1], c = H[2], e = H[4], f = H[5], g = H[6], h = H[7], dd = H[3];
    // 80 rounds as 5 passes of 16 (the first without message expansion): the
    // inner 16 are unrolled so every W index is static (no indexed register
    // access), the outer loop stays rolled to keep the kernel small.
    auto pass = [&](auto expand, int t0) {
      constexpr bool EXPAND = decltype(expand)::value;
      uint64_t K[16];  // this pass's constants: one wait
#pragma unroll
      for (int j = 0; j < 16; ++j) K[j] = kK512[t0 + j];
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        if constexpr (EXPAND) {
          const uint64_t w15 = W[(j + 1) & 15], w2 = W[(j + 14) & 15];
          const uint64_t s0 = xor3_64(rotr64(w15, 1), rotr64(w15, 8), shr64(w15, 7));
          const uint64_t s1 = xor3_64(rotr64(w2, 19), rotr64(w2, 61), shr64(w2, 6));
          W[j] = W[j] + s0 + W[(j + 9) & 15] + s1;
        }
        const uint64_t w = W[j];
        const uint64_t S1 = xor3_64(rotr64(e, 14), rotr64(e, 18), rotr64(e, 41));
        const uint64_t ch = (e & f) ^ (~e & g);
        const uint64_t t1 = h + S1 + ch + K[j] + w;
        const uint64_t S0 = xor3_64(rotr64(a, 28), rotr64(a, 34), rotr64(a, 39));
        const uint64_t maj = maj64(a, b, c);
        const uint64_t t2 = S0 + maj;
        h = g; g = f; f = e; e = dd + t1; dd = c; c = b; b = a; a = t1 + t2;
      }
    };
    pass(std::false_type{}, 0);  // rounds 0-15: no message expansion
#pragma unroll 1
    for (int t0 = 16; t0 < 80; t0 += 16) pass(std::true_type{}, t0);
    H[0] += a; H[1] += b; H[2] += c; H[3] += dd; H[4] += e; H[5] += f; H[6] += g; H[7] += h;
  }
  // SHA-512/256: the first 32 bytes of the big-endian state
  __device__ void out(uint8_t* dst) const {
    uint32_t* o = reinterpret_cast<uint32_t*>(dst);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      o[2 * i] = bswap32((uint32_t)(H[i] >> 32));
      o[2 * i + 1] = bswap32((uint32_t)H[i]);
    }
  }

  // ---- split form (digest_pc_kernel): the message schedule on a producer
  // wave, the 80 rounds on a consumer wave, K[t] + W[t] handed over in LDS
  using Word = uint64_t;
  static constexpr int ROUNDS = 80;
  // kw[t * 64] = K[t] + W[t] for the block d (one lane's column of the LDS buffer)
  __device__ static void schedule(const uint32_t (&d)[32], Word* kw) {
    uint64_t W[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) W[i] = ((uint64_t)d[2 * i] << 32) | d[2 * i + 1];
#pragma unroll
    for (int j = 0; j < 16; ++j) kw[j * 64] = W[j] + kK512[j];
#pragma unroll 1
    for (int t0 = 16; t0 < 80; t0 += 16) {
      uint64_t K[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) K[j] = kK512[t0 + j];
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const uint64_t w15 = W[(j + 1) & 15], w2 = W[(j + 14) & 15];
        const uint64_t s0 = xor3_64(rotr64(w15, 1), rotr64(w15, 8), shr64(w15, 7));
        const uint64_t s1 = xor3_64(rotr64(w2, 19), rotr64(w2, 61), shr64(w2, 6));
        W[j] = W[j] + s0 + W[(j + 9) & 15] + s1;
        kw[(t0 + j) * 64] = W[j] + K[j];
      }
    }
  }
  // the 80 rounds on K[t] + W[t] read from LDS at kw + t * 64 words.  The
  // reads are issued by hand 8 rounds ahead (the compiler placed each one a
  // few instructions before its use, exposing the LDS latency every round);
  // the compiler does not count them, so each use waits explicitly.
  __device__ void compress_kw(const Word* kw) {
    const uint32_t base = (uint32_t)(uintptr_t)(const lds_cvoid_t*)kw;
    uint64_t L[9];
    sfor<8>([&](auto tc) __attribute__((always_inline)) {
      lds_read64<decltype(tc)::value * 512>(L[decltype(tc)::value], base);
    });
    uint64_t a = H[0], b = H[1], c = H[2], dd = H[3], e = H[4], f = H[5], g = H[6], h = H[7];
    sfor<80>([&](auto tc) __attribute__((always_inline)) {
      constexpr int t = decltype(tc)::value;
      lds_wait_for(L[t % 9], 79 - t < 7 ? 79 - t : 7);
      const uint64_t kwt = L[t % 9];
      if constexpr (t + 8 < 80) lds_read64<(t + 8) * 512>(L[(t + 8) % 9], base);
      const uint64_t S1 = xor3_64(rotr64(e, 14), rotr64(e, 18), rotr64(e, 41));
      const uint64_t ch = ch64(e, f, g);
      const uint64_t t1 = h + S1 + ch + kwt;
      const uint64_t S0 = xor3_64(rotr64(a, 28), rotr64(a, 34), rotr64(a, 39));
      const uint64_t t2 = S0 + maj64(a, b, c);
      h = g; g = f; f = e; e = dd + t1; dd = c; c = b; b = a; a = t1 + t2;
    });
    H[0] += a; H[1] += b; H[2] += c; H[3] += dd; H[4] += e; H[5] += f; H[6] += g; H[7] += h;
  }
};

struct Sha256 {
  static constexpr int BLK = 64;
  static constexpr int LENB = 8;
  uint32_t H[8];
  __device__ void init() {
#pragma unroll
    for (int i = 0; i < 8; ++i) H[i] = kIV256[i];
  }
  __device__ void compress(const uint32_t (&d)[32]) {
    uint32_t W[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) W[i] = d[i];
    uint32_t a = H[0], b = H[1], c = H[2], dd = H[3], e = H[4], f = H[5], g = H[6], h = H[7];
    auto pass = [&](auto expand, int t0) {
      constexpr bool EXPAND = decltype(expand)::value;
      uint32_t K[16];  // this pass's constants: one wait
#pragma unroll
      for (int j = 0; j < 16; ++j) K[j] = kK256[t0 + j];
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        if constexpr (EXPAND) {
          const uint32_t w15 = W[(j + 1) & 15], w2 = W[(j + 14) & 15];
          const uint32_t s0 = xor3_32(rotr32(w15, 7), rotr32(w15, 18), w15 >> 3);
          const uint32_t s1 = xor3_32(rotr32(w2, 17), rotr32(w2, 19), w2 >> 10);
          W[j] = W[j] + s0 + W[(j + 9) & 15] + s1;
        }
        const uint32_t w = W[j];
        const uint32_t S1 = xor3_32(rotr32(e, 6), rotr32(e, 11), rotr32(e, 25));
        const uint32_t ch = (e & f) ^ (~e & g);
        const uint32_t t1 = h + S1 + ch + K[j] + w;
        const uint32_t S0 = xor3_32(rotr32(a, 2), rotr32(a, 13), rotr32(a, 22));
        const uint32_t maj = maj32(a, b, c);
        const uint32_t t2 = S0 + maj;
        h = g; g = f; f = e; e = dd + t1; dd = c; c = b; b = a; a = t1 + t2;
      }
    };
    pass(std::false_type{}, 0);  // rounds 0-15: no message expansion
#pragma unroll 1
    for (int t0 = 16; t0 < 64; t0 += 16) pass(std::true_type{}, t0);
    H[0] += a; H[1] += b; H[2] += c; H[3] += dd; H[4] += e; H[5] += f; H[6] += g; H[7] += h;
  }
  __device__ void out(uint8_t* dst) const {
    uint32_t* o = reinterpret_cast<uint32_t*>(dst);
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = bswap32(H[i]);
  }

  using Word = uint32_t;
  static constexpr int ROUNDS = 64;
  __device__ static void schedule(const uint32_t (&d)[32], Word* kw) {
    uint32_t W[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) W[i] = d[i];
#pragma unroll
    for (int j = 0; j < 16; ++j) kw[j * 64] = W[j] + kK256[j];
#pragma unroll 1
    for (int t0 = 16; t0 < 64; t0 += 16) {
      uint32_t K[16];
#pragma unroll
      for (int j = 0; j < 16; ++j) K[j] = kK256[t0 + j];
#pragma unroll
      for (int j = 0; j < 16; ++j) {
        const uint32_t w15 = W[(j + 1) & 15], w2 = W[(j + 14) & 15];
        const uint32_t s0 = xor3_32(rotr32(w15, 7), rotr32(w15, 18), w15 >> 3);
        const uint32_t s1 = xor3_32(rotr32(w2, 17), rotr32(w2, 19), w2 >> 10);
        W[j] = W[j] + s0 + W[(j + 9) & 15] + s1;
        kw[(t0 + j) * 64] = W[j] + K[j];
      }
    }
  }
  __device__ void compress_kw(const Word* kw) {
    const uint32_t base = (uint32_t)(uintptr_t)(const lds_cvoid_t*)kw;
    uint32_t L[9];
    sfor<8>([&](auto tc) __attribute__((always_inline)) {
      lds_read32<decltype(tc)::value * 256>(L[decltype(tc)::value], base);
    });
    uint32_t a = H[0], b = H[1], c = H[2], dd = H[3], e = H[4], f = H[5], g = H[6], h = H[7];
    sfor<64>([&](auto tc) __attribute__((always_inline)) {
      constexpr int t = decltype(tc)::value;
      lds_wait_for(L[t % 9], 63 - t < 7 ? 63 - t : 7);
      const uint32_t kwt = L[t % 9];
      if constexpr (t + 8 < 64) lds_read32<(t + 8) * 256>(L[(t + 8) % 9], base);
      const uint32_t S1 = xor3_32(rotr32(e, 6), rotr32(e, 11), rotr32(e, 25));
      const uint32_t ch = (e & f) ^ (~e & g);
      const uint32_t t1 = h + S1 + ch + kwt;
      const uint32_t S0 = xor3_32(rotr32(a, 2), rotr32(a, 13), rotr32(a, 22));
      const uint32_t t2 = S0 + maj32(a, b, c);
      h = g; g = f; f = e; e = dd + t1; dd = c; c = b; b = a; a = t1 + t2;
    });
    H[0] += a; H[1] += b; H[2] += c; H[3] += dd; H[4] += e; H[5] += f; H[6] += g; H[7] += h;
  }
};

// Full blocks come in two steps so the next block's loads are in flight
// while the current one is compressed (one wave per SIMD at small blobs: the
// load latency would otherwise sit on every block's critical path).
// fetch_raw: the aligned dwordx4 loads over the 16-byte-aligned window of
// [pos, pos + BLK); only valid when fast_ok(pos) (window inside the blob).
template <int BLK>
__device__ __forceinline__ bool fast_ok(uint64_t pos, uint64_t len) {
  return (pos & ~15ull) + BLK + 16 <= len;
}
template <int BLK>
__device__ __forceinline__ void fetch_raw(const uint8_t* blob, uint64_t pos, uint32_t (&raw)[BLK / 4 + 4]) {
  constexpr int ND = BLK / 4;
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  const u32x4* p = reinterpret_cast<const u32x4*>(blob + (pos & ~15ull));
#pragma unroll
  for (int i = 0; i < ND / 4 + 1; ++i) {
    const u32x4 v = __builtin_nontemporal_load(p + i);
    raw[4 * i] = v.x; raw[4 * i + 1] = v.y; raw[4 * i + 2] = v.z; raw[4 * i + 3] = v.w;
  }
}
// align_raw: re-align with v_alignbyte and assemble big-endian dwords.
template <int BLK>
__device__ __forceinline__ void align_raw(const uint32_t (&raw)[BLK / 4 + 4], uint64_t pos,
                                          uint32_t (&d)[32]) {
  constexpr int ND = BLK / 4;
  const uint32_t sh = (uint32_t)(pos & 15u);
  const uint32_t dsh = sh >> 2, bsh = (sh & 3u) * 8u;
#pragma unroll
  for (int i = 0; i < ND; ++i) {
    // dword i of the block = bytes [pos + 4i, pos + 4i + 4): raw[dsh + i], raw[dsh + i + 1]
    uint32_t lo = raw[i], hi = raw[i + 1];
    // select by dsh (0..3) without dynamic register indexing
#pragma unroll
    for (int s = 1; s < 4; ++s) {
      lo = dsh == (uint32_t)s ? raw[i + s] : lo;
      hi = dsh == (uint32_t)s ? raw[i + s + 1] : hi;
    }
    const uint32_t v = bsh ? __builtin_amdgcn_alignbit(hi, lo, bsh) : lo;
    d[i] = bswap32(v);
  }
}
// Near the blob end: byte loads.
template <int BLK>
__device__ __forceinline__ void load_block_bytes(const uint8_t* blob, uint64_t pos, uint32_t (&d)[32]) {
  constexpr int ND = BLK / 4;
#pragma unroll 4
  for (int i = 0; i < ND; ++i) {
    uint32_t v = 0;
    for (int k = 0; k < 4; ++k) v = (v << 8) | blob[pos + 4 * i + k];
    d[i] = v;
  }
}

// Padded tail block: r = remaining message bytes (r < BLK, or r == BLK on no
// path), `marker` = whether the 0x80 byte goes into this block, `lenhere` =
// whether the bit length goes into this block.
template <int BLK, int LENB>
__device__ __forceinline__ void tail_block(const uint8_t* p, uint32_t r, bool marker, bool lenhere,
                                           uint64_t bits, uint32_t (&d)[32]) {
  constexpr int ND = BLK / 4;
  for (int i = 0; i < ND; ++i) {
    uint32_t v = 0;
    for (int k = 0; k < 4; ++k) {
      const uint32_t idx = (uint32_t)(4 * i + k);
      uint32_t byte = 0;
      if (idx < r) byte = p[idx];
      else if (idx == r && marker) byte = 0x80u;
      v = (v << 8) | byte;
    }
    d[i] = v;
  }
  if (lenhere) {  // big-endian bit length in the last LENB bytes (high part 0)
    d[ND - 2] = (uint32_t)(bits >> 32);
    d[ND - 1] = (uint32_t)bits;
  }
}

__global__ void state_snapshot_kernel(const DevState* st, uint64_t* rec) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    rec[0] = st->total;
    rec[1] = st->carry;
  }
}

__global__ void batch_begin_kernel(DevState* st, uint64_t* rec, int fresh, uint64_t carry) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    rec[0] = 0;
    rec[1] = fresh ? carry : st->carry;
    if (!fresh) st->total = 0;
  }
}

// ---- longest-first queue order ---------------------------------------------
// Chunk sizes vary 16x (min..max).  Handed out in index order, the last chunk
// a lane draws may be a long one that its wave then compresses nearly alone
// (a 256 KiB chunk is 2,049 SHA-512 blocks against 513 for the average
// 64 KiB).  Handed out longest first, the long chains start in the first
// round and the short ones fill in behind them (LPT scheduling).  Within a
// size class the order is arbitrary; the IDs land at their chunk index.

// monotone in sz: sz < 8 -> sz, else 8 + 8*(log2(sz) - 3) + the next 3 bits
__device__ __forceinline__ uint32_t size_class(uint64_t sz) {
  if (sz < 8) return (uint32_t)sz;
  const uint32_t lg = 63u - (uint32_t)__builtin_clzll(sz);
  return 8u + 8u * (lg - 3u) + (uint32_t)((sz >> (lg - 3u)) & 7u);
}

// the digest range as digest_kernel resolves it
struct DigestRange {
  uint64_t n, first_start;
  const uint64_t* ends;
};
__device__ __forceinline__ DigestRange digest_range(const DigestArgs& a) {
  DigestRange r{a.n, a.first_start, a.ends};
  if (a.range_lo) {
    const uint64_t i0 = a.range_lo[0], i1 = a.range_hi[0];
    r.n = i1 > i0 ? i1 - i0 : 0;
    r.first_start = a.range_lo[1];
    r.ends += i0;
  }
  return r;
}

__device__ __forceinline__ uint32_t chunk_class(const DigestRange& r, uint64_t i) {
  const uint64_t s = i == 0 ? r.first_start : r.ends[i - 1], e = r.ends[i];
  return size_class(e > s ? e - s : 0);
}

// pass 1: chunks per size class (block tile of kOrderTile chunks)
__global__ __launch_bounds__(256) void digest_order_count_kernel(DigestArgs a, uint32_t* cls_count) {
  __shared__ uint32_t h[kSizeClasses];
  for (int c = threadIdx.x; c < kSizeClasses; c += blockDim.x) h[c] = 0;
  __syncthreads();
  const DigestRange r = digest_range(a);
  const uint64_t t0 = (uint64_t)blockIdx.x * kOrderTile;
  for (uint64_t i = t0 + threadIdx.x; i < r.n && i < t0 + kOrderTile; i += blockDim.x)
    atomicAdd(&h[chunk_class(r, i)], 1u);
  __syncthreads();
  for (int c = threadIdx.x; c < kSizeClasses; c += blockDim.x)
    if (h[c]) atomicAdd(&cls_count[c], h[c]);
}

// pass 2 (one block of kSizeClasses threads): cls_off[c] = chunks in classes
// above c (largest class first)
__global__ __launch_bounds__(kSizeClasses) void digest_order_scan_kernel(const uint32_t* cls_count,
                                                                         uint32_t* cls_off) {
  __shared__ uint32_t v[kSizeClasses];
  const int t = threadIdx.x;              // position in descending class order
  const int c = kSizeClasses - 1 - t;     // its class
  v[t] = cls_count[c];
  __syncthreads();
  for (int d = 1; d < kSizeClasses; d <<= 1) {  // inclusive scan (Hillis-Steele)
    const uint32_t x = t >= d ? v[t - d] : 0u;
    __syncthreads();
    v[t] += x;
    __syncthreads();
  }
  cls_off[c] = v[t] - cls_count[c];
}

// pass 3: each block reserves its tile's slots per class, then places its
// chunks (order within a class: arbitrary)
__global__ __launch_bounds__(256) void digest_order_scatter_kernel(DigestArgs a, uint32_t* cls_off,
                                                                   uint32_t* order) {
  constexpr int PER = kOrderTile / 256;
  __shared__ uint32_t h[kSizeClasses], base[kSizeClasses];
  for (int c = threadIdx.x; c < kSizeClasses; c += blockDim.x) h[c] = 0;
  __syncthreads();
  const DigestRange r = digest_range(a);
  const uint64_t t0 = (uint64_t)blockIdx.x * kOrderTile;
  uint32_t cls[PER], rank[PER];
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const uint64_t i = t0 + (uint64_t)q * 256u + threadIdx.x;
    cls[q] = i < r.n ? chunk_class(r, i) : 0u;
    rank[q] = i < r.n ? atomicAdd(&h[cls[q]], 1u) : 0u;
  }
  __syncthreads();
  for (int c = threadIdx.x; c < kSizeClasses; c += blockDim.x)
    base[c] = h[c] ? atomicAdd(&cls_off[c], h[c]) : 0u;
  __syncthreads();
#pragma unroll
  for (int q = 0; q < PER; ++q) {
    const uint64_t i = t0 + (uint64_t)q * 256u + threadIdx.x;
    if (i < r.n) order[base[cls[q]] + rank[q]] = (uint32_t)i;
  }
}

// PF: prefetch the next full block of the chunk while the current one is
// compressed (its 36-dword window stays live across the compression: SHA-512
// 201 VGPRs, 2 waves per SIMD).  Without it SHA-512 fits 3 waves per SIMD
// (165 VGPRs), and is slower all the same (diagnostic build only).
template <class H, bool PF>
__global__ __launch_bounds__(kDigestThreads) void digest_kernel(DigestArgs a) {
  constexpr int BLK = H::BLK;
  const uint32_t lane = threadIdx.x & 63u;
  // chunk range: host-given, or device-side snapshots of the chain state
  uint64_t n = a.n, first_start = a.first_start;
  uint32_t nfirst = a.nfirst;
  const uint64_t* ends = a.ends;
  uint8_t* ids = a.ids;
  if (a.range_lo) {
    const uint64_t i0 = a.range_lo[0], i1 = a.range_hi[0];
    n = i1 > i0 ? i1 - i0 : 0;
    first_start = a.range_lo[1];
    ends += i0;
    ids += i0 * 32u;
    const uint64_t lanes = (uint64_t)gridDim.x * blockDim.x;
    nfirst = (uint32_t)(n < lanes ? n : lanes);
  }
  // chunk state (s, e, pos relative to blob[0]); k = queue position (the
  // first one static), ci = its chunk (a.order: longest first)
  uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint64_t ci = n;
  uint64_t s = 0, e = 0, pos = 0;
  uint32_t phase = 0;  // 0 = data blocks, 1 = tail with marker, 2 = length-only block
  uint32_t raw[BLK / 4 + 4];  // prefetched window of the next full block
  bool have_next = false;
  H st;
  auto start_chunk = [&]() {
    ci = n;
    while (k < n) {
      ci = a.order ? (uint64_t)a.order[k] : k;
      const uint64_t sa = ci == 0 ? first_start : ends[ci - 1], ea = ends[ci];
      if (a.skip_above && sa <= ea && ea - sa > a.skip_above) {  // hashed on the host
        k = (uint64_t)nfirst + atomicAdd(a.queue, 1u);
        continue;
      }
      // a chunk outside the readable bytes (malformed ends) is skipped and
      // gets no ID instead of reading out of bounds
      if (sa >= a.base_off && sa <= ea && ea - a.base_off <= a.len) {
        s = sa - a.base_off;
        e = ea - a.base_off;
        pos = s;
        phase = 0;
        have_next = false;
        st.init();
        return;
      }
      k = n;  // (this lane takes no further chunk)
      ci = n;
    }
  };
  if (k >= nfirst) k = n;  // (grid larger than the static share)
  start_chunk();
  while (true) {
    const bool live = k < n;
    if (__ballot(live) == 0) break;
    uint32_t d[32];
    bool finished = false;
    have_next = have_next && live;
    if (live) {
      const uint64_t r = e - pos;
      if (phase == 0 && r >= (uint64_t)BLK) {
        if (have_next) {
          align_raw<BLK>(raw, pos, d);
        } else if (fast_ok<BLK>(pos, a.len)) {
          fetch_raw<BLK>(a.blob, pos, raw);
          align_raw<BLK>(raw, pos, d);
        } else {
          load_block_bytes<BLK>(a.blob, pos, d);
        }
        pos += BLK;
        // prefetch the next full block of this chunk
        have_next = PF && e - pos >= (uint64_t)BLK && fast_ok<BLK>(pos, a.len);
        if (have_next) fetch_raw<BLK>(a.blob, pos, raw);
      } else {
        const uint64_t bits = (e - s) * 8u;
        if (phase == 0) {
          // r < BLK message bytes + 0x80; the length fits if r < BLK - LENB
          const bool fits = r < (uint64_t)(BLK - H::LENB);
          tail_block<BLK, H::LENB>(a.blob + pos, (uint32_t)r, true, fits, bits, d);
          pos = e;
          phase = fits ? 3 : 2;
        } else {  // phase 2: zeros + length
          tail_block<BLK, H::LENB>(a.blob + pos, 0u, false, true, bits, d);
          phase = 3;
        }
      }
    }
    st.compress(d);  // (dead lanes compress garbage; their state is discarded)
    if (live && phase == 3) {
      st.out(ids + ci * 32u);
      finished = true;
    }
    // refill the finished lanes from the queue (one atomic per wave)
    const uint64_t fm = __ballot(finished);
    if (fm) {
      const uint32_t nf = (uint32_t)__popcll(fm);
      uint32_t base = 0;
      if (lane == (uint32_t)(__ffsll((long long)fm) - 1)) base = atomicAdd(a.queue, nf);
      base = __shfl(base, __ffsll((long long)fm) - 1, 64);
      if (finished) {
        const uint32_t rank = (uint32_t)__popcll(fm & ((1ull << lane) - 1ull));
        k = (uint64_t)nfirst + base + rank;
        start_chunk();
      }
    }
  }
}

template __global__ void digest_kernel<Sha512, true>(DigestArgs);
template __global__ void digest_kernel<Sha256, true>(DigestArgs);
#if DSX_DIAG
// without the prefetch (DSX_DIGEST_PF=0): 3 waves per SIMD for SHA-512, and
// 11-13 % slower at 4-16 GiB (profiles/r04e)
template __global__ void digest_kernel<Sha512, false>(DigestArgs);
template __global__ void digest_kernel<Sha256, false>(DigestArgs);
#endif

// ---------------------------------------------------------------------------
// digest_pc_kernel -- the same IDs with each chunk's work split over two waves.
//
// A lone wave issues one VALU instruction every ~5 cycles (tools/ubench_hash),
// and at small blobs the time is the longest chunk's serial chain of block
// compressions (2048 blocks for a 256 KiB chunk).  A block is ~40 % message
// schedule, which does not depend on the chaining state: here a producer wave
// (wave 0) assembles each lane's next block and writes its 80 (64) round
// inputs K[t] + W[t] to LDS while the consumer wave (wave 1) runs the rounds
// of the previous block on them.  Lane l of both waves serves the same chunk
// sequence; the producer owns the chunk state machine and the queue, and
// hands each block over with a record {flags, chunk index}.  One barrier per
// block; two LDS buffers.  The LDS size keeps one workgroup per CU, so the
// consumer wave has its SIMD to itself.
// ---------------------------------------------------------------------------
constexpr uint32_t kPcLds = 84 * 1024;
template <class H>
__global__ __launch_bounds__(128, 1) void digest_pc_kernel(DigestArgs a) {
  using Word = typename H::Word;
  constexpr int BLK = H::BLK;
  constexpr int R = H::ROUNDS;
  constexpr uint32_t KWB = (uint32_t)R * 64u * sizeof(Word);  // one buffer
  static_assert(2 * KWB + 1024 + 16 <= kPcLds, "LDS layout");
  __shared__ __attribute__((aligned(16))) uint8_t lds[kPcLds];
  Word* kwbuf = reinterpret_cast<Word*>(lds);                   // [2][R][64]
  uint32_t* rflag = reinterpret_cast<uint32_t*>(lds + 2 * KWB);  // [2][64]
  uint32_t* rci = rflag + 128;                                   // [2][64]
  uint32_t* live = rci + 128;                                    // [2]
  const uint32_t lane = threadIdx.x & 63u;
  const bool producer = threadIdx.x < 64u;
  uint64_t n = a.n, first_start = a.first_start;
  uint32_t nfirst = a.nfirst;
  const uint64_t* ends = a.ends;
  uint8_t* ids = a.ids;
  if (a.range_lo) {
    const uint64_t i0 = a.range_lo[0], i1 = a.range_hi[0];
    n = i1 > i0 ? i1 - i0 : 0;
    first_start = a.range_lo[1];
    ends += i0;
    ids += i0 * 32u;
    const uint64_t lanes = (uint64_t)gridDim.x * 64u;
    nfirst = (uint32_t)(n < lanes ? n : lanes);
  }
  // producer: chunk state (s, e, pos relative to blob[0])
  uint64_t ci = (uint64_t)blockIdx.x * 64u + lane;
  uint64_t s = 0, e = 0, pos = 0;
  uint32_t phase = 0;
  uint32_t raw[BLK / 4 + 4];
  bool have_next = false, fresh = true;
  auto start_chunk = [&]() {
    while (ci < n) {
      const uint64_t sa = ci == 0 ? first_start : ends[ci - 1], ea = ends[ci];
      if (a.skip_above && sa <= ea && ea - sa > a.skip_above) {  // hashed on the host
        ci = (uint64_t)nfirst + atomicAdd(a.queue, 1u);
        continue;
      }
      if (sa >= a.base_off && sa <= ea && ea - a.base_off <= a.len) {
        s = sa - a.base_off;
        e = ea - a.base_off;
        pos = s;
        phase = 0;
        have_next = false;
        fresh = true;
        return;
      }
      ci = n;
    }
  };
  if (producer) {
    if (ci >= nfirst) ci = n;
    start_chunk();
  }
  H st;  // consumer: chaining state of the lane's current chunk
  for (uint32_t k = 0;; ++k) {
    const uint32_t b = k & 1u;
    if (producer) {
      const bool lv = ci < n;
      bool fin = false;
      if (lv) {
        uint32_t d[32];
        const uint64_t r = e - pos;
        if (phase == 0 && r >= (uint64_t)BLK) {
          if (have_next) {
            align_raw<BLK>(raw, pos, d);
          } else if (fast_ok<BLK>(pos, a.len)) {
            fetch_raw<BLK>(a.blob, pos, raw);
            align_raw<BLK>(raw, pos, d);
          } else {
            load_block_bytes<BLK>(a.blob, pos, d);
          }
          pos += BLK;
          have_next = e - pos >= (uint64_t)BLK && fast_ok<BLK>(pos, a.len);
          if (have_next) fetch_raw<BLK>(a.blob, pos, raw);
        } else {
          const uint64_t bits = (e - s) * 8u;
          if (phase == 0) {
            const bool fits = r < (uint64_t)(BLK - H::LENB);
            tail_block<BLK, H::LENB>(a.blob + pos, (uint32_t)r, true, fits, bits, d);
            pos = e;
            phase = fits ? 3 : 2;
          } else {
            tail_block<BLK, H::LENB>(a.blob + pos, 0u, false, true, bits, d);
            phase = 3;
          }
        }
        H::schedule(d, kwbuf + b * (uint32_t)R * 64u + lane);
        fin = phase == 3;
      }
      rflag[b * 64u + lane] = lv ? (1u | (fresh ? 2u : 0u) | (fin ? 4u : 0u)) : 0u;
      rci[b * 64u + lane] = (uint32_t)ci;
      fresh = false;
      const uint64_t lm = __ballot(lv);
      if (lane == 0) live[b] = lm != 0 ? 1u : 0u;
      // refill the lanes whose chunk ended with this block (one atomic per wave)
      const uint64_t fm = __ballot(fin);
      if (fm) {
        const uint32_t nf = (uint32_t)__popcll(fm);
        uint32_t base = 0;
        if (lane == (uint32_t)(__ffsll((long long)fm) - 1)) base = atomicAdd(a.queue, nf);
        base = __shfl(base, __ffsll((long long)fm) - 1, 64);
        if (fin) {
          const uint32_t rank = (uint32_t)__popcll(fm & ((1ull << lane) - 1ull));
          ci = (uint64_t)nfirst + base + rank;
          start_chunk();
        }
      }
    } else if (k > 0) {
      const uint32_t pb = b ^ 1u;
      if (live[pb]) {
        const uint32_t f = rflag[pb * 64u + lane];
        if (f & 2u) st.init();
        st.compress_kw(kwbuf + pb * (uint32_t)R * 64u + lane);
        if (f & 4u) st.out(ids + (uint64_t)rci[pb * 64u + lane] * 32u);
      }
    }
    __syncthreads();
    if (!live[b]) break;
  }
}
template __global__ void digest_pc_kernel<Sha512>(DigestArgs);
template __global__ void digest_pc_kernel<Sha256>(DigestArgs);

}  // namespace dsx
