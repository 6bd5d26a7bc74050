// dsx_hostsha.cpp -- SHA-512/256 chunk IDs on the host (Digest.Sum,
// digest.go:22; FIPS 180-4 sec. 6.4 and 5.3.6.2) for the index pipeline's
// longest chunks at the end of a file (dsx_index.cpp): a GPU
// lane hashes one SHA-512 block per ~5 us, so the last window's digest lasts
// its longest chunk's chain (~10 ms for 256 KiB); a host core hashes 8 chunks
// at once in the qword lanes of AVX-512 registers at ~1-2 GB/s.
//
// Multi-buffer form: block b of 8 messages in step, message words gathered
// from 8 addresses, a lane whose message has no block b any more keeps its
// state (masked adds).  Scalar form for one message (and CPUs without
// AVX-512: the pipeline then leaves every chunk to the GPU).
#include <immintrin.h>

#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstring>
#include <vector>

#include "dsx_engine.h"

namespace {

constexpr uint64_t kK[80] = {
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
constexpr uint64_t kIV[8] = {0x22312194fc2bf72cull, 0x9f555fa3c84c64c2ull, 0x2393b86b6f53b151ull,
                             0x963877195940eabdull, 0x96283ee2a88effe3ull, 0xbe5e1e2553863992ull,
                             0x2b0199fc2c85b8aaull, 0x0eb72ddc81c52ca2ull};

// The padded end of a message of n bytes: its last n % 128 bytes, 0x80,
// zeros and the 128-bit bit length; 1 or 2 blocks (returned).
uint64_t pad_tail(const uint8_t* p, uint64_t n, uint8_t tail[256]) {
  const uint64_t r = n % 128;
  const uint64_t nt = r + 17 > 128 ? 2 : 1;
  memset(tail, 0, 256);
  if (r) memcpy(tail, p + (n - r), r);
  tail[r] = 0x80;
  const uint64_t bits = n << 3;
  uint8_t* l = tail + 128 * nt - 16;
  l[7] = (uint8_t)(n >> 61);  // (the high 64-bit length word)
  for (int i = 0; i < 8; ++i) l[15 - i] = (uint8_t)(bits >> (8 * i));
  return nt;
}

inline uint64_t rotr(uint64_t x, int n) { return (x >> n) | (x << (64 - n)); }
inline uint64_t load_be(const uint8_t* p) {
  uint64_t v;
  memcpy(&v, p, 8);
  return __builtin_bswap64(v);
}

void blocks_scalar(uint64_t H[8], const uint8_t* p, uint64_t nb) {
  for (uint64_t b = 0; b < nb; ++b, p += 128) {
    uint64_t W[80];
    for (int t = 0; t < 16; ++t) W[t] = load_be(p + 8 * t);
    for (int t = 16; t < 80; ++t) {
      const uint64_t s0 = rotr(W[t - 15], 1) ^ rotr(W[t - 15], 8) ^ (W[t - 15] >> 7);
      const uint64_t s1 = rotr(W[t - 2], 19) ^ rotr(W[t - 2], 61) ^ (W[t - 2] >> 6);
      W[t] = W[t - 16] + s0 + W[t - 7] + s1;
    }
    uint64_t a = H[0], bb = H[1], c = H[2], d = H[3], e = H[4], f = H[5], g = H[6], h = H[7];
    for (int t = 0; t < 80; ++t) {
      const uint64_t t1 =
          h + (rotr(e, 14) ^ rotr(e, 18) ^ rotr(e, 41)) + ((e & f) ^ (~e & g)) + kK[t] + W[t];
      const uint64_t t2 = (rotr(a, 28) ^ rotr(a, 34) ^ rotr(a, 39)) + ((a & bb) ^ (a & c) ^ (bb & c));
      h = g;
      g = f;
      f = e;
      e = d + t1;
      d = c;
      c = bb;
      bb = a;
      a = t1 + t2;
    }
    H[0] += a;
    H[1] += bb;
    H[2] += c;
    H[3] += d;
    H[4] += e;
    H[5] += f;
    H[6] += g;
    H[7] += h;
  }
}

#define DSX_AVX512 __attribute__((target("avx512f,avx512bw")))
#define DSX_XOR3(a, b, c) _mm512_ternarylogic_epi64(a, b, c, 0x96)

}  // namespace

bool host_sha_vec() {
  static const bool v = __builtin_cpu_supports("avx512f") && __builtin_cpu_supports("avx512bw");
  return v;
}

void host_sha512_256_one(const uint8_t* p, uint64_t n, uint8_t* out) {
  uint64_t H[8];
  memcpy(H, kIV, sizeof H);
  blocks_scalar(H, p, n / 128);
  alignas(64) uint8_t tail[256];
  blocks_scalar(H, tail, pad_tail(p, n, tail));
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 8; ++j) out[8 * i + j] = (uint8_t)(H[i] >> (56 - 8 * j));
}

// 8 messages (n[i] == UINT64_MAX: an unused lane), out[i] 32 bytes each.
DSX_AVX512 void host_sha512_256_x8(const uint8_t* const p[8], const uint64_t n[8],
                                   uint8_t* const out[8]) {
  alignas(64) uint8_t tail[8][256];
  uint64_t nfull[8], nb[8], maxnb = 0;
  for (int i = 0; i < 8; ++i) {
    if (n[i] == UINT64_MAX) {
      nfull[i] = nb[i] = 0;
      continue;
    }
    nfull[i] = n[i] / 128;
    nb[i] = nfull[i] + pad_tail(p[i], n[i], tail[i]);
    maxnb = std::max(maxnb, nb[i]);
  }
  // big-endian qwords: reverse the bytes of each 64-bit lane
  const __m512i bswap = _mm512_set_epi8(
      8, 9, 10, 11, 12, 13, 14, 15, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 0, 1, 2, 3,
      4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15,
      0, 1, 2, 3, 4, 5, 6, 7);
  __m512i H[8];
  for (int j = 0; j < 8; ++j) H[j] = _mm512_set1_epi64((long long)kIV[j]);
  const uint8_t* base = &tail[0][0];
  for (uint64_t b = 0; b < maxnb; ++b) {
    alignas(64) int64_t off[8];
    __mmask8 act = 0;
    for (int i = 0; i < 8; ++i) {
      const uint8_t* a =
          b < nfull[i] ? p[i] + 128 * b : (b < nb[i] ? tail[i] + 128 * (b - nfull[i]) : tail[i]);
      off[i] = (int64_t)(a - base);
      act |= (__mmask8)((b < nb[i] ? 1u : 0u) << i);
    }
    const __m512i vo = _mm512_load_si512(off);
    __m512i W[16];
    for (int t = 0; t < 16; ++t)
      W[t] = _mm512_shuffle_epi8(
          _mm512_i64gather_epi64(_mm512_add_epi64(vo, _mm512_set1_epi64(8 * t)), base, 1), bswap);
    __m512i a = H[0], bb = H[1], c = H[2], d = H[3], e = H[4], f = H[5], g = H[6], h = H[7];
    for (int t = 0; t < 80; ++t) {
      __m512i w;
      if (t < 16) {
        w = W[t];
      } else {
        const __m512i w15 = W[(t - 15) & 15], w2 = W[(t - 2) & 15];
        const __m512i s0 =
            DSX_XOR3(_mm512_ror_epi64(w15, 1), _mm512_ror_epi64(w15, 8), _mm512_srli_epi64(w15, 7));
        const __m512i s1 =
            DSX_XOR3(_mm512_ror_epi64(w2, 19), _mm512_ror_epi64(w2, 61), _mm512_srli_epi64(w2, 6));
        w = _mm512_add_epi64(_mm512_add_epi64(W[t & 15], s0), _mm512_add_epi64(W[(t - 7) & 15], s1));
        W[t & 15] = w;
      }
      const __m512i S1 =
          DSX_XOR3(_mm512_ror_epi64(e, 14), _mm512_ror_epi64(e, 18), _mm512_ror_epi64(e, 41));
      const __m512i ch = _mm512_ternarylogic_epi64(e, f, g, 0xCA);  // e ? f : g
      const __m512i t1 = _mm512_add_epi64(
          _mm512_add_epi64(h, S1),
          _mm512_add_epi64(_mm512_add_epi64(ch, w), _mm512_set1_epi64((long long)kK[t])));
      const __m512i S0 =
          DSX_XOR3(_mm512_ror_epi64(a, 28), _mm512_ror_epi64(a, 34), _mm512_ror_epi64(a, 39));
      const __m512i maj = _mm512_ternarylogic_epi64(a, bb, c, 0xE8);
      h = g;
      g = f;
      f = e;
      e = _mm512_add_epi64(d, t1);
      d = c;
      c = bb;
      bb = a;
      a = _mm512_add_epi64(t1, _mm512_add_epi64(S0, maj));
    }
    H[0] = _mm512_mask_add_epi64(H[0], act, H[0], a);
    H[1] = _mm512_mask_add_epi64(H[1], act, H[1], bb);
    H[2] = _mm512_mask_add_epi64(H[2], act, H[2], c);
    H[3] = _mm512_mask_add_epi64(H[3], act, H[3], d);
    H[4] = _mm512_mask_add_epi64(H[4], act, H[4], e);
    H[5] = _mm512_mask_add_epi64(H[5], act, H[5], f);
    H[6] = _mm512_mask_add_epi64(H[6], act, H[6], g);
    H[7] = _mm512_mask_add_epi64(H[7], act, H[7], h);
  }
  alignas(64) uint64_t hv[4][8];
  for (int j = 0; j < 4; ++j) _mm512_store_si512(hv[j], H[j]);
  for (int i = 0; i < 8; ++i) {
    if (n[i] == UINT64_MAX) continue;
    for (int j = 0; j < 4; ++j)
      for (int k = 0; k < 8; ++k) out[i][8 * j + k] = (uint8_t)(hv[j][i] >> (56 - 8 * k));
  }
}

// The same from C (include/dsx.h): groups of 8 longest first over the host pool.
extern "C" int dsx_host_sha512_256(const uint8_t* const* ptrs, const uint64_t* lens, uint64_t n,
                                   uint8_t* ids, int threads, int flags) {
  if (n && (!ptrs || !lens || !ids)) return DSX_E_INVAL;
  if (flags & ~DSX_HOST_SHA_SCALAR) return DSX_E_INVAL;
  for (uint64_t i = 0; i < n; ++i)
    if (!ptrs[i] && lens[i]) return DSX_E_INVAL;
  if (!n) return DSX_OK;
  const bool vec = !(flags & DSX_HOST_SHA_SCALAR) && host_sha_vec();
  std::vector<uint64_t> order(n);
  for (uint64_t i = 0; i < n; ++i) order[i] = i;
  std::sort(order.begin(), order.end(), [&](uint64_t x, uint64_t y) { return lens[x] > lens[y]; });
  const uint64_t per = vec ? 8 : 1, groups = (n + per - 1) / per;
  std::atomic<uint64_t> next{0};
  host_parallel((int)std::min<uint64_t>((uint64_t)std::max(1, threads), groups), [&](int) {
    for (uint64_t g; (g = next.fetch_add(1)) < groups;) {
      if (!vec) {
        const uint64_t i = order[g];
        host_sha512_256_one(ptrs[i], lens[i], ids + 32 * i);
        continue;
      }
      const uint8_t* p[8];
      uint64_t l[8];
      uint8_t* o[8];
      for (int k = 0; k < 8; ++k) {
        const uint64_t j = 8 * g + k;
        p[k] = j < n ? ptrs[order[j]] : nullptr;
        l[k] = j < n ? lens[order[j]] : UINT64_MAX;
        o[k] = j < n ? ids + 32 * order[j] : nullptr;
      }
      host_sha512_256_x8(p, l, o);
    }
  });
  return DSX_OK;
}
