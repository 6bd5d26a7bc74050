// dsx_gen.hip -- on-device synthetic inputs for the BASELINE configs.
//
// Uniform stream: 8-byte word w = splitmix64(seed * 2^40 + word_index), little
// endian; identical to oracle/oracle.py:synth_uniform so any window of it can
// be regenerated on the CPU for parity checks.
// Dedup stream (BASELINE.json config 3): 1 MiB blocks; block i is, with
// probability p, a byte copy of block j = h2(i) mod i (j < i), else fresh.
// The content of block i is the uniform stream's block root(i), where root()
// follows the copy chain down to a fresh block.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dsx {

__host__ __device__ inline uint64_t splitmix64(uint64_t z) {
  z = z * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E5A1ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__host__ __device__ inline uint64_t dedup_root(uint64_t blk, uint64_t seed, uint32_t p_thresh) {
  // p_thresh = p * 2^32
  while (blk > 0) {
    const uint64_t r = splitmix64((seed << 40) ^ (blk * 0x2545F4914F6CDD1Dull) ^ 0xD1B54A32D192ED03ull);
    if ((uint32_t)r >= p_thresh) break;  // fresh block
    blk = (r >> 32) % blk;               // copy of an earlier block
  }
  return blk;
}

__global__ void gen_uniform_kernel(uint8_t* dst, uint64_t offset, uint64_t len, uint64_t seed) {
  // each thread produces 16 bytes of output starting at output byte 16*t
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x * 16;
  const uint64_t sbase = seed << 40;
  for (uint64_t o = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 16; o < len; o += stride) {
    const uint64_t abs0 = offset + o;
    const uint64_t w0 = abs0 >> 3;
    const uint32_t sh = (uint32_t)(abs0 & 7);
    const uint64_t a = splitmix64(sbase + w0), b = splitmix64(sbase + w0 + 1),
                   c = splitmix64(sbase + w0 + 2);
    uint8_t tmp[24];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      tmp[i] = (uint8_t)(a >> (8 * i));
      tmp[8 + i] = (uint8_t)(b >> (8 * i));
      tmp[16 + i] = (uint8_t)(c >> (8 * i));
    }
    const uint64_t n = len - o < 16 ? len - o : 16;
    for (uint64_t i = 0; i < n; ++i) dst[o + i] = tmp[sh + i];
  }
}

__global__ void gen_dedup_kernel(uint8_t* dst, uint64_t offset, uint64_t len, uint64_t seed,
                                 uint32_t p_thresh) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x * 16;
  const uint64_t sbase = seed << 40;
  for (uint64_t o = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) * 16; o < len; o += stride) {
    const uint64_t n = len - o < 16 ? len - o : 16;
    for (uint64_t i = 0; i < n; ++i) {
      const uint64_t abs = offset + o + i;
      const uint64_t blk = abs >> 20;
      const uint64_t root = dedup_root(blk, seed, p_thresh);
      const uint64_t src = (root << 20) | (abs & 0xFFFFFull);
      const uint64_t w = splitmix64(sbase + (src >> 3));
      dst[o + i] = (uint8_t)(w >> (8 * (src & 7)));
    }
  }
}

}  // namespace dsx
