// dsx_digest.h -- chunk-ID kernel interface shared by dsx_digest.hip and the
// host engine (dsx_api.cpp).
#pragma once
#include <stdint.h>

namespace dsx {

struct Sha512;  // SHA-512/256 (digest.go:22)
struct Sha256;  // SHA-256 (digest.go:28)

struct DigestArgs {
  const uint8_t* blob;
  uint64_t len;
  const uint64_t* ends;  // [n] chunk end offsets (device)
  uint64_t first_start;  // start of chunk 0
  uint64_t n;
  uint8_t* ids;          // [n][32] (device)
  uint32_t* queue;       // chunk queue counter, zero at launch
  uint32_t nfirst;       // chunks handed out statically (one per lane of the grid)
  uint32_t pad;
};

#ifndef DSX_DIGEST_THREADS
#define DSX_DIGEST_THREADS 256
#endif
constexpr int kDigestThreads = DSX_DIGEST_THREADS;

}  // namespace dsx
