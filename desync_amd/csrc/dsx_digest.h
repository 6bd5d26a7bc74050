// dsx_digest.h -- chunk-ID kernel interface shared by dsx_digest.hip and the
// host engine (dsx_api.cpp).
#pragma once
#include <stdint.h>

namespace dsx {

struct Sha512;  // SHA-512/256 (digest.go:22)
struct Sha256;  // SHA-256 (digest.go:28)

struct DigestArgs {
  const uint8_t* blob;   // blob[0] is absolute position base_off
  uint64_t len;          // readable bytes at blob
  const uint64_t* ends;  // [n] chunk end offsets, absolute (device)
  uint64_t first_start;  // start of chunk 0, absolute
  uint64_t n;
  uint8_t* ids;          // [n][32] (device)
  uint32_t* queue;       // chunk queue counter, zero at launch
  uint32_t nfirst;       // chunks handed out statically (one per lane of the grid)
  uint32_t pad;
  uint64_t base_off;     // absolute position of blob[0]
  // device-side range (the pipelined IndexFromFile, dsx_index.cpp): when
  // range_lo is set, the chunks are ends[range_lo[0] .. range_hi[0]) with the
  // first one starting at range_lo[1]; ids are written at the same indices.
  // Records are {total cuts, carried cut} snapshots of the chain state.
  const uint64_t* range_lo;
  const uint64_t* range_hi;
  // longest-first queue order (digest_order_*_kernel): queue position k takes
  // chunk order[k]; null: index order
  const uint32_t* order;
  // chunks longer than this get no ID here (0: none): the index pipeline
  // hashes them on the host (dsx_index.cpp, host tail)
  uint64_t skip_above;
};

// Longest-first order of a digest range (LPT): a counting sort of the chunks
// by size class (8 per octave), largest class first.
constexpr int kSizeClasses = 512;
constexpr int kOrderTile = 2048;  // chunks per workgroup of the count / scatter passes
__global__ void digest_order_count_kernel(DigestArgs a, uint32_t* cls_count);
__global__ void digest_order_scan_kernel(const uint32_t* cls_count, uint32_t* cls_off);
__global__ void digest_order_scatter_kernel(DigestArgs a, uint32_t* cls_off, uint32_t* order);

// copies {DevState.total, DevState.carry} into rec[0..1] (the digest range
// snapshot after a window's stitch)
struct DevState;
__global__ void state_snapshot_kernel(const DevState* st, uint64_t* rec);
// a streaming batch starts: rec = {0, entry cut} (fresh: `carry`, else the
// carried chain position), and a carried chain's cut count restarts at 0
__global__ void batch_begin_kernel(DevState* st, uint64_t* rec, int fresh, uint64_t carry);

#ifndef DSX_DIGEST_THREADS
#define DSX_DIGEST_THREADS 256
#endif
constexpr int kDigestThreads = DSX_DIGEST_THREADS;

}  // namespace dsx
