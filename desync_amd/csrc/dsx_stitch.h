// dsx_stitch.h -- device structures shared by the stitch kernels and the host
// engine (dsx_api.cpp).
#pragma once
#include <stdint.h>

namespace dsx {

// Where a piece's candidates live: sorted per-region lists written by the
// scan.  Region r covers positions (P + r*RB, P + (r+1)*RB]; candidate =
// P + r*RB + list entry.
struct PieceCands {
  uint64_t P;             // absolute position of the region grid's origin
  uint64_t RB;            // region bytes (64 * lane segment) of regions [0, nbig)
  uint32_t nregions;
  uint32_t region_cap;
  const uint32_t* region_cnt;
  const uint32_t* region_list;
  const uint32_t* overflow;
  uint64_t RB2;           // region bytes of the tail regions [nbig, nregions); 0: one size
  uint32_t nbig;
  uint32_t pad;
};

// Region r covers grid-relative positions (base(r), base(r) + bytes(r)].
__host__ __device__ __forceinline__ uint64_t pc_region_base(const PieceCands& pc, uint64_t r) {
  return (pc.RB2 == 0 || r <= pc.nbig) ? r * pc.RB
                                       : (uint64_t)pc.nbig * pc.RB + (r - pc.nbig) * pc.RB2;
}
// the region whose bytes hold grid-relative offset x, i.e. the first region
// with base(r) + bytes(r) > x (may be >= nregions past the end)
__host__ __device__ __forceinline__ uint64_t pc_region_of(const PieceCands& pc, uint64_t x) {
  const uint64_t big = (uint64_t)pc.nbig * pc.RB;
  return (pc.RB2 == 0 || x < big) ? x / pc.RB : pc.nbig + (x - big) / pc.RB2;
}

// Chain rule inputs (chunker.go:206-277): L is the blob length (known only on
// the final piece), PE the absolute end of the scanned bytes.
struct ChainParams {
  uint64_t min, max;
  uint64_t L;   // valid if is_last
  uint64_t PE;  // piece end (absolute)
  uint32_t is_last;
  uint32_t pad;
};

struct SegInfo {
  uint64_t E;      // entry cut used for staged(k) (= X_{k-1}, or s0 for k == 0)
  uint64_t X;      // exit of the speculative chain started at seg_start(k)
  uint64_t Z;      // exit of staged(k)
  uint32_t cnt;    // cuts in staged(k)
  uint32_t flags;  // kSeg*
};
constexpr uint32_t kSegEnd = 1u;       // staged chain reached the blob end
constexpr uint32_t kSegUndet = 2u;     // stopped: successor beyond the piece
constexpr uint32_t kSegDense = 4u;     // candidates did not fit LDS: repair walks it
constexpr uint32_t kSegOverflow = 8u;  // more cuts than staging capacity

// Chain state carried across pieces and kernels (device memory).
struct DevState {
  uint64_t carry;       // last true cut (chain position)
  uint64_t total;       // cuts emitted so far in this call
  uint64_t piece_cuts;  // cuts emitted by the current piece
  uint64_t repaired;    // segments repaired (stats)
  uint32_t done;        // chain reached the blob end
  uint32_t err;         // kErr* bits
  uint32_t active;      // current piece was processed (K3 ran its body)
  uint32_t pad;
  // snapshots taken by walk_kernel for finish_kernel, whose workgroups must
  // not read fields its last workgroup updates
  uint64_t base;        // total at the start of the piece's stitch
  uint32_t skip;        // done or overflow at that point
  uint32_t pad2;
  uint64_t discarded;   // staged cuts a repair replaced (ChunksProduced - ChunksAccepted)
};

// Published by the last kernel of a piece into pinned host memory.
struct HostState {
  uint64_t carry, total, repaired, discarded;
  uint32_t done, err;
  uint64_t seq;  // piece sequence number, for the host to check freshness
};
constexpr uint32_t kErrCapacity = 1u;  // output capacity exceeded
constexpr uint32_t kErrDense = 2u;     // a lane overflowed its candidate slots
constexpr uint32_t kErrRedo = 4u;      // stitch tasks met a suspect segment: redo the call

// ---- stitch behind the scan --------------------------------
// A queued call (DSX_NO_SYNC, one piece, chain from 0) is stitched by wave
// tasks that run inside the next calls' scans, on wave slots the scan leaves
// idle: call j's scan kernel also walks call j-1's segments and finishes call
// j-2 (offsets, cut list, published state).  Both read only what earlier
// kernels wrote, so no task waits for another.
// A task-walked segment (in the SegInfo buffer, same size): staged(k) is
// P2 = stage[0..n2) (the chain entering from X_{k-1}, up to where it meets
// the speculative chain S1) followed by S1's cuts spec[f1..]; cnt in all.
struct TaskSeg {
  uint64_t X, Z;
  uint32_t cnt, flags;
  uint32_t n2, f1;
};
struct WalkJob {
  PieceCands pc;
  uint64_t min, max, L;  // chain from 0 to the blob end L (one final piece)
  uint64_t seg;          // segment k = [k*seg, min((k+1)*seg, L)) (anchor 0)
  uint32_t nseg, scap;
  SegInfo* seg_info;     // [nseg] (as TaskSeg)
  uint64_t* stage;       // [nseg * scap] P2 lists
  uint64_t* spec;        // [nseg * scap] S1 lists
};
struct FinishJob {
  const SegInfo* seg_info;
  const uint64_t* stage;
  const uint64_t* spec;
  const uint32_t* overflow;  // the scan's list overflow word
  uint32_t nseg, scap;
  uint64_t* out;             // contiguous cut list (device)
  uint64_t out_cap;
  HostState* host_state;     // pinned: published by the last finish task
  uint64_t seq;
};
struct TaskArgs {
  WalkJob w;
  FinishJob f;
  uint32_t nw, nf;       // walk / finish task counts (0: none)
  uint32_t wseg, fseg;   // segments per walk / finish task
  uint32_t* counter;     // task tickets (the fused scan: zeroed by the previous scan)
  uint32_t* farrive;     // finish tasks' arrival counter (0 before, reset by the last)
};
constexpr uint32_t kTaskCand = 2048;  // candidates a walk task stages (8 KiB of LDS)
constexpr uint64_t kSeamPeerFailed = 0x7FFFFFFFFFFFFFFFull;  // seam_resolve_kernel statuses
constexpr uint64_t kSeamRedo = 0x7FFFFFFFFFFFFFFEull;

constexpr uint32_t kMaxSpg = 255;  // segments per walk workgroup (+1 redundant)

struct StitchArgs {
  ChainParams chain;
  PieceCands pc;
  uint64_t anchor;   // seg_start(k) = anchor + k*seg for k >= 1
  uint64_t seg;      // SEG bytes
  uint32_t nseg;     // T
  uint32_t spg;      // segments per K2 workgroup
  uint32_t lds_cap;  // candidates per K2 workgroup (LDS)
  uint32_t scap;     // cut capacity per segment (SEG/min + 2)
  SegInfo* seg_info;
  uint64_t* stage;   // [nseg * scap]
  uint64_t* rep;     // [nseg * scap]
  uint32_t* rep_cnt;
  uint32_t* rep_from;
  uint32_t* flag_list;
  uint64_t* out_off;
  uint64_t* out;     // contiguous cut list (device)
  uint64_t out_cap;
  DevState* state;
  HostState* host_state;  // pinned, written by fixup_kernel (may be null)
  uint64_t seq;
  uint64_t* trace;        // diagnostics: per walk workgroup 5 timestamps (may be null)
  uint64_t init_carry;    // init: the chain origin
  uint32_t init;          // first piece of a call: walk_kernel resets the chain state
  uint32_t pad_init;
};

}  // namespace dsx
