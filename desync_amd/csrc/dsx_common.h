// dsx_common.h -- shared device/host definitions of the MI355X chunker.
//
// Terms (desync's domain):
//   candidate  position p whose 48-byte window [p-48,p) hashes to H(p) with
//              H(p) % d == d-1 (chunker.go:265-268); depends on p only.
//   cut        chunk end offset on the chain 0 -> next(0) -> ... -> len.
//   piece      contiguous byte range scanned by one scan launch.
//   lane seg   S contiguous bytes owned by one wavefront lane in the scan.
//   region     64 consecutive lane segments (one wavefront's work unit).
//   segment    stitch work unit: SEG bytes of cut-chain positions.
#pragma once
#include <stdint.h>

namespace dsx {

constexpr int kWave = 64;
// ---- scan kernel geometry (see DESIGN.md "Scan kernel") --------------------
constexpr int kRound = 48;                    // bytes per lane per round == window
constexpr int kTableBytes = 256 * 256;        // 256 byte values x 32 lane slots x {T,Trot}
constexpr int kScanLds = 163840;              // LDS per CU: table + per-wave staging
constexpr int kLaneSlots = 32;                // candidate slots per lane segment
// lane segment = 48*(BR*k-1) bytes, BR = rounds per DMA batch (warm-up round +
// segment = whole batches);
// offsets stay in u16
constexpr uint32_t kMaxLaneBytes = 48u * (2u * 682u - 1u);  // 65424


// Division-free boundary test constants (host-computed, chunker.go:147-170).
struct TestConsts {
  uint32_t d;      // discriminator
  uint32_t dm1;    // d - 1
  uint32_t madc;   // MODE 1: d - 1 - (d << 22) (folds the float offset, see is_cand)
  uint32_t ninv;   // MODE 2, scanl: 2^32 - inv, so (~h)*ninv = (h+1)*inv = t + 1
  uint32_t inv;    // inverse of odd part of d mod 2^32
  uint32_t qmax;   // (2^32-1)/d - qbias
  uint32_t qbias;
  uint32_t rot;    // k = ctz(d): rotate right by k
  float rcp;       // fl(1/d)
  float c0;        // MODE 1 magic offset 1.5*2^23 - 1
  uint32_t tadd;   // MODE 2: inv - 1, so t = h*inv + tadd = (h+1)*inv - 1
  uint32_t vmax;   // MODE 2: 2^k * floor(2^32/d); candidate => t < vmax
  uint32_t dodd;   // MODE 2: d >> k (h = (t - tadd) * dodd recovers h)
  uint32_t vmax1;  // MODE 2, scanl: vmax + 1 (candidate => t + 1 < vmax1; d >= 3 keeps it < 2^32)
};

struct TaskArgs;   // dsx_stitch.h
struct DevState;   // dsx_stitch.h
struct HostState;  // dsx_stitch.h

struct ScanArgs {
  const uint8_t* base;   // device pointer of the piece's first byte
  uint64_t halo;         // readable bytes before base (0 only at blob start)
  uint64_t piece_abs;    // absolute blob position of base[0]
  uint64_t len;          // piece length in bytes
  uint32_t lane_bytes;   // S = 48*(BR*batches - 1)
  uint32_t batches;      // (S/48 + 1) / BR
  uint32_t nregions;     // ceil(len / (64*S))
  uint32_t region_cap;   // list capacity per region
  TestConsts tc;
  uint64_t min_pos;      // candidates at absolute p < min_pos are dropped (origin + 49)
  uint32_t lane_slots;   // slot capacity per lane (kLaneSlots, or S on the dense path)
  uint32_t pf_batches;   // L2 prefetch distance in batches (PF kernels only)
  uint32_t* lane_slot;   // scratch [nregions*64*lane_slots]: per-lane hit entries (rare writes)
  uint32_t* region_cnt;  // [nregions] candidates per region (exact)
  uint32_t* region_list; // [nregions*region_cap] sorted offsets in (0, 64*S] from region base
  uint32_t* overflow;    // regions whose lanes or list overflowed (-> dense path)
  uint32_t* overflow_next;  // the next piece's counter: zeroed here (parity buffers)
  uint32_t* queue;       // region work queue (regions beyond the first wave slot pass):
                         // 8 counters (one per XCD) at queue[32*x]
  uint32_t* queue_next;  // the next piece's queue counters: zeroed here
  // line-aligned scan (scanl_kernel): the lane grid starts at base - delta,
  // the 128-B line holding base[0]; region 0's descriptor starts shift0 bytes
  // into its warm-up line (bytes before it read as zeros)
  uint32_t delta;
  uint32_t shift0;
  uint64_t* trace;       // diagnostics (DSX_SCAN_TRACE): per wave slot {start, end, regions}
  uint32_t wave_major;   // first regions wave-major over the grid (DSX_WAVE_MAJOR, default 1)
  uint32_t nt_loads;     // line DMA cache policy 0..3 (DSX_SCAN_NT, see dma16x8)
  uint32_t pad_;
  // scanl_kernel<FUSE>: the stitch tasks it carries, in pinned host memory
  // (read once per task; by value they held ~90 more SGPRs through the scan)
  const TaskArgs* tasks;
  // the previous queued piece's chain state, published by block 0 at the
  // start of this scan (a kernel boundary after that piece's stitch) instead
  // of by a publish_kernel of its own (pub_host null: nothing to publish)
  const DevState* pub_state;
  HostState* pub_host;
  uint64_t pub_seq;
  // measurement (dsx_stamps_begin): this launch's per-wave stamp records
  // (kStampWords words per wave slot blockIdx.x * W + wave), or null.  Every
  // wave writes its start/end s_memrealtime (100 MHz) and s_memtime (shader
  // clock) once, taken at its first and last instruction.
  uint64_t* stamp;
  // scanl_kernel, two region sizes: regions [nbig, nregions) have lane
  // segments of lane_bytes2 bytes (batches2 trips) after the nbig regions of
  // lane_bytes; lane_bytes2 == 0: one size
  uint32_t nbig;
  uint32_t lane_bytes2;
  uint32_t batches2;
  uint32_t pad3;
};

constexpr int kStampWords = 4;  // per wave: start rt, end rt, start cycles, end cycles

// line-aligned scan geometry: lane segments of S = 384*m bytes (3 DMA batches
// of one 128-B line per lane, so the ring phase repeats), offsets in u16
constexpr int kLine = 128;
constexpr int kScanTraceWords = 6;  // per wave: start, end, info, entry, region-end cycles, region-start waits
constexpr int kQueueSlots = 4;                  // overflow / queue slots (piece seq mod 4)
constexpr int kQueueWords = 32 + kQueueSlots * 256;  // overflow words + 4 x 8 queue counters
constexpr int kArriveWord = 16;                 // stitch_task_kernel's arrival counter (word 17)
constexpr uint32_t kLineLaneMax = 384u * 170u;  // 65280

// Sentinel for "successor depends on bytes beyond the piece" (non-final piece).
constexpr uint64_t kUndet = ~0ull;

}  // namespace dsx
