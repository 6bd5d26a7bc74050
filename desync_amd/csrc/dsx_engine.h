// dsx_engine.h -- host engine internals shared by the C-ABI translation
// units (dsx_api.cpp: cut lists, streaming, shards; dsx_index.cpp: file ->
// cut list + chunk IDs).  Not part of the ABI (include/dsx.h is).
#pragma once
#include <hip/hip_runtime.h>

#include <array>
#include <atomic>
#include <deque>
#include <functional>
#include <string>
#include <vector>

#include "../../include/dsx.h"
#include "dsx_common.h"
#include "dsx_digest.h"
#include "dsx_stitch.h"

namespace dsx {
template <class H, bool PF>
__global__ void digest_kernel(DigestArgs a);
template <class H>
__global__ void digest_pc_kernel(DigestArgs a);
template <int MODE, int VARIANT, int BR, int NBUF, int W, int SUB, bool PF>
__global__ void scan_kernel(ScanArgs a);
template <int MODE, int VARIANT, int W, int SUB, int D, bool FUSE, bool TWO>
__global__ void scanl_kernel(ScanArgs a);  // TWO: two region sizes (ScanArgs.lane_bytes2)
__global__ void stitch_task_kernel(TaskArgs b);
template <int NT>
__global__ void walk_kernel(StitchArgs a);
__global__ void fixup_kernel(StitchArgs a);
template <int PER>
__global__ void fixup_fast_kernel(StitchArgs a);  // PER = 1, 2, 4, 5, 8, 9
template <int PER>
__global__ void finish_kernel(StitchArgs a);
__global__ void gather_kernel(StitchArgs a);
__global__ void publish_kernel(StitchArgs a);
__global__ void noop_kernel();
__global__ void state_init_kernel(DevState* st, uint64_t carry);
__global__ void gen_uniform_kernel(uint8_t* dst, uint64_t offset, uint64_t len, uint64_t seed);
__global__ void gen_dedup_kernel(uint8_t* dst, uint64_t offset, uint64_t len, uint64_t seed,
                                 uint32_t p_thresh);
__global__ void boundary_selftest_kernel(TestConsts tc, int mode, uint64_t h0, uint64_t n,
                                         unsigned long long* mismatches);
__global__ void seam_cands_kernel(PieceCands pc, uint64_t lo, uint64_t wend, dsx_seam_t* seam);
__global__ void seam_finalize_kernel(dsx_seam_t* seam, const uint64_t* cuts, const DevState* st,
                                     uint64_t shard_start, uint64_t shard_len, uint64_t total,
                                     uint64_t wend0, uint64_t entry, uint32_t flags);
__global__ void seam_resolve_kernel(const dsx_seam_t* all, int nranks, int rank, uint64_t min,
                                    uint64_t max, uint64_t* ext, uint64_t* info);
__global__ void shard_emit_kernel(const uint64_t* info, const uint64_t* ext, const uint64_t* spec,
                                  const DevState* st, uint64_t* out, uint64_t cap,
                                  volatile uint64_t* res, int32_t* code);

}  // namespace dsx

using namespace dsx;

namespace dsx_host {

constexpr uint64_t kPieceMax = 8ull << 30;       // bytes per scan launch
constexpr uint64_t kStreamBatch = 16ull << 20;   // streaming: bytes per device batch
constexpr uint32_t kQueueDepth = 8;              // DSX_NO_SYNC calls queued per context
constexpr uint32_t kWalkLdsCap = 8192;           // candidates per walk workgroup (2 workgroups per CU)
constexpr uint32_t kDenseS = 48 * 9;             // dense path lane bytes (= slot cap)
constexpr uint64_t kDensePiece = 32ull << 20;    // dense path piece size

template <class T>
struct DevBuf {
  T* p = nullptr;
  size_t n = 0;
  hipError_t ensure(size_t want) {
    if (want <= n && p) return hipSuccess;
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
    size_t sz = want < 16 ? 16 : want;
    hipError_t e = hipMalloc((void**)&p, sz * sizeof(T));
    if (e == hipSuccess) n = sz;
    return e;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    n = 0;
  }
};

}  // namespace dsx_host
using namespace dsx_host;

// A piece's candidate lists kept past its call (shards: the O(candidates)
// re-walk re-runs only the stitch over them)
struct KeptPiece {
  DevBuf<uint32_t> cnt, list;
  PieceCands pc{};
  uint64_t P = 0, len = 0;
};

struct dsx_ctx {
  int device = 0;
  int ncu = 256;
  hipStream_t stream = nullptr, copy_stream = nullptr;
  // Scans run on scan_stream (highest priority; their grid leaves
  // `stitch_cus` CUs free) and everything else (the stitch, digests, copies,
  // host syncs) on `stream`: a piece's stitch then overlaps the next piece's
  // scan on the CUs the scan leaves free.  stitch_cus == 0:
  // scan_stream == stream.
  hipStream_t scan_stream = nullptr;
  int stitch_cus = 0;                      // DSX_STITCH_CUS (experiment, off: DESIGN.md 4.2)
  bool scan_mask = false;                  // DSX_SCAN_MASK: CU-masked scan stream (experiment)
  hipEvent_t ev_scan[2] = {}, ev_stitch[2] = {};  // per region-list set (piece parity)
  bool timing = true;  // record the per-piece scan/stitch events (stats.scan_ms/stitch_ms)
  std::atomic<int> cancel{0};
  // dsx_progress (another thread may read it while an index/cut call runs):
  // bytes up to the last confirmed cut of the running or last call
  std::atomic<uint64_t> prog_done{0};
  std::atomic<uint64_t> prog_len{0};
  std::atomic<int> prog_active{0};  // the running call's pieces publish into h_state
  std::string err;
  int force_mode = -1;  // DSX_TEST_MODE env override
  int variant = 0;      // DSX_SCAN_VARIANT: diagnostic scan ablations (wrong results)
  uint32_t lane_bytes_override = 0;  // DSX_LANE_BYTES (tuning; multiple of 48)
  int prefetch_batches = 0;           // DSX_PREFETCH: L2 prefetch distance in DMA batches (0 = off)
  int regions_per_slot = 1;           // DSX_REGIONS_PER_SLOT: scan work units per wave slot
  int scan_cfg = 0;                   // DSX_SCAN_CFG: index into kCfg* (waves, rounds/batch, LDS buffers)
  bool scan_line = true;              // DSX_SCAN_LINE=0: 96-B-row scan_kernel instead of scanl_kernel
  int digest_pc = -1;                 // DSX_DIGEST_PC: 1 producer/consumer digest kernel, 0 the one-wave kernel, -1 by size
  int digest_pc_chunks = 2;           // DSX_DIGEST_PC_CHUNKS: auto uses it up to this many chunks per grid lane
  int scanl_waves = 8;                // waves per workgroup of scanl_kernel
  uint32_t lane_target = 8448;        // DSX_LANE_TARGET: longest line-scan lane segment
  int tail_split = 4;                 // DSX_TAIL_SPLIT=k: tail regions with k x shorter lane segments (0/1: one size)
  int tail_mult = 1;                  // DSX_TAIL_MULT=j: the split tail is j big regions per wave slot
  uint64_t seg_max_mult = 4;          // DSX_SEG_MAX: stitch segment = max(mult * max, floor)
  uint64_t seg_floor = 1ull << 20;    // DSX_SEG_FLOOR
  uint64_t seg_target = 4096;         // DSX_SEG_TARGET: double the segment while a span has more (0: off)
  int walk_wgs = 2;                   // DSX_WALK_WGS: walk workgroups per CU the segments are spread over
  int walk_nt = 576;                  // DSX_WALK_NT: 576 = one wave per chain at 8 segments per workgroup (256: 4 waves)
  bool scan_trace = false;            // DSX_SCAN_TRACE: per-wave timestamps of the last scan
  bool wave_major = true;             // DSX_WAVE_MAJOR: scanl's first regions wave-major
  int scan_nt = 1;                    // DSX_SCAN_NT: line DMA cache policy (0 none, 1 nt: default, 2 sc1, 3 sc0 sc1 nt)
  bool finish = true;                 // DSX_FINISH=0: fixup_fast_kernel + gather_kernel instead of finish_kernel
  bool fixup_fast = true;             // DSX_FIXUP_FAST=0: fixup_kernel for every piece
  DevBuf<uint64_t> trace;       // [4 * trace_n scan records][10 * trace_walk_n walk records]
  uint64_t trace_n = 0, trace_walk_n = 0;
  bool trace_keep = false;            // DSX_SCAN_TRACE=2: a trace slot per piece (seq % 4)
  uint64_t trace_base = 0;            // word offset of the current piece's slot
  uint64_t last_grid_P = 0;           // region grid origin of the last enqueued piece

  DevBuf<uint32_t> region_cnt, region_list, overflow, rep_cnt, rep_from, flag_list;
  DevBuf<uint32_t> region_cnt2, region_list2;  // the second region-list set (split streams)
  const uint32_t* last_rcnt = nullptr;          // region lists of the last enqueued piece
  const uint32_t* last_rlist = nullptr;
  DevBuf<uint32_t> lane_slot;
  DevBuf<SegInfo> seg_info;
  DevBuf<uint64_t> stage, rep, out_off, out;
  DevBuf<uint64_t> dg_ends;   // chunk IDs: staged chunk ends
  DevBuf<uint8_t> dg_ids;     // chunk IDs: staged digests
  DevBuf<uint32_t> dg_queue;  // chunk IDs: lane work queue
  DevBuf<uint32_t> dg_order;  // chunk IDs: longest-first queue order (ctx-stream launches)
  DevBuf<uint32_t> dg_cls;    // chunk IDs: [kSizeClasses] counts, [kSizeClasses] offsets
  int digest_lpt = 1;         // DSX_DIGEST_LPT=0: digest_kernel's queue in index order
  int digest_pf = 1;          // DSX_DIGEST_PF=0: digest_kernel without the block prefetch
  DevBuf<DevState> state;
  HostState* h_state = nullptr;  // pinned mirror published by fixup_kernel
  uint64_t piece_seq = 0;        // global piece counter (overflow parity, freshness)
  bool init_pending = false;     // next scan initialises DevState with init_carry
  uint64_t last_region_bytes = 0;  // geometry of the last enqueued piece's region lists
  uint32_t last_nregions = 0, last_region_cap = 0;
  uint32_t last_nbig = 0;           // (two region sizes: regions [last_nbig, ...) have
  uint64_t last_region_bytes2 = 0;  //  last_region_bytes2 bytes; 0: one size)
  uint64_t init_carry = 0;
  bool last_finish = false;  // the last stitch publishes its state (the host may poll)
  // a queued call's final state is published by the next scan's block 0
  // (no publish_kernel of its own); flush_publish() launches it otherwise
  bool defer_publish = false;       // set while a queued cut_device call is enqueued
  HostState* pub_host = nullptr;    // pending: slot ...
  uint64_t pub_seq = 0;             // ... and piece seq
  // stitch behind the scan (DSX_FUSE=1, opt-in, off by default): queued one-piece calls
  // whose walk (walked = false) or finish (walked = true) runs as tasks in
  // the next queued call's scan; flush_behind() launches them on their own
  struct Behind {
    WalkJob w;
    FinishJob f;
    uint32_t nw = 0, nf = 0, wseg = 1, fseg = 1;
    bool walked = false;
    uint64_t seq = 0;
  };
  std::deque<Behind> behind;
  bool fuse = false;  // DSX_FUSE=1, libdsx_diag.so only (throughput-neutral under the board's power cap)
  static constexpr uint32_t kTaskRing = 16;  // > the launches a queued call can be behind
  TaskArgs* h_tasks = nullptr;               // pinned ring: the TaskArgs of fused scans
  uint64_t fuse_seq = 0;                     // fused calls enqueued (ring index)
  DevBuf<SegInfo> seg_info2;  // the second segment set (calls of odd piece seq)
  DevBuf<uint64_t> stage2;
  DevBuf<uint64_t> spec, spec2;  // stitch tasks' speculative chains (per set)

  // streaming state (Chunker.Next over an io.Reader)
  struct Stream {
    static constexpr int kSlots = 3;  // batches on the GPU at once
    struct Batch {
      uint64_t P, len, seq;
      bool last, ids;
      int slot;
    };
    bool active = false, eof = false, done = false, final_pending = false;
    bool fresh = true;   // the next batch starts the chain at fresh_carry
    bool dense = false;  // dense-candidate mode (after a lane overflow)
    dsx_params_t p{};
    uint64_t batch = 32ull << 20;  // DSX_STREAM_BATCH: bytes per device batch
    uint8_t* h = nullptr;          // pinned host buffer: stream bytes [hbase, hend)
    uint64_t hcap = 0, hbase = 0, hend = 0;
    uint64_t cur = 0;     // consumer position (start of the next chunk)
    uint64_t pin = 0;     // start of the chunks the last pop returned (kept until the next pop)
    std::vector<uint64_t> grp;                    // ends the last pop_many returned ...
    std::vector<std::array<uint8_t, 32>> grp_ids; // ... and their IDs (dsx_stream_unpop)
    uint64_t origin = 0;  // chain origin (0, an Advance target, a read-error restart)
    uint64_t sched = 0;   // bytes before this have been handed to the GPU
    uint64_t carry = 0;   // chain position after the collected batches
    uint64_t fresh_carry = 0;
    uint64_t skip = 0;    // Advance past the held bytes: future bytes to drop
    std::deque<uint64_t> cuts;  // confirmed chunk ends not yet popped
    std::deque<Batch> fly;      // batches on the GPU, oldest first
    int next_slot = 0;
    const uint8_t* last_chunk = nullptr;
    // chunk IDs computed next to the cuts (ChunkStream, dsx_stream_ids)
    int ids = -1;                                  // DSX_DIGEST_* or -1
    std::deque<std::array<uint8_t, 32>> idq;       // IDs of the queued cuts
    uint8_t last_id[32] = {};
    bool has_id = false;
    hipStream_t dg_stream = nullptr;               // digests overlap the next batch's scan
    // per-slot resources
    DevBuf<uint8_t> dbuf[kSlots];
    DevBuf<uint64_t> dout[kSlots];
    uint64_t* hcut[kSlots] = {};
    uint64_t hcut_cap[kSlots] = {};
    HostState* hstate = nullptr;  // pinned, kSlots entries
    hipEvent_t copy_ev[kSlots] = {}, done_ev[kSlots] = {}, stitch_ev[kSlots] = {};
    DevBuf<uint8_t> dids[kSlots];
    uint8_t* hids[kSlots] = {};
    uint64_t hids_cap[kSlots] = {};
    DevBuf<uint64_t> rng;     // per slot {0, entry cut} {cuts, exit cut}: the digest range
    DevBuf<uint32_t> dq;      // per slot digest queue counters
  } st;

  // multi-GPU shard state (dsx_shard_local -> dsx_shard_resolve)
  struct Shard {
    const uint8_t* d = nullptr;  // caller's shard bytes (valid until resolve returns OK)
    uint64_t halo = 0, start = 0, len = 0, total = 0;
    dsx_params_t p{};
    uint64_t nspec = 0;  // speculative cuts in ctx->out (~0: unknown, asynchronous local)
    bool pending = false;              // dsx_shard_resolve_async awaits dsx_shard_collect
    int pend_rank = 0;
    uint64_t pend_cap = 0;
    bool valid = false;
    bool dense = false;                // scanned on the dense path (lists not kept)
    // the shard's pieces' region lists: kept[0 .. nkept) of this run; the
    // buffers stay allocated across runs (a hipFree per step would wait for
    // the whole device, serialising the bench's pipeline lanes)
    std::vector<KeptPiece> kept;
    size_t nkept = 0;
  } sh;
  DevBuf<dsx_seam_t> d_seam, d_all;
  DevBuf<uint32_t> zero_word;  // an overflow flag that stays 0 (stitch-only re-runs)
  DevBuf<uint64_t> d_ext, d_info, d_emit;
  uint64_t* h_res = nullptr;  // pinned: shard_emit_kernel status / count / entry

  dsx_stats_t stats{};
  // in-kernel stamps of the scan launches (dsx_stamps_begin .. dsx_stamps_end):
  // launch i's per-wave records (stamp_slots x kStampWords words from
  // i * stamp_slots * kStampWords) belong to stamp_meta[i] = {seq, bytes}
  DevBuf<uint64_t> stamp_ring;
  uint64_t stamp_slots = 0;
  bool stamping = false;
  uint64_t stamp_cap = 0;
  std::vector<std::pair<uint64_t, uint64_t>> stamp_meta;
  // per-piece timing events of the current call: {before scan, after scan, after gather}
  std::vector<hipEvent_t> pev;
  uint32_t npiece_call = 0;

  // queued DSX_NO_SYNC calls, oldest first (each is re-run synchronously on
  // the dense path if needed).  They run in order on the ctx stream and each
  // publishes its chain state into its own pinned slot of h_ring.
  struct Pending {
    const void* d_blob = nullptr;
    uint64_t len = 0, cap = 0;
    dsx_params_t p{};
    uint64_t* out = nullptr;
    uint32_t slot = 0;
    uint64_t seq = 0;       // piece sequence number of the call's last piece
    hipEvent_t done = nullptr;  // recorded after the call (null: poll the published seq)
    bool behind = false;        // stitched behind later scans (c->behind)
    uint32_t npiece = 0;    // DSX_TIMED: pieces whose events are in q_pev[slot]
  };
  std::vector<hipEvent_t> q_pev[kQueueDepth];  // DSX_TIMED queued calls' piece events
  std::deque<Pending> pend;
  HostState* h_ring = nullptr;   // pinned, kQueueDepth slots
  HostState* h_cur = nullptr;    // slot the next enqueued piece publishes into

  // IndexFromFile pipeline (dsx_index.cpp): pinned read slots, two HBM
  // windows, chain-state snapshots that delimit each window's digest range
  static constexpr int kIdxSlots = 8;
  uint64_t index_window = 1ull << 30;  // DSX_INDEX_WINDOW: bytes per HBM window
  uint64_t index_slot = 32ull << 20;   // DSX_INDEX_SLOT: bytes per pinned read slot
  int index_readers = 4;               // DSX_INDEX_READERS: reader threads
  int64_t index_host_tail = -1;       // DSX_INDEX_HOST_TAIL: -1 auto, 0 off, > 0 chunks longer than this on the host
  uint8_t* idx_slots[kIdxSlots] = {};
  uint64_t idx_slot_bytes = 0;
  DevBuf<uint8_t> idx_win[2];
  DevBuf<uint64_t> idx_snap;
  hipEvent_t idx_copy_ev[kIdxSlots] = {};
  hipEvent_t idx_win_ev[2] = {};      // (recorded on idx_dg_stream after a window's digest)
  hipEvent_t idx_stitch_ev[2] = {};   // a window's last stitch + snapshot (on stream)
  // dsx_index_*'s digests run here, so a window's digest (its longest chunk's
  // chain, ~10-15 ms) does not hold the next window's scans and stitches on
  // `stream` (nor the tail feeder, which follows their published totals)
  // (= idx_side[0])
  hipStream_t idx_dg_stream = nullptr;
  // the GPU's shares of a one-window call during its read (dsx_index.cpp), one
  // stream each so that they run side by side, each with its queue counter
  // (idx_side_q[32 k], one 128-B line each; [32 kIdxSide]: the last window's
  // digest on `stream`); lowest priority: the runtime's
  // low-priority pool of GPU_MAX_HW_QUEUES (4) HSA queues holds exactly these,
  // none shared with `stream` or `copy_stream` (tools/queue_probe.hip)
  static constexpr int kIdxSide = 4;
  hipStream_t idx_side[kIdxSide] = {};
  DevBuf<uint32_t> idx_side_q;
  hipEvent_t q_ev[kQueueDepth] = {};
  uint32_t q_next = 0;
};

// Grow a device buffer; outstanding work may still use the old allocation, so
// drain both streams before freeing it.  Allocates 25% headroom.
template <class T>
inline hipError_t grow(dsx_ctx* c, DevBuf<T>& b, size_t n) {
  if (b.p && b.n >= n) return hipSuccess;
  if (b.p) {
    (void)hipStreamSynchronize(c->stream);
    (void)hipStreamSynchronize(c->copy_stream);
    if (c->scan_stream != c->stream) (void)hipStreamSynchronize(c->scan_stream);
  }
  return b.ensure(n + n / 4 + 64);
}

// The stream a piece's scan waits on for its input bytes (an H2D copy event,
// dsx_index.cpp / dsx_stream.cpp): the scan stream.
inline hipError_t scan_wait(dsx_ctx* c, hipEvent_t ev) {
  return hipStreamWaitEvent(c->scan_stream, ev, 0);
}

int set_hip_err(dsx_ctx* c, hipError_t e, const char* what);

#define HIPCHK(ctx, expr)                                  \
  do {                                                     \
    hipError_t e_ = (expr);                                \
    if (e_ != hipSuccess) return set_hip_err(ctx, e_, #expr); \
  } while (0)

struct CallCfg {
  const dsx_params_t* p;
  uint64_t L;        // blob length (final piece knows it)
  uint64_t origin;   // chain origin: first cut position (0, Advance target, shard start)
  uint64_t min_pos;  // candidates below this absolute position are not real windows
  uint64_t* d_out;   // device output
  uint64_t out_cap;
  bool dense;        // dense-candidate path
  uint64_t halo0 = 0;  // readable bytes before the first piece (shards)
  std::vector<KeptPiece>* keep = nullptr;  // keep every piece's region lists here (sh.nkept counts them)
  bool behind = false;  // one queued piece from 0: stitch behind later scans
};

// engine entry points (dsx_api.cpp)
int reset_state(dsx_ctx* c, uint64_t carry);
int read_state(dsx_ctx* c, HostState* out);
int enqueue_piece(dsx_ctx* c, const CallCfg& cc, const uint8_t* d_piece, uint64_t halo,
                  uint64_t P, uint64_t len, bool is_last);
int ensure_attr_walk(dsx_ctx* c);
// host threads (dsx_stream.cpp): fn(0) on the caller, fn(1..parts-1) on a
// persistent pool; returns when all have returned
void host_parallel(int parts, const std::function<void(int)>& fn);
// host CPUs this process may use (dsx_stream.cpp): the affinity mask, a
// cgroup v2 quota and OMP_NUM_THREADS (the GPU box's per-GPU share), or
// DSX_HOST_THREADS when set
int host_cpu_share();
// a stream for work beside the pipeline (window digests, the tail feeder's
// copies; dsx_stream.cpp): the lowest priority, so it takes an HSA queue of
// the runtime's low-priority pool instead of sharing one with the scan or
// copy stream (GPU_MAX_HW_QUEUES per pool, 4 on the box, tools/queue_probe)
hipError_t side_stream_create(hipStream_t* s);
// SHA-512/256 on the host (dsx_hostsha.cpp): one message, or 8 at once in
// AVX-512 lanes (only when host_sha_vec(); n[i] == UINT64_MAX: unused lane)
bool host_sha_vec();
void host_sha512_256_one(const uint8_t* p, uint64_t n, uint8_t* out);
void host_sha512_256_x8(const uint8_t* const p[8], const uint64_t n[8], uint8_t* const out[8]);
// launch the stitch tasks of the queued calls still behind (before any other
// work on the context, and when such a call is collected)
int flush_behind(dsx_ctx* c);
int flush_tasks(dsx_ctx* c);    // flush_behind without the pending publish
int flush_publish(dsx_ctx* c);  // launch the pending publish, if any
#define DSX_FLUSH_BEHIND(c)                  \
  do {                                       \
    if (c) {                                 \
      const int rc_fb_ = flush_behind(c);    \
      if (rc_fb_) return rc_fb_;             \
    }                                        \
  } while (0)
int launch_stitch(dsx_ctx* c, const CallCfg& cc, const PieceCands& pc, uint64_t P, uint64_t len,
                  bool is_last, uint64_t seq, bool trace);
// digest_kernel on `stream` (null: the ctx stream) with queue counter `queue`
// (null: the ctx's); max_n bounds the chunk count (sizes the grid); pc: 1
// digest_pc_kernel, 0 digest_kernel, -1 by max_n (DSX_DIGEST_PC overrides)
int launch_digest(dsx_ctx* c, DigestArgs da, uint64_t max_n, int algo, hipStream_t stream = nullptr,
                  uint32_t* queue = nullptr, bool serial = false, uint32_t max_blocks = 0, int pc = -1);
void index_release(dsx_ctx* c);   // dsx_index.cpp: frees the pipeline's buffers
void stream_release(dsx_ctx* c);  // dsx_stream.cpp: frees the stream's buffers
