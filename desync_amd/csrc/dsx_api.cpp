// dsx_api.cpp -- C ABI (include/dsx.h) and host engine of libdsx.so.
//
// The engine splits a blob into pieces, and per piece enqueues on the
// context's HIP stream: scan (dsx_scan.hip) -> walk -> fixup -> gather
// (dsx_stitch.hip).  The chain position is carried between pieces in device
// memory (DevState.carry), so a multi-piece call needs no host round trip
// until the end.  Reference interfaces replaced are listed in include/dsx.h.
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <string>
#include <vector>

#include "dsx_engine.h"

using namespace dsx;

// the seam record is exchanged as raw bytes between ranks (and mirrored by
// desync_amd/_lib.py::Seam): its layout is part of the ABI
static_assert(sizeof(dsx_seam_t) == 7 * 8 + 4 * 4 + 8 * (DSX_SEAM_MAX_CANDS + DSX_SEAM_MAX_CUTS),
              "dsx_seam_t layout");

static void release_kept(dsx_ctx* c);


int set_hip_err(dsx_ctx* c, hipError_t e, const char* what) {
  char buf[256];
  snprintf(buf, sizeof buf, "%s: %s", what, hipGetErrorString(e));
  c->err = buf;
  return e == hipErrorOutOfMemory || e == hipErrorMemoryAllocation ? DSX_E_NOMEM : DSX_E_HIP;
}

// --------------------------------------------------------------------------
// parameters (chunker.go:13-28, 134-171)
// --------------------------------------------------------------------------
static uint32_t discriminator_from_avg(uint64_t avg) {
  // float64, evaluated without FMA contraction (built with -ffp-contract=off)
  volatile double a = (double)avg;
  volatile double den = -1.42888852e-7 * a;
  den = den + 1.33237515;
  volatile double q = a / den;
  if (!(q >= 1.0 && q < 4294967296.0)) return 0u;
  return (uint32_t)q;
}

static uint32_t mod_inverse32(uint32_t d) {
  uint32_t x = d;
  for (int i = 0; i < 5; ++i) x *= 2u - d * x;
  return x;
}

extern "C" int dsx_abi_version(void) { return DSX_ABI_VERSION; }

extern "C" int dsx_params_init(uint64_t min, uint64_t avg, uint64_t max, dsx_params_t* out) {
  if (!out) return DSX_E_INVAL;
  if (min < 48) return DSX_E_MIN_TOO_SMALL;
  if (min > max) return DSX_E_MIN_GT_MAX;
  if (min > avg) return DSX_E_MIN_GT_AVG;
  if (avg > max) return DSX_E_AVG_GT_MAX;
  const uint32_t d = discriminator_from_avg(avg);
  if (d == 0) return DSX_E_AVG_RANGE;
  const uint32_t k = (uint32_t)__builtin_ctz(d);
  const uint32_t odd = d >> k;
  memset(out, 0, sizeof *out);
  out->min = min;
  out->avg = avg;
  out->max = max;
  out->discriminator = d;
  out->inverse_odd = mod_inverse32(odd);
  out->qbias = odd > 1u ? 1u : 0u;
  out->qmax = 0xFFFFFFFFu / d - out->qbias;
  out->rot = (int32_t)k;
  return DSX_OK;
}

extern "C" const char* dsx_strerror(int code) {
  switch (code) {
    case DSX_OK: return "ok";
    case DSX_E_MIN_TOO_SMALL: return "min chunk size too small, must be over 48";
    case DSX_E_MIN_GT_MAX: return "min chunk size must not be greater than max";
    case DSX_E_MIN_GT_AVG: return "min chunk size must not be greater than avg";
    case DSX_E_AVG_GT_MAX: return "avg chunk size must not be greater than max";
    case DSX_E_AVG_RANGE: return "avg chunk size out of range for discriminatorFromAvg";
    case DSX_E_INVAL: return "invalid argument";
    case DSX_E_CAPACITY: return "output capacity too small";
    case DSX_E_HIP: return "HIP runtime error";
    case DSX_E_NOMEM: return "out of memory";
    case DSX_E_INTERRUPTED: return "interrupted";
    case DSX_E_IO: return "I/O error";
    case DSX_E_STATE: return "invalid stream state";
    case DSX_E_INTERNAL: return "internal error";
    case DSX_E_RESYNC: return "seam records changed: all-gather them again and resolve again";
    case DSX_E_PEER: return "another rank failed (its seam record carries DSX_SEAM_ERROR)";
    default: return "unknown error";
  }
}

static TestConsts make_tc(const dsx_params_t* p) {
  TestConsts tc;
  tc.d = p->discriminator;
  tc.dm1 = p->discriminator - 1u;
  tc.inv = p->inverse_odd;
  tc.qmax = p->qmax;
  tc.qbias = p->qbias;
  tc.rot = (uint32_t)p->rot;
  tc.rcp = 1.0f / (float)p->discriminator;
  // MODE 1 (is_cand in dsx_scan.hip): fma(h, 1/d, 1.5*2^23 - 1) puts
  // round(h/d) - 1 + 0x400000 in the low mantissa bits; madc folds the
  // 0x400000*d offset and the -1 back into the exact 24-bit check.
  tc.c0 = 12582911.0f;
  tc.madc = p->discriminator - 1u - (p->discriminator << 22);
  // MODE 2 prefilter: with d = 2^k * dodd, h + 1 = d*m (1 <= m <= 2^32/d)
  // gives t = (h+1)*inv - 1 = 2^k*m - 1 < 2^k*floor(2^32/d) = vmax (exact
  // for odd d; for even d the rare path re-checks h % d == d-1)
  const uint32_t k = (uint32_t)p->rot;
  tc.tadd = p->inverse_odd - 1u;
  tc.vmax = (uint32_t)(((1ull << 32) / p->discriminator) << k);
  tc.dodd = p->discriminator >> k;
  // scanl keeps ~h in the hash register (the same recurrence from ~0), so
  // t + 1 = (h+1)*inv = (~h)*(2^32 - inv) is one v_mul_lo_u32
  tc.ninv = 0u - p->inverse_odd;
  tc.vmax1 = tc.vmax + 1u;
  return tc;
}

// MODE 2 (multiply-inverse prefilter, DESIGN.md "Boundary test") for every d
// that is not a power of two; MODE 1 (float, exact for 1024 < d < 2^22) or
// MODE 0 (Go's form) otherwise
static int pick_mode(const dsx_ctx* c, uint32_t d) {
  if (c->force_mode >= 0 && c->force_mode <= 2) {
    if (c->force_mode != 2 || (d & (d - 1u)) != 0) return c->force_mode;
  }
  if ((d & (d - 1u)) != 0) return 2;
  return (d > 1024u && d < (1u << 22)) ? 1 : 0;
}

// --------------------------------------------------------------------------
// context
// --------------------------------------------------------------------------
static char g_create_err[256];

extern "C" int dsx_ctx_create(int device, dsx_ctx_t** out) {
  if (!out) return DSX_E_INVAL;
  *out = nullptr;
  g_create_err[0] = 0;
  dsx_ctx* c = new dsx_ctx();
  c->device = device;
#define CREATE_STEP(expr)                                                              \
  do {                                                                                 \
    hipError_t e_ = (expr);                                                            \
    if (e_ != hipSuccess) {                                                            \
      snprintf(g_create_err, sizeof g_create_err, "%s: %s (%d)", #expr,                \
               hipGetErrorString(e_), (int)e_);                                        \
      dsx_ctx_destroy(c);                                                              \
      return e_ == hipErrorOutOfMemory ? DSX_E_NOMEM : DSX_E_HIP;                      \
    }                                                                                  \
  } while (0)
  CREATE_STEP(hipSetDevice(device));
  hipDeviceProp_t prop;
  CREATE_STEP(hipGetDeviceProperties(&prop, device));
  c->ncu = prop.multiProcessorCount;
  // The product library reads only these DSX_* settings (INTEGRATION.md,
  // "Environment"; each has a test).  Everything measured and rejected, and
  // every diagnostic geometry, is read by libdsx_diag.so only.
  if (const char* v = getenv("DSX_TAIL_SPLIT")) c->tail_split = std::max(0, std::min(8, atoi(v)));
  if (const char* v = getenv("DSX_LANE_TARGET"))
    c->lane_target = (uint32_t)std::max(384, std::min((int)kLineLaneMax, atoi(v)));
  if (const char* v = getenv("DSX_SEG_FLOOR")) c->seg_floor = (uint64_t)std::max(0L, atol(v));
  if (const char* v = getenv("DSX_SCAN_NT")) c->scan_nt = atoi(v) & 3;
  if (const char* v = getenv("DSX_DIGEST_PC")) c->digest_pc = atoi(v);
  if (const char* v = getenv("DSX_DIGEST_LPT")) c->digest_lpt = atoi(v) != 0;
  if (const char* v = getenv("DSX_INDEX_WINDOW")) c->index_window = (uint64_t)std::max(1L << 16, atol(v));
  if (const char* v = getenv("DSX_INDEX_SLOT")) c->index_slot = (uint64_t)std::max(1L << 12, atol(v));
  if (const char* v = getenv("DSX_INDEX_READERS")) c->index_readers = std::max(1, std::min(32, atoi(v)));
  if (const char* v = getenv("DSX_INDEX_HOST_TAIL")) c->index_host_tail = std::max(-1L, atol(v));
#if DSX_DIAG
  // ablation variants, alternative geometries and rejected experiments
  if (const char* m = getenv("DSX_TEST_MODE")) c->force_mode = atoi(m);
  if (const char* v = getenv("DSX_SCAN_VARIANT")) c->variant = atoi(v);
  if (const char* v = getenv("DSX_SCAN_CFG")) c->scan_cfg = std::min(5, std::max(0, atoi(v)));
  if (const char* v = getenv("DSX_DIGEST_PC_CHUNKS")) c->digest_pc_chunks = std::max(1, atoi(v));
  if (const char* v = getenv("DSX_PREFETCH")) c->prefetch_batches = std::max(0, atoi(v));
  if (const char* v = getenv("DSX_REGIONS_PER_SLOT")) c->regions_per_slot = std::max(1, atoi(v));
  if (const char* v = getenv("DSX_SCAN_LINE")) c->scan_line = atoi(v) != 0;
  if (const char* v = getenv("DSX_SCAN_TRACE")) {
    c->scan_trace = atoi(v) != 0;
    c->trace_keep = atoi(v) == 2;  // keep the traces of the last 4 pieces (slot = seq % 4)
  }
  if (const char* v = getenv("DSX_WAVE_MAJOR")) c->wave_major = atoi(v) != 0;
  if (const char* v = getenv("DSX_FIXUP_FAST")) c->fixup_fast = atoi(v) != 0;
  if (const char* v = getenv("DSX_FINISH")) c->finish = atoi(v) != 0;
  // the stitch behind the scan (tasks inside later scans)
  if (const char* v = getenv("DSX_FUSE")) c->fuse = atoi(v) != 0;
  if (const char* v = getenv("DSX_SEG_MAX")) c->seg_max_mult = std::max(1, atoi(v));
  if (const char* v = getenv("DSX_SEG_TARGET")) c->seg_target = (uint64_t)std::max(0L, atol(v));
  if (const char* v = getenv("DSX_WALK_WGS")) c->walk_wgs = std::max(1, std::min(4, atoi(v)));
  if (const char* v = getenv("DSX_WALK_NT")) c->walk_nt = atoi(v) == 576 ? 576 : 256;
  if (const char* v = getenv("DSX_DIGEST_PF")) c->digest_pf = atoi(v) != 0;
  if (const char* v = getenv("DSX_TAIL_MULT")) c->tail_mult = std::max(1, std::min(4, atoi(v)));
  if (const char* v = getenv("DSX_LANE_BYTES")) {
    const long lb = atol(v);
    if (lb >= 48 && lb % 48 == 0 && lb <= (long)kMaxLaneBytes) c->lane_bytes_override = (uint32_t)lb;
  }
  // split streams: the scan on a high-priority (or CU-masked) stream, the
  // stitch beside it on the CUs the scan leaves free
  if (const char* v = getenv("DSX_STITCH_CUS")) c->stitch_cus = std::max(0, std::min(c->ncu / 2, atoi(v)));
  if (const char* v = getenv("DSX_SCAN_MASK")) c->scan_mask = atoi(v) != 0;
#endif
  // The pipeline's streams at the highest priority: the runtime keeps
  // GPU_MAX_HW_QUEUES (4 on the box) HSA queues per priority and hands a
  // stream one at its first launch, sharing a queue once the pool is full,
  // and a kernel on a shared queue waits for the kernel ahead of it
  // (tools/queue_probe.hip, profiles/r06w, r06ai).  The default pool holds the
  // null stream and torch's streams (RCCL's among them: bench.py's N > 1
  // lanes would queue their scans behind another lane's collective); the
  // high pool holds the contexts' streams alone (copy_stream takes a queue
  // only where it is used, the file pipelines), the low pool the index
  // pipeline's digests (side_stream_create).
  {
    int least = 0, greatest = 0;
    CREATE_STEP(hipDeviceGetStreamPriorityRange(&least, &greatest));
#if DSX_DIAG
    if (const char* v = getenv("DSX_CTX_PRIO"))  // (A/B: 0 the default priority)
      if (atoi(v) == 0) greatest = 0;
#endif
    CREATE_STEP(hipStreamCreateWithPriority(&c->stream, hipStreamNonBlocking, greatest));
    CREATE_STEP(hipStreamCreateWithPriority(&c->copy_stream, hipStreamNonBlocking, greatest));
  }
  c->scan_stream = c->stream;
#if DSX_DIAG
  if (c->stitch_cus > 0) {
    // The scan's grid leaves stitch_cus CUs free (one per XCD at 8), and its
    // stream has the highest priority, so the dispatcher places a scan's
    // workgroups ahead of a concurrent stitch's, which fills the free CUs.
    // (A CU mask instead -- bit i is a CU of XCD i % 8 -- left one shader
    // engine per XCD a CU short of its round-robin share of the grid: a few
    // workgroups started only after the others ended, 1.9x the scan time.)
    hipStream_t ss = nullptr;
    if (c->scan_mask) {
      std::vector<uint32_t> mask((c->ncu + 31) / 32, 0u);
      for (int i = 0; i < c->ncu - c->stitch_cus; ++i) mask[i / 32] |= 1u << (i % 32);
      CREATE_STEP(hipExtStreamCreateWithCUMask(&ss, (uint32_t)mask.size(), mask.data()));
    } else {
      int least = 0, greatest = 0;
      CREATE_STEP(hipDeviceGetStreamPriorityRange(&least, &greatest));
      const char* pv = getenv("DSX_SCAN_PRIO");
      CREATE_STEP(hipStreamCreateWithPriority(&ss, hipStreamNonBlocking,
                                              pv && atoi(pv) == 0 ? least : greatest));
    }
    c->scan_stream = ss;
    for (int i = 0; i < 2; ++i) {
      CREATE_STEP(hipEventCreateWithFlags(&c->ev_scan[i], hipEventDisableTiming));
      CREATE_STEP(hipEventCreateWithFlags(&c->ev_stitch[i], hipEventDisableTiming));
    }
  }
#endif
  // coherent, like h_ring: the tail feeder (dsx_index.cpp) and dsx_progress
  // poll it while the stitch publishes into it mid-call
  CREATE_STEP(hipHostMalloc((void**)&c->h_state, sizeof(HostState), hipHostMallocCoherent));
  // coherent: dsx_result polls the seq the GPU publishes here
  CREATE_STEP(hipHostMalloc((void**)&c->h_ring, kQueueDepth * sizeof(HostState), hipHostMallocCoherent));
  memset(c->h_ring, 0, kQueueDepth * sizeof(HostState));
  c->h_cur = c->h_state;
  for (uint32_t i = 0; i < kQueueDepth; ++i)
    CREATE_STEP(hipEventCreateWithFlags(&c->q_ev[i], hipEventDisableTiming));
  CREATE_STEP(hipHostMalloc((void**)&c->h_res, 4 * sizeof(uint64_t)));
#if DSX_DIAG
  CREATE_STEP(hipHostMalloc((void**)&c->h_tasks, dsx_ctx::kTaskRing * sizeof(TaskArgs), hipHostMallocCoherent));
#endif
  memset(c->h_state, 0, sizeof(HostState));
  CREATE_STEP(c->state.ensure(1));
  // [0..1] overflow (piece parity); [32 + 256*parity + 32*x] the scan's work
  // queue counter x = 0..7 (one per XCD, each on its own 128-B line)
  CREATE_STEP(c->overflow.ensure(kQueueWords));
  CREATE_STEP(hipMemset(c->overflow.p, 0, kQueueWords * sizeof(uint32_t)));
  CREATE_STEP(hipMemset(c->state.p, 0, sizeof(DevState)));
#undef CREATE_STEP
  *out = c;
  return DSX_OK;
}

extern "C" int dsx_ctx_destroy(dsx_ctx_t* c) {
  if (!c) return DSX_OK;
  (void)hipSetDevice(c->device);
  if (c->stream) (void)hipStreamSynchronize(c->stream);
  if (c->copy_stream) (void)hipStreamSynchronize(c->copy_stream);
  if (c->scan_stream && c->scan_stream != c->stream) (void)hipStreamSynchronize(c->scan_stream);
  c->region_cnt.release(); c->region_list.release(); c->overflow.release(); c->rep_cnt.release(); c->rep_from.release();
  c->region_cnt2.release(); c->region_list2.release();
  c->flag_list.release(); c->lane_slot.release(); c->seg_info.release(); c->stage.release();
  c->dg_ends.release(); c->dg_ids.release(); c->dg_queue.release();
  c->dg_order.release(); c->dg_cls.release();
  c->rep.release(); c->out_off.release(); c->out.release(); c->state.release();
  c->seg_info2.release(); c->stage2.release(); c->spec.release(); c->spec2.release();
  release_kept(c);
  c->zero_word.release();
  c->d_seam.release(); c->d_all.release(); c->d_ext.release(); c->d_info.release(); c->d_emit.release();
  if (c->h_res) (void)hipHostFree(c->h_res);
  if (c->h_tasks) (void)hipHostFree(c->h_tasks);
  index_release(c);
  stream_release(c);
  if (c->h_state) (void)hipHostFree(c->h_state);
  if (c->h_ring) (void)hipHostFree(c->h_ring);
  for (uint32_t i = 0; i < kQueueDepth; ++i)
    if (c->q_ev[i]) (void)hipEventDestroy(c->q_ev[i]);
  for (hipEvent_t e : c->pev) (void)hipEventDestroy(e);
  for (auto& v : c->q_pev)
    for (hipEvent_t e : v) (void)hipEventDestroy(e);
  for (int i = 0; i < 2; ++i) {
    if (c->ev_scan[i]) (void)hipEventDestroy(c->ev_scan[i]);
    if (c->ev_stitch[i]) (void)hipEventDestroy(c->ev_stitch[i]);
  }
  if (c->scan_stream && c->scan_stream != c->stream) (void)hipStreamDestroy(c->scan_stream);
  if (c->stream) (void)hipStreamDestroy(c->stream);
  if (c->copy_stream) (void)hipStreamDestroy(c->copy_stream);
  delete c;
  return DSX_OK;
}

extern "C" const char* dsx_last_error(dsx_ctx_t* c) { return c ? c->err.c_str() : g_create_err; }

extern "C" int dsx_cancel(dsx_ctx_t* c) {
  if (!c) return DSX_E_INVAL;
  c->cancel.store(1);
  return DSX_OK;
}

// pb.Set(chunk.Start + chunk.Size) per assembled chunk (make.go:134-140): the
// end of the last confirmed chunk of the running (or last) index / cut call.
// Each piece's last stitch kernel publishes the chain position into pinned
// host memory; this reads it without touching the context's streams, so a
// second thread may call it while the call runs.  Monotone within a call.
extern "C" int dsx_progress(dsx_ctx_t* c, uint64_t* bytes) {
  if (!c || !bytes) return DSX_E_INVAL;
  uint64_t v = c->prog_done.load();
  if (c->prog_active.load()) {
    const uint64_t cur = ((volatile HostState*)c->h_state)->carry;
    if (cur > v && cur <= c->prog_len.load()) {
      uint64_t seen = v;
      while (seen < cur && !c->prog_done.compare_exchange_weak(seen, cur)) {
      }
      v = seen > cur ? seen : cur;
    }
  }
  *bytes = v;
  return DSX_OK;
}

extern "C" int dsx_debug_trace(dsx_ctx_t* c, uint64_t* out, uint64_t cap, uint64_t* n_scan,
                               uint64_t* n_walk) {
  DSX_FLUSH_BEHIND(c);
  if (!c || !n_scan || !n_walk) return DSX_E_INVAL;
  *n_scan = c->trace_n;
  *n_walk = c->trace_walk_n;
  const uint64_t words = c->trace_keep ? 4 * (kScanTraceWords * c->trace_n + 10 * 65536ull)
                                       : kScanTraceWords * c->trace_n + 10 * c->trace_walk_n;
  if (!words || !out) return DSX_OK;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  const uint64_t k = std::min<uint64_t>(cap, words);
  HIPCHK(c, hipMemcpy(out, c->trace.p, k * sizeof(uint64_t), hipMemcpyDeviceToHost));
  return DSX_OK;
}

extern "C" int dsx_copy(dsx_ctx_t* c, void* dst, const void* src, uint64_t n) {
  DSX_FLUSH_BEHIND(c);
  if (!c || (n && (!dst || !src))) return DSX_E_INVAL;
  if (!n) return DSX_OK;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  HIPCHK(c, hipMemcpy(dst, src, n, hipMemcpyDefault));
  return DSX_OK;
}

// Every device buffer a context holds (all of them are DevBufs, dsx_engine.h;
// tests/test_gpu_multiproc.py checks the sum against hipMemGetInfo).
static uint64_t ctx_device_bytes(const dsx_ctx* c) {
  uint64_t b = 0;
  auto add = [&](const auto& d) { b += d.n * sizeof(*d.p); };
  add(c->trace);
  add(c->region_cnt), add(c->region_list), add(c->overflow), add(c->rep_cnt), add(c->rep_from);
  add(c->flag_list), add(c->region_cnt2), add(c->region_list2), add(c->lane_slot);
  add(c->seg_info), add(c->stage), add(c->rep), add(c->out_off), add(c->out);
  add(c->dg_ends), add(c->dg_ids), add(c->dg_queue), add(c->dg_order), add(c->dg_cls);
  add(c->state), add(c->seg_info2), add(c->stage2), add(c->spec), add(c->spec2);
  for (int i = 0; i < dsx_ctx::Stream::kSlots; ++i)
    add(c->st.dbuf[i]), add(c->st.dout[i]), add(c->st.dids[i]);
  add(c->st.rng), add(c->st.dq);
  for (const auto& k : c->sh.kept) add(k.cnt), add(k.list);
  add(c->d_seam), add(c->d_all), add(c->zero_word), add(c->d_ext), add(c->d_info), add(c->d_emit);
  add(c->stamp_ring), add(c->idx_win[0]), add(c->idx_win[1]), add(c->idx_snap);
  return b;
}

extern "C" int dsx_get_stats(dsx_ctx_t* c, dsx_stats_t* out) {
  if (!c || !out) return DSX_E_INVAL;
  *out = c->stats;
  out->device_bytes = ctx_device_bytes(c);
  return DSX_OK;
}

// In-kernel stamps of the next max_launches line-scan launches (bench.py's
// roofline: the durations of exactly the launches its timed loop runs, with
// no event between them).  Waits for the context's queued work first.
extern "C" int dsx_stamps_begin(dsx_ctx_t* c, uint64_t max_launches) {
  if (!c || max_launches == 0 || max_launches > 65536) return DSX_E_INVAL;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (c->scan_stream != c->stream) HIPCHK(c, hipStreamSynchronize(c->scan_stream));
  c->stamp_slots = (uint64_t)c->ncu * (uint64_t)c->scanl_waves;  // wave slots of a line scan
  const uint64_t words = max_launches * c->stamp_slots * kStampWords;
  HIPCHK(c, grow(c, c->stamp_ring, words));
  HIPCHK(c, hipMemset(c->stamp_ring.p, 0, words * sizeof(uint64_t)));  // (end 0: slot unused)
  c->stamp_meta.clear();
  c->stamp_cap = max_launches;
  c->stamping = true;
  return DSX_OK;
}

// Stops stamping, waits for the stamped launches and reduces each one's
// per-wave records (first start, last end, summed spans) into min(cap, n)
// records in launch order; *n = the launches stamped.
extern "C" int dsx_stamps_end(dsx_ctx_t* c, dsx_scan_stamp_t* out, uint64_t cap, uint64_t* n) {
  if (!c || !n || (cap && !out)) return DSX_E_INVAL;
  const bool was = c->stamping;
  c->stamping = false;
  *n = 0;
  if (!was) return DSX_E_STATE;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (c->scan_stream != c->stream) HIPCHK(c, hipStreamSynchronize(c->scan_stream));
  const uint64_t k = c->stamp_meta.size();
  *n = k;
  const uint64_t m = std::min(cap, k);
  if (!m) return DSX_OK;
  const uint64_t per = c->stamp_slots * kStampWords;
  std::vector<uint64_t> raw(m * per);
  HIPCHK(c, hipMemcpy(raw.data(), c->stamp_ring.p, raw.size() * sizeof(uint64_t), hipMemcpyDeviceToHost));
  for (uint64_t i = 0; i < m; ++i) {
    dsx_scan_stamp_t s{};
    s.seq = c->stamp_meta[i].first;
    s.bytes = c->stamp_meta[i].second;
    s.t_first = ~0ull;
    for (uint64_t w = 0; w < c->stamp_slots; ++w) {
      const uint64_t* r = &raw[i * per + w * kStampWords];
      if (r[1] == 0) continue;  // (no wave in this slot)
      s.t_first = std::min(s.t_first, r[0]);
      s.t_last = std::max(s.t_last, r[1]);
      s.wave_ticks += r[1] - r[0];
      s.wave_cycles += r[3] - r[2];
      ++s.waves;
    }
    if (!s.waves) s.t_first = 0;
    out[i] = s;
  }
  return DSX_OK;
}

// --------------------------------------------------------------------------
// engine
// --------------------------------------------------------------------------

// Stitch segment for a span of n bytes: max(mult * max, floor), doubled while
// the span would have more than seg_target + 1 segments.  An 8 GiB piece gets
// 2 MiB segments (4096-4097 of them): walk 31 + fixup 13.7 + gather 5.0 us
// against 32.5 + 22.5 + 6.8 with 1 MiB, +0.45 % on the bench line; 4 MiB
// lengthens the walks' chains (walk 55.6 us) (profiles/r04k).
static uint64_t stitch_seg(const dsx_ctx* c, const dsx_params_t* p, uint64_t n) {
  uint64_t seg = std::max<uint64_t>(c->seg_max_mult * p->max, c->seg_floor);
  if (c->seg_target)
    while ((n + seg - 1) / seg > c->seg_target + 1 && seg < (1ull << 26)) seg <<= 1;
  return seg;
}

// The next scan launch initialises the device chain state (no memcpy).
int reset_state(dsx_ctx* c, uint64_t carry) {
  c->npiece_call = 0;
  c->init_pending = true;
  c->init_carry = carry;
  return DSX_OK;
}

// Wait for the stream; the last fixup_kernel published the state into pinned
// host memory.
int read_state(dsx_ctx* c, HostState* out) {
  HIPCHK(c, hipStreamSynchronize(c->stream));
  memcpy(out, (const void*)c->h_state, sizeof(HostState));
  if (out->seq != c->piece_seq) {
    c->err = "stale chain state (no piece completed)";
    return DSX_E_INTERNAL;
  }
  return DSX_OK;
}

// Enqueue scan + stitch for one piece [P, P+len) whose bytes are at d_piece
// (with `halo` readable bytes before it).
int enqueue_piece(dsx_ctx* c, const CallCfg& cc, const uint8_t* d_piece, uint64_t halo,
                         uint64_t P, uint64_t len, bool is_last) {
  const dsx_params_t* p = cc.p;
  // ---- scan geometry: balance regions over the persistent grid ----
  // lane segment S = 48*(4k-1): the warm-up round plus S/48 rounds fill k
  // whole 4-round DMA batches
  // scan configs: {waves per workgroup, rounds per DMA batch}
  static const int kCfgWaves[6] = {8, 12, 16, 12, 8, 16};
  static const int kCfgBR[6] = {2, 1, 1, 2, 2, 2};
  // line-aligned scan (scanl_kernel) unless disabled, on the dense path, or
  // when the grid origin P - delta would precede position 0
  const uint32_t delta = (uint32_t)((uintptr_t)d_piece & (kLine - 1));
  const bool line = c->scan_line && !cc.dense && P >= delta;
  const int W = line ? c->scanl_waves : kCfgWaves[c->scan_cfg];
  const int cfgBR = kCfgBR[c->scan_cfg];
  const bool split = c->scan_stream != c->stream;
  const int ncu_scan = c->ncu - (split ? c->stitch_cus : 0);  // CUs of the scan's mask
  const uint64_t slots_total = (uint64_t)ncu_scan * W;         // wave slots
  const uint64_t span = line ? len + delta : len;       // grid bytes
  uint32_t S, LS;
  uint32_t batches;
  if (cc.dense) {
    S = kDenseS;
    LS = S;
  } else if (line) {
    // S = 384*m: about regions_per_slot regions per wave slot
    const uint64_t lanes_min = slots_total * 64 * (uint64_t)c->regions_per_slot;
    const uint64_t per_lane = (span + lanes_min - 1) / lanes_min;
    const uint64_t rounds_needed = (per_lane + kLineLaneMax - 1) / kLineLaneMax;
    const uint64_t s = (span + rounds_needed * lanes_min - 1) / (rounds_needed * lanes_min);
    uint64_t m = (s + 3 * kLine - 1) / (3 * kLine);
    // lane segments longer than the target lose HBM efficiency (lane stride
    // 33 KB: 4.85 TB/s staging vs 6.24 TB/s at 8448 B, tools/ubench_staging.hip);
    // bigger pieces take more regions per wave slot from the work queue
    // (up to two trips past the target when that keeps every region in the
    // first pass: a second pass for a few regions costs a whole region time)
    const uint64_t mcap = c->lane_target / (3 * kLine);
    if (m > mcap + mcap / 4 || rounds_needed > 1) m = std::min<uint64_t>(m, mcap);
    m = std::max<uint64_t>(1, std::min<uint64_t>(m, kLineLaneMax / (3 * kLine)));
    S = (uint32_t)(3 * kLine * m);
    if (c->lane_bytes_override && c->lane_bytes_override % (3 * kLine) == 0 &&
        c->lane_bytes_override <= kLineLaneMax)
      S = c->lane_bytes_override;
    LS = kLaneSlots;
  } else {
    // about regions_per_slot regions per wave slot (dynamic queue balances
    // them), more if a lane segment would exceed kMaxLaneBytes
    const uint64_t lanes_min = slots_total * 64 * (uint64_t)c->regions_per_slot;
    const uint64_t per_lane = (len + lanes_min - 1) / lanes_min;
    const uint64_t rounds_needed = (per_lane + kMaxLaneBytes - 1) / kMaxLaneBytes;
    uint64_t s = (len + rounds_needed * lanes_min - 1) / (rounds_needed * lanes_min);
    const uint64_t BR = (uint64_t)cfgBR;
    uint64_t kb = (s / kRound + 1 + BR - 1) / BR;  // batches
    if (kb < 4) kb = 4;
    while (kRound * (BR * kb - 1) > kMaxLaneBytes) --kb;
    s = (uint64_t)kRound * (BR * kb - 1);
    if (c->lane_bytes_override && (c->lane_bytes_override / kRound + 1) % BR == 0)
      s = c->lane_bytes_override;
    S = (uint32_t)s;
    LS = kLaneSlots;
  }
  batches = line ? S / (3 * kLine) : (S / kRound + 1) / (uint32_t)cfgBR;
  const uint64_t region_bytes = 64ull * S;
  uint64_t nregions = len == 0 ? 0 : (span + region_bytes - 1) / region_bytes;
  // Two region sizes (DSX_TAIL_SPLIT = k > 1, default 4; line scan, pieces of
  // at least three big regions per wave slot): the last ~one big region's
  // worth of bytes per wave slot is cut into regions with k times shorter lane
  // segments, so the waves that drain the work queue last hold small regions
  // (DSX_TAIL_MULT = j: j big regions' worth per wave slot).  On the 8 GiB
  // pieces the waves end together (wave_busy 0.947 -> 0.98) and the scan is
  // 1 % faster; k = 2, 6, 8 and j = 2 less (profiles/r04d, r04e, r04g, r04aa).
  // (k = 3 was the default while every lane read a warm-up line: k = 4 read
  // 1.021 x the input against 1.018; since the warm-up handoff only lane 0 of
  // a region does, and k = 4 is 0.4-0.5 % ahead, profiles/r04ab.)
  uint64_t nbig = nregions, S2 = 0;
  if (line && !cc.dense && !cc.behind && c->tail_split > 1 && len > 0) {
    const uint64_t m = S / (3 * kLine), m2 = std::max<uint64_t>(1, m / (uint64_t)c->tail_split);
    const uint64_t tail = slots_total * region_bytes * (uint64_t)c->tail_mult;
    if (m2 < m && span >= 3 * tail) {
      const uint64_t rb2 = 64ull * 3 * kLine * m2;
      nbig = (span - tail) / region_bytes;
      nregions = nbig + (span - nbig * region_bytes + rb2 - 1) / rb2;
      S2 = 3 * kLine * m2;
    }
  }
  const uint64_t nlanes = nregions * 64;
  uint32_t rcap;
  if (cc.dense) {
    rcap = 64u * S;
  } else {
    const double expct = (double)region_bytes / (double)p->discriminator;
    rcap = (uint32_t)std::min<double>(64.0 * S, 4.0 * expct + 64.0);
    rcap = (rcap + 63u) & ~63u;
  }
  c->last_region_bytes = region_bytes;
  c->last_nregions = (uint32_t)nregions;
  c->last_region_cap = rcap;
  c->last_nbig = (uint32_t)nbig;
  c->last_region_bytes2 = S2 ? 64ull * S2 : 0;
  HIPCHK(c, grow(c, c->lane_slot, nlanes * LS));
  // region lists: the context's scratch, or (cc.keep: shards) buffers of
  // their own that outlive the call, so a re-walk can re-run the stitch
  // without scanning the bytes again
  uint32_t *rcnt, *rlist;
  KeptPiece* kp = nullptr;
  if (cc.keep) {
    if (c->sh.nkept == cc.keep->size()) cc.keep->emplace_back();
    kp = &(*cc.keep)[c->sh.nkept++];
    HIPCHK(c, grow(c, kp->cnt, nregions));  // (reused across runs: grows once)
    HIPCHK(c, grow(c, kp->list, nregions * rcap));
    rcnt = kp->cnt.p;
    rlist = kp->list.p;
  } else {
    // split streams: two region-list sets, so the next piece's scan writes
    // one while this piece's stitch reads the other
    // (and stitch behind: the next scan writes one while its tasks walk
    // the other)
    const bool second = (split || cc.behind) && (c->piece_seq + 1) % 2 == 1;
    auto& bc = second ? c->region_cnt2 : c->region_cnt;
    auto& bl = second ? c->region_list2 : c->region_list;
    HIPCHK(c, grow(c, bc, nregions));
    HIPCHK(c, grow(c, bl, nregions * rcap));
    rcnt = bc.p;
    rlist = bl.p;
  }
  c->last_rcnt = rcnt;
  c->last_rlist = rlist;
  // stitch behind: this call's segment set (by piece parity), and the tasks
  // of the calls behind it that this scan carries
  dsx_ctx::Behind me;
  TaskArgs tb{};
#if DSX_DIAG
  if (cc.behind) {
    const bool second = (c->piece_seq + 1) % 2 == 1;
    const uint64_t seg = stitch_seg(c, p, len);
    const uint64_t nseg = (len + seg - 1) / seg;
    const uint32_t scap = (uint32_t)(seg / p->min + 3);
    auto& bs = second ? c->seg_info2 : c->seg_info;
    auto& bt = second ? c->stage2 : c->stage;
    auto& bp = second ? c->spec2 : c->spec;
    if (bs.n < nseg || bt.n < nseg * scap || bp.n < nseg * scap) {
      // the call two back may still have to finish from this set: launch it
      // on its own before the set is reallocated
      int rc = flush_behind(c);
      if (rc) return rc;
      HIPCHK(c, grow(c, bs, nseg));
      HIPCHK(c, grow(c, bt, nseg * scap));
      HIPCHK(c, grow(c, bp, nseg * scap));
    }
    // segments per walk task (one lane each, up to 63): the task's
    // candidates fill at most half of its LDS on average
    const double exp_per_seg = (double)seg / (double)p->discriminator + 8.0;
    me.wseg = (uint32_t)std::max(1.0, std::min(32.0, std::floor(kTaskCand / (2.0 * exp_per_seg)) - 1.0));
    me.fseg = 32;
    me.nw = (uint32_t)((nseg + me.wseg - 1) / me.wseg);
    me.nf = (uint32_t)((nseg + me.fseg - 1) / me.fseg);
    me.w.min = p->min;
    me.w.max = p->max;
    me.w.L = len;
    me.w.seg = seg;
    me.w.nseg = (uint32_t)nseg;
    me.w.scap = scap;
    me.w.seg_info = bs.p;
    me.w.stage = bt.p;
    me.w.spec = bp.p;
    me.f.seg_info = bs.p;
    me.f.stage = bt.p;
    me.f.spec = bp.p;
    me.f.nseg = (uint32_t)nseg;
    me.f.scap = scap;
    me.f.out = cc.d_out;
    me.f.out_cap = cc.out_cap;
    me.f.host_state = c->h_cur;
    for (const auto& b : c->behind) {
      if (!b.walked) {
        tb.w = b.w;
        tb.nw = b.nw;
        tb.wseg = b.wseg;
      } else {
        tb.f = b.f;
        tb.nf = b.nf;
        tb.fseg = b.fseg;
      }
    }
  }
#endif
  const uint64_t seq = ++c->piece_seq;
  const int par = (int)(seq & 1);
  hipStream_t ss = c->scan_stream;

  ScanArgs sa{};
  sa.base = d_piece;
  sa.halo = halo;
  sa.piece_abs = P;
  sa.len = len;
  sa.lane_bytes = S;
  sa.batches = batches;
  sa.nregions = (uint32_t)nregions;
  if (S2) {
    sa.nbig = (uint32_t)nbig;
    sa.lane_bytes2 = (uint32_t)S2;
    sa.batches2 = (uint32_t)(S2 / (3 * kLine));
  }
  sa.region_cap = rcap;
  sa.tc = make_tc(p);
  sa.min_pos = cc.min_pos;
  sa.lane_slots = LS;
  sa.pf_batches = (uint32_t)c->prefetch_batches;
  sa.lane_slot = c->lane_slot.p;
  sa.region_cnt = rcnt;
  sa.region_list = rlist;
  // overflow word and queue counters: slot seq % 4; the scan zeroes the next
  // piece's slot (the stitch of the previous piece may still read its own)
  sa.overflow = c->overflow.p + (seq % kQueueSlots);
  sa.overflow_next = c->overflow.p + ((seq + 1) % kQueueSlots);
  sa.queue = c->overflow.p + 32 + 256 * (seq % kQueueSlots);
  sa.queue_next = c->overflow.p + 32 + 256 * ((seq + 1) % kQueueSlots);
  sa.wave_major = c->wave_major ? (cc.behind ? 2u : 1u) : 0u;
  sa.nt_loads = (uint32_t)c->scan_nt;
  if (c->pub_host) {  // the previous queued piece's state, published by this scan
    sa.pub_state = c->state.p;
    sa.pub_host = c->pub_host;
    sa.pub_seq = c->pub_seq;
    c->pub_host = nullptr;
  }
  tb.counter = sa.queue + 1;  // (zeroed by the previous scan, with the queue)
  tb.farrive = sa.queue + 2;

#if DSX_DIAG
  if (cc.behind) {
    // the ring advances with fused calls only: the slot was last read by the
    // scan of the fused call kTaskRing (16) fused calls ago, which completed
    // before the call kQueueDepth (8) queued calls ago was collected (a
    // non-fused multi-piece call between them does not move the index)
    TaskArgs* slot = c->h_tasks + (c->fuse_seq++ % dsx_ctx::kTaskRing);
    *slot = tb;
    sa.tasks = slot;
  }
#endif
  if (line) {
    // region 0's descriptor: the warm-up line unless it would start before
    // the readable bytes (then the 16-B step at or below base - min(halo, 48))
    const uint64_t hmin = std::min<uint64_t>(halo, kRound);
    sa.delta = delta;
    sa.shift0 = halo >= (uint64_t)delta + kLine
                    ? 0u
                    : (uint32_t)(16 * (((uint64_t)kLine + delta - hmin) / 16));
  }
  c->last_grid_P = line ? P - delta : P;
  if (c->stamping && line && c->stamp_meta.size() < c->stamp_cap && W == c->scanl_waves) {
    sa.stamp = c->stamp_ring.p + c->stamp_slots * kStampWords * c->stamp_meta.size();
    c->stamp_meta.emplace_back(seq, len);
  }
  if (c->scan_trace && line) {
    c->trace_n = (uint64_t)c->ncu * W;
    const uint64_t slot_words = kScanTraceWords * c->trace_n + 10 * 65536ull;
    HIPCHK(c, grow(c, c->trace, (c->trace_keep ? 4 : 1) * slot_words));
    c->trace_base = c->trace_keep ? (seq % 4) * slot_words : 0;
    // (stitch behind: 6 task words per wave slot follow, read as walk records)
    const uint64_t tw = cc.behind ? 6 * c->trace_n : 0;
    HIPCHK(c, hipMemsetAsync(c->trace.p + c->trace_base, 0, (kScanTraceWords * c->trace_n + tw) * sizeof(uint64_t), ss));
    sa.trace = c->trace.p + c->trace_base;
    if (cc.behind) c->trace_walk_n = (tw + 9) / 10;
  }
  const uint32_t pi = c->npiece_call++;
  while (c->pev.size() < 3 * (size_t)(pi + 1)) {
    hipEvent_t e;
    HIPCHK(c, hipEventCreate(&e));
    c->pev.push_back(e);
  }
  // the region lists this scan writes were read by the stitch two pieces ago
  if (split) HIPCHK(c, hipStreamWaitEvent(ss, c->ev_stitch[par], 0));
  if (c->timing) HIPCHK(c, hipEventRecord(c->pev[3 * pi], ss));
#if DSX_DIAG
  if (getenv("DSX_NOOP_BEFORE_SCAN")) hipLaunchKernelGGL(noop_kernel, dim3(1), dim3(64), 0, ss);
#endif
  {
    const uint64_t need_wg = std::max<uint64_t>(1, (nregions + W - 1) / W);
    // (stitch behind: every CU, so the wave slots beyond the regions -- spread
    // over the grid by the wave-major order -- run the tasks from the start)
    const uint32_t grid = cc.behind ? (uint32_t)ncu_scan
                                    : (uint32_t)std::min<uint64_t>(need_wg, (uint64_t)ncu_scan);
    const dim3 g(grid), b(W * kWave);
    const int mode = pick_mode(c, p->discriminator);
#if DSX_DIAG
#define DSX_ABLATE(K, ...)                                                                 \
  if (c->variant == 1) hipLaunchKernelGGL((K<2, 1, __VA_ARGS__>), g, b, 0, ss, sa); \
  else if (c->variant == 3) hipLaunchKernelGGL((K<2, 3, __VA_ARGS__>), g, b, 0, ss, sa); \
  else if (c->variant == 4) hipLaunchKernelGGL((K<2, 4, __VA_ARGS__>), g, b, 0, ss, sa); \
  else
// (the piece's region geometry picks TWO, as for the exact kernel: a one-size
// instantiation over a two-size region list reads past the piece)
#define DSX_LV(K, V, ...)                                                                  \
  do {                                                                                     \
    if (sa.lane_bytes2) hipLaunchKernelGGL((K<2, V, __VA_ARGS__, false, true>), g, b, 0, ss, sa); \
    else hipLaunchKernelGGL((K<2, V, __VA_ARGS__, false, false>), g, b, 0, ss, sa);      \
  } while (0)
#define DSX_ABLATEL(K, ...)                                                                \
  if (c->variant == 1) DSX_LV(K, 1, __VA_ARGS__);                                        \
  else if (c->variant == 3) DSX_LV(K, 3, __VA_ARGS__);                                   \
  else if (c->variant == 4) DSX_LV(K, 4, __VA_ARGS__);                                   \
  else if (c->variant == 7 && mode == 2) DSX_LV(K, 7, __VA_ARGS__);                      \
  else if (c->variant == 8 && mode == 2) DSX_LV(K, 8, __VA_ARGS__);                      \
  else if (c->variant == 9 && mode == 2) DSX_LV(K, 9, __VA_ARGS__);                      \
  else if (c->variant == 10 && mode == 2) DSX_LV(K, 10, __VA_ARGS__);                    \
  else
#else
#define DSX_ABLATE(K, ...)
#define DSX_ABLATEL(K, ...)
#endif
#define DSX_LAUNCH(BR, NB, WV, SUB, PF)                                                    \
  do {                                                                                     \
    DSX_ABLATE(scan_kernel, BR, NB, WV, SUB, PF)                                           \
    if (mode == 2)                                                                         \
      hipLaunchKernelGGL((scan_kernel<2, 0, BR, NB, WV, SUB, PF>), g, b, 0, ss, sa); \
    else if (mode == 1)                                                                    \
      hipLaunchKernelGGL((scan_kernel<1, 0, BR, NB, WV, SUB, PF>), g, b, 0, ss, sa); \
    else                                                                                   \
      hipLaunchKernelGGL((scan_kernel<0, 0, BR, NB, WV, SUB, PF>), g, b, 0, ss, sa); \
  } while (0)
#if DSX_DIAG
#define DSX_TRACE_VARIANTS(WV, SUB, D)                                                    \
  if (c->variant == 5) DSX_LV(scanl_kernel, 5, WV, SUB, D);                               \
  else if (c->variant == 6 && mode == 2) DSX_LV(scanl_kernel, 6, WV, SUB, D);             \
  else
#else
#define DSX_TRACE_VARIANTS(WV, SUB, D)
#endif
#define DSX_LAUNCHL(WV, SUB, D, FU, TW)                                                   \
  do {                                                                                    \
    if (mode == 2)                                                                        \
      hipLaunchKernelGGL((scanl_kernel<2, 0, WV, SUB, D, FU, TW>), g, b, 0, ss, sa);      \
    else if (mode == 1)                                                                   \
      hipLaunchKernelGGL((scanl_kernel<1, 0, WV, SUB, D, FU, TW>), g, b, 0, ss, sa);      \
    else                                                                                  \
      hipLaunchKernelGGL((scanl_kernel<0, 0, WV, SUB, D, FU, TW>), g, b, 0, ss, sa);      \
  } while (0)
#if DSX_DIAG
    if (line && cc.behind) {
      DSX_LAUNCHL(8, 8, 1, true, false);
    } else
#endif
    if (line) {
      DSX_ABLATEL(scanl_kernel, 8, 8, 1)
      DSX_TRACE_VARIANTS(8, 8, 1)
      if (sa.lane_bytes2) DSX_LAUNCHL(8, 8, 1, false, true);  // two region sizes
      else DSX_LAUNCHL(8, 8, 1, false, false);
    } else {
#if DSX_DIAG
      switch (c->scan_cfg) {
        case 1: DSX_LAUNCH(1, 2, 12, 4, false); break;
        case 2: DSX_LAUNCH(1, 2, 16, 4, false); break;
        case 3: DSX_LAUNCH(2, 1, 12, 8, false); break;
        case 4: DSX_LAUNCH(2, 1, 8, 8, false); break;
        case 5: DSX_LAUNCH(2, 1, 16, 4, false); break;
        default:
          if (c->prefetch_batches > 0) DSX_LAUNCH(2, 2, 8, 8, true);
          else DSX_LAUNCH(2, 2, 8, 8, false);
      }
#else
      DSX_LAUNCH(2, 2, 8, 8, false);
#endif
    }
#undef DSX_LAUNCH
#undef DSX_LAUNCHL
#undef DSX_ABLATE
#undef DSX_ABLATEL
#ifdef DSX_LV
#undef DSX_LV
#endif
#undef DSX_TRACE_VARIANTS
    HIPCHK(c, hipGetLastError());
  }
  if (c->timing) HIPCHK(c, hipEventRecord(c->pev[3 * pi + 1], ss));
  if (split) {  // the stitch (ctx stream) after the scan (scan stream)
    HIPCHK(c, hipEventRecord(c->ev_scan[par], ss));
    HIPCHK(c, hipStreamWaitEvent(c->stream, c->ev_scan[par], 0));
  }
  PieceCands pc{};
  pc.P = c->last_grid_P;  // region r covers (P' + base(r), P' + base(r) + bytes(r)]
  pc.RB = region_bytes;
  pc.RB2 = c->last_region_bytes2;
  pc.nbig = c->last_nbig;
  pc.nregions = (uint32_t)nregions;
  pc.region_cap = rcap;
  pc.region_cnt = rcnt;
  pc.region_list = rlist;
  pc.overflow = sa.overflow;
  if (kp) {
    kp->pc = pc;
    kp->P = P;
    kp->len = len;
  }
#if DSX_DIAG
  if (cc.behind) {
    // the call two back finished in this scan, the last one walked in it;
    // this one waits for the next scan (or flush_behind)
    me.w.pc = pc;
    me.f.overflow = sa.overflow;
    me.f.seq = seq;
    me.seq = seq;
    std::deque<dsx_ctx::Behind> next;
    for (auto& b : c->behind)
      if (!b.walked) {
        b.walked = true;
        next.push_back(b);
      }
    next.push_back(me);
    c->behind.swap(next);
    c->init_pending = false;
    c->last_finish = false;
    if (c->timing) HIPCHK(c, hipEventRecord(c->pev[3 * pi + 2], c->stream));
    c->stats.pieces++;
    return DSX_OK;
  }
#endif
  int rc = launch_stitch(c, cc, pc, P, len, is_last, seq, line && c->scan_trace);
  if (rc) return rc;
  if (split) HIPCHK(c, hipEventRecord(c->ev_stitch[par], c->stream));
  if (c->timing) HIPCHK(c, hipEventRecord(c->pev[3 * pi + 2], c->stream));
  c->stats.pieces++;
  return DSX_OK;
}

// The piece's state into the pinned host slot after its stitch (the host
// polls it for queued calls, reads it after a sync otherwise).
static int launch_publish(dsx_ctx* c, const StitchArgs& ta) {
  c->last_finish = ta.host_state != nullptr;
  if (!ta.host_state) return DSX_OK;
  if (c->defer_publish) {  // a queued call: the next scan publishes it
    c->pub_host = ta.host_state;
    c->pub_seq = ta.seq;
    return DSX_OK;
  }
  hipLaunchKernelGGL(publish_kernel, dim3(1), dim3(64), 0, c->stream, ta);
  HIPCHK(c, hipGetLastError());
  return DSX_OK;
}

int flush_publish(dsx_ctx* c) {
  if (!c->pub_host) return DSX_OK;
  StitchArgs ta{};
  ta.state = c->state.p;
  ta.host_state = c->pub_host;
  ta.seq = c->pub_seq;
  c->pub_host = nullptr;
  HIPCHK(c, hipSetDevice(c->device));
  hipLaunchKernelGGL(publish_kernel, dim3(1), dim3(64), 0, c->stream, ta);
  HIPCHK(c, hipGetLastError());
  return DSX_OK;
}

// walk -> fixup -> gather for one piece whose candidates are in pc.
int launch_stitch(dsx_ctx* c, const CallCfg& cc, const PieceCands& pc, uint64_t P, uint64_t len,
                  bool is_last, uint64_t seq, bool trace) {
  const dsx_params_t* p = cc.p;
  const uint64_t region_bytes = pc.RB;
  StitchArgs ta{};
  ta.chain.min = p->min;
  ta.chain.max = p->max;
  ta.chain.L = cc.L;
  ta.chain.PE = P + len;
  ta.chain.is_last = is_last ? 1u : 0u;
  ta.pc = pc;
  // the carried cut lies in (P - max, P] (its successor needed bytes >= P)
  const uint64_t anchor = (P > cc.origin + p->max) ? P - p->max : cc.origin;
  const uint64_t end = is_last ? cc.L : P + len;
  const uint64_t seg = stitch_seg(c, p, end > anchor ? end - anchor : 1);
  const uint64_t nseg = end > anchor ? (end - anchor + seg - 1) / seg : 1;
  ta.anchor = anchor;
  ta.seg = seg;
  ta.nseg = (uint32_t)nseg;
  const double exp_per_seg = (double)seg / (double)p->discriminator + 8.0;
  // segments per walk workgroup: about two workgroups per CU (the walks are
  // latency-bound), within the LDS candidate and region budgets
  uint64_t spg = std::max<uint64_t>(2, nseg / ((uint64_t)c->walk_wgs * (uint64_t)c->ncu));
  // split streams: the walk runs beside the next piece's scan on the CUs the
  // scan leaves free, two 1024-thread workgroups per CU (LDS: ~69 KiB each)
  const bool wide = c->scan_stream != c->stream;
  if (wide)
    spg = std::max<uint64_t>(spg, (nseg + 2ull * c->stitch_cus - 1) / (2ull * c->stitch_cus));
  spg = std::min<uint64_t>(spg, (uint64_t)((double)kWalkLdsCap / (2.0 * exp_per_seg)) - 1);
  // (the smaller region size bounds the regions a workgroup's span covers:
  // two region sizes put the short tail regions at the piece's end)
  const uint64_t rb_min = pc.RB2 ? std::min<uint64_t>(region_bytes, pc.RB2) : region_bytes;
  const uint64_t max_spg_reg = rb_min ? (4000ull * rb_min) / seg : kMaxSpg;
  spg = std::min<uint64_t>(spg, max_spg_reg > 2 ? max_spg_reg - 2 : 1);
  spg = std::max<uint64_t>(1, std::min<uint64_t>(spg, kMaxSpg));
  ta.spg = (uint32_t)spg;
  ta.lds_cap = kWalkLdsCap;
  ta.scap = (uint32_t)(seg / p->min + 3);
  HIPCHK(c, grow(c, c->seg_info, nseg));
  HIPCHK(c, grow(c, c->stage, nseg * ta.scap));
  HIPCHK(c, grow(c, c->rep, nseg * ta.scap));
  HIPCHK(c, grow(c, c->rep_cnt, nseg));
  HIPCHK(c, grow(c, c->rep_from, nseg));
  HIPCHK(c, grow(c, c->flag_list, nseg));
  HIPCHK(c, grow(c, c->out_off, nseg));
  ta.seg_info = c->seg_info.p;
  ta.stage = c->stage.p;
  ta.rep = c->rep.p;
  ta.rep_cnt = c->rep_cnt.p;
  ta.rep_from = c->rep_from.p;
  ta.flag_list = c->flag_list.p;
  ta.out_off = c->out_off.p;
  ta.out = cc.d_out;
  ta.out_cap = cc.out_cap;
  ta.state = c->state.p;
  ta.host_state = c->h_cur;
  ta.seq = seq;
  ta.init = c->init_pending ? 1u : 0u;  // the call's first piece: walk_kernel resets the state
  ta.init_carry = c->init_carry;
  c->init_pending = false;
  c->last_finish = false;
  const uint32_t walk_grid = (uint32_t)((nseg + spg - 1) / spg);
  if (trace && walk_grid <= 65536) {
    ta.trace = c->trace.p + c->trace_base + kScanTraceWords * c->trace_n;
    c->trace_walk_n = walk_grid;
  }
  const size_t walk_lds = (size_t)kWalkLdsCap * 4 + (kMaxSpg + 1) * 8;
  if (wide)
    hipLaunchKernelGGL(walk_kernel<1024>, dim3(walk_grid), dim3(1024), walk_lds, c->stream, ta);
  else if (c->walk_nt == 576 && spg == 8)  // (the 8 GiB pieces: 8 segments + the redundant one, a wave each)
    hipLaunchKernelGGL(walk_kernel<576>, dim3(walk_grid), dim3(576), walk_lds, c->stream, ta);
  else
    hipLaunchKernelGGL(walk_kernel<256>, dim3(walk_grid), dim3(256), walk_lds, c->stream, ta);
  HIPCHK(c, hipGetLastError());
  if (c->finish && nseg <= 2048) {  // fixup + gather over nseg/16 workgroups
    const dim3 fg((uint32_t)((nseg + 15) / 16));
    if (nseg <= 256) hipLaunchKernelGGL(finish_kernel<1>, fg, dim3(256), 0, c->stream, ta);
    else if (nseg <= 512) hipLaunchKernelGGL(finish_kernel<2>, fg, dim3(256), 0, c->stream, ta);
    else if (nseg <= 1024) hipLaunchKernelGGL(finish_kernel<4>, fg, dim3(256), 0, c->stream, ta);
    else hipLaunchKernelGGL(finish_kernel<8>, fg, dim3(256), 0, c->stream, ta);
    HIPCHK(c, hipGetLastError());
    return launch_publish(c, ta);
  }
  if (c->fixup_fast && nseg <= 9 * 1024) {
    if (nseg <= 1024) hipLaunchKernelGGL(fixup_fast_kernel<1>, dim3(1), dim3(1024), 0, c->stream, ta);
    else if (nseg <= 2048) hipLaunchKernelGGL(fixup_fast_kernel<2>, dim3(1), dim3(1024), 0, c->stream, ta);
    else if (nseg <= 4096) hipLaunchKernelGGL(fixup_fast_kernel<4>, dim3(1), dim3(1024), 0, c->stream, ta);
    else if (nseg <= 5120) hipLaunchKernelGGL(fixup_fast_kernel<5>, dim3(1), dim3(1024), 0, c->stream, ta);
    else if (nseg <= 8192) hipLaunchKernelGGL(fixup_fast_kernel<8>, dim3(1), dim3(1024), 0, c->stream, ta);
    else hipLaunchKernelGGL(fixup_fast_kernel<9>, dim3(1), dim3(1024), 0, c->stream, ta);
  } else {
    hipLaunchKernelGGL(fixup_kernel, dim3(1), dim3(1024), 0, c->stream, ta);
  }
  HIPCHK(c, hipGetLastError());
  hipLaunchKernelGGL(gather_kernel, dim3((uint32_t)nseg), dim3(256), 0, c->stream, ta);
  HIPCHK(c, hipGetLastError());
  return launch_publish(c, ta);
}

// Runs a whole device-resident blob [origin.., origin+len) through the engine.
static int run_device(dsx_ctx* c, const uint8_t* d_blob, uint64_t len, CallCfg cc) {
  HIPCHK(c, hipSetDevice(c->device));
  int rc = reset_state(c, cc.origin);
  if (rc) return rc;
  const uint64_t piece = cc.dense ? kDensePiece : kPieceMax;
  for (uint64_t off = 0; off < len; off += piece) {
    if (c->cancel.load()) return DSX_E_INTERRUPTED;
    const uint64_t n = std::min(piece, len - off);
    rc = enqueue_piece(c, cc, d_blob + off, off + cc.halo0, cc.origin + off, n, off + n == len);
    if (rc) return rc;
  }
  return DSX_OK;
}

int ensure_attr_walk(dsx_ctx* c) {
  static bool done = false;
  if (!done) {
    HIPCHK(c, hipFuncSetAttribute((const void*)walk_kernel<256>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)(kWalkLdsCap * 4 + (kMaxSpg + 1) * 8)));
    HIPCHK(c, hipFuncSetAttribute((const void*)walk_kernel<576>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)(kWalkLdsCap * 4 + (kMaxSpg + 1) * 8)));
    HIPCHK(c, hipFuncSetAttribute((const void*)walk_kernel<1024>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)(kWalkLdsCap * 4 + (kMaxSpg + 1) * 8)));
    done = true;
  }
  return DSX_OK;
}

int flush_behind(dsx_ctx* c) {
  const int rc = flush_tasks(c);
  return rc ? rc : flush_publish(c);
}

int flush_tasks(dsx_ctx* c) {
  if (c->behind.empty()) return DSX_OK;
#if DSX_DIAG
  HIPCHK(c, hipSetDevice(c->device));
  // round 1: the walked call's finish and the other's walk (independent);
  // round 2: the latter's finish
  while (!c->behind.empty()) {
    TaskArgs tb{};
    tb.farrive = c->overflow.p + kArriveWord + 1;
    for (const auto& b : c->behind) {
      if (!b.walked) {
        tb.w = b.w;
        tb.nw = b.nw;
        tb.wseg = b.wseg;
      } else {
        tb.f = b.f;
        tb.nf = b.nf;
        tb.fseg = b.fseg;
      }
    }
    const uint32_t n = tb.nw + tb.nf;
    if (n) {
      hipLaunchKernelGGL(stitch_task_kernel, dim3((n + 3) / 4), dim3(256), 0, c->stream, tb);
      HIPCHK(c, hipGetLastError());
    }
    std::deque<dsx_ctx::Behind> next;
    for (auto& b : c->behind)
      if (!b.walked) {
        b.walked = true;
        next.push_back(b);
      }
    c->behind.swap(next);
  }
#endif
  return DSX_OK;
}

// A queued cut_device call that can be stitched behind later scans: one
// line-aligned piece from 0, a candidate density the walk tasks' LDS holds.
static bool behind_ok(dsx_ctx* c, const void* d_blob, uint64_t len, const dsx_params_t* p) {
#if !DSX_DIAG
  return false;  // the stitch behind the scan is in libdsx_diag.so only
#endif
  if (!c->fuse || !c->scan_line || c->stitch_cus > 0 || c->variant) return false;
  if (len == 0 || len > kPieceMax || ((uintptr_t)d_blob & (kLine - 1)) != 0) return false;
  const uint64_t seg = stitch_seg(c, p, len);
  const double exp_per_seg = (double)seg / (double)p->discriminator + 8.0;
  return 4.0 * exp_per_seg <= (double)kTaskCand;  // wseg >= 1 with room to spare
}

static int finish_call(dsx_ctx* c, uint64_t* n_out, uint64_t cap, bool* dense_retry) {
  HostState s;
  int rc = read_state(c, &s);
  if (rc) return rc;
  *dense_retry = false;
  if (s.err & kErrDense) {
    *dense_retry = true;
    return DSX_OK;
  }
  c->stats.chunks = s.total;
  c->stats.repaired_segments = s.repaired;
  c->stats.chunks_discarded = s.discarded;
  float scan = 0, stitch = 0;
  for (uint32_t i = 0; i < c->npiece_call; ++i) {
    float a = 0, b = 0;
    (void)hipEventElapsedTime(&a, c->pev[3 * i], c->pev[3 * i + 1]);
    (void)hipEventElapsedTime(&b, c->pev[3 * i + 1], c->pev[3 * i + 2]);
    scan += a;
    stitch += b;
  }
  c->stats.scan_ms = scan;
  c->stats.stitch_ms = stitch;
  *n_out = s.total;
  if ((s.err & kErrCapacity) || s.total > cap) return DSX_E_CAPACITY;
  return DSX_OK;
}

extern "C" int dsx_sync(dsx_ctx_t* c) {
  if (!c) return DSX_E_INVAL;
  int rc = flush_behind(c);
  if (rc) return rc;
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return DSX_OK;
}

extern "C" int dsx_cut_device(dsx_ctx_t* c, const void* d_blob, uint64_t len, const dsx_params_t* p,
                              uint64_t* out_ends, uint64_t cap, uint64_t* n_out, uint32_t flags);

extern "C" int dsx_result(dsx_ctx_t* c, uint64_t* n_out) {
  if (!c || !n_out) return DSX_E_INVAL;
  if (c->pend.empty()) return DSX_E_STATE;
  const dsx_ctx::Pending q = c->pend.front();
  c->pend.pop_front();
  HIPCHK(c, hipSetDevice(c->device));
  if (q.behind) {  // its stitch still waits for a later scan: run it now
    for (const auto& b : c->behind)
      if (b.seq == q.seq) {
        const int rc = flush_behind(c);
        if (rc) return rc;
        break;
      }
  }
  if (c->pub_host && c->pub_seq == q.seq) {  // no later scan carried its publish
    const int rc = flush_publish(c);
    if (rc) return rc;
  }
  if (q.done) HIPCHK(c, hipEventSynchronize(q.done));
  {
    // poll the published seq (published after the event when a later scan
    // or flush_publish carries it); the stream going idle without it is an error
    const volatile uint64_t* sp = &c->h_ring[q.slot].seq;
    for (uint32_t spins = 1; *sp != q.seq; ++spins) {
      if (spins % 4096u == 0) {
        const hipError_t e = hipStreamQuery(c->stream);
        if (e == hipSuccess) break;  // (seq checked below)
        if (e != hipErrorNotReady) return set_hip_err(c, e, "hipStreamQuery");
      }
      __builtin_ia32_pause();
    }
    std::atomic_thread_fence(std::memory_order_acquire);
  }
  HostState s;
  memcpy(&s, (const void*)&c->h_ring[q.slot], sizeof(HostState));
  if (s.seq != q.seq) {
    c->err = "stale chain state (queued call did not complete)";
    return DSX_E_INTERNAL;
  }
  if (s.err & (kErrDense | kErrRedo)) {
    // rare: redo synchronously (dense-candidate path, or the general stitch
    // with fixup_kernel's repair when a behind-the-scan stitch met a suspect
    // segment)
    if (s.err & kErrDense) c->stats.dense_fallbacks++;
    dsx_params_t p = q.p;
    return dsx_cut_device(c, q.d_blob, q.len, &p, q.out, q.cap, n_out, DSX_OUT_DEVICE);
  }
  c->stats.chunks = s.total;
  c->stats.repaired_segments = s.repaired;
  c->stats.chunks_discarded = s.discarded;
  float scan = 0, stitch = 0;  // untimed queued calls record no events
  for (uint32_t i = 0; i < q.npiece; ++i) {
    float a = 0, b = 0;
    (void)hipEventElapsedTime(&a, c->q_pev[q.slot][3 * i], c->q_pev[q.slot][3 * i + 1]);
    (void)hipEventElapsedTime(&b, c->q_pev[q.slot][3 * i + 1], c->q_pev[q.slot][3 * i + 2]);
    scan += a;
    stitch += b;
  }
  c->stats.scan_ms = scan;
  c->stats.stitch_ms = q.behind ? 0.0f : stitch;  // (inside later scans)
  *n_out = s.total;
  if ((s.err & kErrCapacity) || s.total > q.cap) return DSX_E_CAPACITY;
  return DSX_OK;
}

extern "C" int dsx_cut_device(dsx_ctx_t* c, const void* d_blob, uint64_t len, const dsx_params_t* p,
                              uint64_t* out_ends, uint64_t cap, uint64_t* n_out, uint32_t flags) {
  if (!c || !p || !n_out || (len && !d_blob) || (cap && !out_ends)) return DSX_E_INVAL;
  c->cancel.store(0);
  int rc = ensure_attr_walk(c);
  if (rc) return rc;
  *n_out = 0;
  if (len == 0) return DSX_OK;  // TestChunkerEmptyFile: no chunks
  const bool dev_out = (flags & DSX_OUT_DEVICE) != 0;
  const uint64_t need = len / p->min + 2;
  const bool queued = (flags & DSX_NO_SYNC) && dev_out;
  const bool fuse = queued && behind_ok(c, d_blob, len, p);
  if (!fuse) {  // every other call starts after the stitches still behind
    rc = flush_tasks(c);
    if (rc) return rc;
  }
  if (!queued) {  // (a queued call's first scan publishes the previous one's state)
    rc = flush_publish(c);
    if (rc) return rc;
  }
  if (queued) {
    if (c->pend.size() >= kQueueDepth) {
      c->err = "too many queued DSX_NO_SYNC calls (collect them with dsx_result)";
      return DSX_E_STATE;
    }
    CallCfg cc{p, len, 0, kRound, out_ends, cap, false};
    cc.behind = fuse;
    dsx_ctx::Pending q;
    q.d_blob = d_blob;
    q.len = len;
    q.cap = cap;
    q.p = *p;
    q.out = out_ends;
    q.slot = c->q_next++ % kQueueDepth;
    q.done = c->q_ev[q.slot];
    c->h_cur = &c->h_ring[q.slot];
    // queued calls record no timing events unless DSX_TIMED: an event record
    // between two kernels of a stream costs ~6 us of GPU time (rocprofv3
    // kernel trace).  A timed call records into its slot's own events.
    const bool timed = (flags & DSX_TIMED) != 0;
    c->timing = timed;
    if (timed) std::swap(c->pev, c->q_pev[q.slot]);
    // (split streams: the next scan runs on scan_stream and waits only for
    // the stitch two pieces back, so it could publish a state the previous
    // stitch is still writing; publish_kernel then runs on the ctx stream)
    c->defer_publish = c->scan_stream == c->stream;
    rc = run_device(c, (const uint8_t*)d_blob, len, cc);
    c->defer_publish = false;
    if (timed) std::swap(c->pev, c->q_pev[q.slot]);
    q.npiece = timed ? c->npiece_call : 0u;
    c->timing = true;
    c->h_cur = c->h_state;
    if (rc) return rc;
    // an event record costs ~6 us of stream time between two jobs (rocprofv3
    // kernel trace): when finish_kernel ended the call, its last workgroup
    // publishes the state after every cut is written, and dsx_result polls it
    q.behind = fuse;
    if (fuse || (!timed && c->last_finish)) q.done = nullptr;
    else HIPCHK(c, hipEventRecord(q.done, c->stream));
    q.seq = c->piece_seq;
    c->pend.push_back(q);
    return DSX_OK;
  }
  for (int attempt = 0; attempt < 2; ++attempt) {
    CallCfg cc{p, len, 0, kRound, nullptr, 0, attempt == 1};
    if (dev_out) {
      cc.d_out = out_ends;
      cc.out_cap = cap;
    } else {
      HIPCHK(c, grow(c, c->out, need));
      cc.d_out = c->out.p;
      cc.out_cap = need;
    }
    rc = run_device(c, (const uint8_t*)d_blob, len, cc);
    if (rc) return rc;
    bool dense = false;
    rc = finish_call(c, n_out, dev_out ? cap : need, &dense);
    if (dense) {
      c->stats.dense_fallbacks++;
      continue;
    }
    if (rc) return rc;
    if (!dev_out && *n_out > cap) return DSX_E_CAPACITY;
    if (!dev_out && *n_out) {
      HIPCHK(c, hipMemcpy(out_ends, c->out.p, *n_out * sizeof(uint64_t), hipMemcpyDeviceToHost));
    }
    return DSX_OK;
  }
  c->err = "dense-candidate path overflowed";
  return DSX_E_INTERNAL;
}

// --------------------------------------------------------------------------
// synthetic data
// --------------------------------------------------------------------------
extern "C" int dsx_gen_uniform(dsx_ctx_t* c, void* d_dst, uint64_t offset, uint64_t len,
                               uint64_t seed) {
  if (!c || (len && !d_dst)) return DSX_E_INVAL;
  HIPCHK(c, hipSetDevice(c->device));
  if (!len) return DSX_OK;
  const uint64_t threads = (len + 15) / 16;
  const uint32_t grid = (uint32_t)std::min<uint64_t>((threads + 255) / 256, 65536);
  hipLaunchKernelGGL(gen_uniform_kernel, dim3(grid), dim3(256), 0, c->stream, (uint8_t*)d_dst,
                     offset, len, seed);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return DSX_OK;
}

extern "C" int dsx_gen_dedup(dsx_ctx_t* c, void* d_dst, uint64_t offset, uint64_t len,
                             uint64_t seed, double p_repeat) {
  if (!c || (len && !d_dst) || !(p_repeat >= 0.0 && p_repeat < 1.0)) return DSX_E_INVAL;
  HIPCHK(c, hipSetDevice(c->device));
  if (!len) return DSX_OK;
  const uint32_t thresh = (uint32_t)std::min(4294967295.0, p_repeat * 4294967296.0);
  const uint64_t threads = (len + 15) / 16;
  const uint32_t grid = (uint32_t)std::min<uint64_t>((threads + 255) / 256, 65536);
  hipLaunchKernelGGL(gen_dedup_kernel, dim3(grid), dim3(256), 0, c->stream, (uint8_t*)d_dst,
                     offset, len, seed, thresh);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return DSX_OK;
}

// --------------------------------------------------------------------------
// chunk IDs (Digest.Sum per chunk: digest.go:11-29, make.go:223)
// --------------------------------------------------------------------------
// Enqueues digest_kernel on the ctx stream.  max_n bounds the chunk count
// (the grid is sized from it; with da.range_lo the count is read on the
// device).
int launch_digest(dsx_ctx* c, DigestArgs da, uint64_t max_n, int algo, hipStream_t stream,
                  uint32_t* queue, bool serial, uint32_t max_blocks, int pc) {
  // the ctx stream, or a stream whose digests the caller runs one after
  // another (serial: dsx_index_*'s digest stream): the size-order scratch
  // (dg_order, dg_cls) is then never used by two launches at once
  const bool own = stream == nullptr || serial;
  if (!stream) stream = c->stream;
  if (!queue) {
    HIPCHK(c, c->dg_queue.ensure(1));
    queue = c->dg_queue.p;
  }
  // split producer/consumer kernel: one workgroup (producer + consumer wave)
  // per CU, up to digest_pc_chunks chunks per lane of the grid
  const uint64_t pc_lanes = (uint64_t)c->ncu * 64u;
  if (c->digest_pc >= 0) pc = c->digest_pc > 0 ? 1 : 0;  // (DSX_DIGEST_PC)
  if (pc > 0 || (pc < 0 && max_n <= pc_lanes * (uint64_t)c->digest_pc_chunks)) {
    uint64_t blocks = std::max<uint64_t>(1, std::min<uint64_t>((max_n + 63) / 64, c->ncu));
    if (max_blocks) blocks = std::min<uint64_t>(blocks, max_blocks);
    HIPCHK(c, hipMemsetAsync(queue, 0, 4, stream));
    da.queue = queue;
    da.nfirst = (uint32_t)std::min<uint64_t>(da.n, blocks * 64u);
    if (algo == DSX_DIGEST_SHA512_256)
      hipLaunchKernelGGL(digest_pc_kernel<Sha512>, dim3((uint32_t)blocks), dim3(128), 0, stream, da);
    else
      hipLaunchKernelGGL(digest_pc_kernel<Sha256>, dim3((uint32_t)blocks), dim3(128), 0, stream, da);
    HIPCHK(c, hipGetLastError());
    return DSX_OK;
  }
  // Lanes: exactly the workgroups that are resident at once (occupancy is set
  // by VGPRs: 2 per CU for SHA-512, 3 without the prefetch, 4 for SHA-256),
  // every lane pulling chunks
  // from the queue.  A larger grid would hand its non-resident workgroups a
  // static share that starts only when the first wave of workgroups is done.
  int per_cu = 0;
  const bool sha512 = algo == DSX_DIGEST_SHA512_256;
#if DSX_DIAG
  const bool pf = c->digest_pf != 0;
#else
  constexpr bool pf = true;
#endif
  const void* kern = sha512 ? (const void*)digest_kernel<Sha512, true>
                            : (const void*)digest_kernel<Sha256, true>;
#if DSX_DIAG
  if (!pf)
    kern = sha512 ? (const void*)digest_kernel<Sha512, false>
                  : (const void*)digest_kernel<Sha256, false>;
#endif
  HIPCHK(c, hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, kDigestThreads, 0));
  if (per_cu < 1) per_cu = 1;
  uint64_t blocks = std::max<uint64_t>(
      1, std::min<uint64_t>((max_n + kDigestThreads - 1) / kDigestThreads,
                            (uint64_t)per_cu * (uint64_t)c->ncu));
  if (max_blocks) blocks = std::min<uint64_t>(blocks, max_blocks);
  HIPCHK(c, hipMemsetAsync(queue, 0, 4, stream));
  da.queue = queue;
  da.nfirst = (uint32_t)std::min<uint64_t>(da.n, blocks * kDigestThreads);
  // the chunks go out longest first (a counting sort by size class, three
  // small passes on the same stream): with more chunks than lanes the long
  // chains start in the first round; with fewer, each wave's 64 static chunks
  // are of one size, so no lane idles behind a longer neighbour
  if (own && c->digest_lpt && max_n >= 8u * kDigestThreads && max_n < (1ull << 32)) {
    HIPCHK(c, grow(c, c->dg_order, max_n));
    HIPCHK(c, c->dg_cls.ensure(2 * kSizeClasses));
    HIPCHK(c, hipMemsetAsync(c->dg_cls.p, 0, kSizeClasses * sizeof(uint32_t), stream));
    const dim3 tiles((uint32_t)((max_n + kOrderTile - 1) / kOrderTile));
    hipLaunchKernelGGL(digest_order_count_kernel, tiles, dim3(256), 0, stream, da, c->dg_cls.p);
    hipLaunchKernelGGL(digest_order_scan_kernel, dim3(1), dim3(kSizeClasses), 0, stream,
                       (const uint32_t*)c->dg_cls.p, c->dg_cls.p + kSizeClasses);
    hipLaunchKernelGGL(digest_order_scatter_kernel, tiles, dim3(256), 0, stream, da,
                       c->dg_cls.p + kSizeClasses, c->dg_order.p);
    HIPCHK(c, hipGetLastError());
    da.order = c->dg_order.p;
  }
  if (sha512 && pf)
    hipLaunchKernelGGL((digest_kernel<Sha512, true>), dim3((uint32_t)blocks), dim3(kDigestThreads),
                       0, stream, da);
  else if (pf)
    hipLaunchKernelGGL((digest_kernel<Sha256, true>), dim3((uint32_t)blocks), dim3(kDigestThreads),
                       0, stream, da);
#if DSX_DIAG
  else if (sha512)
    hipLaunchKernelGGL((digest_kernel<Sha512, false>), dim3((uint32_t)blocks), dim3(kDigestThreads),
                       0, stream, da);
  else
    hipLaunchKernelGGL((digest_kernel<Sha256, false>), dim3((uint32_t)blocks), dim3(kDigestThreads),
                       0, stream, da);
#endif
  HIPCHK(c, hipGetLastError());
  return DSX_OK;
}

extern "C" int dsx_chunk_ids(dsx_ctx_t* c, const void* d_blob, uint64_t len, uint64_t start,
                             const uint64_t* ends, uint64_t n, void* ids, uint32_t flags,
                             int algo) {
  DSX_FLUSH_BEHIND(c);
  if (!c || (n && (!d_blob || !ends || !ids)) || (algo != DSX_DIGEST_SHA512_256 &&
                                                   algo != DSX_DIGEST_SHA256))
    return DSX_E_INVAL;
  if ((flags & ~(DSX_OUT_DEVICE | DSX_ENDS_DEVICE)) != 0) return DSX_E_INVAL;
  if (n == 0) return DSX_OK;
  if (n > 0xFFFFFFF0ull) return DSX_E_INVAL;
  if (!(flags & DSX_ENDS_DEVICE)) {
    // chunks must lie inside the blob, in order (a hand-built index could
    // otherwise send the kernel past the end of the buffer); device-resident
    // ends are bounds-checked per chunk by the kernel instead
    uint64_t prev = start;
    for (uint64_t i = 0; i < n; ++i) {
      if (ends[i] < prev || ends[i] > len) {
        c->err = "chunk ends must be non-decreasing, start <= ends[0], ends[n-1] <= len";
        return DSX_E_INVAL;
      }
      prev = ends[i];
    }
  }
  HIPCHK(c, hipSetDevice(c->device));
  c->err.clear();
  const uint64_t* d_ends = ends;
  if (!(flags & DSX_ENDS_DEVICE)) {
    HIPCHK(c, grow(c, c->dg_ends, n));
    HIPCHK(c, hipMemcpyAsync(c->dg_ends.p, ends, n * 8, hipMemcpyHostToDevice, c->stream));
    d_ends = c->dg_ends.p;
  }
  uint8_t* d_ids = (uint8_t*)ids;
  if (!(flags & DSX_OUT_DEVICE)) {
    HIPCHK(c, grow(c, c->dg_ids, n * 32));
    d_ids = c->dg_ids.p;
  }
  DigestArgs da{};
  da.blob = (const uint8_t*)d_blob;
  da.len = len;
  da.ends = d_ends;
  da.first_start = start;
  da.n = n;
  da.ids = d_ids;
  int rc = launch_digest(c, da, n, algo);
  if (rc) return rc;
  if (!(flags & DSX_OUT_DEVICE))
    HIPCHK(c, hipMemcpyAsync(ids, d_ids, n * 32, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  return DSX_OK;
}

// --------------------------------------------------------------------------
// diagnostics: GPU boundary predicate vs h % d == d-1
// --------------------------------------------------------------------------
extern "C" int dsx_selftest_boundary(dsx_ctx_t* c, const dsx_params_t* p, int mode, uint64_t h0,
                                     uint64_t n, uint64_t* mismatches) {
  DSX_FLUSH_BEHIND(c);
  if (!c || !p || !mismatches) return DSX_E_INVAL;
  HIPCHK(c, hipSetDevice(c->device));
  if (mode < 0) mode = pick_mode(c, p->discriminator);
  const uint32_t d = p->discriminator;
  if (mode > 2 || (mode == 2 && (d & (d - 1u)) == 0)) return DSX_E_INVAL;  // MODE 2 needs dodd > 1
  DevBuf<unsigned long long> m;
  HIPCHK(c, m.ensure(1));
  HIPCHK(c, hipMemsetAsync(m.p, 0, 8, c->stream));
  hipLaunchKernelGGL(boundary_selftest_kernel, dim3(4096), dim3(256), 0, c->stream, make_tc(p),
                     mode, h0, n, m.p);
  HIPCHK(c, hipGetLastError());
  unsigned long long v = 0;
  HIPCHK(c, hipMemcpyAsync(&v, m.p, 8, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  m.release();
  *mismatches = v;
  return DSX_OK;
}

// --------------------------------------------------------------------------
// multi-GPU shards (split-and-align across ranks, make.go:22-163 / 277-327)
// --------------------------------------------------------------------------
// Chunks the shard from the cut `entry` (shard_start: speculative, make.go's
// worker at span*i; or the true entry cut on a re-walk), builds the seam
// record in c->d_seam, leaves the shard's cuts in c->out and waits.
static void release_kept(dsx_ctx* c) {
  for (auto& k : c->sh.kept) {
    k.cnt.release();
    k.list.release();
  }
  c->sh.kept.clear();
  c->sh.nkept = 0;
}

// Chunks the shard from the cut `entry` (shard_start: speculative, make.go's
// worker at span*i; or the true entry cut on a re-walk), builds the seam
// record in c->d_seam, leaves the shard's cuts in c->out and waits.
// The first run scans the bytes and keeps every piece's candidate lists; a
// re-walk (rewalk = true) only re-runs the stitch over the kept lists from
// the new entry: O(candidates), no byte is read again.  (Pieces that needed
// the dense-candidate path keep no lists; their re-walk scans again.)
// With async, nothing waits: the chain state is not read back (a stitch
// error, including the overflow that the synchronous path retries on the
// dense path, is published as DSX_SEAM_REDO in the record, see
// seam_finalize_kernel) and sh.nspec stays unknown (the emit kernel reads the
// count on the device).
static int shard_run(dsx_ctx* c, uint64_t entry, uint32_t rec_flags, bool rewalk,
                     bool async = false) {
  auto& sh = c->sh;
  const dsx_params_t* p = &sh.p;
  const bool is_last = sh.start + sh.len == sh.total;
  const uint64_t need = sh.len / p->min + 4;
  const uint64_t wend0 = sh.start + std::min<uint64_t>(sh.len, 32 * p->max);
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, grow(c, c->d_seam, 1));
  const bool stitch_only = rewalk && !sh.dense && sh.nkept > 0;
  for (int attempt = 0; attempt < 2; ++attempt) {
    if (c->cancel.load()) return DSX_E_INTERRUPTED;
    HIPCHK(c, grow(c, c->out, need));
    const bool dense = attempt == 1 || (rewalk && sh.dense);
    CallCfg cc{p, sh.total, entry, kRound, c->out.p, need, dense};
    cc.halo0 = sh.start > 0 ? sh.halo : 0;
    int rc = DSX_OK;
    if (stitch_only) {
      HIPCHK(c, c->zero_word.ensure(1));
      HIPCHK(c, hipMemsetAsync(c->zero_word.p, 0, 4, c->stream));
      hipLaunchKernelGGL(state_init_kernel, dim3(1), dim3(64), 0, c->stream, (DevState*)c->state.p,
                         entry);
      HIPCHK(c, hipGetLastError());
      c->npiece_call = 0;
      for (size_t i = 0; i < sh.nkept && !rc; ++i) {
        PieceCands pc = sh.kept[i].pc;
        pc.overflow = c->zero_word.p;  // (the scan succeeded: no overflow)
        rc = launch_stitch(c, cc, pc, sh.kept[i].P, sh.kept[i].len,
                           is_last && i + 1 == sh.nkept, ++c->piece_seq, false);
      }
      if (rc) return rc;
      hipLaunchKernelGGL(seam_cands_kernel, dim3(1), dim3(64), 0, c->stream, sh.kept[0].pc,
                         sh.start, wend0, c->d_seam.p);
      HIPCHK(c, hipGetLastError());
    } else {
      sh.nkept = 0;  // (the buffers are reused)
      cc.keep = dense ? nullptr : &sh.kept;
      sh.dense = dense;
      rc = reset_state(c, entry);
      if (rc) return rc;
      const uint64_t piece = cc.dense ? kDensePiece : kPieceMax;
      for (uint64_t off = 0; off < sh.len; off += piece) {
        const uint64_t n = std::min(piece, sh.len - off);
        rc = enqueue_piece(c, cc, sh.d + off, off + cc.halo0, sh.start + off, n,
                           is_last && off + n == sh.len);
        if (rc) return rc;
        if (off == 0) {
          // the window candidates come from the first piece's region lists
          PieceCands pc{};
          pc.P = c->last_grid_P;
          pc.RB = c->last_region_bytes;
          pc.RB2 = c->last_region_bytes2;
          pc.nbig = c->last_nbig;
          pc.nregions = c->last_nregions;
          pc.region_cap = c->last_region_cap;
          pc.region_cnt = cc.keep ? sh.kept[0].cnt.p : c->last_rcnt;
          pc.region_list = cc.keep ? sh.kept[0].list.p : c->last_rlist;
          pc.overflow = nullptr;
          hipLaunchKernelGGL(seam_cands_kernel, dim3(1), dim3(64), 0, c->stream, pc, sh.start,
                             wend0, c->d_seam.p);
          HIPCHK(c, hipGetLastError());
        }
      }
    }
    hipLaunchKernelGGL(seam_finalize_kernel, dim3(1), dim3(1), 0, c->stream, c->d_seam.p,
                       (const uint64_t*)c->out.p, (const DevState*)c->state.p, sh.start, sh.len,
                       sh.total, wend0, entry, (is_last ? (uint32_t)DSX_SEAM_LAST : 0u) | rec_flags);
    HIPCHK(c, hipGetLastError());
    if (async) {
      sh.nspec = ~0ull;
      return DSX_OK;
    }
    HostState st;
    rc = read_state(c, &st);
    if (rc) return rc;
    if ((st.err & kErrDense) && !stitch_only) {
      c->stats.dense_fallbacks++;
      continue;
    }
    if (st.err) {
      c->err = "shard: stitch error";
      return DSX_E_INTERNAL;
    }
    sh.nspec = st.total;
    c->stats.chunks = st.total;
    return DSX_OK;
  }
  c->err = "dense-candidate path overflowed";
  return DSX_E_INTERNAL;
}

// Copies the ctx's seam record to the caller's (host or device) record; a
// device record is left in flight on the ctx stream when `wait` is false.
static int seam_out(dsx_ctx* c, dsx_seam_t* seam, bool dev, bool wait = true) {
  HIPCHK(c, hipMemcpyAsync(seam, c->d_seam.p, sizeof(dsx_seam_t),
                           dev ? hipMemcpyDeviceToDevice : hipMemcpyDeviceToHost, c->stream));
  if (wait || !dev) HIPCHK(c, hipStreamSynchronize(c->stream));
  return DSX_OK;
}

extern "C" int dsx_shard_local(dsx_ctx_t* c, const void* d_shard, uint64_t halo,
                               uint64_t shard_start, uint64_t shard_len, uint64_t total,
                               const dsx_params_t* p, dsx_seam_t* seam, uint32_t flags) {
  DSX_FLUSH_BEHIND(c);
  if (!c || !p || !seam || (shard_len && !d_shard) || shard_start + shard_len > total ||
      (flags & ~(DSX_SEAM_DEVICE | DSX_NO_SYNC)) != 0 ||
      ((flags & DSX_NO_SYNC) && !(flags & DSX_SEAM_DEVICE)))
    return DSX_E_INVAL;
  const bool async = (flags & DSX_NO_SYNC) != 0;
  if (shard_start > 0 && halo < kRound) return DSX_E_INVAL;
  c->cancel.store(0);
  int rc = ensure_attr_walk(c);
  if (rc) return rc;
  auto& sh = c->sh;
  sh.d = (const uint8_t*)d_shard;
  sh.halo = halo;
  sh.start = shard_start;
  sh.len = shard_len;
  sh.total = total;
  sh.p = *p;
  sh.nspec = 0;
  sh.valid = false;
  if (shard_len == 0) {
    dsx_seam_t z;
    memset(&z, 0, sizeof z);
    z.shard_start = z.exit_cut = z.window_end = z.entry = shard_start;
    z.total = total;
    z.first_cand_beyond = UINT64_MAX;
    z.flags = shard_start == total ? DSX_SEAM_LAST : 0u;
    HIPCHK(c, grow(c, c->d_seam, 1));
    HIPCHK(c, hipMemcpyAsync(c->d_seam.p, &z, sizeof z, hipMemcpyHostToDevice, c->stream));
    sh.valid = true;
    return seam_out(c, seam, (flags & DSX_SEAM_DEVICE) != 0);
  }
  rc = shard_run(c, shard_start, 0u, false, async);
  if (rc) return rc;
  sh.valid = true;
  return seam_out(c, seam, (flags & DSX_SEAM_DEVICE) != 0, !async);
}

// The resolve outcome published by shard_emit_kernel (h_res), interpreted on
// the host: DSX_OK with the count, DSX_E_PEER, or DSX_E_RESYNC after this
// rank re-walked (a seam that did not converge) or redid (DSX_SEAM_REDO) its
// shard and rewrote `my_seam`.  A failed re-walk / redo marks `my_seam`
// DSX_SEAM_ERROR and returns its error.
static int shard_outcome(dsx_ctx* c, int rank, dsx_seam_t* my_seam, bool seam_dev, uint64_t cap,
                         uint64_t* n_out) {
  const uint64_t status = c->h_res[0], n = c->h_res[1], entry = c->h_res[2];
  *n_out = 0;
  if (status == ~0ull) {
    c->err = "shard: resolve did not publish its result";
    return DSX_E_INTERNAL;
  }
  if (status == kSeamPeerFailed) return DSX_E_PEER;
  if (status != 0) {
    // kSeamRedo: rank `entry` redoes its shard from its own start; otherwise
    // seam `status - 1` did not converge inside its window and its owner
    // re-walks its shard from the true entry cut; either way the owner
    // republishes its record
    const bool redo = status == kSeamRedo;
    const int failing = redo ? (int)entry : (int)(status - 1);
    if (failing == rank) {
      auto& sh = c->sh;
      int rc = redo ? shard_run(c, sh.start, 0u, false) : shard_run(c, entry, DSX_SEAM_REWALKED, true);
      if (rc) {
        // publish the failure in this rank's record: the peers' next resolve
        // returns DSX_E_PEER (no rank waits for a record forever)
        const size_t off = offsetof(dsx_seam_t, flags);
        uint32_t fl = 0;
        const hipMemcpyKind d2h = seam_dev ? hipMemcpyDeviceToHost : hipMemcpyHostToHost;
        const hipMemcpyKind h2d = seam_dev ? hipMemcpyHostToDevice : hipMemcpyHostToHost;
        (void)hipStreamSynchronize(c->stream);
        if (hipMemcpy(&fl, (const uint8_t*)my_seam + off, 4, d2h) == hipSuccess) {
          fl |= DSX_SEAM_ERROR;
          (void)hipMemcpy((uint8_t*)my_seam + off, &fl, 4, h2d);
        }
        return rc;
      }
      if (redo)
        c->stats.dense_fallbacks++;
      else
        c->stats.repaired_segments++;
      rc = seam_out(c, my_seam, seam_dev);
      if (rc) return rc;
    }
    return DSX_E_RESYNC;
  }
  *n_out = n;
  if (n > cap) return DSX_E_CAPACITY;
  return DSX_OK;
}

extern "C" int dsx_shard_resolve(dsx_ctx_t* c, const dsx_seam_t* all, int nranks, int rank,
                                 dsx_seam_t* my_seam, uint64_t* out_ends, uint64_t cap,
                                 uint64_t* n_out, uint32_t flags) {
  DSX_FLUSH_BEHIND(c);
  if (!c || !all || nranks < 1 || rank < 0 || rank >= nranks || !n_out || !my_seam ||
      (cap && !out_ends) || (flags & ~(DSX_SEAM_DEVICE | DSX_OUT_DEVICE)) != 0)
    return DSX_E_INVAL;
  auto& sh = c->sh;
  if (!sh.valid) return DSX_E_STATE;
  HIPCHK(c, hipSetDevice(c->device));
  const bool seam_dev = (flags & DSX_SEAM_DEVICE) != 0, out_dev = (flags & DSX_OUT_DEVICE) != 0;
  const dsx_seam_t* d_all = all;
  if (!seam_dev) {
    HIPCHK(c, grow(c, c->d_all, (size_t)nranks));
    HIPCHK(c, hipMemcpyAsync(c->d_all.p, all, sizeof(dsx_seam_t) * nranks, hipMemcpyHostToDevice,
                             c->stream));
    d_all = c->d_all.p;
  }
  HIPCHK(c, grow(c, c->d_ext, DSX_SEAM_MAX_CUTS + 4));
  HIPCHK(c, grow(c, c->d_info, 8));
  hipLaunchKernelGGL(seam_resolve_kernel, dim3(1), dim3(64), 0, c->stream, d_all, nranks, rank,
                     sh.p.min, sh.p.max, c->d_ext.p, c->d_info.p);
  HIPCHK(c, hipGetLastError());
  const uint64_t most = (sh.nspec == ~0ull ? sh.len / sh.p.min + 4 : sh.nspec) + DSX_SEAM_MAX_CUTS;
  uint64_t* dst = out_ends;
  uint64_t dcap = cap;
  if (!out_dev) {
    HIPCHK(c, grow(c, c->d_emit, most));
    dst = c->d_emit.p;
    dcap = most;
  }
  const uint32_t blocks = (uint32_t)std::min<uint64_t>((most + 255) / 256, 4096);
  c->h_res[0] = ~0ull;
  hipLaunchKernelGGL(shard_emit_kernel, dim3(blocks), dim3(256), 0, c->stream,
                     (const uint64_t*)c->d_info.p, (const uint64_t*)c->d_ext.p,
                     (const uint64_t*)c->out.p, (const DevState*)c->state.p, dst, dcap,
                     (volatile uint64_t*)c->h_res, (int32_t*)nullptr);
  HIPCHK(c, hipGetLastError());
  HIPCHK(c, hipStreamSynchronize(c->stream));
  int rc = shard_outcome(c, rank, my_seam, seam_dev, cap, n_out);
  if (rc) return rc;
  const uint64_t n = *n_out;
  if (!out_dev && n)
    HIPCHK(c, hipMemcpy(out_ends, c->d_emit.p, n * sizeof(uint64_t), hipMemcpyDeviceToHost));
  return DSX_OK;
}

extern "C" int dsx_shard_resolve_async(dsx_ctx_t* c, const dsx_seam_t* all, int nranks, int rank,
                                       uint64_t* out_ends, uint64_t cap, int32_t* d_code) {
  DSX_FLUSH_BEHIND(c);
  if (!c || !all || nranks < 1 || rank < 0 || rank >= nranks || !out_ends || !d_code)
    return DSX_E_INVAL;
  auto& sh = c->sh;
  if (!sh.valid) return DSX_E_STATE;
  HIPCHK(c, hipSetDevice(c->device));
  HIPCHK(c, grow(c, c->d_ext, DSX_SEAM_MAX_CUTS + 4));
  HIPCHK(c, grow(c, c->d_info, 8));
  hipLaunchKernelGGL(seam_resolve_kernel, dim3(1), dim3(64), 0, c->stream, all, nranks, rank,
                     sh.p.min, sh.p.max, c->d_ext.p, c->d_info.p);
  HIPCHK(c, hipGetLastError());
  const uint64_t most = sh.len / sh.p.min + 4 + DSX_SEAM_MAX_CUTS;
  const uint32_t blocks = (uint32_t)std::min<uint64_t>((std::min(most, cap) + 255) / 256 + 1, 4096);
  c->h_res[0] = ~0ull;
  hipLaunchKernelGGL(shard_emit_kernel, dim3(blocks), dim3(256), 0, c->stream,
                     (const uint64_t*)c->d_info.p, (const uint64_t*)c->d_ext.p,
                     (const uint64_t*)c->out.p, (const DevState*)c->state.p, out_ends, cap,
                     (volatile uint64_t*)c->h_res, d_code);
  HIPCHK(c, hipGetLastError());
  sh.pend_rank = rank;
  sh.pend_cap = cap;
  sh.pending = true;
  return DSX_OK;
}

extern "C" int dsx_shard_collect(dsx_ctx_t* c, dsx_seam_t* my_seam, const int32_t* d_agreed,
                                 int32_t* agreed, uint64_t* n_out) {
  DSX_FLUSH_BEHIND(c);
  if (!c || !my_seam || !n_out || (d_agreed && !agreed)) return DSX_E_INVAL;
  auto& sh = c->sh;
  if (!sh.pending) return DSX_E_STATE;
  sh.pending = false;
  HIPCHK(c, hipSetDevice(c->device));
  int32_t* h_code = (int32_t*)(c->h_res + 3);
  if (d_agreed)
    HIPCHK(c, hipMemcpyAsync(h_code, d_agreed, sizeof(int32_t), hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));  // the step's one host wait
  if (d_agreed) *agreed = *h_code;
  if (d_agreed && *h_code >= 2) {
    // a rank failed this round: report this rank's own failure if it has one
    const uint64_t status = c->h_res[0], n = c->h_res[1];
    *n_out = 0;
    if (status == ~0ull) return DSX_E_INTERNAL;
    if (status == 0 && n > sh.pend_cap) {
      *n_out = n;
      return DSX_E_CAPACITY;
    }
    return DSX_E_PEER;
  }
  int rc = shard_outcome(c, sh.pend_rank, my_seam, true, sh.pend_cap, n_out);
  if (rc == DSX_OK) c->stats.chunks = *n_out;
  return rc;
}

extern "C" int dsx_ctx_stream(dsx_ctx_t* c, void** stream) {
  DSX_FLUSH_BEHIND(c);
  if (!c || !stream) return DSX_E_INVAL;
  *stream = (void*)c->stream;
  return DSX_OK;
}
