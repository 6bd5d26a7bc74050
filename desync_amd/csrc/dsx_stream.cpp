// dsx_stream.cpp -- Chunker.Next / Advance over an io.Reader
// (chunker.go:175-309; the stdin / pipe path of `desync tar -i`,
// cmd/desync/tar.go:140, and `desync chunk`, cmd/desync/chunk.go:63).
//
// The reader's bytes land in a pinned host buffer (dsx_stream_buffer hands
// out the write pointer, so a reader can fill it directly; dsx_stream_push
// copies).  Every `batch` bytes (8 MiB) the library enqueues, without
// waiting: H2D of the batch on the copy stream, then scan + stitch on the
// compute stream with the chain state carried on the device, then D2H of the
// batch's cuts into pinned memory.  Up to three batches are on the GPU while
// the reader fills the next one; dsx_stream_pop collects a batch only when
// its cuts are needed and no more input can be taken first.  A chunk is
// confirmed once the bytes up to its start + max are scanned, as in the
// reference where Next() needs len(buf) >= max (chunker.go:207, 221).
// Popped chunk bytes alias the host buffer until the next call (Next's rule,
// chunker.go:202-205).
#include <hip/hip_runtime.h>
#include <sched.h>

#include <algorithm>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

#include "dsx_engine.h"

namespace {

using Stream = dsx_ctx::Stream;
constexpr int kSlots = Stream::kSlots;
constexpr uint64_t kHalo = 64;  // bytes re-sent before a batch (the scan's 48-byte warm-up)

int st_setup(dsx_ctx* c) {
  auto& s = c->st;
  if (!s.hstate) HIPCHK(c, hipHostMalloc((void**)&s.hstate, kSlots * sizeof(HostState)));
  for (int i = 0; i < kSlots; ++i) {
    if (!s.copy_ev[i]) HIPCHK(c, hipEventCreateWithFlags(&s.copy_ev[i], hipEventDisableTiming));
    if (!s.done_ev[i]) HIPCHK(c, hipEventCreateWithFlags(&s.done_ev[i], hipEventDisableTiming));
    if (!s.stitch_ev[i]) HIPCHK(c, hipEventCreateWithFlags(&s.stitch_ev[i], hipEventDisableTiming));
  }
  if (!s.dg_stream) HIPCHK(c, hipStreamCreateWithFlags(&s.dg_stream, hipStreamNonBlocking));
  HIPCHK(c, grow(c, s.rng, 4 * kSlots));
  HIPCHK(c, grow(c, s.dq, kSlots));
  return DSX_OK;
}

// Bytes re-sent in front of a batch: the scan's 48-byte warm-up, and with
// chunk IDs the whole unfinished chunk (the carried cut is > P - max).
uint64_t st_halo(const Stream& s) {
  return s.ids >= 0 ? (s.p.max + 64 + kLine - 1) / kLine * kLine : kHalo;
}

// Waits for every batch on the GPU and forgets their results.
int st_drain(dsx_ctx* c) {
  auto& s = c->st;
  HIPCHK(c, hipStreamSynchronize(c->copy_stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
  if (s.dg_stream) HIPCHK(c, hipStreamSynchronize(s.dg_stream));
  s.fly.clear();
  return DSX_OK;
}

// Room for `want` more bytes at the tail of the host buffer.  Bytes below
// keep_from are dropped: nothing needs them (the consumer is past them, and
// every batch that could still be re-sent starts after them).
int st_room(dsx_ctx* c, uint64_t want) {
  auto& s = c->st;
  if (s.h && s.hend - s.hbase + want <= s.hcap) return DSX_OK;
  const uint64_t H = st_halo(s);
  uint64_t keep = std::min(std::min(s.cur, s.pin), s.sched >= H ? s.sched - H : 0);
  if (!s.fly.empty()) keep = std::min(keep, s.fly.front().P >= H ? s.fly.front().P - H : 0);
  keep = std::max(keep, s.hbase);
  const uint64_t held = s.hend - keep;
  // queued H2D copies read the buffer: they must have landed before it moves
  for (const auto& b : s.fly) HIPCHK(c, hipEventSynchronize(s.copy_ev[b.slot]));
  // move the held bytes down while that is cheap (at most a quarter of the
  // buffer); otherwise grow the buffer (up to 32 batches) so that moves stay
  // rare next to the bytes streamed through
  const bool cheap = 4 * (held + want) <= s.hcap || s.hcap >= 32 * s.batch;
  if (held + want <= s.hcap && keep > s.hbase && cheap) {
    memmove(s.h, s.h + (keep - s.hbase), held);
    s.hbase = keep;
    return DSX_OK;
  }
  uint64_t ncap = std::max<uint64_t>(s.hcap ? 2 * s.hcap : 4 * s.batch, 4 * s.batch);
  while (ncap < held + want) ncap *= 2;
  uint8_t* n = nullptr;
  HIPCHK(c, hipHostMalloc((void**)&n, ncap));
  if (held) memcpy(n, s.h + (keep - s.hbase), held);
  if (s.h) (void)hipHostFree(s.h);
  s.h = n;
  s.hcap = ncap;
  s.hbase = keep;
  return DSX_OK;
}

// Enqueue the next batch [sched, sched + len) (last: it ends the stream).
int st_collect(dsx_ctx* c);
int st_issue(dsx_ctx* c, uint64_t len, bool last) {
  auto& s = c->st;
  if ((int)s.fly.size() >= kSlots) return st_collect(c);  // st_pump comes back (its sched may move)
  const int slot = s.next_slot;
  s.next_slot = (slot + 1) % kSlots;
  const uint64_t P = s.sched;
  const uint64_t halo = std::min<uint64_t>(st_halo(s), P - std::max(s.hbase, s.origin));
  const bool ids = s.ids >= 0;
  const uint64_t bound = len / s.p.min + 4;
  HIPCHK(c, grow(c, s.dbuf[slot], halo + len + 64));
  HIPCHK(c, grow(c, s.dout[slot], bound));
  if (s.hcut_cap[slot] < bound) {
    if (s.hcut[slot]) (void)hipHostFree(s.hcut[slot]);
    s.hcut[slot] = nullptr;
    s.hcut_cap[slot] = 0;
    const uint64_t cap = bound + bound / 4 + 64;
    HIPCHK(c, hipHostMalloc((void**)&s.hcut[slot], cap * sizeof(uint64_t)));
    s.hcut_cap[slot] = cap;
  }
  if (ids) {
    HIPCHK(c, grow(c, s.dids[slot], 32 * bound));
    if (s.hids_cap[slot] < bound) {
      if (s.hids[slot]) (void)hipHostFree(s.hids[slot]);
      s.hids[slot] = nullptr;
      s.hids_cap[slot] = 0;
      const uint64_t cap = bound + bound / 4 + 64;
      HIPCHK(c, hipHostMalloc((void**)&s.hids[slot], 32 * cap));
      s.hids_cap[slot] = cap;
    }
  }
  HIPCHK(c, hipMemcpyAsync(s.dbuf[slot].p, s.h + (P - halo - s.hbase), halo + len,
                           hipMemcpyHostToDevice, c->copy_stream));
  HIPCHK(c, hipEventRecord(s.copy_ev[slot], c->copy_stream));
  HIPCHK(c, scan_wait(c, s.copy_ev[slot]));  // the scan reads the batch (the stitch follows it)
  // the batch's entry cut (the digest range starts there) and, for a carried
  // chain, its cut count restarting at 0 (the batch's cuts start at out[0])
  uint64_t* rng = s.rng.p + 4 * slot;
  hipLaunchKernelGGL(batch_begin_kernel, dim3(1), dim3(64), 0, c->stream, (DevState*)c->state.p,
                     rng, s.fresh ? 1 : 0, s.fresh_carry);
  HIPCHK(c, hipGetLastError());
  if (s.fresh) {
    int rc = reset_state(c, s.fresh_carry);  // the scan initialises the chain state
    if (rc) return rc;
    s.fresh = false;
  } else {
    c->npiece_call = 0;
  }
  CallCfg cc{&s.p, P + len, s.origin, s.origin + kRound, s.dout[slot].p, bound, s.dense};
  c->h_cur = &s.hstate[slot];
  c->timing = false;  // (no event records between the batches' kernels)
  int rc = DSX_OK;
  if (!s.dense) {
    rc = enqueue_piece(c, cc, s.dbuf[slot].p + halo, halo, P, len, last);
  } else {
    for (uint64_t o = 0; o < len && !rc; o += kDensePiece) {
      const uint64_t n = std::min(kDensePiece, len - o);
      rc = enqueue_piece(c, cc, s.dbuf[slot].p + halo + o, halo + o, P + o, n, last && o + n == len);
    }
  }
  c->h_cur = c->h_state;
  c->timing = true;
  if (rc) return rc;
  hipStream_t out_stream = c->stream;
  if (ids) {
    // Digest.Sum of the batch's chunks on a side stream, overlapping the next
    // batch's scan: [rng[0], rng[2]) from rng[1], all inside dbuf (the halo
    // holds the unfinished chunk)
    hipLaunchKernelGGL(state_snapshot_kernel, dim3(1), dim3(64), 0, c->stream,
                       (const DevState*)c->state.p, rng + 2);
    HIPCHK(c, hipGetLastError());
    HIPCHK(c, hipEventRecord(s.stitch_ev[slot], c->stream));
    HIPCHK(c, hipStreamWaitEvent(s.dg_stream, s.stitch_ev[slot], 0));
    DigestArgs da{};
    da.blob = s.dbuf[slot].p;
    da.base_off = P - halo;
    da.len = halo + len;
    da.ends = s.dout[slot].p;
    da.ids = s.dids[slot].p;
    da.range_lo = rng;
    da.range_hi = rng + 2;
    rc = launch_digest(c, da, bound, s.ids, s.dg_stream, s.dq.p + slot);
    if (rc) return rc;
    HIPCHK(c, hipMemcpyAsync(s.hids[slot], s.dids[slot].p, 32 * bound, hipMemcpyDeviceToHost,
                             s.dg_stream));
    out_stream = s.dg_stream;
  }
  HIPCHK(c, hipMemcpyAsync(s.hcut[slot], s.dout[slot].p, bound * sizeof(uint64_t),
                           hipMemcpyDeviceToHost, out_stream));
  HIPCHK(c, hipEventRecord(s.done_ev[slot], out_stream));
  s.fly.push_back({P, len, c->piece_seq, last, ids, slot});
  s.sched = P + len;
  return DSX_OK;
}

// Collect the oldest batch: its cuts join the queue.
int st_collect(dsx_ctx* c) {
  auto& s = c->st;
  const Stream::Batch b = s.fly.front();
  HIPCHK(c, hipEventSynchronize(s.done_ev[b.slot]));
  HostState hs;
  memcpy(&hs, (const void*)&s.hstate[b.slot], sizeof hs);
  if (hs.seq != b.seq) {
    c->err = "stream: stale batch state";
    return DSX_E_INTERNAL;
  }
  if (hs.err & kErrDense) {
    // rare: a scan lane overflowed its candidate slots.  Every batch after
    // this one ran on a wrong chain; redo from this batch on the dense path
    // (its bytes are still held: st_room keeps the oldest batch's bytes)
    int rc = st_drain(c);
    if (rc) return rc;
    c->stats.dense_fallbacks++;
    s.dense = true;
    s.fresh = true;
    s.fresh_carry = s.carry;
    s.sched = b.P;
    return DSX_OK;  // the caller re-issues (st_pump)
  }
  if (hs.err) {
    c->err = "stream: stitch error";
    return DSX_E_INTERNAL;
  }
  for (uint64_t i = 0; i < hs.total; ++i) s.cuts.push_back(s.hcut[b.slot][i]);
  if (b.ids) {
    for (uint64_t i = 0; i < hs.total; ++i) {
      std::array<uint8_t, 32> id;
      memcpy(id.data(), s.hids[b.slot] + 32 * i, 32);
      s.idq.push_back(id);
    }
  }
  s.carry = hs.carry;
  if (b.last) s.done = true;
  s.fly.pop_front();
  c->stats.chunks += hs.total;
  return DSX_OK;
}

// Hand the held bytes to the GPU in batches (all of them at the end of the
// stream or on a sync).
int st_pump(dsx_ctx* c, bool sync) {
  auto& s = c->st;
  while (true) {
    const uint64_t avail = s.hend - s.sched;
    int rc = DSX_OK;
    if (avail > s.batch) {  // (one byte is held back: the final batch is never empty)
      rc = st_issue(c, s.batch, false);
    } else if (s.eof) {
      if (avail > 0) {
        rc = st_issue(c, avail, true);
      } else {
        if (!s.done && (s.fly.empty() || !s.fly.back().last)) s.final_pending = true;
        return DSX_OK;
      }
    } else if (sync && avail > 0) {
      rc = st_issue(c, avail, false);
    } else {
      return DSX_OK;
    }
    if (rc) return rc;
  }
}

// End of stream exactly at the last scanned byte: the chain's last chunk
// ends there (no candidate after the carried cut, or it would have been
// emitted: dsx_stitch.hip's undetermined-successor rule).
void st_finish(dsx_ctx* c) {
  auto& s = c->st;
  if (s.carry < s.hend) {
    s.cuts.push_back(s.hend);
    s.carry = s.hend;
  }
  s.final_pending = false;
  s.done = true;
}

void st_restart(dsx_ctx* c, uint64_t at) {
  auto& s = c->st;
  s.cuts.clear();
  s.idq.clear();
  s.has_id = false;
  s.pin = at;
  s.grp.clear();
  s.grp_ids.clear();
  s.origin = s.sched = s.carry = s.fresh_carry = at;
  s.fresh = true;
  s.done = s.final_pending = false;
}

}  // namespace

void stream_release(dsx_ctx* c) {
  auto& s = c->st;
  if (s.h) (void)hipHostFree(s.h);
  s.h = nullptr;
  for (int i = 0; i < kSlots; ++i) {
    s.dbuf[i].release();
    s.dout[i].release();
    if (s.hcut[i]) (void)hipHostFree(s.hcut[i]);
    s.hcut[i] = nullptr;
    if (s.copy_ev[i]) (void)hipEventDestroy(s.copy_ev[i]);
    if (s.done_ev[i]) (void)hipEventDestroy(s.done_ev[i]);
    if (s.stitch_ev[i]) (void)hipEventDestroy(s.stitch_ev[i]);
    s.copy_ev[i] = s.done_ev[i] = s.stitch_ev[i] = nullptr;
    s.dids[i].release();
    if (s.hids[i]) (void)hipHostFree(s.hids[i]);
    s.hids[i] = nullptr;
    s.hids_cap[i] = 0;
  }
  s.rng.release();
  s.dq.release();
  if (s.dg_stream) (void)hipStreamDestroy(s.dg_stream);
  s.dg_stream = nullptr;
  if (s.hstate) (void)hipHostFree(s.hstate);
  s.hstate = nullptr;
}

extern "C" int dsx_stream_begin(dsx_ctx_t* c, const dsx_params_t* p) {
  DSX_FLUSH_BEHIND(c);
  if (!c || !p) return DSX_E_INVAL;
  auto& s = c->st;
  // one stream per context (its scratch and carried state live here): a
  // second Chunker on a context whose stream is still being read is refused
  // instead of silently resetting the first one
  if (s.active && !(s.done && s.cuts.empty())) {
    c->err = "a stream is already active on this context (dsx_stream_end it first)";
    return DSX_E_STATE;
  }
  HIPCHK(c, hipSetDevice(c->device));
  int rc = ensure_attr_walk(c);
  if (!rc) rc = st_setup(c);
  if (!rc) rc = st_drain(c);
  if (rc) return rc;
  s.active = true;
  s.eof = false;
  s.dense = false;
  s.ids = -1;
  s.p = *p;
  s.batch = 8ull << 20;
#if DSX_DIAG
  if (const char* v = getenv("DSX_STREAM_BATCH"))
    s.batch = std::max<uint64_t>(4096, (uint64_t)atoll(v));
#endif
  s.hbase = s.hend = s.cur = s.skip = 0;
  s.next_slot = 0;
  s.last_chunk = nullptr;
  st_restart(c, 0);
  c->stats.chunks = 0;
  return DSX_OK;
}

extern "C" int dsx_stream_end(dsx_ctx_t* c) {
  if (!c) return DSX_E_INVAL;
  auto& s = c->st;
  if (s.active) {
    (void)hipSetDevice(c->device);
    int rc = st_drain(c);
    if (rc) return rc;
  }
  s.active = s.eof = false;
  st_restart(c, 0);
  s.done = false;
  s.last_chunk = nullptr;
  return DSX_OK;
}

extern "C" int dsx_stream_buffer(dsx_ctx_t* c, uint64_t want, uint8_t** ptr) {
  if (!c || !ptr) return DSX_E_INVAL;
  auto& s = c->st;
  if (!s.active || s.eof) return DSX_E_STATE;
  HIPCHK(c, hipSetDevice(c->device));
  s.last_chunk = nullptr;
  int rc = st_room(c, want);
  if (rc) return rc;
  *ptr = s.h + (s.hend - s.hbase);
  return DSX_OK;
}

extern "C" int dsx_stream_commit(dsx_ctx_t* c, uint64_t n, int flags) {
  if (!c) return DSX_E_INVAL;
  auto& s = c->st;
  if (!s.active || s.eof) return DSX_E_STATE;
  if (n && (!s.h || s.hend - s.hbase + n > s.hcap)) return DSX_E_INVAL;
  HIPCHK(c, hipSetDevice(c->device));
  s.last_chunk = nullptr;
  if (s.skip && n) {  // Advance() beyond the held bytes drops future input
    uint8_t* tail = s.h + (s.hend - s.hbase);
    const uint64_t d = std::min(s.skip, n);
    s.skip -= d;
    n -= d;
    if (n) memmove(tail, tail + d, n);
  }
  s.hend += n;
  if (flags & DSX_STREAM_EOF) s.eof = true;
  const bool sync = (flags & DSX_STREAM_SYNC) != 0;
  int rc = st_pump(c, sync);
  // SYNC: no more input for now (the reader failed): everything held is
  // scanned and collected, so pop returns every chunk it can confirm
  while (!rc && sync && !s.fly.empty()) {
    rc = st_collect(c);
    if (!rc) rc = st_pump(c, true);
  }
  return rc;
}

extern "C" int dsx_stream_push(dsx_ctx_t* c, const void* bytes, uint64_t len, int eof) {
  if (!c || (len && !bytes)) return DSX_E_INVAL;
  uint8_t* dst = nullptr;
  int rc = dsx_stream_buffer(c, len, &dst);
  if (rc) return rc;
  if (len) memcpy(dst, bytes, len);
  return dsx_stream_commit(c, len, eof ? DSX_STREAM_EOF : 0);
}

extern "C" int dsx_stream_pop(dsx_ctx_t* c, uint64_t* start, uint64_t* size) {
  if (!c || !start || !size) return DSX_E_INVAL;
  auto& s = c->st;
  if (!s.active) return DSX_E_STATE;
  while (s.cuts.empty()) {
    if (!s.fly.empty()) {
      // collect now if the oldest batch is finished, if no more input can
      // come, or if enough batches are queued; otherwise ask for input
      // first, so the reader works while the GPU does.  With IDs every slot
      // may fill first: the first batch's IDs take ~15 ms (its longest
      // chunk's SHA chain), which the reader spends reading the next batch
      // instead of waiting (ChunkStream)
      const bool ready = hipEventQuery(s.done_ev[s.fly.front().slot]) == hipSuccess;
      const size_t enough = s.ids >= 0 ? (size_t)kSlots : 2;
      if (!(ready || s.eof || s.fly.size() >= enough)) break;
      HIPCHK(c, hipSetDevice(c->device));
      int rc = st_collect(c);
      if (!rc) rc = st_pump(c, false);  // (re-issues after a dense redo)
      if (rc) return rc;
      continue;
    }
    if (s.final_pending) {
      st_finish(c);
      continue;
    }
    break;
  }
  if (s.cuts.empty()) {
    *start = s.cur;
    *size = 0;
    return 0;
  }
  const uint64_t e = s.cuts.front();
  s.cuts.pop_front();
  s.has_id = false;
  if (!s.idq.empty() && s.idq.size() > s.cuts.size()) {  // (cuts and IDs stay aligned from the back)
    memcpy(s.last_id, s.idq.front().data(), 32);
    s.idq.pop_front();
    s.has_id = true;
  }
  *start = s.cur;
  *size = e - s.cur;
  s.last_chunk = s.h + (s.cur - s.hbase);
  s.pin = s.cur;
  s.cur = e;
  return 1;
}

extern "C" const uint8_t* dsx_stream_chunk_data(dsx_ctx_t* c) { return c ? c->st.last_chunk : nullptr; }

extern "C" int dsx_stream_pop_many(dsx_ctx_t* c, uint64_t* ends, uint8_t* ids, uint64_t cap,
                                   uint64_t* start, uint64_t* n) {
  if (!c || !start || !n || !cap || !ends) return DSX_E_INVAL;  // (nothing is popped)
  *n = 0;
  if (ids && c->st.ids < 0) return DSX_E_STATE;  // IDs were not switched on
  uint64_t size = 0;
  int rc = dsx_stream_pop(c, start, &size);  // collects a batch if needed
  if (rc <= 0) return rc;
  auto& s = c->st;
  const uint64_t first = *start;
  uint64_t k = 0;
  s.grp.clear();
  s.grp_ids.clear();
  while (true) {
    ends[k] = s.cur;
    s.grp.push_back(s.cur);
    if (s.has_id) {
      std::array<uint8_t, 32> id;
      memcpy(id.data(), s.last_id, 32);
      s.grp_ids.push_back(id);
    }
    if (ids && !s.has_id) {
      // a chunk without an ID where IDs are asked for: the group ends before
      // it and the chunk goes back to the queue (nothing popped is lost)
      s.last_chunk = s.h + (first - s.hbase);
      s.pin = first;
      s.grp_ids.clear();  // (unpop then re-queues ends alone)
      rc = dsx_stream_unpop(c, k ? ends[k - 1] : first);
      if (rc) return rc;
      *n = k;
      return k ? 1 : DSX_E_STATE;
    }
    if (ids) memcpy(ids + 32 * k, s.last_id, 32);
    ++k;
    if (k >= cap || s.cuts.empty()) break;
    uint64_t st0, sz;
    rc = dsx_stream_pop(c, &st0, &sz);
    if (rc <= 0) break;
  }
  *n = k;
  s.last_chunk = s.h + (first - s.hbase);  // the popped chunks, contiguous from here
  s.pin = first;                            // ... and held until the next pop
  return 1;
}

extern "C" int dsx_stream_unpop(dsx_ctx_t* c, uint64_t pos) {
  if (!c) return DSX_E_INVAL;
  auto& s = c->st;
  if (!s.active) return DSX_E_STATE;
  if (pos == s.cur) return DSX_OK;
  if (pos < s.pin || pos > s.cur) return DSX_E_INVAL;
  // the chunks of the last group that end after pos go back to the queue
  const bool with_ids = s.grp_ids.size() == s.grp.size();
  for (size_t i = s.grp.size(); i-- > 0;) {
    if (s.grp[i] <= pos) break;
    s.cuts.push_front(s.grp[i]);
    if (with_ids) s.idq.push_front(s.grp_ids[i]);
  }
  s.cur = pos;
  s.grp.clear();
  s.grp_ids.clear();
  return DSX_OK;
}

extern "C" int dsx_stream_window(dsx_ctx_t* c, const uint8_t** base, uint64_t* base_pos,
                                 uint64_t* len) {
  if (!c || !base || !base_pos || !len) return DSX_E_INVAL;
  const auto& s = c->st;
  *base = s.h;
  *base_pos = s.hbase;
  *len = s.hend - s.hbase;
  return DSX_OK;
}

extern "C" int dsx_stream_ids(dsx_ctx_t* c, int algo) {
  if (!c || (algo != -1 && algo != DSX_DIGEST_SHA512_256 && algo != DSX_DIGEST_SHA256))
    return DSX_E_INVAL;
  auto& s = c->st;
  if (!s.active) return DSX_E_STATE;
  // only before the first batch of a chain: every chunk then has an ID
  if (!s.fly.empty() || s.sched != s.origin || !s.cuts.empty()) {
    c->err = "dsx_stream_ids: chunks were already scanned without IDs";
    return DSX_E_STATE;
  }
  s.ids = algo;
#if DSX_DIAG
  if (getenv("DSX_STREAM_BATCH")) return DSX_OK;
#endif
  if (algo >= 0) s.batch = std::max<uint64_t>(s.batch, 128ull << 20);  // digests are latency-bound: bigger batches
  return DSX_OK;
}

extern "C" const uint8_t* dsx_stream_chunk_id(dsx_ctx_t* c) {
  return c && c->st.has_id ? c->st.last_id : nullptr;
}

extern "C" int dsx_stream_done(dsx_ctx_t* c) {
  if (!c) return 0;
  const auto& s = c->st;
  return s.active && s.done && s.cuts.empty() ? 1 : 0;
}

extern "C" int dsx_stream_flush(dsx_ctx_t* c, uint64_t* start, uint64_t* size) {
  if (!c || !start || !size) return DSX_E_INVAL;
  auto& s = c->st;
  if (!s.active) return DSX_E_STATE;
  HIPCHK(c, hipSetDevice(c->device));
  int rc = st_drain(c);
  if (rc) return rc;
  // Next()'s read-error path (chunker.go:207-211 -> split(n, err)): every
  // held byte after the consumer position is one chunk, and chunking starts
  // over behind it
  *start = s.cur;
  *size = s.hend - s.cur;
  s.last_chunk = s.h ? s.h + (s.cur - s.hbase) : nullptr;
  s.cur = s.hend;
  st_restart(c, s.hend);
  s.eof = false;
  return DSX_OK;
}

extern "C" int dsx_stream_advance(dsx_ctx_t* c, uint64_t n) {
  if (!c) return DSX_E_INVAL;
  auto& s = c->st;
  if (!s.active) return DSX_E_STATE;
  HIPCHK(c, hipSetDevice(c->device));
  int rc = st_drain(c);
  if (rc) return rc;
  // Advance (chunker.go:292-309): the held bytes count first, then the
  // reader's; the chunker behaves as if the stream started at cur + n
  const uint64_t target = s.cur + n;
  s.last_chunk = nullptr;
  if (target <= s.hend) {
    s.skip = 0;
  } else {
    s.skip = target - s.hend;
    s.hbase = s.hend = target;  // nothing held
  }
  s.cur = target;
  st_restart(c, target);
  if (s.eof) {
    s.skip = 0;
    return st_pump(c, false);  // the remaining held bytes are the rest of the stream
  }
  return DSX_OK;
}

// ---- host_parallel: a persistent pool of host threads ----------------------
// One job at a time: fn(0) on the calling thread, fn(1..parts-1) on pool
// threads.  The threads persist (one per call would cost more than a
// ChunkStream slab's copy); they are detached and the pool is never
// destroyed, so process exit does not wait on them.
namespace {
class HostPool {
 public:
  void run(int parts, const std::function<void(int)>& fn) {
    std::lock_guard<std::mutex> call(call_mu_);  // one job at a time through the pool
    while ((int)threads_ < parts - 1) {
      const int idx = ++threads_;
      std::thread([this, idx] { loop(idx); }).detach();
    }
    {
      std::lock_guard<std::mutex> g(mu_);
      fn_ = &fn;
      parts_ = parts;
      pending_ = parts - 1;
      ++gen_;
    }
    cv_.notify_all();
    fn(0);
    std::unique_lock<std::mutex> g(mu_);
    done_.wait(g, [&] { return pending_ == 0; });
  }

 private:
  void loop(int idx) {
    uint64_t seen = 0;
    std::unique_lock<std::mutex> g(mu_);
    for (;;) {
      cv_.wait(g, [&] { return gen_ != seen; });
      seen = gen_;
      if (idx >= parts_) continue;  // (no part for this thread in this job)
      const std::function<void(int)>* fn = fn_;
      g.unlock();
      (*fn)(idx);
      g.lock();
      if (--pending_ == 0) done_.notify_one();
    }
  }
  std::mutex call_mu_, mu_;
  std::condition_variable cv_, done_;
  int threads_ = 0, parts_ = 0, pending_ = 0;
  uint64_t gen_ = 0;
  const std::function<void(int)>* fn_ = nullptr;
};
}  // namespace

hipError_t side_stream_create(hipStream_t* s) {
#if DSX_DIAG
  if (const char* v = getenv("DSX_SIDE_PRIO"))
    if (atoi(v) == 0) return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
#endif
  int least = 0, greatest = 0;
  hipError_t e = hipDeviceGetStreamPriorityRange(&least, &greatest);
  if (e != hipSuccess) return e;
  return hipStreamCreateWithPriority(s, hipStreamNonBlocking, least);
}

int host_cpu_share() {
  const int share = [] {
    if (const char* v = getenv("DSX_HOST_THREADS")) {
      const int o = atoi(v);
      if (o > 0) return std::min(o, 256);
    }
    int n = 0;
    cpu_set_t set;
    CPU_ZERO(&set);
    if (sched_getaffinity(0, sizeof set, &set) == 0) n = CPU_COUNT(&set);
    if (n <= 0) n = (int)std::thread::hardware_concurrency();
    if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {  // "quota period" or "max period"
      char q[32] = {0};
      long long period = 0;
      if (fscanf(f, "%31s %lld", q, &period) == 2 && strcmp(q, "max") != 0 && period > 0) {
        const long long quota = atoll(q);
        if (quota > 0) n = (int)std::min<long long>(n, std::max(1LL, (quota + period - 1) / period));
      }
      fclose(f);
    } else if (FILE* fq = fopen("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "r")) {  // cgroup v1
      long long quota = -1, period = 0;
      if (fscanf(fq, "%lld", &quota) != 1) quota = -1;
      fclose(fq);
      if (FILE* fp = fopen("/sys/fs/cgroup/cpu/cpu.cfs_period_us", "r")) {
        if (fscanf(fp, "%lld", &period) != 1) period = 0;
        fclose(fp);
      }
      if (quota > 0 && period > 0)
        n = (int)std::min<long long>(n, std::max(1LL, (quota + period - 1) / period));
    }
    // (the GPU box exports its CPU share per GPU here; its affinity mask and
    // nproc show the whole machine)
    if (const char* v = getenv("OMP_NUM_THREADS")) {
      const int o = atoi(v);
      if (o > 0) n = std::min(n, o);
    }
    return std::max(1, n);
  }();
  return share;
}

void host_parallel(int parts, const std::function<void(int)>& fn) {
  if (parts <= 1) {
    fn(0);
    return;
  }
  static HostPool* pool = new HostPool;  // (never destroyed: detached threads wait on it)
  pool->run(std::min(parts, 64), fn);
}

// ---- dsx_host_copy: ChunkStream's clone of a run (index.go:196-200) -------
// One memcpy thread moves ~15 GB/s out of the pinned buffer: 512 MiB of
// clones were 16 ms of ChunkStream's 65 (profiles/r05v/cs.json).
extern "C" int dsx_host_copy(void* dst, const void* src, uint64_t n, int threads) {
  if (n && (!dst || !src)) return DSX_E_INVAL;
  const uint8_t* s = (const uint8_t*)src;
  uint8_t* d = (uint8_t*)dst;
  if (d < s + n && s < d + n) return DSX_E_INVAL;  // (overlap)
  const int parts = (int)std::min<uint64_t>(std::max(1, std::min(threads, 64)), (n + (1u << 20) - 1) >> 20);
  if (parts <= 1) {
    if (n) memcpy(d, s, n);
    return DSX_OK;
  }
  const uint64_t step = ((n + parts - 1) / parts + 4095) & ~uint64_t(4095);
  host_parallel(parts, [&](int i) {
    const uint64_t off = (uint64_t)i * step;
    if (off < n) memcpy(d + off, s + off, std::min(step, n - off));
  });
  return DSX_OK;
}
