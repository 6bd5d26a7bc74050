// dsx_index.cpp -- IndexFromFile on the GPU: bytes from a file descriptor or
// host memory -> cut list + chunk IDs (include/dsx.h: dsx_index_fd,
// dsx_index_host).
//
// Reference: IndexFromFile (make.go:22-163) chunks the file with n goroutines
// (split-and-align) and computes Digest.Sum of every chunk (make.go:223,
// digest.go:11-29); GetFileSize (ioctl_linux.go:63-84) sizes regular files
// and block devices.
//
// Pipeline (one context, reader threads, HIP streams in three priority pools
// so that none shares an HSA queue with another -- tools/queue_probe.hip):
//   reader threads  pread/memcpy 32 MiB pieces into a ring of pinned slots
//                   (the file's last 32 MiB in 8 MiB pieces);
//   copy_stream     H2D of each piece into the current HBM window (high);
//   stream          scan + stitch (dsx_scan.hip, dsx_stitch.hip) every
//                   32 MiB, the chain state carried on the device; at the
//                   end of a window a snapshot of {total cuts, carried cut}
//                   (high);
//   idx_side[0..3]  the windows' digests (idx_side[0] = idx_dg_stream) and,
//                   in a one-window call, the GPU's shares of the window
//                   during the read (low);
//   tail feeder     the last window's long chunks hashed on the host as the
//                   stitches confirm them (its copy stream at the default
//                   priority), the GPU's last digest skipping them.
// Two windows alternate, so the digest of window w overlaps the H2D and scan
// of window w+1.  A window starts with the last max + 128 bytes of the
// previous one: the carried cut lies in (P - max, P] (dsx_stitch.hip), so the
// unfinished chunk and the scan's 48-byte warm-up are always in HBM.  No host
// round trip happens until the end of the file but the feeder's (DESIGN.md
// 5.1).
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <algorithm>
#include <deque>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <memory>
#include <cerrno>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "dsx_engine.h"

namespace {

using FillFn = int (*)(void* ud, uint8_t* dst, uint64_t off, uint64_t n);

// Reads pieces [k*piece, (k+1)*piece) of the source into slot k % K on
// reader threads, ahead of the consumer, never more than K pieces ahead; from
// fine_from on (a multiple of piece) the pieces are `fine` bytes.
// Pieces [0, len): `piece` bytes each up to fine_from (a multiple of piece),
// `fine` bytes from there on (none when fine_from >= len).
struct PieceMap {
  uint64_t len, piece, fine_from, fine, kf, np;
  PieceMap(uint64_t n, uint64_t pc, uint64_t ff = UINT64_MAX, uint64_t fn = 0)
      : len(n), piece(pc), fine_from(fn && ff < n ? ff : UINT64_MAX), fine(fn ? fn : pc),
        kf(fine_from < n ? fine_from / pc : (n + pc - 1) / pc),
        np(kf + (fine_from < n ? (n - fine_from + fine - 1) / fine : 0)) {}
  uint64_t off(uint64_t k) const { return k < kf ? k * piece : fine_from + (k - kf) * fine; }
  uint64_t size(uint64_t k) const { return std::min(k < kf ? piece : fine, len - off(k)); }
};

class Prefetcher {
 public:
  Prefetcher(FillFn fill, void* ud, uint64_t len, uint64_t piece, uint8_t* const* slots, int nslots,
             int nthreads, uint64_t fine_from = UINT64_MAX, uint64_t fine = 0)
      : fill_(fill), ud_(ud), map_(len, piece, fine_from, fine), np_(map_.np),
        slots_(slots, slots + nslots), have_(nslots, -1), allow_(nslots), rc_(nslots, 0) {
    for (int s = 0; s < nslots; ++s) allow_[s] = s;
    const int nt = std::max(1, std::min<int>(nthreads, (int)std::min<uint64_t>(np_, 64)));
    for (int i = 0; i < nt; ++i) th_.emplace_back([this] { run(); });
  }
  ~Prefetcher() { stop(); }
  // blocks until piece k is in its slot; returns the fill status
  int wait(uint64_t k, uint8_t** p, uint64_t* n) {
    const size_t s = k % slots_.size();
    std::unique_lock<std::mutex> lk(m_);
    cv_.wait(lk, [&] { return have_[s] == (int64_t)k; });
    *p = slots_[s];
    *n = map_.size(k);
    return rc_[s];
  }
  // the slot holding piece k may be refilled (its H2D copy has landed)
  void release(uint64_t k) {
    const size_t s = k % slots_.size();
    {
      std::lock_guard<std::mutex> lk(m_);
      allow_[s] = (int64_t)(k + slots_.size());
    }
    cv_.notify_all();
  }
  void stop() {
    {
      std::lock_guard<std::mutex> lk(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
    th_.clear();
  }

 private:
  void run() {
    while (true) {
      uint64_t k;
      size_t s;
      {
        std::unique_lock<std::mutex> lk(m_);
        if (stop_ || next_ >= np_) return;
        k = next_++;
        s = k % slots_.size();
        cv_.wait(lk, [&] { return stop_ || allow_[s] == (int64_t)k; });
        if (stop_) return;
      }
      const int rc = fill_(ud_, slots_[s], map_.off(k), map_.size(k));
      {
        std::lock_guard<std::mutex> lk(m_);
        rc_[s] = rc;
        have_[s] = (int64_t)k;
      }
      cv_.notify_all();
    }
  }
  FillFn fill_;
  void* ud_;
  PieceMap map_;
  uint64_t np_;
  std::vector<uint8_t*> slots_;
  std::vector<int64_t> have_, allow_;
  std::vector<int> rc_;
  std::mutex m_;
  std::condition_variable cv_;
  uint64_t next_ = 0;
  bool stop_ = false;
  std::vector<std::thread> th_;
};

struct MemSrc {
  const uint8_t* p;
};
int fill_mem(void* ud, uint8_t* dst, uint64_t off, uint64_t n) {
  memcpy(dst, ((const MemSrc*)ud)->p + off, n);
  return DSX_OK;
}
struct FdSrc {
  int fd;
  uint64_t base;
};
int fill_fd(void* ud, uint8_t* dst, uint64_t off, uint64_t n) {
  const FdSrc* s = (const FdSrc*)ud;
  uint64_t got = 0;
  while (got < n) {
    const ssize_t r = pread(s->fd, dst + got, n - got, (off_t)(s->base + off + got));
    if (r < 0) {
      if (errno == EINTR) continue;
      return DSX_E_IO;
    }
    if (r == 0) return DSX_E_IO;  // the file shrank underneath us
    got += (uint64_t)r;
  }
  return DSX_OK;
}

// bytes per scan + stitch launch: each stitch publishes the chain position
// (dsx_progress), so 32 per GiB, make.go:138's pb.Set per chunk in steps of
// 32 MiB; the GPU work per step (~40 us) is far below its PCIe time (~1 ms)
constexpr uint64_t kScanStep = 32ull << 20;

int index_setup(dsx_ctx* c, uint64_t slot_bytes) {
  if (c->idx_slot_bytes < slot_bytes) {
    HIPCHK(c, hipStreamSynchronize(c->copy_stream));
    for (auto& s : c->idx_slots) {
      if (s) (void)hipHostFree(s);
      s = nullptr;
    }
    c->idx_slot_bytes = 0;
    for (auto& s : c->idx_slots) HIPCHK(c, hipHostMalloc((void**)&s, slot_bytes));
    c->idx_slot_bytes = slot_bytes;
  }
  for (auto& e : c->idx_copy_ev)
    if (!e) HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
  for (auto& e : c->idx_win_ev)
    if (!e) HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
  for (auto& e : c->idx_stitch_ev)
    if (!e) HIPCHK(c, hipEventCreateWithFlags(&e, hipEventDisableTiming));
  for (auto& s : c->idx_side)
    if (!s) HIPCHK(c, side_stream_create(&s));
  c->idx_dg_stream = c->idx_side[0];
  HIPCHK(c, c->idx_side_q.ensure(32 * (dsx_ctx::kIdxSide + 1)));  // (+ the end digest's)
  return DSX_OK;
}

// A window's digest on the digest stream, after the window's last stitch and
// snapshot (recorded on `stream`); then the event the copy stream waits for
// before it refills the window's buffer.
int launch_window_digest(dsx_ctx* c, const DigestArgs& da, uint64_t max_n, int algo, int slot,
                         uint32_t max_blocks = 0) {
  HIPCHK(c, hipEventRecord(c->idx_stitch_ev[slot], c->stream));
  HIPCHK(c, hipStreamWaitEvent(c->idx_dg_stream, c->idx_stitch_ev[slot], 0));
  const int rc = launch_digest(c, da, max_n, algo, c->idx_dg_stream, nullptr, true, max_blocks);
  if (rc) return rc;
  HIPCHK(c, hipEventRecord(c->idx_win_ev[slot], c->idx_dg_stream));
  return DSX_OK;
}

// Drains both streams (after an error or a cancel: nothing may still read the
// pinned slots or the windows when the call returns).
int drain(dsx_ctx* c, Prefetcher& pf, int rc) {
  pf.stop();
  (void)hipStreamSynchronize(c->copy_stream);
  (void)hipStreamSynchronize(c->scan_stream);
  (void)hipStreamSynchronize(c->stream);
  for (auto& s : c->idx_side)  // (idx_dg_stream among them)
    if (s) (void)hipStreamSynchronize(s);
  return rc;
}

// Marks the progress of a run_index call (dsx_progress) for its lifetime.
struct ProgressScope {
  dsx_ctx* c;
  ProgressScope(dsx_ctx* cc, uint64_t len) : c(cc) {
    c->prog_active.store(0);
    c->prog_done.store(0);
    c->prog_len.store(len);
    ((volatile HostState*)c->h_state)->carry = 0;
    c->prog_active.store(1);
  }
  ~ProgressScope() { c->prog_active.store(0); }
  void set(uint64_t v) { c->prog_done.store(v); }
};

// ---- host tail --------------------------
// The last window's digest starts when the read ends and lasts its longest
// chunk's SHA chain: ~38 ns per byte on one GPU lane, ~10 ms for 256 KiB.
// The longest chunks of that window go to the host instead (AVX-512, 8 per
// core at once), the GPU skipping them (DigestArgs.skip_above): the cut L is
// where the host's bytes over its threads take as long as the GPU's longest
// remaining chain.
// (measured at the end of a 1 GiB file call, profiles/r05ao: the GPU's chain
// runs at the clock an idle-ish GPU has then, ~58 ns per byte, against ~38 ns
// on a busy one; 16 host threads read and hash ~43 GB/s)
constexpr double kGpuNsPerByte = 58.0;   // digest_pc_kernel, one lane, end of a file call
constexpr double kShareNsPerByte = 45.0;  // the same beside the read's scans (37-40, r06an)
constexpr double kReadBytesPerNs = 45.0;  // page cache -> HBM through the pinned slots (dsx_cut_fd, ~42 GiB/s)
constexpr double kHostNsPerByte = 0.38;  // one host thread, read + hash (AVX-512)

// This host's SHA-512/256 rate, ns per byte on one thread (8 lanes of 128 KiB
// hashed once per process, ~0.5 ms), plus the read: the VerifyIndex budget
// takes the slower of it and kHostNsPerByte, so a slower host gets fewer
// bytes instead of a call that waits for its early hash.
double host_ns_per_byte() {
  static const double v = [] {
    if (!host_sha_vec()) return 4.0 * kHostNsPerByte;  // (the scalar path)
    constexpr uint64_t n = 128 << 10;
    std::vector<uint8_t> buf(8 * n, 0x5a), out(8 * 32);
    const uint8_t* p[8];
    uint64_t len[8];
    uint8_t* o[8];
    for (int i = 0; i < 8; ++i) p[i] = buf.data() + i * n, len[i] = n, o[i] = out.data() + 32 * i;
    host_sha512_256_x8(p, len, o);  // (warm)
    const auto t0 = std::chrono::steady_clock::now();
    host_sha512_256_x8(p, len, o);
    const double ns = std::chrono::duration<double, std::nano>(std::chrono::steady_clock::now() - t0).count();
    return 1.15 * ns / (8.0 * (double)n);  // (+15 %: the read through `fill`)
  }();
  return std::max(v, kHostNsPerByte);
}
constexpr double kTailMinGainNs = 5e5;   // worth a host pass only above this
constexpr int kTailThreads = 16;
constexpr size_t kMaxMids = dsx_ctx::kIdxSide;  // GPU shares of a one-window call during its read
constexpr uint64_t kFineTail = 32ull << 20;      // the call's last bytes in smaller pieces
constexpr uint64_t kFineDiv = 4;                 // of piece / kFineDiv bytes

struct TailChunk {
  uint64_t idx, start, len;
};

// The chunks of ranges [i0, i1) (ends e, the first starting at first) that the
// host hashes, longest first; empty: none.  *cut = the GPU's skip_above.
std::vector<TailChunk> plan_tail(const dsx_ctx* c, const std::vector<uint64_t>& e, uint64_t i0,
                                 uint64_t first, int threads, uint64_t* cut) {
  std::vector<TailChunk> t(e.size());
  for (size_t i = 0; i < e.size(); ++i) {
    const uint64_t s = i ? e[i - 1] : first;
    t[i] = {i0 + i, s, e[i] - s};
  }
  std::sort(t.begin(), t.end(), [](const TailChunk& a, const TailChunk& b) { return a.len > b.len; });
  *cut = 0;
  if (t.empty()) return {};
  size_t k = 0;
  if (c->index_host_tail > 0) {  // forced cut (tests)
    while (k < t.size() && t[k].len > (uint64_t)c->index_host_tail) ++k;
    *cut = (uint64_t)c->index_host_tail;
  } else {
    // k chunks to the host: time max(host bytes / threads, GPU's longest chain)
    const double now = kGpuNsPerByte * (double)t[0].len;
    double best = now, bytes = 0;
    for (size_t j = 0; j + 1 < t.size(); ++j) {
      bytes += (double)t[j].len;
      const double tj = std::max(bytes * kHostNsPerByte / threads, kGpuNsPerByte * (double)t[j + 1].len);
      if (tj < best) {
        best = tj;
        k = j + 1;
      }
      if (bytes * kHostNsPerByte / threads > now) break;
    }
    if (now - best < kTailMinGainNs) k = 0;
    // (chunks as long as the first one left to the GPU stay there)
    while (k > 0 && t[k - 1].len == t[k].len) --k;
    if (k) *cut = t[k].len;
  }
  t.resize(k);
  return t;
}

// Hashes the planned chunks (their bytes read again through `fill`) into
// ids[32 j] for t[j]; 8 at a time per thread.
// Where the host tail takes a chunk's bytes: straight from the caller's
// memory (dsx_*_host), else read again through the call's fill function
// (dsx_*_fd: the pages the readers just brought into the page cache).
// (Taking them from the pinned read slots instead, each slot kept three
// pieces longer for the feeder, saved the copy of ~0.7 GB per GiB and
// measured no gain, in-process A/B at three cuts, profiles/r06n/: the SHA
// rounds, not the copy, hold the host threads.)
struct TailSrc {
  FillFn fill;
  void* ud;
  const uint8_t* direct = nullptr;  // the source's bytes [0, len) in host memory
};

// Hashes chunks t[0, cnt) (cnt <= 8: one AVX-512 group, else cnt == 1 on the
// scalar path) into ids[32 j]; their bytes from the caller's memory or read
// again through `fill` into buf.
int hash_group(const TailSrc& src, const TailChunk* t, uint64_t cnt, uint8_t* ids,
               std::vector<uint8_t>& buf) {
  const bool vec = host_sha_vec();
  const uint64_t per = vec ? 8 : 1;
  uint64_t total = 0;
  for (uint64_t j = 0; j < cnt; ++j) total += t[j].len;
  if (!src.direct && buf.size() < total + 1) buf.resize(total + 1);
  const uint8_t* p[8];
  uint64_t n[8];
  uint8_t* o[8];
  uint64_t at = 0;
  int rc = DSX_OK;
  for (uint64_t j = 0; j < per; ++j) {
    if (j >= cnt) {
      p[j] = nullptr;
      n[j] = UINT64_MAX;
      o[j] = nullptr;
      continue;
    }
    n[j] = t[j].len;
    o[j] = ids + 32 * j;
    if (src.direct) {
      p[j] = src.direct + t[j].start;
      continue;
    }
    if (t[j].len && rc == DSX_OK) rc = src.fill(src.ud, buf.data() + at, t[j].start, t[j].len);
    p[j] = buf.data() + at;
    at += t[j].len;
  }
  if (rc) return rc;
  if (vec)
    host_sha512_256_x8(p, n, o);
  else
    host_sha512_256_one(p[0], n[0], o[0]);
  return DSX_OK;
}

// Stops with DSX_E_INTERRUPTED between groups once `halt` (the caller's: a
// feeder told to stop, an error path joining it) or `cancel` (dsx_cancel) is
// set, so a cancelled call does not wait for a whole window's host hash.
int hash_tail(const TailSrc& src, const std::vector<TailChunk>& t, uint8_t* ids, int threads,
              const std::atomic<int>* halt, const std::atomic<int>* cancel) {
  const uint64_t per = host_sha_vec() ? 8 : 1;
  const uint64_t groups = (t.size() + per - 1) / per;
  std::atomic<uint64_t> next{0};
  std::atomic<int> err{DSX_OK};
  host_parallel((int)std::min<uint64_t>((uint64_t)threads, groups), [&](int) {
    std::vector<uint8_t> buf;
    for (uint64_t g; err.load() == DSX_OK && (g = next.fetch_add(1)) < groups;) {
      if ((halt && halt->load(std::memory_order_relaxed)) ||
          (cancel && cancel->load(std::memory_order_relaxed))) {
        err.store(DSX_E_INTERRUPTED);
        return;
      }
      const uint64_t j0 = g * per, j1 = std::min<uint64_t>(t.size(), j0 + per);
      const int rc = hash_group(src, t.data() + j0, j1 - j0, ids + 32 * j0, buf);
      if (rc) {
        err.store(rc);
        return;
      }
    }
  });
  return err.load();
}

// The long chunks of a call's last window (the whole file up to the window
// size) hashed on the host while that window is still being read: a thread follows the chain state each stitch publishes
// (HostState.total, seq written last), copies the newly final cut ends to the
// host and hashes the chunks longer than `cut` (read again through the
// call's fill function) on the host pool.  After the read, the GPU digest
// skips those chunks (DigestArgs.skip_above = cut) and hashes the rest, a
// chain of at most `cut` bytes; finish() hands the feeder the final count.
class TailFeeder {
 public:
  // (the last of several windows: start_ev marks the previous window's
  // snapshot dsnap = {cuts before this window, their last end})
  // (`cut`: the cut of the chunks before the first boundary; a boundary, a
  // snapshot the GPU hashed the shorter chunks before during the read, sets
  // the cut of those after it)
  // (cap: at most this many chunks in the window; extra: hashers that join
  // once reads_done() -- the readers' CPUs)
  TailFeeder(dsx_ctx* c, const TailSrc& src, uint64_t len, uint64_t cut, int threads, uint64_t cap,
             uint64_t seq0, hipEvent_t start_ev = nullptr, const uint64_t* dsnap = nullptr,
             int extra = 0)
      : c_(c), src_(src), len_(len), cut_(cut), cap_(cap), threads_(threads), extra_(extra),
        seq0_(seq0), start_ev_(start_ev), dsnap_(dsnap) {
    th_ = std::thread([this] { run(); });
  }
  // a snapshot {total, carry} was enqueued (ev after it): chunks from its
  // total on take `cut_after`.  Called before the pieces after the snapshot
  // are enqueued, so no total the feeder reads after it can come from them
  // without it knowing the boundary.
  void add_boundary(hipEvent_t ev, const uint64_t* snap, uint64_t cut_after) {
    std::lock_guard<std::mutex> g(m_);
    bounds_.push_back({ev, snap, cut_after, 0});
  }
  ~TailFeeder() { stop(); }
  // the call's reads are done: the extra hashers start
  void reads_done() { reads_done_.store(1); }
  void finish(uint64_t total) {
    {
      std::lock_guard<std::mutex> g(m_);
      final_ = total;
      have_final_ = true;
    }
    cv_.notify_all();
  }
  // joins; the hashed chunks and their IDs, or an error
  int join() {
    if (th_.joinable()) th_.join();
    return err_;
  }
  void stop() {
    halt_.store(1);  // (the hashers stop at their next group of 8)
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
    }
    cv_.notify_all();
    if (th_.joinable()) th_.join();
  }
  std::vector<TailChunk> chunks;
  std::vector<uint8_t> ids;

 private:
  // cuts the device has published as final, 0 if none of this call yet
  uint64_t published() const {
    const volatile HostState* h = (const volatile HostState*)c_->h_state;
    const uint64_t q0 = h->seq;
    const uint64_t t = h->total;
    const uint64_t q1 = h->seq;
    return (q0 == q1 && q0 > seq0_) ? t : 0;
  }
  // This thread follows the published totals and queues each new batch's
  // long chunks, longest first, in groups of 8 (part 0 of the host pool);
  // threads_ more parts hash the groups as they come.  (Until round 6 each
  // batch was hashed whole before the next was fetched: the threads idled at
  // every batch's end, and the call's last batch waited for the one before.)
  void run() {
    if (hipSetDevice(c_->device) != hipSuccess) {
      err_ = DSX_E_HIP;
      return;
    }
    // (default priority: beside the null stream in that pool; `stream` and
    // `copy_stream` are in the high pool, the digests in the low one)
    hipStream_t s = nullptr;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) {
      err_ = DSX_E_HIP;
      return;
    }
    chunks.reserve(cap_);  // (never reallocated: the hashers read it while it grows)
    ids.assign(32 * cap_, 0);
    const uint64_t per = host_sha_vec() ? 8 : 1;
    std::mutex qm;
    std::condition_variable qcv;
    std::deque<std::pair<size_t, uint64_t>> q;  // {first chunk, count}
    bool qdone = false;
    std::atomic<int> herr{DSX_OK};
    auto fail = [&](int rc) {
      int ok = DSX_OK;
      herr.compare_exchange_strong(ok, rc);
      qcv.notify_all();
    };
    host_parallel(threads_ + 1 + extra_, [&](int part) {
      if (part == 0) {
        const int rc = produce(s, [&](std::vector<TailChunk>& batch) -> int {
          if (chunks.size() + batch.size() > cap_) return DSX_E_INTERNAL;
          std::sort(batch.begin(), batch.end(),
                    [](const TailChunk& a, const TailChunk& b) { return a.len > b.len; });
          {
            std::lock_guard<std::mutex> g(qm);
            const size_t at = chunks.size();
            chunks.insert(chunks.end(), batch.begin(), batch.end());
            for (uint64_t j = 0; j < batch.size(); j += per)
              q.push_back({at + j, std::min<uint64_t>(per, batch.size() - j)});
          }
          qcv.notify_all();
          return herr.load();
        });
        if (rc) fail(rc);
        {
          std::lock_guard<std::mutex> g(qm);
          qdone = true;
        }
        qcv.notify_all();
        return;
      }
      std::vector<uint8_t> buf;
      if (part > threads_) {  // (the readers' CPUs: only once the reads are done)
        std::unique_lock<std::mutex> lk(qm);
        while (!reads_done_.load() && !qdone && herr.load() == DSX_OK)
          qcv.wait_for(lk, std::chrono::microseconds(200));
      }
      for (;;) {
        std::pair<size_t, uint64_t> g;
        {
          std::unique_lock<std::mutex> lk(qm);
          qcv.wait(lk, [&] { return !q.empty() || qdone || herr.load() != DSX_OK; });
          if (herr.load() != DSX_OK || q.empty()) return;
          g = q.front();
          q.pop_front();
        }
        if (halt_.load(std::memory_order_relaxed) || c_->cancel.load(std::memory_order_relaxed)) {
          fail(DSX_E_INTERRUPTED);
          return;
        }
        const int rc = hash_group(src_, chunks.data() + g.first, g.second, ids.data() + 32 * g.first, buf);
        if (rc) {
          fail(rc);
          return;
        }
      }
    });
    ids.resize(32 * chunks.size());
    if (!err_) err_ = herr.load();
    (void)hipStreamDestroy(s);
  }
  // the follower: each batch of newly final chunks above their cut goes to
  // `put` (which returns non-zero to stop); returns a HIP error, or OK once
  // the final count is in
  template <class Put>
  int produce(hipStream_t s, Put&& put) {
    std::vector<uint64_t> e;
    uint64_t seen = 0, prev = 0;
    if (start_ev_) {
      uint64_t sn[2] = {0, 0};
      if (hipEventSynchronize(start_ev_) != hipSuccess ||
          hipMemcpyAsync(sn, dsnap_, sizeof sn, hipMemcpyDeviceToHost, s) != hipSuccess ||
          hipStreamSynchronize(s) != hipSuccess)
        return DSX_E_HIP;
      seen = sn[0];
      prev = sn[1];
    }
    std::vector<Bound> known;  // the boundaries resolved so far (their totals read)
    while (true) {
      uint64_t target;
      bool last;
      std::vector<Bound> fresh;
      {
        std::unique_lock<std::mutex> g(m_);
        cv_.wait_for(g, std::chrono::microseconds(200), [&] { return stop_ || have_final_; });
        if (stop_) return DSX_E_INTERRUPTED;
        last = have_final_;
        // (read with the boundaries under one lock: a total published before
        // add_boundary cannot come from a piece after that snapshot)
        target = last ? final_ : std::max(seen, published());
        fresh.assign(bounds_.begin() + (long)known.size(), bounds_.end());
      }
      for (Bound& b : fresh) {
        uint64_t sn[2] = {0, 0};
        if (hipEventSynchronize(b.ev) != hipSuccess ||
            hipMemcpyAsync(sn, b.snap, sizeof sn, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
          return DSX_E_HIP;
        b.total = sn[0];
        known.push_back(b);
      }
      if (target > seen) {
        e.resize(target - seen);
        if (hipMemcpyAsync(e.data(), c_->out.p + seen, e.size() * 8, hipMemcpyDeviceToHost, s) !=
                hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
          return DSX_E_HIP;
        std::vector<TailChunk> batch;
        for (uint64_t i = 0; i < e.size(); ++i) {
          const uint64_t st = i ? e[i - 1] : prev;
          // (a call that overflows its candidate slots reruns and drops these:
          // never read outside the source for them)
          uint64_t cut = cut_;
          for (const Bound& b : known)
            if (seen + i >= b.total) cut = b.cut_after;
          if (e[i] > st && e[i] <= len_ && e[i] - st > cut) batch.push_back({seen + i, st, e[i] - st});
        }
        prev = e.back();
        seen = target;
        if (!batch.empty()) {
          const int rc = put(batch);
          if (rc) return rc;
        }
      }
      if (last) return DSX_OK;
    }
  }
  dsx_ctx* c_;
  TailSrc src_;
  uint64_t len_;
  uint64_t cut_, cap_;
  struct Bound {
    hipEvent_t ev;
    const uint64_t* snap;
    uint64_t cut_after, total;
  };
  std::vector<Bound> bounds_;  // (add_boundary, under m_)
  int threads_, extra_;
  std::atomic<int> reads_done_{0};
  uint64_t seq0_;
  hipEvent_t start_ev_;
  const uint64_t* dsnap_;
  std::thread th_;
  std::mutex m_;
  std::condition_variable cv_;
  bool stop_ = false, have_final_ = false;
  std::atomic<int> halt_{0};
  uint64_t final_ = 0;
  int err_ = DSX_OK;
};
// The GPU's shares of a one-window call during its read (run_index,
// run_ids): the points f_k = 1/2, 3/4, ... of the window where a digest on side
// stream k hashes the chunks completed since the previous point up to cut_k =
// the read time left after f_k over the GPU's ns per byte (its chain ends
// about when the read does; digest_pc_kernel beside the scans ran 37-40 ns
// per byte, profiles/r06an, so 45 with a margin: 0.892 against 0.872 x
// dsx_cut_fd at 58, profiles/r06ao).  They stop where cut_k falls below 1.5 x
// `feed_cut`, the host's usual cut (two points at 1 GiB and 12 threads; a
// third slowed the read, r06ab, r06am, r06ao); none when the first is below
// 2 x it.
struct Mid {
  uint64_t at, cut;
};
std::vector<Mid> plan_shares(uint64_t len, uint64_t max_chunk, uint64_t feed_cut) {
  double share_ns = kShareNsPerByte;  // the shares' chain, ns per byte
  double slack_ns = 0;              // a share may end this long after the read
  const double t_read = (double)len / kReadBytesPerNs;  // ns
  std::vector<double> fr;
  for (double f = 0.5; f < 0.99 && fr.size() < kMaxMids; f = 0.5 * (1.0 + f)) fr.push_back(f);
#if DSX_DIAG
  if (const char* v = getenv("DSX_SHARE_NS")) share_ns = std::max(10.0, atof(v));
  if (const char* v = getenv("DSX_SHARE_SLACK")) slack_ns = 1e3 * atof(v);  // (us)
  if (const char* v = getenv("DSX_FEED_MID")) {  // (A/B: "0" off, else a list "0.5,0.75")
    fr.clear();
    for (const char* q = v; *q && fr.size() < kMaxMids;) {
      char* nx = nullptr;
      const double f = strtod(q, &nx);
      if (nx == q) break;
      if (f > 0.05 && f < 0.99 && (fr.empty() || f > fr.back())) fr.push_back(f);
      q = *nx == ',' ? nx + 1 : nx;
    }
  }
#endif
  std::vector<Mid> mids;
  for (double f : fr) {
    const double ck = ((1.0 - f) * t_read + slack_ns) / share_ns;
    if (ck < (mids.empty() ? 2.0 : 1.5) * (double)feed_cut) break;
    mids.push_back({(uint64_t)(f * (double)len), std::min<uint64_t>(max_chunk, (uint64_t)ck & ~4095ull)});
  }
  return mids;
}

// The host's share of the tail: feed_threads() SHA threads beside the
// readers, within the process's CPU share (host_cpu_share: 16 on the GPU box,
// whose affinity mask shows the whole machine); the GPU keeps the chunks up
// to feed_cut() bytes (a 58 ns/B chain at the end of the call), the host the
// longer ones.  Fewer threads hash less per ms, so the cut rises with them:
// 28 KiB at 28 threads (round 5's setting, above the share), 64 KiB at 12
// (tools/feed_ab.py).
constexpr uint64_t kFeedCutBase = 28ull << 10;  // at kFeedThreadsBase threads
constexpr int kFeedThreadsBase = 28;
int feed_threads(const dsx_ctx* c) {
  int t = std::max(1, host_cpu_share() - c->index_readers);
#if DSX_DIAG
  if (const char* v = getenv("DSX_FEED_THREADS")) t = std::max(1, std::min(64, atoi(v)));
#endif
  return t;
}
uint64_t feed_cut_for(int64_t host_tail, int threads) {
  if (host_tail > 0) return (uint64_t)host_tail;  // forced (tests, A/B)
  const uint64_t cut = kFeedCutBase * (uint64_t)kFeedThreadsBase / (uint64_t)std::max(1, threads);
  return std::min<uint64_t>(128ull << 10, std::max<uint64_t>(kFeedCutBase, (cut + 2047) & ~4095ull));
}
uint64_t feed_cut(const dsx_ctx* c, int threads) { return feed_cut_for(c->index_host_tail, threads); }

// run_index's geometry: pieces (pinned slots) tile the windows exactly; a
// window keeps `pre` bytes of its predecessor in front (>= max + 64, line
// aligned).  The file's last kFineTail bytes (in its last window) are read,
// copied and scanned in pieces of piece / kFineDiv when the tail feeder runs
// (`feeds`): it then sees the long chunks of the call's last piece, the
// host's last batch, a few MB sooner.  (Smaller pieces throughout slow the
// read: 8 MiB slots, 28 against 45 GiB/s for dsx_cut_fd, profiles/r06ad.)
struct IndexGeom {
  uint64_t pre, piece, W, nwin, fine, fine_from = UINT64_MAX;
  IndexGeom(uint64_t len, uint64_t max_chunk, uint64_t slot, uint64_t window, bool feeds) {
    pre = (max_chunk + 64 + kLine - 1) / kLine * kLine;
    piece = std::min<uint64_t>(slot, std::max<uint64_t>(len, 4096));
    piece = (piece + 4095) & ~4095ull;
    W = std::max<uint64_t>(window, 2 * pre);
    W = (W + piece - 1) / piece * piece;
    if (W >= len) W = (len + piece - 1) / piece * piece;  // one window
    nwin = (len + W - 1) / W;
    uint64_t fine_tail = kFineTail, fine_div = kFineDiv;
#if DSX_DIAG
    if (const char* v = getenv("DSX_FINE_TAIL")) fine_tail = (uint64_t)atol(v);
    if (const char* v = getenv("DSX_FINE_DIV")) fine_div = std::max<uint64_t>(1, atol(v));
#endif
    fine = std::max<uint64_t>(4096, (piece / fine_div) & ~4095ull);
    if (feeds && fine_tail && fine < piece) {
      const uint64_t last_ws = (nwin - 1) * W;
      fine_from = std::max(last_ws, (len - std::min(len, fine_tail)) / piece * piece);
    }
  }
};

// With the GPU's shares the host has fewer bytes: after the last point the
// feeder takes 11/16 of its usual cut (64 -> 44 KiB at 12 threads; 3/4:
// profiles/r06af, r06ag, 0.882 / 0.898 x dsx_cut_fd against 0.874 / 0.894 at
// 64; 44 against 48 / 40 / 36 KiB, r06aq: the call's end 1.88 ms after the
// last stitch against 2.04 / 1.89 / 2.07).
uint64_t share_end_cut(uint64_t fcut) { return std::max<uint64_t>(kFeedCutBase, (fcut * 11 / 16) & ~4095ull); }

int run_index(dsx_ctx* c, const dsx_params_t* p, int algo, uint64_t len, FillFn fill, void* ud,
              uint64_t* out_ends, uint8_t* out_ids, uint64_t cap, uint64_t* n_out,
              const uint8_t* direct = nullptr) {
  HIPCHK(c, hipSetDevice(c->device));
  c->err.clear();
  int rc = ensure_attr_walk(c);
  if (rc) return rc;
  *n_out = 0;
  c->stats.host_tail_chunks = 0;
  if (len == 0) return DSX_OK;  // empty file: no chunks (TestChunkerEmptyFile)
  const uint64_t need = len / p->min + 2;
  const bool feeds = algo == DSX_DIGEST_SHA512_256 && out_ids &&
                     (c->index_host_tail > 0 || (c->index_host_tail < 0 && host_sha_vec()));
  const IndexGeom g(len, p->max, c->index_slot, c->index_window, feeds);
  const uint64_t pre = g.pre, piece = g.piece, W = g.W, nwin = g.nwin;
  const uint64_t fine = g.fine, fine_from = g.fine_from;
  const uint64_t scan_step = std::max<uint64_t>(piece, kScanStep / piece * piece);
  rc = index_setup(c, piece);
  if (rc) return rc;
  HIPCHK(c, grow(c, c->idx_win[0], pre + W));
  if (nwin > 1) HIPCHK(c, grow(c, c->idx_win[1], pre + W));
  HIPCHK(c, grow(c, c->idx_snap, 2 * (nwin + 1 + kMaxMids)));  // (+ the one window's mid snapshots)
  HIPCHK(c, grow(c, c->out, need));
  if (algo >= 0) HIPCHK(c, grow(c, c->dg_ids, need * 32));
  const int K = dsx_ctx::kIdxSlots;

  ProgressScope prog(c, len);
#if DSX_DIAG
  const auto call_t0 = std::chrono::steady_clock::now();
#endif
  for (int attempt = 0; attempt < 2; ++attempt) {
    CallCfg cc{p, len, 0, kRound, c->out.p, need, attempt == 1};
    rc = reset_state(c, 0);
    if (rc) return rc;
    HIPCHK(c, hipMemsetAsync(c->idx_snap.p, 0, 2 * sizeof(uint64_t), c->stream));  // {0 cuts, cut 0}
    Prefetcher pf(fill, ud, len, piece, c->idx_slots, K, c->index_readers, fine_from, fine);
    const TailSrc tsrc{fill, ud, direct};  // (the host tail's bytes)
    uint64_t k = 0;  // piece index
    uint64_t w = 0, ws = 0, wl = 0;
    // Interrupted{} or a read error (make.go:133-162, :201-203): the chunks
    // confirmed so far -- the chain up to the last stitched piece, a prefix
    // of the true chain -- are returned with the error, IDs included: the
    // current window's confirmed chunks are hashed first.
    auto partial = [&](int err) -> int {
      drain(c, pf, err);
      if (algo >= 0) {
        hipLaunchKernelGGL(state_snapshot_kernel, dim3(1), dim3(64), 0, c->stream,
                           (const DevState*)c->state.p, c->idx_snap.p + 2 * (w + 1));
        DigestArgs da{};
        uint8_t* buf = c->idx_win[w & 1].p;
        da.blob = w == 0 ? buf + pre : buf;
        da.base_off = w == 0 ? 0 : ws - pre;
        da.len = w == 0 ? wl : pre + wl;
        da.ends = c->out.p;
        da.ids = c->dg_ids.p;
        da.range_lo = c->idx_snap.p + 2 * w;
        da.range_hi = c->idx_snap.p + 2 * (w + 1);
        if (launch_window_digest(c, da, (pre + wl) / p->min + 2, algo, (int)(w & 1))) return err;
      }
      HostState st;
      (void)hipStreamSynchronize(c->stream);
      (void)hipStreamSynchronize(c->idx_dg_stream);
      if (read_state(c, &st) || st.err) return err;  // (no piece stitched yet: nothing)
      const uint64_t n = std::min<uint64_t>(st.total, cap);
      if (n && hipMemcpy(out_ends, c->out.p, n * 8, hipMemcpyDeviceToHost) != hipSuccess) return err;
      if (n && out_ids && hipMemcpy(out_ids, c->dg_ids.p, n * 32, hipMemcpyDeviceToHost) != hipSuccess)
        return err;
      *n_out = n;
      prog.set(n ? out_ends[n - 1] : 0);
      return err;
    };
    // the host tail of the last window (SHA-512/256 only; auto needs AVX-512)
    const bool tail_on = feeds;
    std::vector<TailChunk> tail;
    std::vector<uint8_t> tail_ids;
    // the last window's long chunks are hashed on the host during its read;
    // with several windows the feeder starts from the previous window's
    // snapshot (feed_ev: recorded after it)
    struct Ev {
      hipEvent_t e = nullptr;
      ~Ev() {
        if (e) (void)hipEventDestroy(e);
      }
    } feed_ev;
    if (tail_on) HIPCHK(c, hipEventCreateWithFlags(&feed_ev.e, hipEventDisableTiming));
    std::unique_ptr<TailFeeder> feed;
    const int fth = feed_threads(c);
    const uint64_t fcut = feed_cut(c, fth);
    // the readers' CPUs join the feeder's hashers once the reads are done
    int feed_extra = std::max(0, std::min(c->index_readers, host_cpu_share() - fth));
#if DSX_DIAG
    if (const char* v = getenv("DSX_FEED_EXTRA")) feed_extra = std::max(0, std::min(16, atoi(v)));
#endif
    // One window (a file up to DSX_INDEX_WINDOW): the GPU hashes most of it
    // DURING the read.  At the points f_k of the window (1/2, 3/4, ...) a
    // snapshot follows the piece's stitch and a digest on side stream k (a
    // "share") hashes the chunks confirmed since the previous point, all but
    // those longer than cut_k = the read time left after f_k over the GPU's
    // ns per byte (plan_shares): its chain ends about when the read does.  The feeder
    // hashes, from the call's start, each segment's chunks above its cut and
    // the last segment's above fcut_end; the digest after the read (on
    // `stream`, digest_pc_kernel) takes the last segment's short chunks, a
    // chain of at most fcut_end bytes.  The points stop where cut_k would
    // fall below 1.5 x fcut (two points at 1 GiB and 12 threads); none
    // when the first is below 2 x fcut (files below ~0.5 GiB), for
    // SHA-256, or without the host tail.  At 1 GiB and 12 threads the host
    // takes 2,985 chunks against 6,060 without the shares, and the call
    // reads 0.87-0.90 x dsx_cut_fd against 0.78-0.84.
    // The side streams have hardware queues of their own (side_stream_create):
    // on one shared with the pipeline's streams the shares held the next
    // pieces' scans and the call fell to 0.58-0.63 x dsx_cut_fd
    // (profiles/r06q, r06x).  Four shares (down to 7/8 and 15/16) slowed the
    // read: 0.87 against 0.89 (profiles/r06ag).
    // (A first form gave the GPU every chunk of the first half and started
    // the feeder at mid: the host then had less time for the same work, 0.66-
    // 0.72 x dsx_cut_fd against 0.78, profiles/r06e, r06f.)
    uint64_t fcut_end = fcut;
    int share_pc = 1;
#if DSX_DIAG
    if (const char* v = getenv("DSX_SHARE_PC")) share_pc = atoi(v);
#endif
    // (several windows: the last one's shares, on side streams 1.. -- side
    // stream 0 carries the previous window's digest meanwhile)
    bool share_multi = true;
#if DSX_DIAG
    if (const char* v = getenv("DSX_SHARE_MULTI")) share_multi = atoi(v) != 0;
#endif
    const uint64_t last_ws = (nwin - 1) * W, last_wl = len - last_ws;
    const size_t side0 = nwin > 1 ? 1 : 0;  // the first side stream of the shares
    std::vector<Mid> mids;
    if (tail_on && (nwin == 1 || share_multi) && c->index_host_tail < 0) {
      fcut_end = share_end_cut(fcut);
#if DSX_DIAG
      if (const char* v = getenv("DSX_FEED_CUT_END")) fcut_end = std::max<uint64_t>(4096, atol(v));
#endif
      mids = plan_shares(last_wl, p->max, fcut);
      if (mids.size() > (size_t)dsx_ctx::kIdxSide - side0) mids.resize(dsx_ctx::kIdxSide - side0);
      for (Mid& m : mids) m.at += last_ws;
      if (mids.empty()) fcut_end = fcut;
    }
    std::vector<Ev> mid_ev(mids.size());
    for (auto& x : mid_ev) HIPCHK(c, hipEventCreateWithFlags(&x.e, hipEventDisableTiming));
    size_t mids_done = 0;
    // snapshot k: after the piece at mids[k].at (the window's start is idx_snap[0])
    auto mid_snap = [&](size_t k) { return c->idx_snap.p + 2 * (nwin + 1 + k); };
    for (w = 0; w < nwin; ++w) {
      ws = w * W;
      wl = std::min(W, len - ws);
      uint8_t* buf = c->idx_win[w & 1].p;
      bool feed_on = tail_on && w + 1 == nwin;
#if DSX_DIAG
      if (nwin > 1 && getenv("DSX_FEED_MULTI") && atoi(getenv("DSX_FEED_MULTI")) == 0) feed_on = false;
#endif
      if (feed_on) {
        feed.reset(new TailFeeder(c, tsrc, len, mids.empty() ? fcut : mids[0].cut, fth,
                                  (pre + wl) / p->min + 2, c->piece_seq, nwin > 1 ? feed_ev.e : nullptr,
                                  c->idx_snap.p + 2 * w, feed_extra));
      }
      // the digest of window w-2 read this buffer; the copy stream waits for it
      if (w >= 2) HIPCHK(c, hipStreamWaitEvent(c->copy_stream, c->idx_win_ev[w & 1], 0));
      if (w >= 1)  // the previous window's last `pre` bytes (it was a full window)
        HIPCHK(c, hipMemcpyAsync(buf, c->idx_win[(w - 1) & 1].p + W, pre,
                                 hipMemcpyDeviceToDevice, c->copy_stream));
      uint64_t scanned = ws;
      for (uint64_t off = ws, hn = 0; off < ws + wl; off += hn, ++k) {
        if (c->cancel.load()) return partial(DSX_E_INTERRUPTED);
        uint8_t* hp = nullptr;
        hn = 0;
        rc = pf.wait(k, &hp, &hn);
        if (rc) return partial(rc);
        if (feed && off + hn == len) feed->reads_done();  // (the readers are idle now)
        hipError_t e = hipMemcpyAsync(buf + pre + (off - ws), hp, hn, hipMemcpyHostToDevice,
                                      c->copy_stream);
        if (e == hipSuccess) e = hipEventRecord(c->idx_copy_ev[k % K], c->copy_stream);
        // keep two copies queued: the previous slot returns to the readers
        // once its copy has landed
        if (e == hipSuccess && k >= 1) e = hipEventSynchronize(c->idx_copy_ev[(k - 1) % K]);
        if (e != hipSuccess) return drain(c, pf, set_hip_err(c, e, "index: H2D"));
        if (k >= 1) pf.release(k - 1);
        const uint64_t end = off + hn;
        if (end == ws + wl || end - scanned >= scan_step || end > fine_from) {
          e = scan_wait(c, c->idx_copy_ev[k % K]);  // (the stitch follows the scan)
          if (e != hipSuccess) return drain(c, pf, set_hip_err(c, e, "index: wait"));
          const uint64_t halo = w == 0 ? scanned : pre + (scanned - ws);
          c->timing = false;  // (no event records between the pipeline's kernels)
          rc = enqueue_piece(c, cc, buf + pre + (scanned - ws), halo, scanned, end - scanned,
                             end == len);
          c->timing = true;
          if (rc) return drain(c, pf, rc);
          scanned = end;
          if (mids_done < mids.size() && end >= mids[mids_done].at && end < len && feed) {
            // the GPU's share of segment k: chunks [snap[k-1].total,
            // snap[k].total) up to its cut, on the digest stream, on 3/4 of
            // the CUs (the rest keep room for the next pieces' scans)
            const size_t m = mids_done++;
            hipLaunchKernelGGL(state_snapshot_kernel, dim3(1), dim3(64), 0, c->stream,
                               (const DevState*)c->state.p, mid_snap(m));
            e = hipEventRecord(mid_ev[m].e, c->stream);
            if (e != hipSuccess) return drain(c, pf, set_hip_err(c, e, "index: record"));
            DigestArgs dm{};
            dm.blob = w == 0 ? buf + pre : buf;
            dm.base_off = w == 0 ? 0 : ws - pre;
            dm.len = w == 0 ? end : pre + (end - ws);
            dm.ends = c->out.p;
            dm.ids = c->dg_ids.p;
            dm.range_lo = m ? mid_snap(m - 1) : c->idx_snap.p + 2 * w;
            dm.range_hi = mid_snap(m);
            dm.skip_above = mids[m].cut >= p->max ? 0 : mids[m].cut;
            // (on its own side stream after this stitch: the shares run side by side)
            hipStream_t ss = c->idx_side[side0 + m];
            e = hipStreamWaitEvent(ss, mid_ev[m].e, 0);
            if (e != hipSuccess) return drain(c, pf, set_hip_err(c, e, "index: wait"));
            // (digest_pc_kernel: its chain ran ~45 ns/B during the read,
            // digest_kernel's ~85, profiles/r06aa, r06ab)
            const uint64_t from = m ? mids[m - 1].at : ws;
            rc = launch_digest(c, dm, (end - from + 2 * p->max) / p->min + 2, algo, ss,
                               c->idx_side_q.p + 32 * (side0 + m), false, (uint32_t)(c->ncu * 3 / 4),
                               share_pc);
            if (rc) return drain(c, pf, rc);
            feed->add_boundary(mid_ev[m].e, mid_snap(m), m + 1 < mids.size() ? mids[m + 1].cut : fcut_end);
#if DSX_DIAG
            if (getenv("DSX_TAIL_LOG"))
              fprintf(stderr, "index: GPU share %zu up to %.1f MB (cut %lu), %.2f ms into the call\n",
                      m, end / 1e6, (unsigned long)mids[m].cut,
                      std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - call_t0).count());
#endif
          }
#if DSX_DIAG
          if (end == len && getenv("DSX_TAIL_LOG"))
            fprintf(stderr, "index: last piece enqueued %.2f ms into the call\n",
                    std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - call_t0).count());
#endif
        }
      }
      // the window's finished chunks: [snap[w].total, snap[w+1].total) from
      // snap[w].carry, all inside this window's bytes
      if (algo < 0) {  // cut list only (dsx_cut_host / dsx_cut_fd)
        hipError_t e = hipEventRecord(c->idx_win_ev[w & 1], c->stream);
        if (e != hipSuccess) return drain(c, pf, set_hip_err(c, e, "index: record"));
        continue;
      }
      hipLaunchKernelGGL(state_snapshot_kernel, dim3(1), dim3(64), 0, c->stream,
                         (const DevState*)c->state.p, c->idx_snap.p + 2 * (w + 1));
      if (tail_on && w + 2 == nwin) {  // (the last window's feeder starts from this snapshot)
        hipError_t e = hipEventRecord(feed_ev.e, c->stream);
        if (e != hipSuccess) return drain(c, pf, set_hip_err(c, e, "index: record"));
      }
      DigestArgs da{};
      da.blob = w == 0 ? buf + pre : buf;
      da.base_off = w == 0 ? 0 : ws - pre;
      da.len = w == 0 ? wl : pre + wl;
      da.ends = c->out.p;
      da.ids = c->dg_ids.p;
      da.range_lo = mids_done ? mid_snap(mids_done - 1) : c->idx_snap.p + 2 * w;  // (after the GPU's shares)
      da.range_hi = c->idx_snap.p + 2 * (w + 1);
      if (tail_on && w + 1 == nwin) {
        // the window's chunk ends (the stitch is done once the stream is)
        uint64_t snap[4];
        hipError_t e = hipStreamSynchronize(c->stream);
        if (e == hipSuccess)
          e = hipMemcpy(snap, c->idx_snap.p + 2 * w, sizeof snap, hipMemcpyDeviceToHost);
        if (e != hipSuccess) return drain(c, pf, set_hip_err(c, e, "index: tail range"));
        const uint64_t i0 = snap[0], i1 = std::max(snap[0], snap[2]);
        std::vector<uint64_t> ends(i1 - i0);
        if (i1 > i0)
          e = hipMemcpy(ends.data(), c->out.p + i0, (i1 - i0) * 8, hipMemcpyDeviceToHost);
        if (e != hipSuccess) return drain(c, pf, set_hip_err(c, e, "index: tail ends"));
        const int threads = std::max(1, std::min(kTailThreads, host_cpu_share()));
        if (feed) {  // the feeder has the long chunks: the GPU the rest
          // on `stream` after the last stitch (nothing follows it there; the
          // shares hold the side streams), sized by the count of the
          // window's chunks up to the cut, so that a window's ~10 K of them
          // run on digest_pc_kernel (its chain ~38 ns/B at the end of a call,
          // digest_kernel's ~58; profiles/r06aa)
          da.skip_above = fcut_end;
          uint64_t short_n = 0;
          for (uint64_t i = 0, st = snap[1]; i < ends.size(); st = ends[i++]) short_n += ends[i] - st <= fcut_end;
          // (its own queue counter: the previous window's digest may still
          // run on idx_dg_stream with the ctx's)
          rc = launch_digest(c, da, short_n + 2, algo, c->stream, c->idx_side_q.p + 32 * dsx_ctx::kIdxSide,
                             false);
          if (rc) return drain(c, pf, rc);
#if DSX_DIAG
          const auto tf0 = std::chrono::steady_clock::now();
          if (getenv("DSX_TAIL_LOG"))
            fprintf(stderr, "feed: last piece stitched %.2f ms into the call\n",
                    std::chrono::duration<double, std::milli>(tf0 - call_t0).count());
#endif
          feed->finish(i1);
          rc = feed->join();
          if (rc == DSX_E_INTERRUPTED) return partial(rc);  // (dsx_cancel during the host hash)
          if (rc) return drain(c, pf, rc);
          tail = std::move(feed->chunks);
          tail_ids = std::move(feed->ids);
          c->stats.host_tail_chunks = tail.size();
#if DSX_DIAG
          if (getenv("DSX_TAIL_LOG")) {
            const double hms =
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tf0).count();
            (void)hipStreamSynchronize(c->stream);
            const double gms =
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tf0).count();
            for (size_t m = 0; m < mids_done; ++m) (void)hipStreamSynchronize(c->idx_side[side0 + m]);
            const double sms =
                std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - tf0).count();
            fprintf(stderr, "feed: chunks %lu host %zu (cut %lu) host done %.2f ms, GPU done %.2f ms, shares done %.2f ms\n",
                    (unsigned long)i1, tail.size(), (unsigned long)fcut_end, hms, gms, sms);
          }
#endif
          continue;
        }
        // (the end tail: reached only with the last-window feeder switched off,
        // DSX_FEED_MULTI=0 in the diagnostic build, the comparison of r05bt)
        tail = plan_tail(c, ends, i0, snap[1], threads, &da.skip_above);
        rc = launch_window_digest(c, da, (pre + wl) / p->min + 2, algo, (int)(w & 1));
        if (rc) return drain(c, pf, rc);
        // the host's share while the GPU hashes the rest
        tail_ids.assign(32 * tail.size(), 0);
#if DSX_DIAG
        const auto th0 = std::chrono::steady_clock::now();
#endif
        if (!tail.empty()) rc = hash_tail(tsrc, tail, tail_ids.data(), threads, nullptr, &c->cancel);
        if (rc) return drain(c, pf, rc);
        c->stats.host_tail_chunks = tail.size();
#if DSX_DIAG
        if (getenv("DSX_TAIL_LOG")) {
          uint64_t hb = 0;
          for (const auto& x : tail) hb += x.len;
          const double hms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - th0).count();
          (void)hipStreamSynchronize(c->idx_dg_stream);
          const double gms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - th0).count();
          fprintf(stderr, "tail: window chunks %lu host %zu (%.1f MB, cut %lu) host %.2f ms, GPU done %.2f ms\n",
                  (unsigned long)ends.size(), tail.size(), hb / 1e6, (unsigned long)da.skip_above, hms, gms);
        }
#endif
      } else {
        rc = launch_window_digest(c, da, (pre + wl) / p->min + 2, algo, (int)(w & 1));
        if (rc) return drain(c, pf, rc);
      }
    }
    pf.stop();
    HostState st;
    rc = read_state(c, &st);  // (the stitches)
    HIPCHK(c, hipStreamSynchronize(c->copy_stream));
    HIPCHK(c, hipStreamSynchronize(c->idx_dg_stream));  // (the digests)
    for (size_t m = 0; m < mids_done; ++m) HIPCHK(c, hipStreamSynchronize(c->idx_side[side0 + m]));
    if (rc) return rc;
    if (st.err & kErrDense) {  // rare: a lane overflowed its candidate slots
      c->stats.dense_fallbacks++;
      continue;
    }
    if (st.err) {
      c->err = "index: stitch error";
      return DSX_E_INTERNAL;
    }
#if DSX_DIAG
    if (getenv("DSX_TAIL_LOG"))
      fprintf(stderr, "index: done %.2f ms into the call\n",
              std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - call_t0).count());
#endif
    c->stats.chunks = st.total;
    c->stats.repaired_segments = st.repaired;
    c->stats.chunks_discarded = st.discarded;
    *n_out = st.total;
    if (st.total > cap) return DSX_E_CAPACITY;
    if (st.total) {
      HIPCHK(c, hipMemcpy(out_ends, c->out.p, st.total * 8, hipMemcpyDeviceToHost));
      if (out_ids) HIPCHK(c, hipMemcpy(out_ids, c->dg_ids.p, st.total * 32, hipMemcpyDeviceToHost));
      for (size_t j = 0; j < tail.size(); ++j)  // (the GPU skipped these)
        if (tail[j].idx < st.total) memcpy(out_ids + 32 * tail[j].idx, tail_ids.data() + 32 * j, 32);
    }
    prog.set(len);
    return DSX_OK;
  }
  c->err = "dense-candidate path overflowed";
  return DSX_E_INTERNAL;
}

// IDs of a given contiguous chunk list [start, ends[0]), [ends[0], ends[1]),
// ... of the source's bytes [0, len): the same reader / window pipeline as
// run_index without the scan.  The source is read from `start` to the last
// end; a window's halo is the longest chunk, so every chunk is hashed in the
// window where it ends, with all its bytes resident.  The ranges per window
// come from the host's list (no device snapshots).
int run_ids(dsx_ctx* c, int algo, uint64_t len, FillFn fill, void* ud, uint64_t start,
            const uint64_t* ends, uint64_t n, uint8_t* out_ids, const uint8_t* direct = nullptr) {
  HIPCHK(c, hipSetDevice(c->device));
  c->err.clear();
  if (n == 0) return DSX_OK;
  if (n > 0xFFFFFFF0ull) return DSX_E_INVAL;
  uint64_t prev = start, maxc = 0;
  for (uint64_t i = 0; i < n; ++i) {
    if (ends[i] < prev || ends[i] > len) {
      c->err = "chunk ends must be non-decreasing, start <= ends[0], ends[n-1] <= len";
      return DSX_E_INVAL;
    }
    maxc = std::max(maxc, ends[i] - prev);
    prev = ends[i];
  }
  // bytes [start, last) relative to `start` from here on
  const uint64_t L = ends[n - 1] - start;
  const uint64_t pre = (maxc + kLine - 1) / kLine * kLine;
  uint64_t piece = std::min<uint64_t>(c->index_slot, std::max<uint64_t>(L, 4096));
  piece = (piece + 4095) & ~4095ull;
  uint64_t W = std::max<uint64_t>(c->index_window, 2 * pre);
  W = (W + piece - 1) / piece * piece;
  if (W >= L) W = std::max<uint64_t>(piece, (L + piece - 1) / piece * piece);  // one window
  const uint64_t nwin = std::max<uint64_t>(1, (L + W - 1) / W);
  int rc = index_setup(c, piece);
  if (rc) return rc;
  HIPCHK(c, grow(c, c->idx_win[0], pre + W));
  if (nwin > 1) HIPCHK(c, grow(c, c->idx_win[1], pre + W));
  HIPCHK(c, grow(c, c->dg_ends, n));
  HIPCHK(c, grow(c, c->dg_ids, n * 32));
  // the list, relative to `start`, on the device
  {
    std::vector<uint64_t> rel(n);
    for (uint64_t i = 0; i < n; ++i) rel[i] = ends[i] - start;
    HIPCHK(c, hipMemcpyAsync(c->dg_ends.p, rel.data(), n * 8, hipMemcpyHostToDevice, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
  }
  struct Shifted {
    FillFn fill;
    void* ud;
    uint64_t start;
  } sh{fill, ud, start};
  auto fill_shifted = [](void* u, uint8_t* dst, uint64_t off, uint64_t cnt) {
    const Shifted* s = (const Shifted*)u;
    return s->fill(s->ud, dst, s->start + off, cnt);
  };
  const int K = dsx_ctx::kIdxSlots;
#if DSX_DIAG
  // (DSX_TAIL_LOG: the call's phases, to find which one a slow call spends
  // its time in -- the reads, the wait for the early host hash, the GPU)
  const bool tlog = getenv("DSX_TAIL_LOG") != nullptr;
  const auto t0 = std::chrono::steady_clock::now();
  auto ms = [&] { return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count(); };
  double t_read = 0, t_join0 = 0, t_join1 = 0;
#endif
  Prefetcher pf(fill_shifted, &sh, L, piece, c->idx_slots, K, c->index_readers);
  uint64_t k = 0, i0 = 0;
  // the host tail of the last window, as in run_index (the list is known here)
  const bool tail_on = algo == DSX_DIGEST_SHA512_256 &&
                       (c->index_host_tail > 0 || (c->index_host_tail < 0 && host_sha_vec()));
  std::vector<TailChunk> tail;
  std::vector<uint8_t> tail_ids;
  c->stats.host_tail_chunks = 0;
  // The list is known up front, so the host hashes the last window's long
  // chunks (all of them in one window) from the start, beside the read (the
  // tail feeder of run_index without the wait for the stitch); that window's
  // digest skips them.
  const int eth = feed_threads(c);
  const uint64_t early_cut = feed_cut(c, eth);
  std::vector<TailChunk> early;
  std::vector<uint8_t> early_ids;
  int early_rc = DSX_OK;
  struct Joiner {  // (an error return stops the early hash at its next group, then joins)
    std::thread t;
    std::atomic<int> halt{0};
    ~Joiner() {
      halt.store(1);
      if (t.joinable()) t.join();
    }
  } early_th;
  // One window: the GPU's shares during the read (plan_shares, as in
  // run_index; here the chunk ranges are known on the host: share k takes the
  // chunks that end in the pieces landed by its point, up to its cut), and
  // the host the longer ones from the call's start, with the last segment's
  // above end_cut -- the lowest cut whose host bytes the threads finish within
  // ~3/4 of the read (the list is known, so the host can start on the last
  // segment at once); the digest after the read takes the rest, a chain of
  // at most end_cut bytes.
  struct IdShare {
    uint64_t landed, cut, i1;  // chunks [previous i1, i1) end at or before `landed`
  };
  std::vector<IdShare> shares;
  uint64_t end_cut = early_cut;
  // (several windows: the last one's, on side streams 0.., planned over its
  // length; the windows' digests run on `stream` here)
  const uint64_t last_ws = (nwin - 1) * W;
  uint64_t i_last = 0;  // the last window's first chunk (the first ending past last_ws)
  while (nwin > 1 && i_last < n && ends[i_last] - start <= last_ws) ++i_last;
  bool share_multi = true;
#if DSX_DIAG
  if (const char* v = getenv("DSX_SHARE_MULTI")) share_multi = atoi(v) != 0;
#endif
  if (tail_on && (nwin == 1 || share_multi) && c->index_host_tail < 0) {
    for (const Mid& m : plan_shares(L - last_ws, maxc, early_cut)) {
      const uint64_t landed = std::min(L, (last_ws + m.at + piece - 1) / piece * piece);
      if (landed >= L || shares.size() >= (size_t)dsx_ctx::kIdxSide) break;
      uint64_t i1 = shares.empty() ? i_last : shares.back().i1;
      while (i1 < n && ends[i1] - start <= landed) ++i1;
      shares.push_back({landed, m.cut, i1});
    }
    if (!shares.empty()) {
      // host bytes: each segment's chunks above its cut, and the last
      // segment's above end_cut
      uint64_t fixed = 0;
      std::vector<uint64_t> last;
      for (uint64_t i = i_last, k = 0; i < n; ++i) {
        while (k < shares.size() && i >= shares[k].i1) ++k;
        const uint64_t ln = ends[i] - (i ? ends[i - 1] : start);
        if (k < shares.size()) {
          if (ln > shares[k].cut) fixed += ln;
        } else {
          last.push_back(ln);
        }
      }
      std::sort(last.begin(), last.end());
      const double budget = 0.75 * (double)L / kReadBytesPerNs * eth / host_ns_per_byte();  // bytes
      // the lowest cut (4 KiB steps up to early_cut) whose host bytes fit
      uint64_t tail_bytes = 0;
      for (uint64_t x : last) tail_bytes += x;
      size_t j = 0;
      end_cut = early_cut;
      for (uint64_t cut = 4096; cut <= early_cut; cut += 4096) {
        while (j < last.size() && last[j] <= cut) tail_bytes -= last[j++];
        if ((double)(fixed + tail_bytes) <= budget) {
          end_cut = cut;
          break;
        }
      }
#if DSX_DIAG
      if (const char* v = getenv("DSX_FEED_CUT_END")) end_cut = std::max<uint64_t>(4096, atol(v));
#endif
    }
  }
  if (tail_on) {  // (the last window: chunks ending past last_ws)
    for (uint64_t i = 0, k = 0; i < n; ++i) {
      const uint64_t s0 = i ? ends[i - 1] - start : 0, e0 = ends[i] - start;
      while (k < shares.size() && i >= shares[k].i1) ++k;
      const uint64_t cut = k < shares.size() ? shares[k].cut : (shares.empty() ? early_cut : end_cut);
      if (i < i_last) continue;  // (k counts segments from the last window's first chunk)
      if ((nwin == 1 || e0 > last_ws) && e0 - s0 > cut) early.push_back({i, s0, e0 - s0});
    }
    std::sort(early.begin(), early.end(), [](const TailChunk& a, const TailChunk& b) { return a.len > b.len; });
    early_ids.assign(32 * early.size(), 0);
    if (!early.empty())
      early_th.t = std::thread([&, eth] {
        const TailSrc esrc{fill_shifted, &sh, direct ? direct + start : nullptr};
        early_rc = hash_tail(esrc, early, early_ids.data(), eth, &early_th.halt, &c->cancel);
      });
  }
  size_t shares_done = 0;
  for (uint64_t w = 0; w < nwin; ++w) {
    const uint64_t ws = w * W, wl = std::min(W, L - ws);
    uint8_t* buf = c->idx_win[w & 1].p;
    if (w >= 2) HIPCHK(c, hipStreamWaitEvent(c->copy_stream, c->idx_win_ev[w & 1], 0));
    if (w >= 1)
      HIPCHK(c, hipMemcpyAsync(buf, c->idx_win[(w - 1) & 1].p + W, pre, hipMemcpyDeviceToDevice,
                               c->copy_stream));
    for (uint64_t off = ws; off < ws + wl; off += piece, ++k) {
      if (c->cancel.load()) return drain(c, pf, DSX_E_INTERRUPTED);
      uint8_t* hp = nullptr;
      uint64_t hn = 0;
      rc = pf.wait(k, &hp, &hn);
      if (rc) return drain(c, pf, rc);
      hipError_t e = hipMemcpyAsync(buf + pre + (off - ws), hp, hn, hipMemcpyHostToDevice,
                                    c->copy_stream);
      if (e == hipSuccess) e = hipEventRecord(c->idx_copy_ev[k % K], c->copy_stream);
      if (e == hipSuccess && k >= 1) e = hipEventSynchronize(c->idx_copy_ev[(k - 1) % K]);
      if (e != hipSuccess) return drain(c, pf, set_hip_err(c, e, "ids: H2D"));
      if (k >= 1) pf.release(k - 1);
      if (shares_done < shares.size() && off + hn >= shares[shares_done].landed) {
        // share m: its chunks' bytes have landed once this copy has
        const size_t m = shares_done++;
        const uint64_t a = m ? shares[m - 1].i1 : i_last, b = shares[m].i1;
        if (b > a) {
          hipStream_t ss = c->idx_side[m];
          e = hipStreamWaitEvent(ss, c->idx_copy_ev[k % K], 0);
          if (e != hipSuccess) return drain(c, pf, set_hip_err(c, e, "ids: wait"));
          DigestArgs dm{};
          dm.blob = w == 0 ? buf + pre : buf;
          dm.base_off = w == 0 ? 0 : ws - pre;
          dm.len = w == 0 ? shares[m].landed : pre + (shares[m].landed - ws);
          dm.ends = c->dg_ends.p + a;
          dm.first_start = a == 0 ? 0 : ends[a - 1] - start;
          dm.n = b - a;
          dm.ids = c->dg_ids.p + a * 32;
          dm.skip_above = shares[m].cut >= maxc ? 0 : shares[m].cut;
          rc = launch_digest(c, dm, b - a, algo, ss, c->idx_side_q.p + 32 * m, false,
                             (uint32_t)(c->ncu * 3 / 4), 1);
          if (rc) return drain(c, pf, rc);
        }
      }
    }
    // chunks ending in (ws, ws + wl] (window 0 also those ending at 0)
    uint64_t i1 = i0;
    while (i1 < n && ends[i1] - start <= ws + wl) ++i1;
    if (w + 1 == nwin) i1 = n;
    if (i1 > i0) {
      hipError_t e = hipSuccess;
      if (k >= 1) e = hipStreamWaitEvent(c->stream, c->idx_copy_ev[(k - 1) % K], 0);
      if (e != hipSuccess) return drain(c, pf, set_hip_err(c, e, "ids: wait"));
      DigestArgs da{};
      da.blob = w == 0 ? buf + pre : buf;
      da.base_off = w == 0 ? 0 : ws - pre;
      da.len = w == 0 ? wl : pre + wl;
      da.ends = c->dg_ends.p + i0;
      da.first_start = i0 == 0 ? 0 : ends[i0 - 1] - start;
      da.n = i1 - i0;
      da.ids = c->dg_ids.p + i0 * 32;
      if (tail_on && w + 1 == nwin) {
        da.skip_above = early_cut;
        if (!shares.empty()) {  // (one window: the chunks after the last share)
          const uint64_t a = shares.back().i1;
          da.ends = c->dg_ends.p + a;
          da.first_start = a == 0 ? 0 : ends[a - 1] - start;
          da.n = i1 - a;
          da.ids = c->dg_ids.p + a * 32;
          da.skip_above = end_cut;
        }
        if (da.n) rc = launch_digest(c, da, da.n, algo);
        if (rc) return drain(c, pf, rc);
#if DSX_DIAG
        t_read = t_join0 = ms();
#endif
        if (early_th.t.joinable()) early_th.t.join();
#if DSX_DIAG
        t_join1 = ms();
#endif
        if (early_rc) return drain(c, pf, early_rc);
        tail = std::move(early);
        tail_ids = std::move(early_ids);
        c->stats.host_tail_chunks = tail.size();
        hipError_t e = hipEventRecord(c->idx_win_ev[w & 1], c->stream);
        if (e != hipSuccess) return drain(c, pf, set_hip_err(c, e, "ids: record"));
        i0 = i1;
        continue;
      }
      rc = launch_digest(c, da, i1 - i0, algo);
      if (rc) return drain(c, pf, rc);
    } else if (k >= 1) {  // (the window's buffer is free once its copies landed)
      hipError_t e = hipStreamWaitEvent(c->stream, c->idx_copy_ev[(k - 1) % K], 0);
      if (e != hipSuccess) return drain(c, pf, set_hip_err(c, e, "ids: wait"));
    }
    hipError_t e = hipEventRecord(c->idx_win_ev[w & 1], c->stream);
    if (e != hipSuccess) return drain(c, pf, set_hip_err(c, e, "ids: record"));
    i0 = i1;
  }
  pf.stop();
  HIPCHK(c, hipStreamSynchronize(c->copy_stream));
  for (size_t m = 0; m < shares_done; ++m) HIPCHK(c, hipStreamSynchronize(c->idx_side[m]));
  HIPCHK(c, hipMemcpyAsync(out_ids, c->dg_ids.p, n * 32, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(c, hipStreamSynchronize(c->stream));
#if DSX_DIAG
  if (tlog) {
    uint64_t hb = 0;
    for (const auto& x : tail) hb += x.len;
    fprintf(stderr, "ids: %.1f MB windows %lu reads+H2D done %.2f ms, early hash joined %.2f ms "
            "(waited %.2f; %zu chunks %.1f MB on %d threads, cut %lu, %zu shares, end cut %lu), GPU done %.2f ms\n",
            L / 1e6, (unsigned long)nwin, t_read, t_join1, t_join1 - t_join0, tail.size(), hb / 1e6, eth,
            (unsigned long)early_cut, shares.size(), (unsigned long)end_cut, ms());
  }
#endif
  for (size_t j = 0; j < tail.size(); ++j)  // (the GPU skipped these)
    memcpy(out_ids + 32 * tail[j].idx, tail_ids.data() + 32 * j, 32);
  return DSX_OK;
}

}  // namespace

#if DSX_DIAG
// The plan a one-window dsx_index_* call of `len` bytes makes with the default
// host tail (-1, AVX-512) at `threads` feeder threads: the feeder's cut, the
// cut after the GPU's last share, and the shares {at, cut} (returns their
// count, at most cap); and the pieces it reads (off, size), for tests on the
// CPU (tests/test_host_logic.py).
extern "C" int dsx_diag_index_plan(uint64_t len, uint64_t max_chunk, int threads, uint64_t* fcut,
                                   uint64_t* fcut_end, uint64_t* at, uint64_t* cut, int cap) {
  *fcut = feed_cut_for(-1, threads);
  const std::vector<Mid> m = plan_shares(len, max_chunk, *fcut);
  *fcut_end = m.empty() ? *fcut : share_end_cut(*fcut);
  const int n = (int)std::min<size_t>(m.size(), (size_t)std::max(0, cap));
  for (int i = 0; i < n; ++i) {
    at[i] = m[i].at;
    cut[i] = m[i].cut;
  }
  return (int)m.size();
}
extern "C" uint64_t dsx_diag_index_pieces(uint64_t len, uint64_t max_chunk, uint64_t slot, uint64_t window,
                                          int feeds, uint64_t* off, uint64_t* size, uint64_t cap) {
  const IndexGeom g(len, max_chunk, slot, window, feeds != 0);
  const PieceMap pm(len, g.piece, g.fine_from, g.fine);
  for (uint64_t k = 0; k < pm.np && k < cap; ++k) {
    off[k] = pm.off(k);
    size[k] = pm.size(k);
  }
  return pm.np;
}
#endif

void index_release(dsx_ctx* c) {
  c->idx_dg_stream = nullptr;  // (idx_side[0])
  for (auto& s : c->idx_side)
    if (s) (void)hipStreamSynchronize(s), (void)hipStreamDestroy(s), s = nullptr;
  c->idx_side_q.release();
  for (auto& e : c->idx_stitch_ev)
    if (e) (void)hipEventDestroy(e), e = nullptr;
  for (auto& s : c->idx_slots) {
    if (s) (void)hipHostFree(s);
    s = nullptr;
  }
  c->idx_slot_bytes = 0;
  c->idx_win[0].release();
  c->idx_win[1].release();
  c->idx_snap.release();
  for (auto& e : c->idx_copy_ev)
    if (e) (void)hipEventDestroy(e), e = nullptr;
  for (auto& e : c->idx_win_ev)
    if (e) (void)hipEventDestroy(e), e = nullptr;
}

static bool bad_algo(int algo) { return algo != DSX_DIGEST_SHA512_256 && algo != DSX_DIGEST_SHA256; }

extern "C" int dsx_index_fd(dsx_ctx_t* c, int fd, uint64_t off, uint64_t len, const dsx_params_t* p,
                            int algo, uint64_t* out_ends, uint8_t* ids, uint64_t cap,
                            uint64_t* n_out) {
  DSX_FLUSH_BEHIND(c);
  if (!c || !p || !n_out || fd < 0 || (cap && (!out_ends || !ids)) || bad_algo(algo))
    return DSX_E_INVAL;
  if (len == UINT64_MAX) {
    // GetFileSize (ioctl_linux.go:63-84): lseek(SEEK_END) gives the size of
    // a regular file and of a block device alike
    const off_t end = lseek(fd, 0, SEEK_END);
    if (end < 0) return DSX_E_IO;
    len = (uint64_t)end > off ? (uint64_t)end - off : 0;
  }
  FdSrc s{fd, off};
  const int rc = run_index(c, p, algo, len, fill_fd, &s, out_ends, ids, cap, n_out);
  c->cancel.store(0);  // a dsx_cancel() issued before or during this call ends here
  return rc;
}

// The cut list alone from a file or host memory: the same pipeline without
// the digests.
extern "C" int dsx_cut_fd(dsx_ctx_t* c, int fd, uint64_t off, uint64_t len, const dsx_params_t* p,
                          uint64_t* out_ends, uint64_t cap, uint64_t* n_out) {
  DSX_FLUSH_BEHIND(c);
  if (!c || !p || !n_out || fd < 0 || (cap && !out_ends)) return DSX_E_INVAL;
  if (len == UINT64_MAX) {
    const off_t end = lseek(fd, 0, SEEK_END);
    if (end < 0) return DSX_E_IO;
    len = (uint64_t)end > off ? (uint64_t)end - off : 0;
  }
  FdSrc s{fd, off};
  const int rc = run_index(c, p, -1, len, fill_fd, &s, out_ends, nullptr, cap, n_out);
  c->cancel.store(0);
  return rc;
}

extern "C" int dsx_cut_host(dsx_ctx_t* c, const void* h_blob, uint64_t len, const dsx_params_t* p,
                            uint64_t* out_ends, uint64_t cap, uint64_t* n_out) {
  DSX_FLUSH_BEHIND(c);
  if (!c || !p || !n_out || (len && !h_blob) || (cap && !out_ends)) return DSX_E_INVAL;
  MemSrc s{(const uint8_t*)h_blob};
  const int rc = run_index(c, p, -1, len, fill_mem, &s, out_ends, nullptr, cap, n_out);
  c->cancel.store(0);
  return rc;
}

extern "C" int dsx_index_host(dsx_ctx_t* c, const void* h_blob, uint64_t len, const dsx_params_t* p,
                              int algo, uint64_t* out_ends, uint8_t* ids, uint64_t cap,
                              uint64_t* n_out) {
  DSX_FLUSH_BEHIND(c);
  if (!c || !p || !n_out || (len && !h_blob) || (cap && (!out_ends || !ids)) || bad_algo(algo))
    return DSX_E_INVAL;
  MemSrc s{(const uint8_t*)h_blob};
  const int rc = run_index(c, p, algo, len, fill_mem, &s, out_ends, ids, cap, n_out, s.p);
  c->cancel.store(0);
  return rc;
}

// IDs of a given chunk list read from a file / host memory (VerifyIndex,
// verifyindex.go:13-79; ChopFile's NewChunkWithID check, chop.go:76-80,
// chunk.go:60-73).
extern "C" int dsx_ids_fd(dsx_ctx_t* c, int fd, uint64_t off, uint64_t len, uint64_t start,
                          const uint64_t* ends, uint64_t n, int algo, uint8_t* ids) {
  DSX_FLUSH_BEHIND(c);
  if (!c || fd < 0 || (n && (!ends || !ids)) || bad_algo(algo)) return DSX_E_INVAL;
  if (len == UINT64_MAX) {
    const off_t end = lseek(fd, 0, SEEK_END);
    if (end < 0) return DSX_E_IO;
    len = (uint64_t)end > off ? (uint64_t)end - off : 0;
  }
  FdSrc s{fd, off};
  const int rc = run_ids(c, algo, len, fill_fd, &s, start, ends, n, ids);
  c->cancel.store(0);
  return rc;
}

extern "C" int dsx_ids_host(dsx_ctx_t* c, const void* h_blob, uint64_t len, uint64_t start,
                            const uint64_t* ends, uint64_t n, int algo, uint8_t* ids) {
  DSX_FLUSH_BEHIND(c);
  if (!c || (len && !h_blob) || (n && (!ends || !ids)) || bad_algo(algo)) return DSX_E_INVAL;
  MemSrc s{(const uint8_t*)h_blob};
  const int rc = run_ids(c, algo, len, fill_mem, &s, start, ends, n, ids, s.p);
  c->cancel.store(0);
  return rc;
}
