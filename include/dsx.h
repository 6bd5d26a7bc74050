/*
 * dsx.h -- C ABI of the MI355X-native content-defined chunker (libdsx.so).
 *
 * Drop-in boundary for desync's chunking hot path.  Each entry point names the
 * reference interface it replaces (paths relative to the desync repository):
 *
 *   dsx_params_init      <- NewChunker validation + constants, chunker.go:134-171
 *                           (discriminatorFromAvg chunker.go:13-15, modInverse32
 *                           chunker.go:20-28)
 *   dsx_cut_device       <- the cut list IndexFromFile assembles, make.go:22-163,
 *                           for a blob already resident in HBM
 *   dsx_cut_host         <- IndexFromFile over an in-memory blob (pinned H2D
 *                           pipeline inside the library)
 *   dsx_cut_fd           <- IndexFromFile(ctx, name, ...) on an open file,
 *                           make.go:49-116 (file read + H2D pipelined)
 *   dsx_stream_*         <- Chunker.Next / Advance over an io.Reader,
 *                           chunker.go:206-309 (stdin/pipe path, tar.go:140)
 *   dsx_cancel           <- ctx cancellation -> Interrupted{}, make.go:201-203,
 *                           errors.go:56-58
 *   dsx_shard_*          <- make.go's split-and-align across GPUs: each rank
 *                           chunks its range, then seams are aligned from a
 *                           small all-gathered seam record (syncWith,
 *                           make.go:277-327)
 *
 * Conventions (cgo-safe): plain pointers and sizes only; no pointer passed in
 * is retained after a call returns; every function returns 0 or a negative
 * DSX_E_* code; cut lists are chunk END offsets (the caibx table offsets,
 * index.go:106-113), strictly increasing, the last one equal to the length.
 * A context is not thread-safe (like a Chunker, one per goroutine/worker).
 */
#ifndef DSX_H
#define DSX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DSX_ABI_VERSION 5

/* ---- error codes (negative) ---------------------------------------------- */
enum {
    DSX_OK = 0,
    DSX_E_MIN_TOO_SMALL = -1,    /* "min chunk size too small, must be over 48"   chunker.go:135-137 */
    DSX_E_MIN_GT_MAX = -2,       /* "min chunk size must not be greater than max"  chunker.go:138-140 */
    DSX_E_MIN_GT_AVG = -3,       /* "min chunk size must not be greater than avg"  chunker.go:141-143 */
    DSX_E_AVG_GT_MAX = -4,       /* "avg chunk size must not be greater than max"  chunker.go:144-146 */
    DSX_E_AVG_RANGE = -5,        /* discriminatorFromAvg() <= 0 (Go: panic / implementation-defined) */
    DSX_E_INVAL = -6,            /* bad argument (NULL pointer, bad flags) */
    DSX_E_CAPACITY = -7,         /* output capacity too small; *n_out holds the required count */
    DSX_E_HIP = -8,              /* HIP runtime error (see dsx_last_error) */
    DSX_E_NOMEM = -9,            /* device or pinned allocation failed */
    DSX_E_INTERRUPTED = -10,     /* dsx_cancel() was called: Interrupted{} errors.go:56-58 */
    DSX_E_IO = -11,              /* read() on the file descriptor failed */
    DSX_E_STATE = -12,           /* call not valid in the current stream state */
    DSX_E_INTERNAL = -13,        /* internal consistency check failed */
    DSX_E_RESYNC = -14,          /* dsx_shard_resolve: exchange the seam records again */
    DSX_E_PEER = -15             /* dsx_shard_resolve: another rank's record carries DSX_SEAM_ERROR */
};

/* ---- chunker parameters ----------------------------------------------------
 * Mirrors the Chunker fields of chunker.go:108-131.  Filled by
 * dsx_params_init(); treat as opaque besides min/avg/max/discriminator. */
typedef struct dsx_params {
    uint64_t min, avg, max;
    uint32_t discriminator; /* hDiscriminator */
    uint32_t inverse_odd;   /* hInverseOdd */
    uint32_t qmax;          /* hQMax */
    uint32_t qbias;         /* hQBias */
    int32_t rot;            /* k = trailing zeros of the discriminator (Go stores -k) */
    uint32_t reserved;
} dsx_params_t;

/* NewChunker(r, min, avg, max) validation and constant derivation.
 * Checks run in the order of chunker.go:135-146 and return the matching
 * DSX_E_* code; dsx_strerror() returns the reference's exact message. */
int dsx_params_init(uint64_t min, uint64_t avg, uint64_t max, dsx_params_t *out);
const char *dsx_strerror(int code);
int dsx_abi_version(void);

/* ---- context ---------------------------------------------------------------- */
typedef struct dsx_ctx dsx_ctx_t;

/* Owns HIP streams, device scratch and pinned staging on `device`. */
int dsx_ctx_create(int device, dsx_ctx_t **out);
int dsx_ctx_destroy(dsx_ctx_t *ctx);
/* Human-readable detail for the last DSX_E_HIP / DSX_E_INTERNAL on ctx
 * (ctx == NULL: the reason the last dsx_ctx_create failed). */
const char *dsx_last_error(dsx_ctx_t *ctx);
/* Request cancellation of the running/next call; it returns DSX_E_INTERRUPTED. */
int dsx_cancel(dsx_ctx_t *ctx);
/* Progress of the running (or last) dsx_index_* / dsx_cut_fd / dsx_cut_host
 * call: *bytes = the end of the last confirmed chunk, relative to the call's
 * `off` -- pb.Set(chunk.Start + chunk.Size) per assembled chunk in
 * IndexFromFile (make.go:134-140).  Monotone within a call, the file length
 * once it succeeded.  Like dsx_cancel, safe to call from another thread while
 * the call runs (it reads pinned memory the device publishes into after each
 * 32 MiB piece's stitch, 32 values per GiB; it never touches the context's
 * streams). */
int dsx_progress(dsx_ctx_t *ctx, uint64_t *bytes);

/* ---- one-shot cut lists ------------------------------------------------------ */
#define DSX_OUT_HOST 0u   /* out_ends is host memory */
#define DSX_OUT_DEVICE 1u /* out_ends is device memory on the ctx's device */
#define DSX_NO_SYNC 2u    /* (device output only) enqueue on the ctx stream and return;
                             up to 8 such calls may be queued (they run in order);
                             dsx_result() waits for the OLDEST and returns its count */
#define DSX_TIMED 16u     /* with DSX_NO_SYNC: record the call's scan/stitch events
                             (dsx_get_stats after its dsx_result reports them); untimed
                             queued calls record none (an event costs ~6 us of stream time) */

/* Device-resident blob (HBM) -> cut list.  d_blob must stay valid until the
 * call (with DSX_NO_SYNC: its dsx_result()) returns -- a queued call that
 * needs the general path (dense candidates, a stitch repair) is re-run from
 * the blob inside dsx_result().  If cap is too small the call returns
 * DSX_E_CAPACITY and *n_out holds the required count (an upper bound of
 * len/min + 2 always suffices).  A queued call's stitch publishes its state
 * into pinned host memory and dsx_result() polls it (no event per call).
 * (The diagnostic build libdsx_diag.so also has DSX_FUSE=1: the stitch of a
 * queued one-piece call as tasks inside the next queued calls' scans; the
 * product library does not read it, INTEGRATION.md "Environment".) */
int dsx_cut_device(dsx_ctx_t *ctx, const void *d_blob, uint64_t len, const dsx_params_t *p,
                   uint64_t *out_ends, uint64_t cap, uint64_t *n_out, uint32_t flags);
int dsx_sync(dsx_ctx_t *ctx);
/* Completes the oldest queued DSX_NO_SYNC dsx_cut_device(): waits for it, then
 * returns its status and cut count (its device cut list is valid once this
 * returns DSX_OK).  DSX_E_STATE if no call is queued. */
int dsx_result(dsx_ctx_t *ctx, uint64_t *n_out);

/* Host-memory blob -> cut list (host).  Pipelined pinned H2D inside. */
int dsx_cut_host(dsx_ctx_t *ctx, const void *h_blob, uint64_t len, const dsx_params_t *p,
                 uint64_t *out_ends, uint64_t cap, uint64_t *n_out);

/* File descriptor range [off, off+len) -> cut list (host).  len == UINT64_MAX
 * means "until EOF".  The fd's file offset is not used or changed (pread). */
int dsx_cut_fd(dsx_ctx_t *ctx, int fd, uint64_t off, uint64_t len, const dsx_params_t *p,
               uint64_t *out_ends, uint64_t cap, uint64_t *n_out);

/* ---- streaming (Chunker.Next / Advance over an io.Reader) -------------------
 * One stream per context (a Chunker owns its context, as each Go Chunker owns
 * its buffer and hash state, chunker.go:108-131).
 * begin:  starts a stream at position 0 with params p (NewChunker).  Returns
 *         DSX_E_STATE while another stream on ctx is unfinished.
 * end:    drops the stream (the context can begin a new one).
 * buffer: room for `want` bytes at the tail of the library's pinned host
 *         buffer; *ptr is where the caller writes them (e.g. the reader
 *         reads straight into it).  Valid until the next call on ctx.
 * commit: the caller wrote n bytes at *ptr.  flags: DSX_STREAM_EOF marks the
 *         end of input; DSX_STREAM_SYNC means no more input is coming for
 *         now (a failed reader): everything held is scanned and collected.
 *         Full 8 MiB batches (128 MiB with chunk IDs) are sent to the GPU
 *         without waiting (H2D + scan + stitch, up to 3 batches in flight).
 * push:   buffer + memcpy + commit (eof != 0: DSX_STREAM_EOF).
 * pop:    start and size of the next confirmed chunk.  Returns 1 if a chunk
 *         was produced, 0 if more input is needed first (or the stream
 *         ended: then dsx_stream_done() is 1), or a negative error.  Blocks
 *         on the GPU only when its result is needed and no input can be
 *         taken first.
 * chunk_data: the bytes of the chunk returned by the last pop or flush (host
 *         memory, valid until the next call on ctx -- Next()'s aliasing
 *         rule, chunker.go:202-205).
 * flush:  Next()'s read-error path (chunker.go:207-211, split(n, err)): all
 *         held bytes after the consumer position as one chunk; chunking then
 *         starts over behind them.
 * advance: Chunker.Advance(n) (chunker.go:292-309): drop n bytes at the
 *         current position (held bytes first, then future input), and
 *         continue as if the stream started there.
 * A chunk is confirmed once the bytes up to its start + max are scanned, as
 * Next() needs len(buf) >= max (chunker.go:207, 221). */
#define DSX_STREAM_EOF 1
#define DSX_STREAM_SYNC 2
int dsx_stream_begin(dsx_ctx_t *ctx, const dsx_params_t *p);
int dsx_stream_end(dsx_ctx_t *ctx);
int dsx_stream_buffer(dsx_ctx_t *ctx, uint64_t want, uint8_t **ptr);
int dsx_stream_commit(dsx_ctx_t *ctx, uint64_t n, int flags);
int dsx_stream_push(dsx_ctx_t *ctx, const void *bytes, uint64_t len, int eof);
int dsx_stream_pop(dsx_ctx_t *ctx, uint64_t *start, uint64_t *size);
int dsx_stream_flush(dsx_ctx_t *ctx, uint64_t *start, uint64_t *size);
int dsx_stream_advance(dsx_ctx_t *ctx, uint64_t n);
int dsx_stream_done(dsx_ctx_t *ctx);
const uint8_t *dsx_stream_chunk_data(dsx_ctx_t *ctx);
/* Chunk IDs next to the cuts (ChunkStream, index.go:138-234: Next() then
 * Digest.Sum of every chunk, index.go:165-169): with algo = DSX_DIGEST_* each
 * batch's chunks are hashed on the GPU right after its stitch, on a side
 * stream that overlaps the next batch.  Only before the first bytes of a
 * chain are scanned (else DSX_E_STATE).  dsx_stream_chunk_id returns the
 * 32-byte ID of the chunk the last pop returned (valid until the next call),
 * or NULL if it has none. */
int dsx_stream_ids(dsx_ctx_t *ctx, int algo);
/* Up to cap confirmed chunks at once (a binding that hands out Next() results
 * without a call per chunk): the first starts at *start, chunk i ends at
 * ends[i]; with ids non-NULL (dsx_stream_ids on) their 32-byte IDs.  Returns
 * 1 with *n >= 1, or what dsx_stream_pop returns (0: input needed / ended).
 * The chunks' bytes are contiguous from dsx_stream_chunk_data(). */
int dsx_stream_pop_many(dsx_ctx_t *ctx, uint64_t *ends, uint8_t *ids, uint64_t cap,
                        uint64_t *start, uint64_t *n);
/* Gives back the chunks of the last pop_many that end after pos (a binding
 * that consumed only some of them before an Advance or a read error): the
 * consumer position returns to pos (a chunk end of that group) and the
 * chunks after it are queued again. */
int dsx_stream_unpop(dsx_ctx_t *ctx, uint64_t pos);
/* The held stream bytes [*base_pos, *base_pos + *len) at *base (host memory,
 * valid until the next buffer/commit/push/advance/flush/end on ctx). */
int dsx_stream_window(dsx_ctx_t *ctx, const uint8_t **base, uint64_t *base_pos, uint64_t *len);
const uint8_t *dsx_stream_chunk_id(dsx_ctx_t *ctx);
/* The clone of a run of chunks out of the held bytes (index.go:196-200,
 * slices.Clone of each chunk: ChunkStream clones a run at once): a host
 * memcpy of n bytes split over up to `threads` threads of a persistent pool
 * (<= 1: the calling thread alone).  dst and src must not overlap.  No
 * context; no GPU. */
int dsx_host_copy(void *dst, const void *src, uint64_t n, int threads);
/* Digest.Sum (digest.go:22, SHA-512/256) of n host messages ptrs[i] of lens[i]
 * bytes into ids[32 i], on up to `threads` host threads: 8 messages per set of
 * AVX-512 registers, longest first (the scalar form without AVX-512, or with
 * DSX_HOST_SHA_SCALAR in flags).  The same code hashes the long chunks of an
 * index call's last window on the host (DSX_INDEX_HOST_TAIL).
 * No context; no GPU. */
#define DSX_HOST_SHA_SCALAR 1
int dsx_host_sha512_256(const uint8_t *const *ptrs, const uint64_t *lens, uint64_t n, uint8_t *ids,
                        int threads, int flags);

/* ---- multi-GPU shards (split-and-align across ranks) ------------------------
 * A blob of total length `total` is range-sharded; rank r holds
 * [shard_start, shard_start+shard_len) in device memory at d_shard, preceded
 * by `halo` readable bytes (halo >= 48, or halo == 0 only when shard_start==0).
 *
 * dsx_shard_local: chunks the shard speculatively from a virtual cut at
 *   shard_start (make.go's worker at span*i, make.go:94-116) and fills a
 *   fixed-size seam record (dsx_seam_t): the candidates and speculative cuts
 *   of the shard's first 32*max bytes and the chain's exit cut.  The record is
 *   built on the device; `seam` is device memory with DSX_SEAM_DEVICE (then it
 *   can be all-gathered by RCCL in place), host memory otherwise.
 * dsx_shard_resolve: given all ranks' seam records (rank order, host or
 *   device memory per DSX_SEAM_DEVICE), walks the true chain across the seams
 *   (syncWith, make.go:277-298) and writes this rank's final cut list: the
 *   cuts c with shard_start < c <= shard_start+shard_len (host memory, or
 *   device memory with DSX_OUT_DEVICE).
 *   Returns DSX_E_RESYNC when a seam did not converge inside its window (a
 *   zero run across a shard boundary, README.md:114-119): the rank owning
 *   that seam has then re-walked its shard from the true entry cut and
 *   rewritten its record `my_seam` (flag DSX_SEAM_REWALKED); every rank
 *   all-gathers the records again and calls dsx_shard_resolve again (at most
 *   nranks rounds).  The re-walk re-runs only the stitch over the shard's
 *   kept candidate lists (O(candidates), no byte is scanned again).  If the
 *   re-walk itself fails, resolve returns that error and marks `my_seam`
 *   DSX_SEAM_ERROR: the caller all-gathers it once more so that every other
 *   rank's resolve returns DSX_E_PEER instead of waiting for a record that
 *   never comes.  d_shard passed to dsx_shard_local must stay valid until
 *   dsx_shard_resolve returns DSX_OK.
 * Seam records are plain bytes. */
#define DSX_SEAM_MAX_CANDS 1024
#define DSX_SEAM_MAX_CUTS 1024
#define DSX_SEAM_DEVICE 8u      /* flag: seam records are device memory */
#define DSX_SEAM_LAST 1u        /* seam flags: the shard ends the blob */
#define DSX_SEAM_REWALKED 2u    /* seam flags: chain re-walked from the true entry `entry` */
#define DSX_SEAM_ERROR 4u       /* seam flags: the owner failed; every rank's resolve returns DSX_E_PEER */
#define DSX_SEAM_REDO 16u       /* seam flags: an asynchronous dsx_shard_local hit a stitch error; the
                                   owner redoes its shard synchronously (dsx_shard_collect) */
typedef struct dsx_seam {
    uint64_t shard_start, shard_len, total;
    uint64_t first_cand_beyond;   /* first candidate > window end, or UINT64_MAX */
    uint64_t exit_cut;            /* the shard chain's last cut <= shard end */
    uint64_t window_end;          /* candidates/cuts below cover (shard_start, window_end] */
    uint64_t entry;               /* DSX_SEAM_REWALKED: the entry cut the chain started from */
    uint32_t ncands, ncuts, flags, pad;
    uint64_t cands[DSX_SEAM_MAX_CANDS]; /* candidate positions in (shard_start, window_end] */
    uint64_t cuts[DSX_SEAM_MAX_CUTS];   /* spec chain cuts in (shard_start, window_end] */
} dsx_seam_t;

int dsx_shard_local(dsx_ctx_t *ctx, const void *d_shard, uint64_t halo, uint64_t shard_start,
                    uint64_t shard_len, uint64_t total, const dsx_params_t *p, dsx_seam_t *seam,
                    uint32_t flags);
int dsx_shard_resolve(dsx_ctx_t *ctx, const dsx_seam_t *all, int nranks, int rank,
                      dsx_seam_t *my_seam, uint64_t *out_ends, uint64_t cap, uint64_t *n_out,
                      uint32_t flags);

/* Asynchronous step (device records, device cut list): at most one host wait
 * per converged step.
 *   dsx_shard_local(..., DSX_SEAM_DEVICE | DSX_NO_SYNC) enqueues the scan,
 *     stitch and record on the ctx stream and returns (a stitch error shows up
 *     as DSX_SEAM_REDO in the record instead of a return code);
 *   the caller all-gathers the records on the ctx stream (dsx_ctx_stream);
 *   dsx_shard_resolve_async enqueues the resolve: this rank's final cuts go to
 *     out_ends (device, cap entries) and the round's outcome to the device
 *     int32 *d_code: 0 done, 1 exchange again, 2 failed (a peer's
 *     DSX_SEAM_ERROR, or cap too small);
 *   the caller all-reduces the code words with MAX on the ctx stream (the
 *     ranks' agreement, so a local failure reaches every rank in this round);
 *   dsx_shard_collect waits once, copies the agreed word (d_agreed, device,
 *     or NULL when the caller agrees on the host) to *agreed and returns what
 *     dsx_shard_resolve would: DSX_OK with *n_out, DSX_E_RESYNC (the owner of
 *     a non-converged or DSX_SEAM_REDO seam has re-walked / redone its shard
 *     and rewritten my_seam, device memory), DSX_E_PEER, or an error (then
 *     my_seam is marked DSX_SEAM_ERROR when the failure happened after the
 *     agreement: exchange once more so the peers learn of it).  With an
 *     agreed code of 2 it returns this rank's own failure (DSX_E_CAPACITY) or
 *     DSX_E_PEER. */
int dsx_shard_resolve_async(dsx_ctx_t *ctx, const dsx_seam_t *all, int nranks, int rank,
                            uint64_t *out_ends, uint64_t cap, int32_t *d_code);
int dsx_shard_collect(dsx_ctx_t *ctx, dsx_seam_t *my_seam, const int32_t *d_agreed,
                      int32_t *agreed, uint64_t *n_out);
/* The ctx's HIP stream (hipStream_t), for ordering a caller's collectives
 * with the library's kernels without host waits.  It is created at the
 * highest stream priority, so it takes an HSA queue of that priority's pool
 * (a caller's streams and RCCL's, at the default priority, do not share it;
 * DESIGN.md 5.1). */
int dsx_ctx_stream(dsx_ctx_t *ctx, void **stream);

/* Synchronous copy of n bytes between any host / device pointers (hipMemcpy
 * with the direction inferred): a binding without its own GPU runtime uses it
 * to move the seam-tail bytes of a shard (the chunk IDs across seams). */
int dsx_copy(dsx_ctx_t *ctx, void *dst, const void *src, uint64_t n);

/* ---- diagnostics ------------------------------------------------------------- */
/* Evaluates the GPU boundary predicate (mode 0: multiply-inverse form of
 * chunker.go:265, mode 1: float-reciprocal form, mode 2: multiply-inverse
 * prefilter + exact re-check (d not a power of two), -1: the one the scan uses)
 * for h in [h0, h0+n) (mod 2^32) against h % d == d-1 and counts mismatches
 * (the check of chunker_test.go:190-213, on the device). */
int dsx_selftest_boundary(dsx_ctx_t *ctx, const dsx_params_t *p, int mode, uint64_t h0,
                          uint64_t n, uint64_t *mismatches);

/* Timeline of the last piece when the context was created with
 * DSX_SCAN_TRACE=1 (libdsx_diag.so only; the product library records none and
 * returns zero records) (s_memrealtime ticks, 100 MHz): *n_scan wave-slot records
 * {start, end, regions} of the line-aligned scan, then *n_walk stitch-walk
 * workgroup records {entry, counts scanned, candidates staged, speculative
 * walks done, staged walks done, s_memtime at staged, s_memtime at
 * speculative walks done, first walk: seek done, first step done, chain
 * done}.  Copies min(cap, 3*n_scan + 10*n_walk) words to out. */
int dsx_debug_trace(dsx_ctx_t *ctx, uint64_t *out, uint64_t cap, uint64_t *n_scan,
                    uint64_t *n_walk);

/* ---- measurement: in-kernel stamps of the scan launches ----------------------
 * (bench.py's roofline; replaces no reference interface.)  Between
 * dsx_stamps_begin and dsx_stamps_end the next max_launches line-scan launches
 * of ctx record, from inside the kernel, the s_memrealtime ticks (100 MHz) of
 * their first wave's first instruction and last wave's last instruction, and
 * the shader-clock cycles (s_memtime) and realtime ticks each wave spent, summed
 * over the waves: duration = (t_last - t_first) / 100 MHz, mean shader clock =
 * wave_cycles / wave_ticks * 100 MHz.  No event or extra kernel runs between
 * the stamped launches.  begin waits for the ctx's queued work; end waits for
 * the stamped launches and copies min(cap, *n) records in launch order. */
typedef struct dsx_scan_stamp {
    uint64_t seq;          /* piece sequence number of the launch */
    uint64_t bytes;        /* bytes the launch scanned (one piece: <= 8 GiB) */
    uint64_t t_first, t_last;
    uint64_t wave_cycles, wave_ticks;
    uint64_t waves;        /* waves of the launch's grid */
    uint64_t reserved;
} dsx_scan_stamp_t;
int dsx_stamps_begin(dsx_ctx_t *ctx, uint64_t max_launches);
int dsx_stamps_end(dsx_ctx_t *ctx, dsx_scan_stamp_t *out, uint64_t cap, uint64_t *n);

/* ---- synthetic inputs (bench / tests; generated on device) ------------------ */
/* bytes [offset, offset+len) of the seeded uniform stream (splitmix64 of the
 * 8-byte word index), written to d_dst. */
int dsx_gen_uniform(dsx_ctx_t *ctx, void *d_dst, uint64_t offset, uint64_t len, uint64_t seed);
/* dedup-realistic stream: 1 MiB blocks; block i is, with probability p_repeat,
 * a copy of a uniformly chosen earlier block j < i, else fresh uniform bytes. */
int dsx_gen_dedup(dsx_ctx_t *ctx, void *d_dst, uint64_t offset, uint64_t len, uint64_t seed,
                  double p_repeat);

/* ---- chunk IDs on the GPU (Digest.Sum per chunk: digest.go:11-29, make.go:223,
 * nullchunk.go:17-23) ------------------------------------------------------- */
#define DSX_DIGEST_SHA512_256 0 /* desync's default Digest (digest.go:22) */
#define DSX_DIGEST_SHA256 1     /* the --digest sha256 alternative (digest.go:28) */
#define DSX_ENDS_DEVICE 4u      /* flag: ends[] is device memory (default: host) */
/* 32-byte IDs of the chunks [start, ends[0]), [ends[0], ends[1]), ... of the
 * device-resident blob d_blob[0..len): ids receives n*32 bytes, host memory
 * by default or device memory with DSX_OUT_DEVICE.  Synchronous. */
int dsx_chunk_ids(dsx_ctx_t *ctx, const void *d_blob, uint64_t len, uint64_t start,
                  const uint64_t *ends, uint64_t n, void *ids, uint32_t flags, int algo);

/* ---- IndexFromFile on the GPU: cut list + chunk IDs ----------------------------
 * The whole of IndexFromFile's data path (make.go:22-163: chunking, then
 * Digest.Sum of every chunk, make.go:223) for a file descriptor range
 * [off, off+len) or a host-memory blob.  len == UINT64_MAX (fd only) means
 * "to the end", for regular files and block devices alike (GetFileSize,
 * ioctl_linux.go:63-84).  Reader threads pread into pinned staging, the bytes
 * are copied to HBM while the next ones are read, chunked there, and hashed
 * there (algo: DSX_DIGEST_*); files larger than the HBM window
 * (DSX_INDEX_WINDOW, 1 GiB) stream through two alternating windows.  The fd's
 * file offset is not used or changed.
 * out_ends: chunk END offsets relative to off (cap entries); ids: 32 bytes per
 * chunk (cap * 32 bytes); both host memory.  DSX_E_CAPACITY sets *n_out to the
 * required count (len/min + 2 always suffices).  Synchronous; dsx_cancel()
 * interrupts it between 32 MiB pieces (DSX_E_INTERRUPTED).
 * Partial results (IndexFromFile returns the chunks assembled so far with
 * chunkErr or Interrupted{}, make.go:133-162, :201-203): on DSX_E_INTERRUPTED
 * and DSX_E_IO, out_ends / ids hold the confirmed prefix of the chain (every
 * chunk of the pieces stitched before the stop, with its ID) and *n_out its
 * length (0 if no piece was done).  dsx_cut_fd / dsx_cut_host do the same
 * with the cut list alone. */
int dsx_index_fd(dsx_ctx_t *ctx, int fd, uint64_t off, uint64_t len, const dsx_params_t *p,
                 int algo, uint64_t *out_ends, uint8_t *ids, uint64_t cap, uint64_t *n_out);
int dsx_index_host(dsx_ctx_t *ctx, const void *h_blob, uint64_t len, const dsx_params_t *p,
                   int algo, uint64_t *out_ends, uint8_t *ids, uint64_t cap, uint64_t *n_out);

/* ---- chunk IDs of a given chunk list from a file or host memory --------------
 * Digest.Sum of the chunks [start, ends[0]), [ends[0], ends[1]), ... of the
 * bytes [off, off+len) of fd (len == UINT64_MAX: to the end) or of
 * h_blob[0..len): the re-hash of VerifyIndex (verifyindex.go:13-79,
 * fileseed.go:183-196) and of ChopFile's NewChunkWithID check (chop.go:66-80,
 * chunk.go:37-73).  Offsets are relative to off; ends must be non-decreasing
 * with start <= ends[0] and ends[n-1] <= len (else DSX_E_INVAL).  The same
 * pipeline as dsx_index_fd without the scan: only [start, ends[n-1]) is read,
 * through pinned staging into two alternating HBM windows whose overlap is the
 * longest chunk.  ids: n * 32 bytes, host memory.  A file shorter than
 * ends[n-1] gives DSX_E_IO.  Synchronous; dsx_cancel() interrupts it. */
int dsx_ids_fd(dsx_ctx_t *ctx, int fd, uint64_t off, uint64_t len, uint64_t start,
               const uint64_t *ends, uint64_t n, int algo, uint8_t *ids);
int dsx_ids_host(dsx_ctx_t *ctx, const void *h_blob, uint64_t len, uint64_t start,
                 const uint64_t *ends, uint64_t n, int algo, uint8_t *ids);

/* ---- statistics (ChunkingStats, make.go:329-341 + scan/stitch timings) ------ */
typedef struct dsx_stats {
    uint64_t chunks;            /* ChunksAccepted */
    uint64_t candidates;        /* boundary candidates found by the scan */
    uint64_t pieces;            /* scan pieces processed */
    uint64_t repaired_segments; /* segments that needed the sequential repair */
    uint64_t dense_fallbacks;   /* pieces processed on the dense-candidate path */
    float scan_ms, stitch_ms;   /* device time of the last synchronous call (HIP events; 0 after dsx_result) */
    uint64_t chunks_discarded;  /* cuts the stitch computed, then replaced by a repair: ChunksProduced
                                   = chunks + chunks_discarded (make.go:329-341 counts the workers'
                                   discarded overlap chunks too) */
    uint64_t device_bytes;      /* HBM the context holds now (its pipeline buffers; filled in by
                                   dsx_get_stats; the caller's blob and cut list are not counted) */
    uint64_t host_tail_chunks;  /* dsx_index_*: chunks of the last window hashed on the host
                                   (DSX_INDEX_HOST_TAIL) while the GPU hashed the others */
} dsx_stats_t;
int dsx_get_stats(dsx_ctx_t *ctx, dsx_stats_t *out);

#ifdef __cplusplus
}
#endif
#endif /* DSX_H */
