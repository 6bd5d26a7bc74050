/*
 * dsx_oracle.c -- CPU restatement of desync's content-defined chunker.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the parity oracle for the MI355X
 * HIP path in desync_amd/csrc and the CPU baseline timed by bench.py's
 * `cpu_baseline` leg.  Nothing in the product path (libdsx.so and the desync_amd Python package)
 * links, loads or calls it.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may use it.
 *
 * Parity is pinned (see tests/test_oracle_golden.py) against the reference's
 * own known-answer data: chunker_test.go:20-67 (TestChunkerLargeFile triples),
 * testdata/chunker.index (index_test.go:55-112), testdata/blob1.caibx,
 * cmd/desync/testdata/blob2.caibx, cmd/desync/testdata/tree.caidx,
 * chunker_test.go:69-131 (empty/small/zero/bounds) and
 * chunker_test.go:190-213 (boundary-test ranges).
 *
 * Two formulations are restated and cross-checked against each other:
 *   (1) dsxo_chunk_stream(): the literal sequential loop of Chunker.Next()
 *       (chunker.go:206-277): per chunk, hash init over [min-48,min), then the
 *       2-bytes-per-iteration roll + multiply-inverse boundary test.
 *   (2) dsxo_candidates() + dsxo_chain(): the position-only candidate
 *       predicate (SURVEY.md sec.0 finding 1) followed by the chain rule
 *       (finding 2).  This is the formulation the GPU implements.
 * plus dsxo_chunk_parallel(): make.go-style split-and-align over pthreads
 * (make.go:22-163), used only as the multi-core CPU baseline.
 *
 * Build: oracle/Makefile (gcc -O3 -ffp-contract=off).  -ffp-contract=off is
 * REQUIRED: discriminatorFromAvg (chunker.go:13-15) must not be fused.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/dsx_buzhash_table.h"

static inline uint32_t rotl32(uint32_t x, unsigned r) {
    r &= 31u;
    return r ? (x << r) | (x >> (32u - r)) : x;
}

static uint32_t T_ROT[256]; /* chunker.go:97-105: rotl32(T, 48) */
static pthread_once_t t_rot_once = PTHREAD_ONCE_INIT;
static void init_trot(void) {
    for (int i = 0; i < 256; i++) T_ROT[i] = rotl32(DSX_BUZHASH_T[i], 48u);
}

/* ---- chunker.go:13-15 discriminatorFromAvg ---------------------------- */
/* float64 arithmetic, no FMA contraction (Makefile: -ffp-contract=off).
 * Go's uint32(float64) on amd64 converts through int64 (CVTTSD2SQ) and keeps
 * the low 32 bits; out-of-int64-range values produce 0x8000000000000000.  We
 * mirror that so the (out-of-spec, avg > ~9.3M) region is at least
 * deterministic; the product API rejects it (DSX_E_AVG_RANGE). */
uint32_t dsxo_discriminator(uint64_t avg) {
    volatile double a = (double)avg;
    volatile double den = -1.42888852e-7 * a;
    den = den + 1.33237515;
    volatile double q = a / den;
    if (!(q > -9.2e18 && q < 9.2e18)) return 0u;
    return (uint32_t)(uint64_t)(int64_t)q;
}

/* ---- chunker.go:20-28 modInverse32 -------------------------------------- */
uint32_t dsxo_mod_inverse32(uint32_t d) {
    uint32_t x = d;
    x *= 2u - d * x;
    x *= 2u - d * x;
    x *= 2u - d * x;
    x *= 2u - d * x;
    x *= 2u - d * x;
    return x;
}

typedef struct {
    uint64_t min, avg, max;
    uint32_t d, inv, qmax, qbias;
    int rot; /* right rotation k (Go stores -k and rotates left by it) */
} dsxo_params_t;

/* chunker.go:134-171 NewChunker.  Returns 0 on success, or the 1-based index
 * of the failing check in the order of chunker.go:135-146:
 *   1 min < 48, 2 min > max, 3 min > avg, 4 avg > max, 5 d == 0 (Go panics). */
int dsxo_params(uint64_t min, uint64_t avg, uint64_t max, dsxo_params_t *p) {
    if (min < DSX_WINDOW) return 1;
    if (min > max) return 2;
    if (min > avg) return 3;
    if (avg > max) return 4;
    uint32_t d = dsxo_discriminator(avg);
    if (d == 0) return 5;
    unsigned k = (unsigned)__builtin_ctz(d);
    uint32_t odd = d >> k;
    p->min = min; p->avg = avg; p->max = max;
    p->d = d;
    p->inv = dsxo_mod_inverse32(odd);
    p->qbias = odd > 1u ? 1u : 0u;
    p->qmax = 0xFFFFFFFFu / d - p->qbias;
    p->rot = (int)k;
    return 0;
}

/* chunker.go:265/268: rotl32((h+1)*inv, -k) - qBias <= qMax  <=> h % d == d-1 */
static inline int is_boundary(const dsxo_params_t *p, uint32_t h) {
    uint32_t v = (h + 1u) * p->inv;
    v = rotl32(v, (unsigned)(32 - p->rot));
    return v - p->qbias <= p->qmax;
}

int dsxo_is_boundary(const dsxo_params_t *p, uint32_t h) { return is_boundary(p, h); }

/* ---- (1) literal Chunker.Next() loop, chunker.go:206-277 --------------------
 * Emits chunk END offsets (the caibx table offsets, index.go:108-113).
 * An in-memory blob has len(c.buf) >= max unless fewer bytes remain
 * (fillBuffer reads 10*max, chunker.go:175-200), so m = min(rem, max). */
uint64_t dsxo_chunk_stream(const uint8_t *buf, uint64_t len, const dsxo_params_t *p,
                           uint64_t *ends, uint64_t cap) {
    pthread_once(&t_rot_once, init_trot);
    uint64_t pos = 0, k = 0;
    const uint64_t min = p->min, max = p->max;
    while (pos < len) {
        uint64_t rem = len - pos, end;
        if (rem <= min) {
            end = len; /* chunker.go:215-217 */
        } else {
            uint64_t m = rem < max ? rem : max; /* chunker.go:221 */
            const uint8_t *c = buf + pos;
            uint32_t h = 0;
            for (unsigned i = 0; i < DSX_WINDOW; i++) /* chunker.go:225-228 */
                h ^= rotl32(DSX_BUZHASH_T[c[min - DSX_WINDOW + i]], DSX_WINDOW - i - 1);
            const uint8_t *in = c + min, *out = c + min - DSX_WINDOW;
            uint64_t n = m - min;
            end = pos + m; /* chunker.go:276 */
            for (uint64_t i = 0; i + 1 < n; i += 2) { /* chunker.go:259-271 */
                uint32_t a0 = T_ROT[out[i]] ^ DSX_BUZHASH_T[in[i]];
                uint32_t a1 = T_ROT[out[i + 1]] ^ DSX_BUZHASH_T[in[i + 1]];
                uint32_t h1 = rotl32(h, 1) ^ a0;
                h = rotl32(h, 2) ^ rotl32(a0, 1) ^ a1;
                if (is_boundary(p, h1)) { end = pos + min + i + 1; break; }
                if (is_boundary(p, h)) { end = pos + min + i + 2; break; }
            }
        }
        if (k < cap) ends[k] = end;
        k++;
        pos = end;
    }
    return k;
}

/* ---- (2a) candidate predicate ---------------------------------------------
 * cand(p) <=> H(p) % d == d-1, H(p) = XOR_{j<48} rotl32(T[b[p-48+j]], 47-j),
 * defined for p in [48, len].  Writes sorted candidate positions. */
uint64_t dsxo_candidates(const uint8_t *buf, uint64_t len, const dsxo_params_t *p,
                         uint64_t *cands, uint64_t cap) {
    pthread_once(&t_rot_once, init_trot);
    if (len < DSX_WINDOW) return 0;
    uint32_t h = 0;
    for (unsigned i = 0; i < DSX_WINDOW; i++)
        h ^= rotl32(DSX_BUZHASH_T[buf[i]], DSX_WINDOW - i - 1);
    uint64_t k = 0;
    if (is_boundary(p, h)) { if (k < cap) cands[k] = DSX_WINDOW; k++; }
    for (uint64_t i = DSX_WINDOW; i < len; i++) {
        h = rotl32(h, 1) ^ T_ROT[buf[i - DSX_WINDOW]] ^ DSX_BUZHASH_T[buf[i]];
        if (is_boundary(p, h)) { if (k < cap) cands[k] = i + 1; k++; }
    }
    return k;
}

/* ---- (2b) chain rule over sorted candidates --------------------------------
 * From cut s: if len-s <= min the tail is one chunk; else the next cut is the
 * first candidate in (s+min, s+min(len-s,max)], else s+min(len-s,max). */
uint64_t dsxo_chain(const uint64_t *cands, uint64_t ncand, uint64_t len, uint64_t min,
                    uint64_t max, uint64_t *ends, uint64_t cap) {
    uint64_t s = 0, k = 0, j = 0;
    while (s < len) {
        uint64_t rem = len - s, next;
        if (rem <= min) {
            next = len;
        } else {
            uint64_t m = rem < max ? rem : max;
            while (j < ncand && cands[j] <= s + min) j++;
            next = (j < ncand && cands[j] <= s + m) ? cands[j] : s + m;
        }
        if (k < cap) ends[k] = next;
        k++;
        s = next;
    }
    return k;
}

/* ---- make.go-style split-and-align (CPU baseline only) ---------------------
 * n workers start span*i apart (make.go:69-116); each chunks its span
 * sequentially with the Chunker.Next() loop (as pChunker.start,
 * make.go:196-258) and then keeps going past its span until one of its cuts
 * coincides with a cut of its successor (the syncWith test, make.go:277-298).
 * The resulting cut list equals the sequential one (make_test.go:16-80). */
typedef struct {
    const uint8_t *buf;
    uint64_t len, start, stop; /* chunk from start; first pass ends at cut >= stop */
    const dsxo_params_t *p;
    uint64_t *cuts;
    uint64_t ncuts, cap;
    int ok;
} pworker_t;

static uint64_t next_cut(const uint8_t *buf, uint64_t len, uint64_t pos, const dsxo_params_t *p) {
    uint64_t rem = len - pos, min = p->min, max = p->max;
    if (rem <= min) return len;
    uint64_t m = rem < max ? rem : max;
    const uint8_t *c = buf + pos;
    uint32_t h = 0;
    for (unsigned i = 0; i < DSX_WINDOW; i++)
        h ^= rotl32(DSX_BUZHASH_T[c[min - DSX_WINDOW + i]], DSX_WINDOW - i - 1);
    const uint8_t *in = c + min, *out = c + min - DSX_WINDOW;
    uint64_t n = m - min;
    for (uint64_t i = 0; i + 1 < n; i += 2) {
        uint32_t a0 = T_ROT[out[i]] ^ DSX_BUZHASH_T[in[i]];
        uint32_t a1 = T_ROT[out[i + 1]] ^ DSX_BUZHASH_T[in[i + 1]];
        uint32_t h1 = rotl32(h, 1) ^ a0;
        h = rotl32(h, 2) ^ rotl32(a0, 1) ^ a1;
        if (is_boundary(p, h1)) return pos + min + i + 1;
        if (is_boundary(p, h)) return pos + min + i + 2;
    }
    return pos + m;
}

static void *pworker_run(void *arg) {
    pworker_t *w = (pworker_t *)arg;
    uint64_t pos = w->start;
    w->ncuts = 0;
    while (pos < w->len && pos < w->stop) {
        pos = next_cut(w->buf, w->len, pos, w->p);
        if (w->ncuts >= w->cap) { w->ok = 0; return NULL; }
        w->cuts[w->ncuts++] = pos;
    }
    w->ok = 1;
    return NULL;
}

static int has_cut(const uint64_t *cuts, uint64_t n, uint64_t x) {
    uint64_t lo = 0, hi = n;
    while (lo < hi) {
        uint64_t mid = (lo + hi) / 2;
        if (cuts[mid] < x) lo = mid + 1; else hi = mid;
    }
    return lo < n && cuts[lo] == x;
}

uint64_t dsxo_chunk_parallel(const uint8_t *buf, uint64_t len, const dsxo_params_t *p,
                             int n, uint64_t *ends, uint64_t cap) {
    pthread_once(&t_rot_once, init_trot);
    if (len == 0) return 0;
    uint64_t nn = len / p->max + 1; /* make.go:70-74 */
    if (nn < (uint64_t)n) n = (int)nn;
    if (n < 1) n = 1;
    uint64_t span = len / (uint64_t)n;
    pworker_t *w = (pworker_t *)calloc((size_t)n, sizeof(pworker_t));
    pthread_t *th = (pthread_t *)calloc((size_t)n, sizeof(pthread_t));
    for (int i = 0; i < n; i++) {
        w[i].buf = buf; w[i].len = len; w[i].p = p;
        w[i].start = span * (uint64_t)i;
        w[i].stop = (i + 1 < n) ? span * (uint64_t)(i + 1) : len;
        w[i].cap = (w[i].stop - w[i].start) / p->min + 4;
        w[i].cuts = (uint64_t *)malloc(w[i].cap * sizeof(uint64_t));
        pthread_create(&th[i], NULL, pworker_run, &w[i]);
    }
    for (int i = 0; i < n; i++) pthread_join(th[i], NULL);
    /* align: the true chain (worker 0's) is extended with next_cut() until it
     * lands on worker i's virtual start or one of its cuts (syncWith,
     * make.go:277-298); from there worker i's cuts are the true ones. */
    uint64_t k = 0, pos = 0;
    for (int i = 0; i < n; i++) {
        int synced = (i == 0);
        if (!synced) {
            if (pos >= len || pos >= w[i].stop) continue;
            synced = (pos == w[i].start) || has_cut(w[i].cuts, w[i].ncuts, pos);
            while (!synced && pos < len && pos < w[i].stop) {
                pos = next_cut(buf, len, pos, p);
                if (k < cap) ends[k] = pos;
                k++;
                synced = (pos == w[i].start) || has_cut(w[i].cuts, w[i].ncuts, pos);
            }
            if (!synced) continue;
        }
        for (uint64_t c = 0; c < w[i].ncuts; c++) {
            if (w[i].cuts[c] <= pos && i > 0) continue;
            if (k < cap) ends[k] = w[i].cuts[c];
            k++;
            pos = w[i].cuts[c];
        }
    }
    while (pos < len) { /* only reachable if the last worker was skipped */
        pos = next_cut(buf, len, pos, p);
        if (k < cap) ends[k] = pos;
        k++;
    }
    for (int i = 0; i < n; i++) free(w[i].cuts);
    free(w); free(th);
    return k;
}

/* ---- synthetic inputs: CPU twins of desync_amd/csrc/dsx_gen.hip ------------
 * These are not reference algorithms (the BASELINE configs only name the
 * shapes: uniform bytes, 30 % repeated 1 MiB blocks); they let the tests
 * regenerate any window of the device-generated workloads on the host and
 * check the device bytes before comparing cut lists.  Stream definition:
 *   uniform: 8-byte word i = splitmix64(seed * 2^40 + i), little endian;
 *   dedup:   1 MiB blocks; block b > 0 is, with probability p, a copy of block
 *            j = hi32(r) mod b (r = splitmix64(seed<<40 ^ b*K ^ C), taken when
 *            lo32(r) < p_thresh), followed down to a fresh block; a fresh
 *            block's bytes are the uniform stream's bytes of that block. */
static inline uint64_t splitmix64(uint64_t z) {
    z = z * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E5A1ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

uint32_t dsxo_dedup_thresh(double p_repeat) {
    double t = p_repeat * 4294967296.0;
    return t >= 4294967295.0 ? 0xFFFFFFFFu : (uint32_t)t;
}

uint64_t dsxo_dedup_root(uint64_t blk, uint64_t seed, uint32_t p_thresh) {
    while (blk > 0) {
        uint64_t r = splitmix64((seed << 40) ^ (blk * 0x2545F4914F6CDD1Dull) ^ 0xD1B54A32D192ED03ull);
        if ((uint32_t)r >= p_thresh) break;
        blk = (r >> 32) % blk;
    }
    return blk;
}

/* bytes [src, src+n) of the uniform stream of `seed` into dst */
static void gen_uniform_at(uint8_t *dst, uint64_t src, uint64_t n, uint64_t seed) {
    const uint64_t sb = seed << 40;
    uint64_t i = 0;
    while (i < n) {
        const uint64_t a = src + i, w = splitmix64(sb + (a >> 3));
        const unsigned s = (unsigned)(a & 7u);
        if (s == 0 && n - i >= 8) {
            memcpy(dst + i, &w, 8); /* little-endian host (x86-64) */
            i += 8;
        } else {
            dst[i++] = (uint8_t)(w >> (8u * s));
        }
    }
}

void dsxo_gen_uniform(uint8_t *dst, uint64_t offset, uint64_t len, uint64_t seed) {
    gen_uniform_at(dst, offset, len, seed);
}

void dsxo_gen_dedup(uint8_t *dst, uint64_t offset, uint64_t len, uint64_t seed, uint32_t p_thresh) {
    uint64_t i = 0;
    while (i < len) {
        const uint64_t a = offset + i, blk = a >> 20, in = a & 0xFFFFFull;
        const uint64_t n = (1ull << 20) - in < len - i ? (1ull << 20) - in : len - i;
        const uint64_t root = dsxo_dedup_root(blk, seed, p_thresh);
        gen_uniform_at(dst + i, (root << 20) | in, n, seed);
        i += n;
    }
}
