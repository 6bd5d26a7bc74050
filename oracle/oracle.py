"""CPU oracle for desync's content-defined chunker -- TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module.  It is the checker, never the thing measured or
shipped: the product path (``desync_amd``) never imports it and fails loudly if
its HIP library is missing.

What it restates (reference file:line):

* ``chunker.go:13-15``  discriminatorFromAvg            -> :func:`discriminator`
* ``chunker.go:20-28``  modInverse32                     -> :func:`mod_inverse32`
* ``chunker.go:134-171`` NewChunker constants + errors   -> :func:`params`
* ``chunker.go:206-277`` Chunker.Next loop               -> :func:`chunk_stream`
  (C, ``dsx_oracle.c``) and :func:`chunk_stream_py` (pure Python, small inputs)
* candidate predicate + chain rule     -> :func:`candidates`,
  :func:`candidates_np`, :func:`chain`
* ``make.go:22-163``    IndexFromFile split-and-align    -> :func:`chunk_parallel`
* ``make.go:35-62``     index feature flags + catar sniff -> :func:`index_flags`
* ``index.go:90-124`` + ``format.go:582-620`` caibx      -> :func:`encode_caibx`
* ``digest.go:11-29``   SHA-512/256 / SHA-256 chunk IDs  -> :func:`chunk_ids`
  (Go stdlib ``crypto/sha512`` go1.25 per go.mod:3; restated by OpenSSL through
  :mod:`hashlib`; pinned by the reference's own chunk IDs in
  chunker_test.go:30-49, chunker.index, blob1/2.caibx and tree.caidx).

Parity is pinned by tests/test_oracle_golden.py against the reference's
golden files, copied as data fixtures under tests/golden/.
"""
from __future__ import annotations

import ctypes
import hashlib
import os
import struct
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
WINDOW = 48  # ChunkerWindowSize, chunker.go:11

# caibx constants (const.go:23-25, 74-77)
CA_FORMAT_ENTRY = 0x1396FABCEA5BBB51
CA_FORMAT_INDEX = 0x96824D9C7B129FF9
CA_FORMAT_TABLE = 0xE75B9E112F17417D
CA_FORMAT_TABLE_TAIL_MARKER = 0x4B4F050E5549ECD1
CA_FORMAT_SHA512256 = 0x2000000000000000
CA_FORMAT_EXCLUDE_NO_DUMP = 0x8000000000000000

# reference error messages, chunker.go:135-146 (in check order)
PARAM_ERRORS = {
    1: "min chunk size too small, must be over 48",
    2: "min chunk size must not be greater than max",
    3: "min chunk size must not be greater than avg",
    4: "avg chunk size must not be greater than max",
}


def _table():
    path = os.path.join(REPO, "include", "dsx_buzhash_table.h")
    txt = open(path).read().split("#define DSX_BUZHASH_TABLE_INIT {")[1].split("}")[0]
    txt = txt.replace("\\", " ").replace("\n", " ")
    vals = [int(t.strip().rstrip("u"), 16) for t in txt.split(",") if t.strip()]
    assert len(vals) == 256
    return np.array(vals, dtype=np.uint32)


T = _table()


def rotl32(x, r):
    r &= 31
    x &= 0xFFFFFFFF
    return ((x << r) | (x >> (32 - r))) & 0xFFFFFFFF if r else x


T_ROT = np.array([rotl32(int(v), 48) for v in T], dtype=np.uint32)


# --------------------------------------------------------------------------
# C library
# --------------------------------------------------------------------------
class _Params(ctypes.Structure):
    _fields_ = [
        ("min", ctypes.c_uint64), ("avg", ctypes.c_uint64), ("max", ctypes.c_uint64),
        ("d", ctypes.c_uint32), ("inv", ctypes.c_uint32), ("qmax", ctypes.c_uint32),
        ("qbias", ctypes.c_uint32), ("rot", ctypes.c_int),
    ]


_LIB = None


def lib():
    """Load (building if needed) oracle/liboracle.so."""
    global _LIB
    if _LIB is None:
        so = os.path.join(HERE, "liboracle.so")
        src = os.path.join(HERE, "dsx_oracle.c")
        if not os.path.exists(so) or os.path.getmtime(so) < os.path.getmtime(src):
            subprocess.check_call(["make", "-s", "-C", HERE])
        L = ctypes.CDLL(so)
        u64, u32, p = ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p
        L.dsxo_discriminator.restype = u32
        L.dsxo_discriminator.argtypes = [u64]
        L.dsxo_mod_inverse32.restype = u32
        L.dsxo_mod_inverse32.argtypes = [u32]
        L.dsxo_params.restype = ctypes.c_int
        L.dsxo_params.argtypes = [u64, u64, u64, ctypes.POINTER(_Params)]
        L.dsxo_is_boundary.restype = ctypes.c_int
        L.dsxo_is_boundary.argtypes = [ctypes.POINTER(_Params), u32]
        for name in ("dsxo_chunk_stream", "dsxo_candidates"):
            f = getattr(L, name)
            f.restype = u64
            f.argtypes = [p, u64, ctypes.POINTER(_Params), p, u64]
        L.dsxo_chain.restype = u64
        L.dsxo_chain.argtypes = [p, u64, u64, u64, u64, p, u64]
        L.dsxo_chunk_parallel.restype = u64
        L.dsxo_chunk_parallel.argtypes = [p, u64, ctypes.POINTER(_Params), ctypes.c_int, p, u64]
        L.dsxo_dedup_thresh.restype = u32
        L.dsxo_dedup_thresh.argtypes = [ctypes.c_double]
        L.dsxo_dedup_root.restype = u64
        L.dsxo_dedup_root.argtypes = [u64, u64, u32]
        L.dsxo_gen_uniform.restype = None
        L.dsxo_gen_uniform.argtypes = [p, u64, u64, u64]
        L.dsxo_gen_dedup.restype = None
        L.dsxo_gen_dedup.argtypes = [p, u64, u64, u64, u32]
        _LIB = L
    return _LIB


class ParamError(ValueError):
    pass


def params(min_size, avg_size, max_size):
    """NewChunker validation + derived constants (chunker.go:134-171)."""
    P = _Params()
    rc = lib().dsxo_params(min_size, avg_size, max_size, ctypes.byref(P))
    if rc:
        raise ParamError(PARAM_ERRORS.get(rc, "discriminator is zero (Go would panic)"))
    return P


def discriminator(avg):
    return int(lib().dsxo_discriminator(avg))


def mod_inverse32(d):
    return int(lib().dsxo_mod_inverse32(d))


def is_boundary(P, h):
    return bool(lib().dsxo_is_boundary(ctypes.byref(P), h & 0xFFFFFFFF))


def _buf(data):
    a = np.frombuffer(data, dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    return np.ascontiguousarray(a, dtype=np.uint8)


def chunk_stream(data, min_size, avg_size, max_size):
    """Chunk END offsets from the literal Chunker.Next() loop (C)."""
    P = params(min_size, avg_size, max_size)
    a = _buf(data)
    n = a.size
    cap = n // min_size + 2
    out = np.zeros(cap, dtype=np.uint64)
    k = lib().dsxo_chunk_stream(a.ctypes.data, n, ctypes.byref(P), out.ctypes.data, cap)
    assert k <= cap
    return out[:k].copy()


def candidates(data, min_size, avg_size, max_size, cap=None):
    """Sorted candidate cut positions p (H(p) % d == d-1), C implementation."""
    P = params(min_size, avg_size, max_size)
    a = _buf(data)
    n = a.size
    if cap is None:
        cap = max(1024, 8 * n // max(P.d, 1) + 1024)
    while True:
        out = np.zeros(cap, dtype=np.uint64)
        k = lib().dsxo_candidates(a.ctypes.data, n, ctypes.byref(P), out.ctypes.data, cap)
        if k <= cap:
            return out[:k].copy()
        cap = int(k)


def chain(cands, length, min_size, max_size):
    """Chain rule over sorted candidates (C)."""
    c = np.ascontiguousarray(cands, dtype=np.uint64)
    cap = length // min_size + 2
    out = np.zeros(cap, dtype=np.uint64)
    k = lib().dsxo_chain(c.ctypes.data, c.size, length, min_size, max_size, out.ctypes.data, cap)
    return out[:k].copy()


def chunk_parallel(data, min_size, avg_size, max_size, n):
    """make.go split-and-align over n pthreads (CPU baseline)."""
    P = params(min_size, avg_size, max_size)
    a = _buf(data)
    cap = a.size // min_size + 2
    out = np.zeros(cap, dtype=np.uint64)
    k = lib().dsxo_chunk_parallel(a.ctypes.data, a.size, ctypes.byref(P), n, out.ctypes.data, cap)
    return out[:k].copy()


# --------------------------------------------------------------------------
# Pure Python / numpy restatements (small inputs; cross-check the C code)
# --------------------------------------------------------------------------
def window_hash(window):
    """chunker.go:225-228: XOR of rotl32(T[b], 47-i) over a 48-byte window."""
    h = 0
    for i, b in enumerate(window):
        h ^= rotl32(int(T[b]), WINDOW - i - 1)
    return h


def is_boundary_py(h, d):
    """The plain form of the test (chunker_test.go:197): h % d == d-1."""
    return h % d == d - 1


def candidates_np(data, d):
    """Vectorised H(p) for every p in [48, len] via 48 rotated-table passes."""
    a = _buf(data)
    n = a.size
    if n < WINDOW:
        return np.zeros(0, dtype=np.uint64)
    m = n - WINDOW + 1  # positions 48..n
    h = np.zeros(m, dtype=np.uint32)
    for j in range(WINDOW):
        r = WINDOW - j - 1
        t = np.array([rotl32(int(v), r) for v in T], dtype=np.uint32)
        h ^= t[a[j:j + m]]
    pos = np.nonzero(h % np.uint32(d) == np.uint32(d - 1))[0]
    return (pos + WINDOW).astype(np.uint64)


def chunk_stream_py(data, min_size, avg_size, max_size):
    """Pure-Python Chunker.Next() (chunker.go:206-277) for small inputs."""
    P = params(min_size, avg_size, max_size)
    a = bytes(_buf(data))
    n = len(a)
    pos, ends = 0, []
    while pos < n:
        rem = n - pos
        if rem <= min_size:
            end = n
        else:
            m = min(rem, max_size)
            h = window_hash(a[pos + min_size - WINDOW:pos + min_size])
            end = pos + m
            for i in range(min_size, m):
                h = rotl32(h, 1) ^ int(T_ROT[a[pos + i - WINDOW]]) ^ int(T[a[pos + i]])
                if h % P.d == P.d - 1:
                    end = pos + i + 1
                    break
        ends.append(end)
        pos = end
    return np.array(ends, dtype=np.uint64)


# --------------------------------------------------------------------------
# Chunk IDs, index flags and caibx encoding
# --------------------------------------------------------------------------
def chunk_ids(data, ends, algo="sha512-256"):
    """Digest.Sum per chunk (digest.go:11-29)."""
    a = bytes(_buf(data)) if not isinstance(data, (bytes, bytearray)) else data
    out, s = [], 0
    for e in ends:
        e = int(e)
        if algo == "sha512-256":
            out.append(hashlib.new("sha512_256", a[s:e]).digest())
        else:
            out.append(hashlib.sha256(a[s:e]).digest())
        s = e
    return out


def index_flags(first_bytes, algo="sha512-256"):
    """make.go:35-62: ExcludeNoDump | SHA512256 (if digest is SHA-512/256) |
    the FeatureFlags of a leading catar FormatEntry (format.go:161-172:
    header size 64, type CaFormatEntry)."""
    flags = CA_FORMAT_EXCLUDE_NO_DUMP
    if algo == "sha512-256":
        flags |= CA_FORMAT_SHA512256
    if len(first_bytes) >= 24:
        size, typ, ff = struct.unpack_from("<QQQ", first_bytes, 0)
        if typ == CA_FORMAT_ENTRY and size == 64 and len(first_bytes) >= 64:
            flags |= ff
    return flags


def encode_caibx(flags, min_size, avg_size, max_size, ends, ids):
    """Index.WriteTo (index.go:90-124) + FormatEncoder.Encode (format.go:582-620)."""
    out = bytearray(struct.pack("<6Q", 48, CA_FORMAT_INDEX, flags, min_size, avg_size, max_size))
    out += struct.pack("<2Q", 0xFFFFFFFFFFFFFFFF, CA_FORMAT_TABLE)
    n = 16
    for e, i in zip(ends, ids):
        out += struct.pack("<Q", int(e)) + i
        n += 40
    out += struct.pack("<5Q", 0, 0, 48, n + 40, CA_FORMAT_TABLE_TAIL_MARKER)
    return bytes(out)


def decode_caibx(blob):
    """Inverse of encode_caibx (format.go:402-447 decoder subset)."""
    size, typ, flags, mn, av, mx = struct.unpack_from("<6Q", blob, 0)
    assert size == 48 and typ == CA_FORMAT_INDEX
    tsize, ttyp = struct.unpack_from("<2Q", blob, 48)
    assert tsize == 0xFFFFFFFFFFFFFFFF and ttyp == CA_FORMAT_TABLE
    off, ends, ids = 64, [], []
    while True:
        (e,) = struct.unpack_from("<Q", blob, off)
        if e == 0:
            break
        ends.append(e)
        ids.append(bytes(blob[off + 8:off + 40]))
        off += 40
    return dict(flags=flags, min=mn, avg=av, max=mx, ends=np.array(ends, dtype=np.uint64), ids=ids)


def make_caibx(data, min_size, avg_size, max_size, algo="sha512-256"):
    """desync make (IndexFromFile + WriteTo) restated end to end."""
    a = _buf(data)
    ends = chunk_stream(a, min_size, avg_size, max_size)
    ids = chunk_ids(a, ends, algo)
    flags = index_flags(bytes(a[:64]), algo)
    return encode_caibx(flags, min_size, avg_size, max_size, ends, ids)


# --------------------------------------------------------------------------
# Deterministic synthetic inputs (shared with the GPU generator, see
# desync_amd/csrc/dsx_gen.hip): splitmix64 of the 8-byte word index.
# --------------------------------------------------------------------------
def splitmix64_words(seed, start_word, nwords):
    """uint64 words w[i] = splitmix64(seed*2^40 + start_word + i)."""
    i = np.arange(start_word, start_word + nwords, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = i + np.uint64(seed) * np.uint64(1 << 40)
        z = z * np.uint64(0x9E3779B97F4A7C15) + np.uint64(0x632BE59BD9B4E5A1)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def synth_uniform(seed, offset, length):
    """Bytes [offset, offset+length) of the seeded uniform stream."""
    w0 = offset // 8
    w1 = (offset + length + 7) // 8
    words = splitmix64_words(seed, w0, w1 - w0)
    b = words.view(np.uint8)
    s = offset - w0 * 8
    return b[s:s + length].copy()


def default_threads():
    """Host threads for the oracle: the GPU box exports OMP_NUM_THREADS (its
    CPU share, 16); os.cpu_count() there reports the whole machine."""
    try:
        n = int(os.environ.get("OMP_NUM_THREADS", "0"))
    except ValueError:
        n = 0
    return max(1, min(n or 16, os.cpu_count() or 1))


def _gen_parallel(fn, args, offset, length, out, threads):
    import concurrent.futures as cf
    a = np.empty(length, dtype=np.uint8) if out is None else out
    assert a.size >= length and a.flags.c_contiguous
    if length == 0:
        return a
    step = max(1 << 20, -(-length // (4 * threads)))
    step = (step + 7) & ~7
    with cf.ThreadPoolExecutor(max_workers=threads) as pool:
        futs = [pool.submit(fn, a.ctypes.data + o, offset + o, min(step, length - o), *args)
                for o in range(0, length, step)]
        for f in futs:
            f.result()
    return a


def synth_uniform_c(seed, offset, length, out=None, threads=None):
    """synth_uniform in C (dsxo_gen_uniform) over host threads, for GiB sizes."""
    return _gen_parallel(lib().dsxo_gen_uniform, (seed,), offset, length, out,
                         threads or default_threads())


def synth_dedup(seed, offset, length, p_repeat=0.30, out=None, threads=None):
    """Bytes [offset, offset+length) of the dedup stream (BASELINE config 3
    shape): the CPU twin of dsx_gen_dedup (desync_amd/csrc/dsx_gen.hip)."""
    th = lib().dsxo_dedup_thresh(p_repeat)
    return _gen_parallel(lib().dsxo_gen_dedup, (seed, th), offset, length, out,
                         threads or default_threads())


def dedup_roots(seed, nblocks, p_repeat=0.30):
    """Source block of every 1 MiB block of the dedup stream (copy chains
    followed down to a fresh block)."""
    th = lib().dsxo_dedup_thresh(p_repeat)
    return np.array([lib().dsxo_dedup_root(b, seed, th) for b in range(nblocks)], dtype=np.uint64)
