"""ctypes binding of libdsx.so (the C ABI declared in include/dsx.h).

This is the same binding a Go maintainer writes with cgo;
here it backs the Python mirror of desync's Chunker / IndexFromFile API.  There
is deliberately no CPU fallback: if the HIP library is missing or no GPU is
visible, calls raise.
"""
from __future__ import annotations

import ctypes
import os
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("DSX_LIB_PATH") or os.path.join(HERE, "libdsx.so")  # (A/B runs)

DSX_OUT_HOST = 0
DSX_OUT_DEVICE = 1
DSX_NO_SYNC = 2
DSX_TIMED = 16
DSX_SEAM_MAX_CANDS = 1024
DSX_SEAM_MAX_CUTS = 1024

# error codes (include/dsx.h)
DSX_OK = 0
DSX_E_MIN_TOO_SMALL = -1
DSX_E_MIN_GT_MAX = -2
DSX_E_MIN_GT_AVG = -3
DSX_E_AVG_GT_MAX = -4
DSX_E_AVG_RANGE = -5
DSX_E_INVAL = -6
DSX_E_CAPACITY = -7
DSX_E_HIP = -8
DSX_E_NOMEM = -9
DSX_E_INTERRUPTED = -10
DSX_E_IO = -11
DSX_E_STATE = -12
DSX_E_INTERNAL = -13
DSX_E_RESYNC = -14
DSX_E_PEER = -15
DSX_STREAM_EOF = 1
DSX_STREAM_SYNC = 2
DSX_SEAM_DEVICE = 8
DSX_SEAM_LAST = 1
DSX_SEAM_REWALKED = 2
DSX_SEAM_ERROR = 4
DSX_SEAM_REDO = 16

# every symbol include/dsx.h declares (tests check the library exports them)
EXPORTS = (
    "dsx_params_init", "dsx_strerror", "dsx_abi_version", "dsx_ctx_create", "dsx_ctx_destroy",
    "dsx_last_error", "dsx_cancel", "dsx_cut_device", "dsx_sync", "dsx_result", "dsx_cut_host",
    "dsx_cut_fd", "dsx_stream_begin", "dsx_stream_push", "dsx_stream_pop", "dsx_stream_advance",
    "dsx_stream_done", "dsx_stream_end", "dsx_stream_chunk_data", "dsx_stream_buffer",
    "dsx_stream_commit", "dsx_stream_flush", "dsx_stream_ids", "dsx_stream_chunk_id",
    "dsx_stream_pop_many", "dsx_stream_window", "dsx_stream_unpop", "dsx_shard_local", "dsx_shard_resolve",
    "dsx_selftest_boundary", "dsx_gen_uniform", "dsx_gen_dedup", "dsx_chunk_ids",
    "dsx_get_stats", "dsx_debug_trace", "dsx_index_fd", "dsx_index_host", "dsx_copy",
    "dsx_ids_fd", "dsx_ids_host", "dsx_progress", "dsx_shard_resolve_async", "dsx_shard_collect",
    "dsx_ctx_stream", "dsx_stamps_begin", "dsx_stamps_end", "dsx_host_copy",
    "dsx_host_sha512_256",
)
DSX_DIGEST_SHA512_256 = 0
DSX_DIGEST_SHA256 = 1
DSX_ENDS_DEVICE = 4
DSX_HOST_SHA_SCALAR = 1


class Params(ctypes.Structure):
    """dsx_params_t (mirrors the Chunker fields of chunker.go:108-131)."""

    _fields_ = [
        ("min", ctypes.c_uint64), ("avg", ctypes.c_uint64), ("max", ctypes.c_uint64),
        ("discriminator", ctypes.c_uint32), ("inverse_odd", ctypes.c_uint32),
        ("qmax", ctypes.c_uint32), ("qbias", ctypes.c_uint32), ("rot", ctypes.c_int32),
        ("reserved", ctypes.c_uint32),
    ]


class Stats(ctypes.Structure):
    _fields_ = [
        ("chunks", ctypes.c_uint64), ("candidates", ctypes.c_uint64), ("pieces", ctypes.c_uint64),
        ("repaired_segments", ctypes.c_uint64), ("dense_fallbacks", ctypes.c_uint64),
        ("scan_ms", ctypes.c_float), ("stitch_ms", ctypes.c_float),
        ("chunks_discarded", ctypes.c_uint64),
        ("device_bytes", ctypes.c_uint64),
        ("host_tail_chunks", ctypes.c_uint64),
    ]


class ScanStamp(ctypes.Structure):
    """dsx_scan_stamp_t: one scan launch timed from inside the kernel."""

    _fields_ = [(n, ctypes.c_uint64) for n in
                ("seq", "bytes", "t_first", "t_last", "wave_cycles", "wave_ticks", "waves", "reserved")]

    @property
    def ms(self):
        return (self.t_last - self.t_first) / 1e5  # s_memrealtime: 100 MHz

    @property
    def mhz(self):
        return 100.0 * self.wave_cycles / self.wave_ticks if self.wave_ticks else 0.0

    @property
    def busy(self):
        """Mean fraction of the launch its waves were running (1 - the
        wave-end spread and start skew)."""
        span = self.t_last - self.t_first
        return self.wave_ticks / (self.waves * span) if self.waves and span else 0.0


class Seam(ctypes.Structure):
    _fields_ = [
        ("shard_start", ctypes.c_uint64), ("shard_len", ctypes.c_uint64), ("total", ctypes.c_uint64),
        ("first_cand_beyond", ctypes.c_uint64), ("exit_cut", ctypes.c_uint64),
        ("window_end", ctypes.c_uint64), ("entry", ctypes.c_uint64),
        ("ncands", ctypes.c_uint32), ("ncuts", ctypes.c_uint32),
        ("flags", ctypes.c_uint32), ("pad", ctypes.c_uint32),
        ("cands", ctypes.c_uint64 * DSX_SEAM_MAX_CANDS),
        ("cuts", ctypes.c_uint64 * DSX_SEAM_MAX_CUTS),
    ]


_lib = None
_lock = threading.RLock()  # (re-entrant: a Chunker's __del__ may return its context to the pool)


def _share_torch_hip_runtime():
    """A process can drive the GPU through ONE HIP runtime.  PyTorch-ROCm ships
    its own libamdhip64.so (SONAME libamdhip64.so.7, the same as ROCm's); load
    it before libdsx.so so that libdsx binds to it and device pointers, streams
    and RCCL from torch interoperate with the library.  Without torch the
    system ROCm runtime (/opt/rocm/lib, libdsx's RUNPATH) is used."""
    try:
        import torch
    except ImportError:
        return
    path = os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so")
    if os.path.exists(path):
        ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)


# The DSX_* settings the product library reads (INTEGRATION.md,
# "Environment"; tests/test_abi.py checks the library's strings against it).
PRODUCT_ENV = ("DSX_TAIL_SPLIT", "DSX_LANE_TARGET", "DSX_SEG_FLOOR", "DSX_SCAN_NT",
               "DSX_DIGEST_PC", "DSX_DIGEST_LPT", "DSX_INDEX_WINDOW", "DSX_INDEX_SLOT",
               "DSX_INDEX_READERS", "DSX_INDEX_HOST_TAIL", "DSX_HOST_THREADS")
# Settings only libdsx_diag.so reads (scan ablations, other geometries,
# rejected experiments), with the value the product library behaves as (None:
# no such value).  Set to anything else with the product library they would
# be silently ignored, so loading it refuses them.
DIAG_ENV = {"DSX_SCAN_VARIANT": "0", "DSX_SCAN_CFG": "0", "DSX_FUSE": "0", "DSX_TEST_MODE": None,
            "DSX_DIGEST_PC_CHUNKS": "2", "DSX_PREFETCH": "0", "DSX_REGIONS_PER_SLOT": "1",
            "DSX_SCAN_LINE": "1", "DSX_SCAN_TRACE": "0", "DSX_WAVE_MAJOR": "1",
            "DSX_FIXUP_FAST": "1", "DSX_FINISH": "1", "DSX_SEG_MAX": "4", "DSX_SEG_TARGET": "4096",
            "DSX_DIGEST_PF": "1", "DSX_TAIL_MULT": "1", "DSX_LANE_BYTES": None,
            "DSX_STITCH_CUS": "0", "DSX_SCAN_MASK": "0", "DSX_SCAN_PRIO": None,
            "DSX_STREAM_BATCH": None, "DSX_NOOP_BEFORE_SCAN": None, "DSX_WALK_WGS": "2",
            "DSX_WALK_NT": "576", "DSX_TAIL_LOG": None, "DSX_FEED_THREADS": None, "DSX_FEED_MULTI": None,
            "DSX_FEED_MID": None, "DSX_SIDE_PRIO": "1",
            "DSX_FEED_CUT_END": None, "DSX_SHARE_NS": "58", "DSX_SHARE_PC": "1", "DSX_SHARE_SLACK": "0", "DSX_CTX_PRIO": "1", "DSX_FEED_EXTRA": None, "DSX_SHARE_MULTI": "1", "DSX_FINE_TAIL": "33554432", "DSX_FINE_DIV": "4"}


def lib():
    """Load libdsx.so; raises ImportError if it has not been built."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is missing: build it with __graft_entry__.build() "
                "(make -C desync_amd/csrc). desync_amd has no CPU fallback.")
        diag_env = [k for k, dflt in DIAG_ENV.items() if os.environ.get(k, "") not in ("", dflt)]
        if diag_env and not os.path.basename(LIB_PATH).startswith("libdsx_diag"):
            raise ImportError(
                f"{', '.join(diag_env)} selects a diagnostic path (scan ablations, other "
                "geometries, rejected experiments), which only the diagnostic build reads: "
                "make -C desync_amd/csrc diag and set "
                "DSX_LIB_PATH=desync_amd/libdsx_diag.so")
        _share_torch_hip_runtime()
        L = ctypes.CDLL(LIB_PATH)
        u64, u32, i32, vp = ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p
        P = ctypes.POINTER
        sig = {
            "dsx_params_init": (i32, [u64, u64, u64, P(Params)]),
            "dsx_strerror": (ctypes.c_char_p, [i32]),
            "dsx_abi_version": (i32, []),
            "dsx_ctx_create": (i32, [i32, P(vp)]),
            "dsx_ctx_destroy": (i32, [vp]),
            "dsx_last_error": (ctypes.c_char_p, [vp]),
            "dsx_cancel": (i32, [vp]),
            "dsx_progress": (i32, [vp, P(u64)]),
            "dsx_cut_device": (i32, [vp, vp, u64, P(Params), vp, u64, P(u64), u32]),
            "dsx_sync": (i32, [vp]),
            "dsx_result": (i32, [vp, P(u64)]),
            "dsx_cut_host": (i32, [vp, vp, u64, P(Params), vp, u64, P(u64)]),
            "dsx_cut_fd": (i32, [vp, i32, u64, u64, P(Params), vp, u64, P(u64)]),
            "dsx_stream_begin": (i32, [vp, P(Params)]),
            "dsx_stream_push": (i32, [vp, vp, u64, i32]),
            "dsx_stream_pop": (i32, [vp, P(u64), P(u64)]),
            "dsx_stream_advance": (i32, [vp, u64]),
            "dsx_stream_done": (i32, [vp]),
            "dsx_stream_end": (i32, [vp]),
            "dsx_stream_buffer": (i32, [vp, u64, P(vp)]),
            "dsx_stream_commit": (i32, [vp, u64, i32]),
            "dsx_stream_flush": (i32, [vp, P(u64), P(u64)]),
            "dsx_stream_ids": (i32, [vp, i32]),
            "dsx_stream_chunk_id": (vp, [vp]),
            "dsx_stream_pop_many": (i32, [vp, vp, vp, u64, P(u64), P(u64)]),
            "dsx_stream_window": (i32, [vp, P(vp), P(u64), P(u64)]),
            "dsx_stream_unpop": (i32, [vp, u64]),
            "dsx_stream_chunk_data": (vp, [vp]),
            "dsx_shard_local": (i32, [vp, vp, u64, u64, u64, u64, P(Params), vp, u32]),
            "dsx_shard_resolve": (i32, [vp, vp, i32, i32, vp, vp, u64, P(u64), u32]),
            "dsx_shard_resolve_async": (i32, [vp, vp, i32, i32, vp, u64, vp]),
            "dsx_shard_collect": (i32, [vp, vp, vp, P(ctypes.c_int32), P(u64)]),
            "dsx_ctx_stream": (i32, [vp, P(vp)]),
            "dsx_selftest_boundary": (i32, [vp, P(Params), i32, u64, u64, P(u64)]),
            "dsx_gen_uniform": (i32, [vp, vp, u64, u64, u64]),
            "dsx_gen_dedup": (i32, [vp, vp, u64, u64, u64, ctypes.c_double]),
            "dsx_chunk_ids": (i32, [vp, vp, u64, u64, vp, u64, vp, u32, i32]),
            "dsx_get_stats": (i32, [vp, P(Stats)]),
            "dsx_copy": (i32, [vp, vp, vp, u64]),
            "dsx_index_fd": (i32, [vp, i32, u64, u64, P(Params), i32, vp, vp, u64, P(u64)]),
            "dsx_index_host": (i32, [vp, vp, u64, P(Params), i32, vp, vp, u64, P(u64)]),
            "dsx_debug_trace": (i32, [vp, vp, u64, P(u64), P(u64)]),
            "dsx_ids_fd": (i32, [vp, i32, u64, u64, u64, vp, u64, i32, vp]),
            "dsx_ids_host": (i32, [vp, vp, u64, u64, vp, u64, i32, vp]),
            "dsx_stamps_begin": (i32, [vp, u64]),
            "dsx_stamps_end": (i32, [vp, vp, u64, P(u64)]),
            "dsx_host_copy": (i32, [vp, vp, u64, i32]),
            "dsx_host_sha512_256": (i32, [vp, vp, u64, vp, i32, i32]),
        }
        for name, (res, args) in sig.items():
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _lib = L
        return L


class DsxError(RuntimeError):
    def __init__(self, code, detail=""):
        self.code = code
        msg = lib().dsx_strerror(code).decode()
        super().__init__(f"{msg}" + (f": {detail}" if detail else ""))


def check(rc, ctx=None):
    if rc < 0:
        detail = ""
        if ctx is not None and rc in (DSX_E_HIP, DSX_E_INTERNAL, DSX_E_NOMEM):
            d = lib().dsx_last_error(ctx)
            detail = d.decode() if d else ""
        raise DsxError(rc, detail)
    return rc


class Context:
    """One dsx_ctx (HIP streams + device scratch) on a GPU; not thread-safe."""

    def __init__(self, device=0):
        h = ctypes.c_void_p()
        rc = lib().dsx_ctx_create(int(device), ctypes.byref(h))
        if rc != DSX_OK:
            why = lib().dsx_last_error(None)
            raise DsxError(rc, f"cannot create a dsx context on HIP device {device}"
                           + (f" ({why.decode()})" if why else ""))
        self.h = h
        self.device = device

    def close(self):
        if self.h:
            lib().dsx_ctx_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def stats(self):
        s = Stats()
        check(lib().dsx_get_stats(self.h, ctypes.byref(s)), self.h)
        return s

    def stamps_begin(self, max_launches):
        """Time the next max_launches scan launches from inside the kernel."""
        check(lib().dsx_stamps_begin(self.h, int(max_launches)), self.h)
        self._stamp_cap = int(max_launches)

    def stamps_end(self):
        """The stamped launches' ScanStamp records, in launch order."""
        cap = getattr(self, "_stamp_cap", 0)
        buf = (ScanStamp * max(1, cap))()
        n = ctypes.c_uint64()
        check(lib().dsx_stamps_end(self.h, buf, cap, ctypes.byref(n)), self.h)
        return list(buf[:min(cap, n.value)])


_default = {}
_pool = {}  # (device, DSX_* env) -> idle contexts (IndexFromFile is re-entrant, a context is not)


def default_context(device=0):
    ctx = _default.get(device)
    if ctx is None:
        ctx = Context(device)
        _default[device] = ctx
    return ctx


_POOL_IDLE = 4  # idle contexts kept per device (each holds its pipeline buffers)


def _env_key(device):
    # a context reads its DSX_* settings from the environment when created:
    # it is handed out again only under the same settings
    return (device, tuple(sorted((k, v) for k, v in os.environ.items() if k.startswith("DSX_"))))


def acquire_context(device=0):
    """A context no other thread uses until release_context(): an idle pooled
    one (its pinned and device buffers already sized by earlier calls) or a
    new one.  A new context costs ~0.2 s of allocations once its pipelines
    run; a pooled one costs nothing."""
    key = _env_key(device)
    ctx = None
    with _lock:
        # idle contexts made under other settings are not handed out again
        # while these hold: close them rather than keep their buffers
        stale = [c for k in list(_pool) if k[0] == device and k != key for c in _pool.pop(k)]
        idle = _pool.setdefault(key, [])
        while idle and ctx is None:
            ctx = idle.pop()
            ctx = ctx if ctx.h else None  # (closed meanwhile: reset_context_pool)
    for c in stale:
        c.close()
    if ctx is None:
        ctx = Context(device)
        ctx._pool_key = key
    return ctx


def release_context(ctx):
    """Returns a context from acquire_context() to its pool (closed instead
    when the pool is full or the context is closed)."""
    if ctx is None or not ctx.h:
        return
    key = getattr(ctx, "_pool_key", None) or _env_key(ctx.device)
    with _lock:
        idle = _pool.setdefault(key, [])
        if len(idle) < _POOL_IDLE:
            idle.append(ctx)
            return
    ctx.close()


class pooled_context:
    """``with pooled_context(dev) as ctx``: a context no other thread uses
    meanwhile (created on demand, returned to a per-device pool afterwards;
    the pipeline buffers a context holds are reused by the next call)."""

    def __init__(self, device=0):
        self.device = device
        self.ctx = None

    def __enter__(self):
        self.ctx = acquire_context(self.device)
        return self.ctx

    def __exit__(self, *exc):
        release_context(self.ctx)
        self.ctx = None
        return False


def reset_context_pool():
    """Closes the idle pooled contexts (settings such as DSX_INDEX_WINDOW are
    read from the environment when a context is created)."""
    with _lock:
        idle = [c for cs in _pool.values() for c in cs]
        _pool.clear()
    for c in idle:
        c.close()
