"""C ABI checks that need no GPU: libdsx.so loads, exports every symbol that
include/dsx.h declares, and NewChunker's validation matches chunker.go."""
import ctypes
import os
import re

import pytest

from desync_amd import _lib
from oracle import oracle as o

HDR = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "dsx.h")


def declared_functions():
    txt = open(HDR).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(dsx_[a-z0-9_]+)\s*\(", txt)))


def test_header_and_binding_agree():
    assert declared_functions() == sorted(_lib.EXPORTS)


def test_library_exports_every_declared_symbol():
    L = _lib.lib()
    for name in declared_functions():
        assert hasattr(L, name), name


def test_abi_version():
    assert _lib.lib().dsx_abi_version() == 5


@pytest.mark.parametrize("args,code,msg", [
    ((47, 64, 128), _lib.DSX_E_MIN_TOO_SMALL, "min chunk size too small, must be over 48"),
    ((200, 300, 100), _lib.DSX_E_MIN_GT_MAX, "min chunk size must not be greater than max"),
    ((200, 100, 300), _lib.DSX_E_MIN_GT_AVG, "min chunk size must not be greater than avg"),
    ((100, 300, 200), _lib.DSX_E_AVG_GT_MAX, "avg chunk size must not be greater than max"),
])
def test_param_validation_order_and_messages(args, code, msg):
    p = _lib.Params()
    assert _lib.lib().dsx_params_init(*args, ctypes.byref(p)) == code
    assert _lib.lib().dsx_strerror(code).decode() == msg
    with pytest.raises(ValueError, match=msg):
        import desync_amd
        desync_amd.Params(*args)


def test_param_constants_match_oracle():
    """dsx_params_init derives the same constants as chunker.go:147-170."""
    avgs = [48, 64, 100, 1000, 4096, 8192, 16384, 65536, 100000, 262144, 1 << 20, 3 << 20,
            8 << 20] + list(range(48, 5000, 37)) + list(range(60000, 70000, 113))
    for avg in avgs:
        p = _lib.Params()
        assert _lib.lib().dsx_params_init(48, avg, avg, ctypes.byref(p)) == 0
        P = o.params(48, avg, avg)
        assert (p.discriminator, p.inverse_odd, p.qmax, p.qbias, p.rot) == \
            (P.d, P.inv, P.qmax, P.qbias, P.rot), avg


def test_no_gpu_context_fails_loudly():
    """Without a GPU the context cannot be created -- there is no CPU path."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(_lib.DsxError):
        _lib.Context(0)


def test_seam_record_layout():
    """dsx_seam_t is exchanged as raw bytes between ranks: the ctypes mirror
    has the C layout (static_assert in dsx_api.cpp)."""
    assert ctypes.sizeof(_lib.Seam) == 7 * 8 + 4 * 4 + 8 * (1024 + 1024)
    assert _lib.Seam.cands.offset == 7 * 8 + 4 * 4


# Message tokens that appear as text in the library (error strings), not as
# environment settings it reads.
_MESSAGE_TOKENS = {"DSX_NO_SYNC", "DSX_SEAM_ERROR", "DSX_SEAM_MAX_CUTS"}
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _dsx_strings(path):
    with open(path, "rb") as f:
        return {m.decode() for m in re.findall(rb"DSX_[A-Z0-9_]+", f.read())}


def test_product_library_reads_only_the_documented_environment():
    """libdsx.so names exactly _lib.PRODUCT_ENV: the
    rejected experiments and diagnostic geometries are compiled into
    libdsx_diag.so only.  INTEGRATION.md documents each product setting, a
    test sets each one, and loading the product library refuses a
    diagnostic setting instead of ignoring it."""
    names = _dsx_strings(_lib.LIB_PATH) - _MESSAGE_TOKENS
    assert names == set(_lib.PRODUCT_ENV), sorted(names ^ set(_lib.PRODUCT_ENV))
    doc = open(os.path.join(REPO, "INTEGRATION.md")).read()
    env_doc = doc[doc.index("## Environment"):]
    tests = "".join(open(os.path.join(REPO, "tests", f)).read()
                    for f in os.listdir(os.path.join(REPO, "tests"))
                    if f.endswith(".py") and f != "test_abi.py")
    for k in _lib.PRODUCT_ENV:
        assert f"`{k}`" in env_doc, k
        assert f'"{k}"' in tests, f"{k}: no test sets it"
    assert not set(_lib.DIAG_ENV) & set(_lib.PRODUCT_ENV)


def test_diagnostic_library_reads_the_diagnostic_environment():
    diag = os.path.join(REPO, "desync_amd", "libdsx_diag.so")
    if not os.path.exists(diag):
        pytest.skip("libdsx_diag.so not built (make -C desync_amd/csrc diag)")
    names = _dsx_strings(diag) - _MESSAGE_TOKENS
    assert set(_lib.DIAG_ENV) | set(_lib.PRODUCT_ENV) == names, sorted(
        names ^ (set(_lib.DIAG_ENV) | set(_lib.PRODUCT_ENV)))


def test_diagnostic_setting_refused_by_the_product_library():
    import subprocess
    import sys
    for k, v in (("DSX_PREFETCH", "1"), ("DSX_SCAN_TRACE", "1"), ("DSX_WAVE_MAJOR", "0")):
        env = dict(os.environ, **{k: v})
        env.pop("DSX_LIB_PATH", None)
        r = subprocess.run([sys.executable, "-c", "from desync_amd import _lib; _lib.lib()"],
                           env=env, capture_output=True, text=True, timeout=120, cwd=REPO)
        assert r.returncode != 0 and k in r.stderr and "libdsx_diag" in r.stderr, (k, r.stderr)
    # the value the product library behaves as is accepted
    env = dict(os.environ, DSX_FUSE="0", DSX_WAVE_MAJOR="1")
    env.pop("DSX_LIB_PATH", None)
    r = subprocess.run([sys.executable, "-c", "from desync_amd import _lib; _lib.lib()"],
                       env=env, capture_output=True, text=True, timeout=120, cwd=REPO)
    assert r.returncode == 0, r.stderr
