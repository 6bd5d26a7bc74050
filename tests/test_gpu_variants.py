"""Every scan variant of the diagnostic build on a two-size piece.

libdsx_diag.so carries ablation variants of scanl_kernel (DSX_SCAN_VARIANT:
1 no boundary test, 3 staging only, 4 no staging, 7-10 the round-5 energy
ablations) and two trace variants (5, 6) with exact results.  Round 5 once
launched a one-size instantiation over a piece whose region list has two
region sizes, and the scan read past the piece (an illegal memory access,
DESIGN.md 10).  The launch macro now picks the instantiation from the
piece's geometry; this test pins that: each variant runs a 4 GiB - 999 B
piece (three big regions per wave slot and more: two region sizes) and must
complete.  Only the trace variants' cut lists are checked (against the exact
kernel's); the ablations' lists are wrong by design.

All variants run in one child process on libdsx_diag.so (the package never
loads the diagnostic build itself).
"""
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DIAG = os.path.join(REPO, "desync_amd", "libdsx_diag.so")
N = (4 << 30) - 999
VARIANTS = (1, 3, 4, 5, 6, 7, 8, 9, 10)
EXACT = (5, 6)


def test_every_diag_variant_on_a_two_size_piece():
    assert os.path.exists(DIAG), "libdsx_diag.so missing: __graft_entry__.build() makes it"
    env = dict(os.environ, DSX_LIB_PATH=DIAG, PYTHONPATH=REPO)
    env.pop("DSX_SCAN_VARIANT", None)
    r = subprocess.run([sys.executable, "-u", os.path.abspath(__file__)], env=env,
                       capture_output=True, text=True, timeout=600, cwd=REPO)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    for v in VARIANTS:
        assert f"variant {v} ok" in r.stdout, r.stdout[-3000:]


def _main():
    import torch

    import desync_amd
    from desync_amd import _lib
    assert os.path.basename(_lib.LIB_PATH).startswith("libdsx_diag")
    L = _lib.lib()
    p = desync_amd.Params(16 << 10, 64 << 10, 256 << 10)
    blob = torch.empty(N, dtype=torch.uint8, device="cuda")
    out = torch.empty(N // (16 << 10) + 4, dtype=torch.int64, device="cuda")
    cnt = ctypes.c_uint64()

    def run(variant):
        os.environ["DSX_SCAN_VARIANT"] = str(variant)
        ctx = _lib.Context(0)
        try:
            if variant == 0:
                _lib.check(L.dsx_gen_uniform(ctx.h, ctypes.c_void_p(blob.data_ptr()), 0, N, 7),
                           ctx.h)
            _lib.check(L.dsx_cut_device(ctx.h, ctypes.c_void_p(blob.data_ptr()), N,
                                        ctypes.byref(p.c), ctypes.c_void_p(out.data_ptr()),
                                        out.numel(), ctypes.byref(cnt), _lib.DSX_OUT_DEVICE),
                       ctx.h)
            torch.cuda.synchronize()
            # the piece had two region sizes (the geometry this test is about)
            assert ctx.stats().pieces == 1
            return out[:cnt.value].cpu().numpy().copy()
        finally:
            ctx.close()

    exact = run(0)
    assert exact.size > N // (128 << 10), exact.size
    for v in VARIANTS:
        got = run(v)
        if v in EXACT:
            assert np.array_equal(got, exact), f"trace variant {v} changed the cut list"
        print(f"variant {v} ok ({got.size} cuts)", flush=True)
    os.environ.pop("DSX_SCAN_VARIANT", None)


if __name__ == "__main__":
    sys.path.insert(0, REPO)
    _main()
