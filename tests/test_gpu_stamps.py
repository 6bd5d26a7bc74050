"""In-kernel stamps of the scan launches (dsx_stamps_begin / dsx_stamps_end),
the timing bench.py's roofline reads: one record per stamped launch, in launch
order, with the launch's bytes, a positive duration, every wave counted, and a
shader clock in the MI355X's range; launches after the budget and after
dsx_stamps_end are not recorded, and stamping does not change a cut list."""
import ctypes

import numpy as np
import pytest

from oracle import oracle as o

pytestmark = pytest.mark.gpu

MIN, AVG, MAX = 16 * 1024, 64 * 1024, 256 * 1024


def test_scan_stamps():
    import torch

    import desync_amd
    from desync_amd import _lib
    ctx = _lib.Context(0)
    try:
        n = (64 << 20) + 4096
        arr = o.synth_uniform(71, 0, n)
        ref = o.chunk_stream(arr, MIN, AVG, MAX)
        t = torch.from_numpy(arr).to("cuda")
        p = desync_amd.Params(MIN, AVG, MAX)
        L = _lib.lib()
        outs = [torch.empty(n // MIN + 4, dtype=torch.int64, device="cuda") for _ in range(6)]
        cnt = ctypes.c_uint64()
        ctx.stamps_begin(4)
        for s in range(6):  # 6 queued jobs, 4 stamped
            _lib.check(L.dsx_cut_device(ctx.h, ctypes.c_void_p(t.data_ptr()), n, ctypes.byref(p.c),
                                        ctypes.c_void_p(outs[s].data_ptr()), n // MIN + 4,
                                        ctypes.byref(cnt), _lib.DSX_OUT_DEVICE | _lib.DSX_NO_SYNC),
                       ctx.h)
        for s in range(6):
            _lib.check(L.dsx_result(ctx.h, ctypes.byref(cnt)), ctx.h)
            assert np.array_equal(outs[s][:cnt.value].cpu().numpy().astype(np.uint64), ref)
        st = ctx.stamps_end()
        assert len(st) == 4
        seqs = [r.seq for r in st]
        assert seqs == sorted(seqs) and len(set(seqs)) == 4
        for r in st:
            assert r.bytes == n
            assert r.t_last > r.t_first and 0.001 < r.ms < 50.0
            assert r.waves >= 64  # every wave of the grid stamps once
            assert 500.0 < r.mhz < 3000.0, r.mhz
        # not stamping: dsx_stamps_end without a begin is a state error
        with pytest.raises(_lib.DsxError):
            ctx.stamps_end()
    finally:
        ctx.close()
