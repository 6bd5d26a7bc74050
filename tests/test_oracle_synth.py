"""The host twins of the device workload generators (oracle/dsx_oracle.c
dsxo_gen_uniform / dsxo_gen_dedup, mirroring desync_amd/csrc/dsx_gen.hip).
The GPU tests compare device bytes with these before comparing cut lists."""
import numpy as np
import pytest

from oracle import oracle as o

MiB = 1 << 20


@pytest.mark.parametrize("offset,length", [(0, 1), (0, 4096), (3, 1000), (12345, 77777),
                                           ((5 << 30) + 7, 3 * MiB + 5)])
def test_uniform_c_equals_numpy(offset, length):
    a = o.synth_uniform_c(1, offset, length, threads=3)
    b = o.synth_uniform(1, offset, length)
    assert np.array_equal(a, b)


def test_dedup_stream_shape():
    """BASELINE config 3: ~30 % of the 1 MiB blocks are byte copies of an
    earlier block; the others are the uniform stream's own bytes."""
    nblk = 16384  # 16 GiB worth of blocks
    roots = o.dedup_roots(2, nblk)
    assert roots[0] == 0 and np.all(roots <= np.arange(nblk, dtype=np.uint64))
    frac = float(np.mean(roots != np.arange(nblk, dtype=np.uint64)))
    assert 0.28 < frac < 0.32, frac
    # bytes: a window straddling fresh and repeated blocks
    rep = [b for b in range(1, 64) if roots[b] != b]
    fresh = [b for b in range(1, 64) if roots[b] == b]
    assert rep and fresh
    for b in rep[:3] + fresh[:3]:
        got = o.synth_dedup(2, b * MiB - 100, MiB + 200, threads=2)
        r0, r1 = int(roots[b - 1]), int(roots[b])
        want = np.concatenate([o.synth_uniform(2, r0 * MiB + MiB - 100, 100),
                               o.synth_uniform(2, r1 * MiB, MiB),
                               o.synth_uniform(2, int(roots[b + 1]) * MiB, 100)])
        assert np.array_equal(got, want), b
