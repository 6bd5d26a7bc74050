"""Pins the CPU oracle to the reference's own golden data (CPU only).

Fixtures in tests/golden/ are byte copies of the reference's test data:
testdata/chunker.input + chunker.index (index_test.go:55-112),
testdata/blob1 + blob1.caibx, cmd/desync/testdata/blob2 + blob2.caibx
(cmd/desync/verifyindex_test.go:13-29), cmd/desync/testdata/tree.catar +
tree.caidx.  The chunk triples are TestChunkerLargeFile's (chunker_test.go:30-49).
"""
import numpy as np
import pytest

from oracle import oracle as o

MIN, AVG, MAX = 16 * 1024, 64 * 1024, 256 * 1024

# chunker_test.go:30-49
LARGE_FILE = [
    (0, 81590, "ad951d7f65c27828ce390f3c81c41d75f80e4527169ad072ad720b56220f5be4"),
    (81590, 46796, "ef6df312072ccefe965f07669b2819902f4e9889ebe7c35a38f1dc11ee99f212"),
    (128386, 36543, "a816e22f4105741972eb34909b6f8ffa569759a1c2cf82ab88394b3db9019f23"),
    (164929, 83172, "8b8e4a274f06dc3c92d49869a699a5a8255c0bf0b48a4d3c3689aaa3e9cff090"),
    (248101, 76749, "583d08fc16d8d191af362a1aaecea6af062cc8afab1b301786bb717aa1b425b4"),
    (324850, 79550, "aefa8c5a3c86896110565b6a3748c2f985892e8ab0073730cac390cb478a913a"),
    (404400, 41484, "8e39f02975c8d0596e46f643b90cd290b7c0386845132eee4d415c63317773a4"),
    (445884, 20326, "d689ca889f2f7ba26896681214f0f0f5f5177d5820d99b1f11ddb76b693bddee"),
    (466210, 31652, "259de367c7ef2f51133d04e744f05918ceb93bd4b9c2bb6621ffeae70501dd09"),
    (497862, 19995, "01ae987ec457cacc8b3528e3254bc9c93b3f0c0b2a51619e15be16e678ef016d"),
    (517857, 103873, "78618b2d0539ecf45c08c7334e1c61051725767a76ba9108ad5298c6fd7cde1b"),
    (621730, 38087, "f44e6992cccadb08d8e18174ba3d6dd6365bdfb9906a58a9f82621ace0461c0d"),
    (659817, 38377, "abbf9935aaa535538c5fbff069481c343c2770207d88b94584314ee33050ae4f"),
    (698194, 23449, "a6c737b95ab514d6538c6ef4c42ef2f08b201c3426a88b95e67e517510cd1fb9"),
    (721643, 47321, "51d44e2d355d5c5b846543d47ba9569f12bbc3d49970c91913a8e3efef45e47e"),
    (768964, 86692, "90f7e061ed2fb1ed9594297851f8528d3ac355c98457b5dce08ee7d88f801b26"),
    (855656, 28268, "2dea144e5d771420e90b6e96c1e97e9c6afeda2c37ae7c95ceaf3ee2550efa08"),
    (883924, 65465, "7a94e051c82ec7abba32883b2eee9a2832e8e9bcc3b3151743fef533e2d46e70"),
    (949389, 33255, "32edd2d382045ad64d5fbd1a574f8191b700b9e0a2406bd90d2eefcf77168846"),
    (982644, 65932, "a8bfdadaecbee1ed16ce23d8bf771d1b3fbca2e631fc71b5adb3846c1bb2d542"),
]

GOLDEN_PAIRS = [
    ("chunker.input", "chunker.index"),
    ("blob1", "blob1.caibx"),
    ("blob2", "blob2.caibx"),
    ("tree.catar", "tree.caidx"),
]


def test_large_file_triples(golden):
    data = golden("chunker.input")
    ends = o.chunk_stream(data, MIN, AVG, MAX)
    starts = [0] + ends[:-1].tolist()
    ids = o.chunk_ids(data, ends)
    got = [(s, int(e) - s, i.hex()) for s, e, i in zip(starts, ends.tolist(), ids)]
    assert got == LARGE_FILE


@pytest.mark.parametrize("inp,idx", GOLDEN_PAIRS)
def test_caibx_bit_identical(golden, inp, idx):
    data, ref = golden(inp), golden(idx)
    d = o.decode_caibx(ref)
    assert o.make_caibx(data, d["min"], d["avg"], d["max"]) == ref


@pytest.mark.parametrize("inp,idx", GOLDEN_PAIRS)
def test_candidate_chain_equals_sequential(golden, inp, idx):
    data = golden(inp)
    d = o.decode_caibx(golden(idx))
    seq = o.chunk_stream(data, d["min"], d["avg"], d["max"])
    cands = o.candidates(data, d["min"], d["avg"], d["max"])
    assert np.array_equal(o.chain(cands, len(data), d["min"], d["max"]), seq)
    assert np.array_equal(seq, d["ends"])


def test_numpy_restatement_matches_c(golden):
    data = golden("blob1")[:300_000]
    P = o.params(2048, 8192, 32768)
    assert np.array_equal(o.candidates_np(data, P.d), o.candidates(data, 2048, 8192, 32768))
    assert np.array_equal(o.chunk_stream_py(data, 2048, 8192, 32768),
                          o.chunk_stream(data, 2048, 8192, 32768))


@pytest.mark.parametrize("n", [1, 2, 3, 5, 8, 10])
def test_parallel_equals_sequential(n):
    """make_test.go:16-80 on reproducible random/null compositions."""
    rng = np.random.default_rng(7)
    null = np.zeros(4 * MAX, np.uint8)
    r1 = rng.integers(0, 256, 4 * MAX, dtype=np.uint8)
    r2 = rng.integers(0, 256, 4 * MAX, dtype=np.uint8)
    for parts in ([r1, r2, r1, r2, r1], [null] * 4 + [r1, r2], [r1, r2] + [null] * 4,
                  [r1] + [null] * 4 + [r2], [r1, null, null, null, r1, null, null, null, r2]):
        data = np.concatenate(parts)
        seq = o.chunk_stream(data, MIN, AVG, MAX)
        assert np.array_equal(o.chunk_parallel(data, MIN, AVG, MAX, n), seq)


def test_edge_cases():
    """chunker_test.go:69-131"""
    assert o.chunk_stream(b"", MIN, AVG, MAX).size == 0  # empty
    assert o.chunk_stream(bytes(range(16)), MIN, AVG, MAX).tolist() == [16]  # small
    zeros = bytes(1024 * 1024)  # no boundary: only max chunks
    ends = o.chunk_stream(zeros, MIN, AVG, MAX)
    assert ends.tolist() == [MAX * (i + 1) for i in range(4)]
    for size in (MIN, AVG, MAX):  # exactly min/avg/max
        assert o.chunk_stream(bytes(size), MIN, AVG, MAX).tolist() == [size]


def test_boundary_test_ranges():
    """chunker_test.go:190-213: multiply-inverse test == h % d == d-1."""
    for avg in (16 * 1024, 64 * 1024, 256 * 1024, 1024 * 1024):
        P = o.params(avg // 4, avg, avg * 4)
        d = P.d
        hs = list(range(0, 3 * d, 997)) + list(range(2**32 - 1 - 3 * d, 2**32, 991))
        hs += [d - 1, 2 * d - 1, 2**32 - 1, (2**32 - 1) // d * d - 1]
        for h in hs:
            assert o.is_boundary(P, h) == (h % d == d - 1), (avg, h)


def test_discriminator_values():
    """d(8K)=6153, d(16K)=12318, d(64K)=49535, ..."""
    assert [o.discriminator(a) for a in (8192, 16384, 65536, 262144, 1 << 20)] == \
        [6153, 12318, 49535, 202440, 886711]


def test_param_errors():
    """chunker.go:135-146 order and messages."""
    with pytest.raises(o.ParamError, match="min chunk size too small, must be over 48"):
        o.params(47, 64, 128)
    with pytest.raises(o.ParamError, match="min chunk size must not be greater than max"):
        o.params(200, 300, 100)
    with pytest.raises(o.ParamError, match="min chunk size must not be greater than avg"):
        o.params(200, 100, 300)
    with pytest.raises(o.ParamError, match="avg chunk size must not be greater than max"):
        o.params(100, 300, 200)


def test_index_test_pattern():
    """index_test.go:119-145 pattern LE64(i*0x9E3779B97F4A7C15) (survey-derived)."""
    i = np.arange(8 * 1024 * 1024 // 8, dtype=np.uint64)
    with np.errstate(over="ignore"):
        data = (i * np.uint64(0x9E3779B97F4A7C15)).view(np.uint8)
    ends = o.chunk_stream(data, MIN, AVG, MAX)
    assert len(ends) == 127
    assert ends[:3].tolist() == [49967, 49967 + 25492, 75459 + 46498]
    assert int(ends[-1]) == 8375948 + 12660 == len(data)
