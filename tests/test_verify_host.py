"""Host logic of VerifyIndex (verifyindex.go:13-79) that runs before any GPU
call: the size check and its exact message, progress-bar bracketing, and an
empty index.  The digest comparison itself is a GPU test
(tests/test_gpu_parity.py::test_verify_index_*)."""
import os

import pytest

import desync_amd

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _read(name):
    with open(os.path.join(GOLDEN, name), "rb") as f:
        return f.read()


class _PB:
    def __init__(self):
        self.calls = []

    def SetTotal(self, n):
        self.calls.append(("SetTotal", n))

    def Start(self):
        self.calls.append(("Start",))

    def Add(self, n):
        self.calls.append(("Add", n))

    def Finish(self):
        self.calls.append(("Finish",))


def test_size_mismatch_message(tmp_path):
    index = desync_amd.IndexFromReader(_read("blob1.caibx"))
    f = tmp_path / "short"
    f.write_bytes(_read("blob1")[:-1])
    pb = _PB()
    with pytest.raises(desync_amd.VerifyError) as e:
        desync_amd.VerifyIndex(None, str(f), index, 10, pb)
    n = index.Length()
    assert str(e.value) == f"index size ({n}) does not match file size ({n - 1})"
    assert pb.calls == [("SetTotal", len(index.Chunks)), ("Start",), ("Finish",)]


def test_missing_file(tmp_path):
    index = desync_amd.IndexFromReader(_read("blob1.caibx"))
    with pytest.raises(FileNotFoundError):
        desync_amd.VerifyIndex(None, str(tmp_path / "nope"), index, 1)


def test_empty_index_empty_file(tmp_path):
    f = tmp_path / "empty"
    f.write_bytes(b"")
    index = desync_amd.Index(desync_amd.FormatIndex(0, 16, 64, 256), [])
    assert desync_amd.VerifyIndex(None, str(f), index, 1) is None


def test_chunk_arrays_and_runs():
    """VerifyIndex's chunk list as arrays: a decoded caibx (ChunkArray) gives
    its arrays without building chunk objects and is one run; a hand-built
    list with a gap and an overlap splits into runs at exactly those chunks,
    and a wrong-length ID is flagged (it can only mismatch)."""
    import numpy as np

    from desync_amd import make
    from desync_amd.index import ChunkArray
    index = desync_amd.IndexFromReader(_read("blob1.caibx"))
    starts, ends, ids, bad = make._chunk_arrays(index.Chunks)  # a list of IndexChunk
    assert bad is None and ids.shape == (len(index.Chunks), 32)
    assert make._contiguous_runs(starts, ends) == [(0, len(index.Chunks))]
    arr = ChunkArray(ends, ids)  # IndexFromFile's form
    s2, e2, i2, b2 = make._chunk_arrays(arr)
    assert arr._list is None  # nothing materialised
    assert b2 is None and np.array_equal(s2, starts) and np.array_equal(e2, ends)
    assert np.array_equal(i2, ids) and bytes(i2[3]) == index.Chunks[3].ID
    c = desync_amd.IndexChunk
    hand = [c(b"a" * 32, 0, 10), c(b"b" * 32, 10, 5), c(b"c" * 32, 20, 4),
            c(b"d" * 31, 22, 8), c(b"e" * 32, 30, 1)]
    starts, ends, ids, bad = make._chunk_arrays(hand)
    assert make._contiguous_runs(starts, ends) == [(0, 2), (2, 3), (3, 5)]
    assert bad.tolist() == [False, False, False, True, False]
    assert bytes(ids[4]) == b"e" * 32 and int(ends[3]) == 30
    assert make._contiguous_runs(np.zeros(0, np.uint64), np.zeros(0, np.uint64)) == [(0, 0)]
