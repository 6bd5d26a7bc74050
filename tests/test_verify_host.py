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
