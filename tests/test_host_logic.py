"""Host-side logic of the desync_amd mirror that needs no GPU."""
import os
import stat
import struct

from desync_amd import make


def test_file_size_regular(tmp_path):
    f = tmp_path / "x"
    f.write_bytes(b"a" * 12345)
    fd = os.open(str(f), os.O_RDONLY)
    try:
        assert make.file_size(fd) == 12345
    finally:
        os.close(fd)


def test_file_size_block_device(monkeypatch, tmp_path):
    """GetFileSize (ioctl_linux.go:63-84): a block device's st_size is 0, its
    size comes from the BLKGETSIZE64 ioctl (mocked: no loop devices here)."""
    import fcntl
    f = tmp_path / "dev"
    f.write_bytes(b"")
    real_fstat = os.fstat

    class St:
        def __init__(self, s):
            self.st_mode = stat.S_IFBLK | 0o660
            self.st_size = 0

    calls = []

    def fake_ioctl(fd, req, arg):
        calls.append(req)
        assert req == 0x80081272  # BLKGETSIZE64 = _IOR(0x12, 114, size_t)
        return struct.pack("Q", 7 << 30)

    monkeypatch.setattr(os, "fstat", lambda fd: St(real_fstat(fd)))
    monkeypatch.setattr(fcntl, "ioctl", fake_ioctl)
    fd = os.open(str(f), os.O_RDONLY)
    try:
        assert make.file_size(fd) == 7 << 30
    finally:
        os.close(fd)
    assert calls == [0x80081272]
