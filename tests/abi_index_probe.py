"""A caller of libdsx.so that uses nothing but the C ABI (ctypes, struct, os):
the shape of the cgo binding in INTEGRATION.md.  Run as a subprocess by
tests/test_gpu_index.py; it must never import torch.

For each (input, golden caibx) pair it calls dsx_index_fd (file -> cut list
+ SHA-512/256 chunk IDs, all on the GPU), writes the caibx bytes the way
Index.WriteTo does (index.go:90-124, format.go:582-620; flags as in
IndexFromFile, make.go:35-62) and compares them with the golden file; then
re-hashes the golden table's own chunk list with dsx_ids_fd (VerifyIndex's
data path, verifyindex.go:13-79) and compares the IDs with the table's.
Prints "ok <n>" per file; exits non-zero on a mismatch.
"""
import ctypes
import os
import struct
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(REPO, "desync_amd", "libdsx.so")
GOLDEN = os.path.join(REPO, "tests", "golden")

CA_FORMAT_ENTRY = 0x1396FABCEA5BBB51
CA_FORMAT_INDEX = 0x96824D9C7B129FF9
CA_FORMAT_TABLE = 0xE75B9E112F17417D
CA_FORMAT_TAIL = 0x4B4F050E5549ECD1
SHA512256 = 0x2000000000000000
EXCLUDE_NO_DUMP = 0x8000000000000000


class Params(ctypes.Structure):
    _fields_ = [("min", ctypes.c_uint64), ("avg", ctypes.c_uint64), ("max", ctypes.c_uint64),
                ("d", ctypes.c_uint32), ("inv", ctypes.c_uint32), ("qmax", ctypes.c_uint32),
                ("qbias", ctypes.c_uint32), ("rot", ctypes.c_int32), ("res", ctypes.c_uint32)]


def caibx(flags, mn, av, mx, ends, ids):
    out = bytearray(struct.pack("<6Q", 48, CA_FORMAT_INDEX, flags, mn, av, mx))
    out += struct.pack("<2Q", 0xFFFFFFFFFFFFFFFF, CA_FORMAT_TABLE)
    for e, i in zip(ends, ids):
        out += struct.pack("<Q", e) + i
    out += struct.pack("<5Q", 0, 0, 48, 16 + 40 * len(ends) + 40, CA_FORMAT_TAIL)
    return bytes(out)


def main():
    L = ctypes.CDLL(LIB)
    u64, vp = ctypes.c_uint64, ctypes.c_void_p
    L.dsx_params_init.argtypes = [u64, u64, u64, ctypes.POINTER(Params)]
    L.dsx_ctx_create.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
    L.dsx_ctx_destroy.argtypes = [vp]
    L.dsx_last_error.restype = ctypes.c_char_p
    L.dsx_last_error.argtypes = [vp]
    L.dsx_index_fd.argtypes = [vp, ctypes.c_int, u64, u64, ctypes.POINTER(Params), ctypes.c_int,
                               vp, vp, u64, ctypes.POINTER(u64)]
    L.dsx_ids_fd.argtypes = [vp, ctypes.c_int, u64, u64, u64, vp, u64, ctypes.c_int, vp]
    ctx = vp()
    assert L.dsx_ctx_create(0, ctypes.byref(ctx)) == 0, L.dsx_last_error(None)
    pairs = [("chunker.input", "chunker.index"), ("blob1", "blob1.caibx"), ("blob2", "blob2.caibx"),
             ("tree.catar", "tree.caidx")]
    bad = 0
    for inp, idx in pairs:
        with open(os.path.join(GOLDEN, idx), "rb") as f:
            want = f.read()
        _, _, _, mn, av, mx = struct.unpack_from("<6Q", want, 0)
        p = Params()
        assert L.dsx_params_init(mn, av, mx, ctypes.byref(p)) == 0
        fd = os.open(os.path.join(GOLDEN, inp), os.O_RDONLY)
        try:
            head = os.pread(fd, 64, 0)
            flags = EXCLUDE_NO_DUMP | SHA512256
            if len(head) >= 64:
                size, typ, ff = struct.unpack_from("<3Q", head, 0)
                if typ == CA_FORMAT_ENTRY and size == 64:
                    flags |= ff
            cap = os.fstat(fd).st_size // mn + 2
            ends = (u64 * cap)()
            ids = (ctypes.c_uint8 * (32 * cap))()
            n = u64()
            rc = L.dsx_index_fd(ctx, fd, 0, 0xFFFFFFFFFFFFFFFF, ctypes.byref(p), 0, ends, ids, cap,
                                ctypes.byref(n))
            # VerifyIndex's re-hash (dsx_ids_fd) over the golden table's own
            # chunk list: items of 40 bytes {end offset, ID} after 64 header bytes
            nt = (len(want) - 64 - 40) // 40
            gends = (u64 * nt)(*[struct.unpack_from("<Q", want, 64 + 40 * i)[0] for i in range(nt)])
            gids = [want[64 + 40 * i + 8:64 + 40 * i + 40] for i in range(nt)]
            vids = (ctypes.c_uint8 * (32 * max(nt, 1)))()
            vrc = L.dsx_ids_fd(ctx, fd, 0, 0xFFFFFFFFFFFFFFFF, 0, gends, nt, 0, vids)
        finally:
            os.close(fd)
        assert rc == 0, (rc, L.dsx_last_error(ctx))
        got = caibx(flags, mn, av, mx, list(ends[:n.value]),
                    [bytes(ids[32 * i:32 * i + 32]) for i in range(n.value)])
        assert vrc == 0, (vrc, L.dsx_last_error(ctx))
        if [bytes(vids[32 * i:32 * i + 32]) for i in range(nt)] != gids:
            bad += 1
            print("IDS MISMATCH", inp)
        elif got != want:
            bad += 1
            print("MISMATCH", inp)
        else:
            print("ok", inp, n.value)
    L.dsx_ctx_destroy(ctx)
    assert "torch" not in sys.modules, "the C-ABI probe must not import torch"
    print("torch imported:", "torch" in sys.modules)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
