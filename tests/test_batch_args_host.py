"""Host side of the batch pack (aql.cpp / kernels.hip `build_aql_batch_args`), on the CPU: the
640-byte argument block of `dora_aql_packb_u4` for several messages — segments sorted by
absolute destination, chunk bounds, each message's stitched-edge bits carried to its segments'
sorted positions, one fill flag / epoch per message — against a Python statement of the same
rules (pack_device.h `segment_chunks`, kernels.hip `edge_mask`)."""
import ctypes
import struct

import pytest

from dora_amd import _lib

ARGS_BYTES = 640
MAX_SEGS = 16
LINE = 128


def segment_chunks(d0, length, chunk):
    a0 = (d0 + 15) & ~15
    a1 = (d0 + length) & ~15
    if a1 <= a0:
        return 1
    o = a0 & ~(LINE - 1)
    return (a1 - o + chunk - 1) // chunk


def edge_mask(segs, dst, cap):
    if not cap:
        return 0
    for k in range(1, len(segs)):
        if segs[k][1] < segs[k - 1][1] + segs[k - 1][2]:
            return 0

    def inside(u):
        return u >= dst and u + 16 <= dst + cap
    m = 0
    for k, (_, off, n) in enumerate(segs):
        d0, d1 = dst + off, dst + off + n
        if d1 == d0:
            continue
        a0 = (d0 + 15) & ~15
        if a0 > d0 and inside(a0 - 16):
            m |= 1 << (2 * k)
        if a0 < d1 and (d1 & 15) and inside(d1 & ~15):
            m |= 2 << (2 * k)
    return m


def build(msgs):
    """msgs: [(dst, cap, flag, epoch, [(src, dst_off, len), ...])] -> (args bytes, grid)."""
    lib = _lib.load_testing()
    n = len(msgs)
    counts = (ctypes.c_size_t * n)(*[len(m[4]) for m in msgs])
    flat = [x for m in msgs for s in m[4] for x in s]
    segs = (ctypes.c_uint64 * max(1, len(flat)))(*flat)
    arr = lambda i: (ctypes.c_uint64 * n)(*[m[i] for m in msgs])  # noqa: E731
    out = ctypes.create_string_buffer(ARGS_BYTES)
    grid = ctypes.c_uint32()
    rc = lib.dora_gpu_test_batch_args(n, counts, segs, arr(0), arr(1), arr(2), arr(3), out,
                                      ARGS_BYTES, ctypes.byref(grid))
    return rc, out.raw, grid.value


def parse(raw):
    dst, flag, done, epoch = struct.unpack_from("<4Q", raw, 0)
    n_chunks, nseg, chunk, grid = struct.unpack_from("<4I", raw, 32)
    edge, = struct.unpack_from("<Q", raw, 48)
    nmsg, = struct.unpack_from("<I", raw, 56)
    chunk_end = struct.unpack_from(f"<{MAX_SEGS}I", raw, 64)
    seg = [struct.unpack_from("<3Q", raw, 128 + 24 * k) for k in range(MAX_SEGS)]
    msg = [struct.unpack_from("<2Q", raw, 512 + 16 * k) for k in range(8)]
    return dict(dst=dst, flag=flag, done=done, epoch=epoch, n_chunks=n_chunks, nseg=nseg,
                chunk=chunk, grid=grid, edge=edge, nmsg=nmsg, chunk_end=chunk_end, seg=seg,
                msg=msg)


MiB2 = 2 << 20


def _msgs():
    # slots out of address order; segments with unaligned heads / tails; the middle message
    # is a nested sample (list offsets at 0, values at 4 mod 16), the others raw payloads
    a, b, c = 0x7F0000400000, 0x7F0000000000, 0x7F0000800000
    return [
        (a, MiB2, 0x1000, 7, [(0x10000003, 0, 100003)]),
        (b, MiB2, 0x1040, 8, [(0x20000000, 0, 68), (0x20001000, 68, 40000),
                              (0x20011000, 40068, 40000), (0x20021000, 80068, 10001)]),
        (c, 0, 0x1080, 9, [(0x30000005, 0, 4096)]),
    ]


def test_batch_args_sorted_segments_chunks_edges_and_flags():
    msgs = _msgs()
    rc, raw, grid = build(msgs)
    assert rc == 0, _lib.load().dora_gpu_last_error()
    p = parse(raw)
    assert p["dst"] == 0 and p["nmsg"] == 3 and p["nseg"] == 6
    # segments: absolute destinations, sorted
    want = []
    for dst, cap, _, _, segs in msgs:
        em = edge_mask(segs, dst, cap)
        for k, (src, off, n) in enumerate(segs):
            want.append((dst + off, src, n, (em >> (2 * k)) & 3))
    want.sort()
    chunk = p["chunk"]
    assert chunk == 8192
    total = 0
    for k, (d, src, n, e) in enumerate(want):
        assert p["seg"][k] == (src, d, n), k
        total += segment_chunks(d, n, chunk)
        assert p["chunk_end"][k] == total, k
        assert (p["edge"] >> (2 * k)) & 3 == e, k
    assert p["n_chunks"] == total and grid == p["grid"] == min(total, 1024)
    # stitched edges exist where the slot can take a whole unit (message 0's ragged tail,
    # message 1's joints) and not for the message without a writable capacity
    assert p["edge"] != 0
    # one flag / epoch per message, the launch's done words and epoch are message 0's
    assert p["msg"][:3] == [(0x1000, 7), (0x1040, 8), (0x1080, 9)]
    assert p["flag"] == 0x1000 and p["epoch"] == 7


def test_batch_args_refuses_mixed_chunks_and_too_many_segments():
    lib = _lib.load_testing()
    small = (0x7F0000000000, MiB2, 0x1000, 1, [(0x10000000, 0, 4096)])
    big = (0x7F0002000000, 1 << 25, 0x1040, 2, [(0x20000000, 0, 30 << 20)])  # 16 KiB chunks
    rc, _, _ = build([small, big])
    assert rc == -1 and b"chunk" in _lib.load().dora_gpu_last_error()
    many = [(0x7F0000000000 + m * MiB2, MiB2, 0x1000 + 64 * m, m,
             [(0x10000000, 4096 * j, 4096) for j in range(3)]) for m in range(6)]
    rc, _, _ = build(many)   # 18 segments > 16
    assert rc == -1 and b"segments" in _lib.load().dora_gpu_last_error()


@pytest.mark.parametrize("n", [1, 8])
def test_batch_args_message_counts(n):
    msgs = [(0x7F0000000000 + m * MiB2, MiB2, 0x1000 + 64 * m, 100 + m,
             [(0x10000000 + m, 0, 65536 + 17 * m)]) for m in range(n)]
    rc, raw, _ = build(msgs)
    assert rc == 0
    p = parse(raw)
    assert p["nmsg"] == n and p["nseg"] == n
    assert [p["msg"][m] for m in range(n)] == [(0x1000 + 64 * m, 100 + m) for m in range(n)]
