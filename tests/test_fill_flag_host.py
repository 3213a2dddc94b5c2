"""The fill-flag completion protocol on the host (no GPU): shm.h FillFlag / fill_reached /
cp_arm through the C-ABI test hooks.  A flag line is 128 bytes: the epoch word the in-kernel
signal stores (offset 0), cp_epoch (24), and an amd_signal_t-shaped line (64: kind, 72: value)
whose value the command processor decrements when a CP-signalled pack's dispatch ends."""
import ctypes
import struct

import pytest

from dora_amd import _lib

EPOCH, CP_EPOCH, KIND, VALUE, MAILBOX = 0, 24, 64, 72, 80


@pytest.fixture()
def line():
    raw = ctypes.create_string_buffer(128 + 64)
    base = (ctypes.addressof(raw) + 63) & ~63
    ctypes.memset(base, 0, 128)
    yield raw, base


def _u64(base, off):
    return struct.unpack("<q", ctypes.string_at(base + off, 8))[0]


def _set(base, off, v):
    ctypes.memmove(base + off, struct.pack("<q", v), 8)


def test_in_kernel_epochs_only_grow():
    lib = _lib.load_testing()
    raw = ctypes.create_string_buffer(256)
    base = (ctypes.addressof(raw) + 63) & ~63
    _set(base, EPOCH, 7)
    assert lib.dora_gpu_test_fill_reached(base, 7) == 1
    assert lib.dora_gpu_test_fill_reached(base, 3) == 1  # a later fill covers earlier ones
    assert lib.dora_gpu_test_fill_reached(base, 8) == 0


def test_cp_fill_completes_on_the_decrement(line):
    lib = _lib.load_testing()
    _, base = line
    _set(base, EPOCH, 3)  # the flag's previous (in-kernel) fill
    assert lib.dora_gpu_test_cp_arm(base, 10) == 0
    # amd_signal_t: a user signal with no mailbox (no interrupt), value 1 while the pack runs
    assert _u64(base, KIND) == 1 and _u64(base, MAILBOX) == 0 and _u64(base, VALUE) == 1
    assert _u64(base, CP_EPOCH) == 10 and _u64(base, EPOCH) == 9
    assert lib.dora_gpu_test_fill_reached(base, 10) == 0
    # every earlier epoch of the flag reads complete at once (the previous fill had completed)
    assert all(lib.dora_gpu_test_fill_reached(base, e) == 1 for e in (1, 3, 9))
    _set(base, VALUE, 0)  # the command processor's decrement at the end of the dispatch
    assert lib.dora_gpu_test_fill_reached(base, 10) == 1
    assert lib.dora_gpu_test_fill_reached(base, 11) == 0


def test_flag_switches_between_rules(line):
    """A flag used by a CP-signalled fill, then an in-kernel one, then a CP one again."""
    lib = _lib.load_testing()
    _, base = line
    lib.dora_gpu_test_cp_arm(base, 5)
    _set(base, VALUE, 0)
    assert lib.dora_gpu_test_fill_reached(base, 5) == 1
    # in-kernel fill 8 in flight: 5 stays complete, 8 is not, until the kernel stores 8
    assert lib.dora_gpu_test_fill_reached(base, 8) == 0
    _set(base, EPOCH, 8)
    assert lib.dora_gpu_test_fill_reached(base, 8) == 1
    lib.dora_gpu_test_cp_arm(base, 12)
    assert _u64(base, EPOCH) == 11  # raised to e - 1, never lowered
    assert lib.dora_gpu_test_fill_reached(base, 12) == 0
    assert lib.dora_gpu_test_fill_reached(base, 8) == 1
    _set(base, VALUE, 0)
    assert lib.dora_gpu_test_fill_reached(base, 12) == 1
    # a stale CP completion never completes a different epoch
    assert lib.dora_gpu_test_fill_reached(base, 13) == 0


def test_misaligned_flag_is_rejected(line):
    lib = _lib.load_testing()
    _, base = line
    assert lib.dora_gpu_test_fill_reached(base + 8, 1) < 0
    assert lib.dora_gpu_test_cp_arm(base + 8, 1) < 0
    assert lib.dora_gpu_test_cp_arm(base, 0) < 0
