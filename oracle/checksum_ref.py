"""TEST INFRASTRUCTURE ONLY — numpy restatement of the payload generator and the parity checksum.

* `splitmix_bytes(n, seed)`: the seeded UInt8 payload of BASELINE.md §2 (splitmix64 with
  seed = 0xD05A + size; the reference uses an unseeded `thread_rng`,
  examples/benchmark/node/src/main.rs:29-33).  Byte k is byte (k % 8) of the little-endian
  64-bit output number k // 8.
* `csum64(data)`: position-sensitive, order-independent-sum checksum used for size-independent
  parity at full sizes (SURVEY.md §8c "checksum over the DFS concatenation"):
      word_i = little-endian u64 i of data (tail zero-padded)
      S      = sum_i fmix64(word_i ^ (i * GOLDEN + SEED))  (mod 2^64)
      csum   = fmix64(S + len(data))
  `combine(acc, c) = fmix64(acc + c * GOLDEN)` folds region checksums in DFS order.
The product computes the same quantities with HIP kernels (dora_amd/csrc/checksum.hip).
"""
from __future__ import annotations

import numpy as np

GOLDEN = np.uint64(0x9E3779B97F4A7C15)
SEED = np.uint64(0xD0A5D0A5D0A5D0A5)
M1 = np.uint64(0xBF58476D1CE4E5B9)
M2 = np.uint64(0x94D049BB133111EB)
MASK = (1 << 64) - 1


def fmix64_np(z):
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * M1
        z = (z ^ (z >> np.uint64(27))) * M2
        return z ^ (z >> np.uint64(31))


def fmix64(z: int) -> int:
    z &= MASK
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & MASK
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & MASK
    return z ^ (z >> 31)


def splitmix_bytes(n: int, seed: int) -> bytes:
    nw = (n + 7) // 8
    with np.errstate(over="ignore"):
        state = np.uint64(seed & MASK) + (np.arange(1, nw + 1, dtype=np.uint64) * GOLDEN)
    words = fmix64_np(state)
    return words.astype("<u8").tobytes()[:n]


def payload_seed(size: int) -> int:
    return 0xD05A + size


def csum64(data) -> int:
    buf = bytes(data) if not isinstance(data, (bytes, bytearray, memoryview)) else data
    n = len(buf)
    nw = (n + 7) // 8
    padded = bytes(buf) + b"\0" * (nw * 8 - n)
    words = np.frombuffer(padded, dtype="<u8").astype(np.uint64)
    with np.errstate(over="ignore"):
        idx = np.arange(nw, dtype=np.uint64) * GOLDEN + SEED
        s = int(fmix64_np(words ^ idx).sum(dtype=np.uint64)) if nw else 0
    return fmix64((s + n) & MASK)


def combine(acc: int, c: int) -> int:
    return fmix64((acc + c * 0x9E3779B97F4A7C15) & MASK)


def regions_csum(regions) -> int:
    acc = 0
    for r in regions:
        acc = combine(acc, csum64(r))
    return acc
