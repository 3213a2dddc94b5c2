/*
 * TEST INFRASTRUCTURE ONLY — plain-C restatement of the reference CPU pack path, used as the
 * checker's C twin of oracle/checksum_ref.py and as the CPU baseline kernel (`bench.py`
 * cpu_baseline leg).  Never linked into the product.
 *
 *  - oracle_copy_segments: the `target_buffer[off..][..len].copy_from_slice(buffer)` loop of
 *    copy_array_into_sample_inner (apis/rust/node/src/node/arrow_utils.rs:48), one memcpy per
 *    buffer, single thread, exactly as the reference runs it.
 *  - oracle_csum64 / oracle_splitmix: the parity checksum and payload generator
 *    (oracle/checksum_ref.py).
 */
#include <stdint.h>
#include <string.h>

#define GOLDEN 0x9E3779B97F4A7C15ull
#define SEED 0xD0A5D0A5D0A5D0A5ull

static inline uint64_t fmix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

void oracle_copy_segments(uint8_t* dst, const void* const* srcs, const uint64_t* offs,
                          const uint64_t* lens, uint64_t n) {
  for (uint64_t i = 0; i < n; ++i) memcpy(dst + offs[i], srcs[i], lens[i]);
}

uint64_t oracle_csum64(const uint8_t* p, uint64_t n) {
  uint64_t s = 0, nw = (n + 7) / 8;
  for (uint64_t i = 0; i < nw; ++i) {
    uint64_t w = 0;
    uint64_t lim = (8 * i + 8 <= n) ? 8 : n - 8 * i;
    memcpy(&w, p + 8 * i, lim);
    s += fmix64(w ^ (i * GOLDEN + SEED));
  }
  return fmix64(s + n);
}

void oracle_splitmix(uint8_t* p, uint64_t n, uint64_t seed) {
  for (uint64_t i = 0; 8 * i < n; ++i) {
    uint64_t w = fmix64(seed + (i + 1) * GOLDEN);
    uint64_t lim = (8 * i + 8 <= n) ? 8 : n - 8 * i;
    memcpy(p + 8 * i, &w, lim);
  }
}
