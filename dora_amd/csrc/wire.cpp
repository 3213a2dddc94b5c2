// DropToken generation: UUIDv7 like `DropToken::generate` (libraries/message/src/common.rs:181-183).
#include <time.h>

#include <atomic>
#include <random>

#include "shm.h"
#include "wire.h"

namespace dora {

// 48-bit ms timestamp, version 7, 74 random bits: a per-thread splitmix64 sequence seeded from
// the OS (each output is a bijection of a distinct counter value, so a thread never repeats one)
// and the coarse realtime clock, which has ms resolution and costs no system call (mt19937 +
// CLOCK_REALTIME cost ~80 ns per token).
DropToken generate_drop_token() {
  thread_local uint64_t state = [] {
    std::random_device rd;
    return (uint64_t(rd()) << 32) ^ uint64_t(rd()) ^ now_ns();
  }();
  auto mix = [](uint64_t z) {
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  };
  timespec ts;
  clock_gettime(CLOCK_REALTIME_COARSE, &ts);
  const uint64_t ms = uint64_t(ts.tv_sec) * 1000u + uint64_t(ts.tv_nsec) / 1000000u;
  state += 0x9E3779B97F4A7C15ull;
  const uint64_t r1 = mix(state);
  const uint64_t r2 = mix(state ^ 0xD1B54A32D192ED03ull);
  DropToken t;
  for (int i = 0; i < 6; ++i) t.b[i] = static_cast<uint8_t>(ms >> (8 * (5 - i)));
  for (int i = 0; i < 2; ++i) t.b[6 + i] = static_cast<uint8_t>(r1 >> (8 * i));
  for (int i = 0; i < 8; ++i) t.b[8 + i] = static_cast<uint8_t>(r2 >> (8 * i));
  t.b[6] = static_cast<uint8_t>(0x70 | (t.b[6] & 0x0F));  // version 7
  t.b[8] = static_cast<uint8_t>(0x80 | (t.b[8] & 0x3F));  // RFC 4122 variant
  return t;
}

}  // namespace dora
