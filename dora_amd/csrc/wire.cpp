// DropToken generation: UUIDv7 like `DropToken::generate` (libraries/message/src/common.rs:181-183).
#include <atomic>
#include <random>

#include "shm.h"
#include "wire.h"

namespace dora {

DropToken generate_drop_token() {
  static std::atomic<uint64_t> counter{0};
  thread_local std::mt19937_64 rng{std::random_device{}() ^
                                   (uint64_t(std::random_device{}()) << 32)};
  DropToken t;
  const uint64_t ms = now_ns() / 1000000;
  for (int i = 0; i < 6; ++i) t.b[i] = static_cast<uint8_t>(ms >> (8 * (5 - i)));
  const uint64_t r1 = rng() ^ counter.fetch_add(1, std::memory_order_relaxed);
  const uint64_t r2 = rng();
  for (int i = 0; i < 2; ++i) t.b[6 + i] = static_cast<uint8_t>(r1 >> (8 * i));
  for (int i = 0; i < 8; ++i) t.b[8 + i] = static_cast<uint8_t>(r2 >> (8 * i));
  t.b[6] = static_cast<uint8_t>(0x70 | (t.b[6] & 0x0F));  // version 7
  t.b[8] = static_cast<uint8_t>(0x80 | (t.b[8] & 0x3F));  // RFC 4122 variant
  return t;
}

}  // namespace dora
