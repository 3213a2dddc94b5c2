// Shared helpers for the dora-gpu C ABI: error reporting and HIP checks.
#pragma once

#include <hip/hip_runtime_api.h>

#include <cstdarg>
#include <cstdio>
#include <string>

#include "dora_gpu.h"

namespace dora {

void set_error(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
void clear_error();

// Return `code` after recording a formatted message.
int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));

// Process-wide diagnostics (dora_gpu_busy_stats): host time spent blocked on an empty control
// ring (idle) and spinning on a producer's fill flag, so a pipeline's bottleneck process shows
// as the one with no idle time.
void add_idle_ns(uint64_t ns);
void add_fill_wait_ns(uint64_t ns);

}  // namespace dora

#define DORA_HIP(expr)                                                                  \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess) {                                                             \
      ::dora::set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e), __FILE__, \
                        __LINE__);                                                      \
      return DORA_ERR_HIP;                                                              \
    }                                                                                   \
  } while (0)

// Wrap a C++ body that may throw into a C status.
#define DORA_GUARD_BEGIN try {
#define DORA_GUARD_END                                                     \
  }                                                                        \
  catch (const std::bad_alloc&) {                                          \
    return ::dora::fail(DORA_ERR_INVALID, "out of host memory");           \
  }                                                                        \
  catch (const std::exception& e) {                                        \
    return ::dora::fail(DORA_ERR_INVALID, "internal error: %s", e.what()); \
  }
