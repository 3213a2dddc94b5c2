// Layouts behind the opaque Input_t / Output_t of the operator ABI (include/dora_operator_api.h),
// shared by the helpers in libdora_gpu.so (operator_api.cpp) and the runtime (dora-gpu-runtime):
// the counterparts of `Input` / `Output` in apis/rust/operator/types/src/lib.rs:99-136.
#pragma once

#include <string>

#include "dora_gpu.h"
#include "dora_operator_api.h"

// An input handed to an operator: its Arrow array in host memory (owned, released with the
// input), read once through dora_read_data like the reference's `data_array.take()`.
struct Input {
  std::string id;
  ArrowArray array{};
  ArrowSchema schema{};
  bool taken = false;
  std::string open_telemetry_context;
  ~Input() {
    if (array.release) array.release(&array);
    if (schema.release) schema.release(&schema);
  }
};

// An output on its way from an operator to the runtime, passed by value through the
// SendOutput closure: plain data, the callee takes ownership of all of it.
struct Output {
  char* id;            // malloc'ed
  ArrowArray array;    // moved in: the callee releases it
  ArrowSchema schema;  // moved in: the callee releases it
};
