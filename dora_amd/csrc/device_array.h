// Internal: receiver-side import of a device sample (used by the node API).
#pragma once

#include <cstddef>
#include <cstdint>
#include <memory>

#include "dora_gpu.h"

namespace dora {

// `keep` is held by every imported ArrowArray node until released (the received slot).
int import_sample(const void* sample, uint64_t sample_len, const uint8_t* type_info,
                  size_t type_info_len, std::shared_ptr<void> keep, ArrowArray* out_array,
                  ArrowSchema* out_schema);

}  // namespace dora
