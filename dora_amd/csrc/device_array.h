// Internal: receiver-side import of a device sample (used by the node API).
#pragma once

#include <cstddef>
#include <cstdint>
#include <memory>
#include <vector>

#include "dora_gpu.h"

namespace dora {

// `keep` is held by every imported ArrowArray node until released (the received slot).
// `ext_len` (>= sample_len, 0 = sample_len): readable bytes of the slot incl. the validity tail
// that type infos with in-sample bitmaps (tag 2) point into.  `host`: the sample is in host
// memory (inline Vec sample): bitmaps and empty buffers are host allocations, no HIP call.
int import_sample(const void* sample, uint64_t sample_len, const uint8_t* type_info,
                  size_t type_info_len, std::shared_ptr<void> keep, ArrowArray* out_array,
                  ArrowSchema* out_schema, uint64_t ext_len = 0, bool host = false);

// The reference (inline) form of a type info: in-sample bitmaps (tag 2) read back from the
// device sample into tag-1 bytes.  `*changed` = false (out untouched) when there were none.
// `host`: the sample is in host memory (a staged copy), read without HIP.
int inline_type_info(const uint8_t* type_info, size_t type_info_len, const void* sample,
                     uint64_t ext_len, std::vector<uint8_t>* out, bool* changed,
                     bool host = false);

}  // namespace dora
