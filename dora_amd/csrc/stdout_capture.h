// `send_stdout_as` (binaries/daemon/src/spawn.rs:280-437): a node's stdout and stderr lines,
// each batch sent as a one-element Utf8 array on one of its outputs.
#pragma once

#include <cstdint>
#include <functional>
#include <string>
#include <vector>

namespace dora {

// Sends one request (kind, payload) on the node's control ring (thread-safe).
using RequestFn = std::function<int(uint32_t, const std::vector<uint8_t>&)>;

class StdoutCapture;

// Redirect fd 1 and 2 through pipes: every byte still reaches the original descriptors, and
// every line batch is sent on `output`.  nullptr (and nothing changed) on failure.
StdoutCapture* stdout_capture_start(const std::string& output, RequestFn request);
// Restore fd 1 and 2, send what is still buffered, join the readers.
void stdout_capture_stop(StdoutCapture* c);

}  // namespace dora
