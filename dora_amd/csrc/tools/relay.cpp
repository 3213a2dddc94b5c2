// dora-gpu-relay: forwards every input `in` to output `out` with the same parameters — one stage
// of the C5 pipeline (BASELINE.json configs[4]: one node per GPU, peer copies over xGMI).  An
// input whose slot lives on another GPU arrives already pulled into a local slot (node.cpp); the
// relay then packs it into its own output slot, which the next stage pulls in turn.
//   env: DORA_GPU_DATAFLOW, DORA_NODE_ID, DORA_GPU_DEVICE
#include <cstdio>

#include "dora_gpu.h"

int main() {
  dora_node* node = nullptr;
  if (dora_node_init_from_env(&node) != 0) {
    std::fprintf(stderr, "relay: init failed: %s\n", dora_gpu_last_error());
    return 1;
  }
  int errors = 0;
  for (;;) {
    dora_event* ev = nullptr;
    if (dora_node_next_event(node, -1, &ev) != 0) break;
    const int type = dora_event_type(ev);
    if (type == DORA_EVENT_INPUT) {
      const void* p = nullptr;
      size_t len = 0;
      const uint8_t* params = nullptr;
      size_t plen = 0;
      const uint8_t* ti = nullptr;
      size_t tilen = 0;
      dora_event_data(ev, &p, &len);
      dora_event_parameters(ev, &params, &plen);
      dora_event_type_info(ev, &ti, &tilen);
      int rc;
      if (len == 0) {
        rc = dora_node_send_output_bytes(node, "out", nullptr, 0, ARROW_DEVICE_ROCM, params, plen);
      } else {
        // same type info, fresh sample: allocate, copy on the node stream, send
        dora_sample* s = nullptr;
        rc = dora_node_allocate_data_sample(node, len, &s);
        if (rc == 0) rc = dora_gpu_memcpy_async(dora_sample_data(s), p, len, dora_node_stream(node));
        if (rc == 0) rc = dora_gpu_stream_sync(dora_node_stream(node));
        if (rc == 0) rc = dora_node_send_output_sample(node, "out", ti, tilen, params, plen, s);
      }
      if (rc != 0) {
        std::fprintf(stderr, "relay: forward failed: %s\n", dora_gpu_last_error());
        ++errors;
      }
    } else if (type == DORA_EVENT_ERROR) {
      std::fprintf(stderr, "relay: error event: %s\n", dora_event_error(ev));
      ++errors;
    }
    const bool end = type == DORA_EVENT_ALL_INPUTS_CLOSED || type == DORA_EVENT_STOP;
    dora_event_free(ev);
    if (end) break;
  }
  uint64_t copies = 0, bytes = 0;
  dora_node_peer_stats(node, &copies, &bytes);
  std::printf("{\"relay_peer_copies\": %llu, \"relay_peer_bytes\": %llu, \"errors\": %d}\n",
              (unsigned long long)copies, (unsigned long long)bytes, errors);
  dora_node_free(node);
  return errors ? 1 : 0;
}
