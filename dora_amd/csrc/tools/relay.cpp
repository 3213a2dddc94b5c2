// dora-gpu-relay: forwards every input to the output of the same name with the same parameters
// (inputs `latency`, `throughput` -> outputs `latency`, `throughput`) — one stage
// of the C5 pipeline (BASELINE.json configs[4]: one node per GPU, peer copies over xGMI).  An
// input whose slot lives on another GPU is copied over xGMI straight into the relay's own output
// slot (dora_node_forward), which the next stage pulls in turn.
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
      const uint8_t* params = nullptr;
      size_t plen = 0;
      dora_event_parameters(ev, &params, &plen);
      // one copy per hop: a cross-GPU input goes from the peer's slot straight into ours
      int rc = dora_node_forward(node, dora_event_id(ev), ev, params, plen);
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
