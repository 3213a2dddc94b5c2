// Host sub-phase profile of the per-message path (diagnostics only): DORA_GPU_TRACE (a trace
// directory, or "subphases") makes
// every process accumulate TSC ticks per named span of send / route / receive and print one JSON
// line {"subphases": {name: [ns per call, calls]}} to stderr at exit.  Off by default: one
// predictable branch per span.
#pragma once

#include <x86intrin.h>

#include <cstdint>

namespace dora {

enum SubPhase : int {
  SP_SEND_PLAN = 0,   // send_output_bytes: one-buffer plan built
  SP_ALLOC_TOKENS,    // alloc_sample: returned tokens handled
  SP_ALLOC_WAIT,      // alloc_sample: in-flight cap wait
  SP_ALLOC_SLOT,      // allocate_slot (cache scan + last-fill check)
  SP_STREAM_QUERY,    // fill_sample: node stream idle check
  SP_AQL_PACK,        // aql_pack total
  SP_AQL_ARGS,        // aql_pack: argument build + copy
  SP_AQL_DISPATCH,    // aql_pack: packet write + doorbell
  SP_SEND_TI,         // pack_and_send: type info bytes
  SP_SEND_TOKENS,     // send_sample: returned tokens handled
  SP_SEND_LOOKUP,     // send_sample: output lookup
  SP_SEND_REQUEST,    // send_sample: descriptor encoded and pushed
  SP_SEND_TRACK,      // send_sample: token -> slot map insert
  SP_RECV_DRAIN,      // next_event: ring drained into events
  SP_RECV_ENCODE,     // encode_event (one event)
  SP_RECV_DROPOLD,    // drop_oldest_inputs
  SP_RECV_FINISH,     // finish_input (fill wait included)
  SP_RECV_RELEASE,    // InputData release: token reported
  SP_DAEMON_ROUTE,    // daemon: one request handled
  SP_SLOT_FLAG,       // allocate_slot: the reused slot's last-fill check
  SP_SAMPLE_NEW,      // alloc_sample: the sample object
  SP_SEND_SOURCE_WAIT,  // pack_and_send: a synchronous send waits for its pack to read the source
  SP_COUNT
};

extern const bool g_subprof_on;  // DORA_GPU_TRACE set, read at load time
inline bool subprof_enabled() { return g_subprof_on; }
void subprof_add(int phase, uint64_t ticks);

struct SubSpan {
  int phase;
  uint64_t t0;
  explicit SubSpan(int p) : phase(p), t0(subprof_enabled() ? __rdtsc() : 0) {}
  void stop() {
    if (t0) subprof_add(phase, __rdtsc() - t0);
    t0 = 0;
  }
  ~SubSpan() { stop(); }
};

}  // namespace dora
