// Lightweight per-process message tracing (the data-plane part of the reference's tracing spans,
// libraries/extensions/telemetry/tracing): when DORA_GPU_TRACE=<dir> is set, every send /
// route / receive / release of a sample is stamped (CLOCK_REALTIME ns, keyed by drop token) into
// a preallocated buffer and written to <dir>/<who>-<pid>.trace.csv at exit.
#pragma once

#include <cstdint>
#include <string>

#include "wire.h"

namespace dora {

enum TracePoint : uint8_t {
  TP_ALLOC_BEGIN = 1,  // sender: allocate_data_sample entered
  TP_ALLOC_END,        // sender: slot in hand
  TP_LAUNCHED,         // sender: pack kernel enqueued
  TP_FILL_ORDERED,     // sender: fill flag / event / sync issued
  TP_SENT,             // sender: descriptor pushed to the daemon
  TP_TOKEN_BACK,       // sender: OutputDropped received
  TP_ROUTED,           // daemon: Input pushed to a receiver
  TP_TOKEN_DONE,       // daemon: token complete, OutputDropped pushed
  TP_POPPED,           // receiver: event popped from the ring
  TP_FILLED,           // receiver: fill observed complete
  TP_RELEASED,         // receiver: drop token reported
  TP_GPU_START,        // receiver: the pack's first workgroup started (host clock via HSA)
  TP_GPU_SIGNAL,       // receiver: the pack signalled its fill (host clock via HSA)
  // r06: the control plane's wake-ups, per message (inline samples too, keyed by ts_key)
  TP_SENT_RANG,        // sender: as TP_SENT, after waking a sleeping daemon (futex)
  TP_ROUTED_WOKE,      // daemon: as TP_ROUTED, in the loop pass that followed a futex sleep
  TP_POPPED_WOKE,      // receiver: as TP_POPPED, its wait for the event slept in the futex
};

// The trace key of a message without a drop token (an inline Vec sample): its metadata
// timestamp, which the sender, the daemon and the receiver all see.
DropToken ts_key(uint64_t ts);
// Whether the calling thread's last RingReader::wait slept in the futex (cleared by the call).
bool ring_take_woke();

bool trace_enabled();
void trace(TracePoint p, const DropToken& t);
void trace_at(TracePoint p, const DropToken& t, uint64_t t_ns);
void trace_set_name(const std::string& who);
void trace_flush();

}  // namespace dora
