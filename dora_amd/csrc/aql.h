// Direct AQL dispatch of signalling packs on a node-owned HSA queue (aql.cpp).
//
// hipLaunchKernel costs ~2.5 us of host time per pack (profiles/r01_launch_probe.jsonl): its
// kernel arguments go to device memory and are made visible with a PCIe read-back, and every
// dispatch acquires at system scope.  Below ~16 MB a send is bound by that host time.  A node
// instead writes the pack's arguments into a device-memory ring (write-combined stores, one HDP
// flush instead of the read-back) and a raw kernel-dispatch packet into its own HSA queue:
// ~1.5 us per send, agent-scope acquire/release (pack sources are device memory of this GPU;
// the pack writes its sample through to device scope and signals the fill flag itself), no
// barrier bit, so consecutive packs overlap (profiles/r01_aql_probe.jsonl).
#pragma once

#include <atomic>
#include <cstddef>
#include <cstdint>

#include "plan.h"

namespace dora {

struct AqlQueue;

// The process's AQL queue for HIP device `device`, created on first use; nullptr when HSA or
// the code object cannot be set up (callers then launch through HIP).
AqlQueue* aql_queue(int device);
// A queue aql_queue returned is still usable (not marked failed): callers may keep the pointer
// (queues are never freed) instead of looking it up under the global lock on every send.
bool aql_usable(const AqlQueue* q);

// Dispatch one signalling pack of `n` (<= 8) device-source copy segments into `dst`; the launch
// stores `sig.epoch` into `sig.flag` when the sample is complete.  `flag_host` is the host view
// of that flag (kernarg slots are recycled once the launch that used them has signalled).
// `dst_cap`: bytes writable from `dst` (0: unknown; see launch_pack).
// With `profile`, the packet carries a completion signal whose dispatch times
// aql_profile_take() reports.  `profile` packs (a timed region's) are signalled by the command
// processor only when `cp_stamps` (device memory, 1 + kCpStampWgs zeroed words, plan.h) takes
// their stamps: [0] the first workgroup's start, [1 + k mod kCpStampWgs] the latest completion of
// the workgroups k that map there (s_memrealtime, atomic max).
//
// `sync`: the caller waits for this pack before it does anything else (a synchronous send,
// node.cpp wait_source_read).  A single-segment pack that is sent synchronously, or that finds
// every queue idle, runs alone on the GPU: its arguments go to the device ring and it reads
// without the acquire fence; a synchronous one is also signalled by the command processor at any
// size >= 1 MiB, with a grid of up to 3584 workgroups (no done words to poll, so no
// 1024-workgroup signalling cap).  A synchronous one of 1-256 MiB of 16-byte-aligned bytes is
// read-signalled (*read_signalled): the pack raises the flag line's read word (FillFlag
// read_epoch) once every source byte is in its workgroups' registers, before its stores drain,
// and the caller may return then.
int aql_pack(AqlQueue* q, const Segment* segs, size_t n, uint8_t* dst, const FillSignal& sig,
             const std::atomic<uint64_t>* flag_host, bool profile, uint64_t dst_cap = 0,
             uint64_t* cp_stamps = nullptr, bool sync = false, bool* read_signalled = nullptr);
// Would a pack of these segments be signalled by the command processor: [1 MiB, 32 MiB), or
// (`lone`: a synchronous send) a single-segment pack of any size from 1 MiB.
bool aql_cp_candidate(const Segment* segs, size_t n, bool lone = false);

// Forget every argument slot whose fill flag lies in [base, base + size) (a node's control
// region about to be unmapped), after waiting (bounded) for those fills to signal.
void aql_forget_flags(int device, const void* base, size_t size);

// Wait (bounded) until every AQL pack dispatched so far in this process has signalled: HIP's
// hipFree waits for the HIP streams of the device, not for these queues, so the library's own
// frees of device memory (dora_gpu_free, device array release) call this first.
void aql_fence_all();

// Diagnostics: the kernels of the AQL code object and the packets dispatched per kernel in
// this process on `device` (dora_gpu_aql_dispatch_counts).
size_t aql_kernel_count();
const char* aql_kernel_name(size_t k);
uint64_t aql_dispatched(int device, size_t k);
// Test tool: while held, every batchable send of this process on `device` waits in the
// backlog; releasing dispatches the backlog as batch packs (tests/test_gpu_dataflow.py).
int aql_hold(int device, bool hold);
// Period of the warm thread's empty packets (aql.cpp warm_main; 0: off; at least 5 us).
void aql_keep_awake(double period_us);
// Test tool: empty packets the warm thread of `device` has published, and whether it is parked.
uint64_t aql_heartbeats(int device, bool* parked);
// Whether the process's packet rings are published with fences (in device memory), and where
// the runtime says they are (pointer type * 4 + owner: 1 CPU agent, 2 this GPU, 3 other).
int aql_ring_write_combined(int device, bool* wc, int* where);
// Packs signalled by the command processor (cp_signal_window, aql.cpp).
uint64_t aql_cp_signalled(int device);
// A pack's own GPU stamp (s_memrealtime ticks) as CLOCK_REALTIME ns, for the message trace
// (DORA_GPU_TRACE): the HSA runtime maps GPU ticks to its system clock, whose offset from
// CLOCK_REALTIME is taken once per process from the tightest of 16 bracketed samples.  0 when
// the device has no AQL queue or the runtime cannot convert.
uint64_t aql_gpu_tick_to_realtime_ns(int device, uint64_t tick);
// Batch packs dispatched, the sends they carried, and sends that waited in the backlog.
int aql_batch_stats(int device, uint64_t* batches, uint64_t* batched_msgs, uint64_t* backlogged);

// Test tool (tests/fence_probe.py): device memory of the GPU's coarse-grained pool that the host
// writes directly through the BAR (bar_write: stores + HDP flush + read-back), i.e. behind every
// XCD's L2 — the writer a pack without an acquire fence cannot see.
int bar_alloc(int device, size_t bytes, void** out);
int bar_write(int device, void* dst, const void* src, size_t bytes);
void bar_free(void* p);

// Host-resident sources written straight into a device slot by the CPU (node.cpp
// host_bar_fill): bar_map makes a hipMalloc'd slot host-accessible through the large BAR (once
// per slot; its IPC export is unaffected), bar_copy writes bytes with streaming stores, and
// bar_publish (sfence + HDP flush + one read-back of `last`) returns once every byte written so
// far has reached HBM.
int bar_map(AqlQueue* q, void* p);
void bar_copy(void* dst, const void* src, size_t n);
void bar_publish(AqlQueue* q, const void* last);

// Region-end reduction of stamp areas (node.cpp): one dispatch of dora_aql_stamp_reduce over
// `n` areas of `area_words` words each at `base` (device memory), area indices in `areas`, writing
// (start, latest end) pairs to `out` (host memory the GPU can write); waits for it (bounded).
int aql_stamp_reduce(int device, const uint64_t* base, uint32_t area_words,
                     const uint32_t* areas, uint32_t n, uint64_t* out);

// One copy-engine copy of `n` bytes between device memory (this process's or IPC-imported) and
// pinned host memory — `to_host`: `src` is the device side, else `dst` — waited for by polling its
// signal: a 4 KB sample to the host in 6.9 us against 17 for hipMemcpyAsync +
// hipStreamSynchronize, equal from ~64 KB (scripts/d2h_copy_probe.py,
// profiles/r06_d2h_copy_probe.jsonl).  DORA_ERR_UNSUPPORTED when the runtime cannot take it (the
// caller uses HIP's copy); DORA_ERR_TIMEOUT after 10 s.
int hsa_copy_host(void* dst, const void* src, uint64_t n, bool to_host);
// Test hooks: the stamp reduction's wait (0: the default 5 s), and the argument slots left to
// reductions that timed out (never written again).
void aql_reduce_timeout(uint64_t ns);
uint32_t aql_abandoned_slots(int device);

// Segments one AQL dispatch takes.
size_t aql_max_segments();

// Enable per-packet timestamps (regions) and collect them: start/end of every profiled dispatch
// since the last take, in ns, after waiting for them to complete.
int aql_profile_enable(AqlQueue* q, bool on);
int aql_profile_take(AqlQueue* q, uint64_t* first_start, uint64_t* last_end, uint64_t* count);

}  // namespace dora
