/*
 * dora_gpu_testing.h — test and microbenchmark hooks of the device data plane, exported by
 * libdora_gpu_testing.so (dora_amd/csrc/testing/testing.cpp), which is built apart from the
 * shipped libdora_gpu.so and links against it.  No reference counterpart: tests/ and scripts/
 * use these to reach internals (the AQL backlog, the BAR, the fill-flag protocol, the RCCL group
 * path, the inter-daemon codec) that the product ABI (dora_gpu.h) does not expose.
 */
#ifndef DORA_GPU_TESTING_H
#define DORA_GPU_TESTING_H

#include "dora_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Tuning knob of the pack kernel (process-wide): 16-B loads in flight per lane (0 = default,
 * 2, 4, 8), non-temporal loads/stores (-1 = default, 0, 1; 2 = the signalling kernels'
 * write-through stores without a signal, a microbenchmark variant), bytes per workgroup (0 =
 * auto, else a multiple of 128: chunks start on cache lines). */
int dora_gpu_test_pack_tune(int unroll, int nontemporal, uint32_t chunk_bytes);
/* Tuning of packs that signal their fill from the kernel (node sends): workgroups of such a
 * launch, which then strides over the chunks (0: up to 4096).  With `bench_signal`,
 * dora_gpu_pack signals a scratch flag too (microbenchmarks). */
int dora_gpu_test_pack_signal_tune(uint32_t grid, int bench_signal);
/* Workgroup cap of packs the command processor signals (0: the default, 3584; a pack has at most
 * one workgroup per chunk). */
int dora_gpu_test_cp_grid(uint32_t grid);
/* Workgroup cap of multi-segment packs the command processor signals (0: the default, 640). */
int dora_gpu_test_cp_grid_multi(uint32_t grid);
/* Samples a sender of this process may have in flight below / from 8 MiB before an allocation
 * waits for a returned token (0: DORA_GPU_MAX_IN_FLIGHT or the defaults 11 / 8). */
int dora_gpu_test_in_flight(long small, long big);

/* Test tool (no reference counterpart): one workgroup per CU reads all of [data, data + len)
 * with plain cached loads, leaving the lines in every XCD's L2 (the acquire-fence negative
 * control of tests/test_gpu_fence.py). */
int dora_gpu_test_l2_touch(const void* data, size_t len, dora_stream_t stream);
/* Test tools (no reference counterpart): device memory of `device`'s coarse-grained pool that
 * the host writes directly through the PCIe BAR (stores + HDP flush + read-back), behind every
 * XCD's L2 — the source rewrite of the acquire-fence negative control. */
int dora_gpu_test_bar_alloc(int device, size_t bytes, void** out);
/* Test tool: while `hold` is set, every batchable AQL send of this process on `device` waits in
 * the backlog; clearing it dispatches the backlog as batch packs.  Only for asynchronous sends
 * (DORA_SEND_ASYNC): a synchronous send waits for its own pack. */
int dora_gpu_test_aql_hold(int device, int hold);
/* Test tool: 1 (default) lets the command processor signal a lone single-segment pack above
 * 32 MiB (a synchronous send's); 0 makes it signal its fill in-kernel. */
int dora_gpu_test_cp_lone(int on);
/* Test tool (latency probe): a host thread that every `period_us` either publishes an empty
 * barrier-AND packet on this process's first AQL queue of `device` (mode 1), reads (2) or writes
 * (3) one word of host-visible device memory over PCIe; until dora_gpu_test_heartbeat_stop or
 * `seconds` (at most 600). */
int dora_gpu_test_heartbeat_start(int device, int mode, double period_us, double seconds,
                                  void** out);
int dora_gpu_test_heartbeat_stop(void* h);
/* Test tool: empty packets the keep-awake thread of `device` has published in this process
 * (dora_gpu_set_keep_awake), and whether it is parked (no send for 100 ms). */
int dora_gpu_test_keep_awake_stats(int device, uint64_t* heartbeats, int* parked);
/* Test tool (latency probe): one resident wave on `device` that sleeps until
 * dora_gpu_test_keep_warm_stop (or `seconds`, at most 600) so the GPU never idles. */
int dora_gpu_test_keep_warm_start(int device, double seconds, void** out);
int dora_gpu_test_keep_warm_stop(void* handle);
/* Test tool: the AQL queues this process creates (effective before its first AQL use; 0 keeps
 * 4, at most 8) and how many of them take packs of 8-32 MiB in turn (0 keeps 4). */
int dora_gpu_test_mid_queues(int create, int use);
/* Test tool: `wc` 1 if `device`'s AQL packet rings are published with store fences (the runtime
 * put them in this GPU's memory), 0 otherwise; `where` (may be NULL): the runtime's pointer type
 * of the ring * 4 + its owner (0 none, 1 the CPU agent, 2 this GPU, 3 another agent). */
int dora_gpu_test_aql_ring_wc(int device, int* wc, int* where);
/* Test tool (host only): the 640-byte argument block of a batch pack (dora_aql_packb_u4) for
 * `n_msgs` (<= 8) messages; message m has seg_counts[m] segments, given as (src, dst_off, len)
 * triples in `segs`, its slot at dsts[m] with dst_caps[m] writable bytes, and fill flag /
 * epoch flags[m] / epochs[m].  *grid = the workgroups the dispatch would launch. */
int dora_gpu_test_batch_args(size_t n_msgs, const size_t* seg_counts, const uint64_t* segs,
                             const uint64_t* dsts, const uint64_t* dst_caps,
                             const uint64_t* flags, const uint64_t* epochs, uint8_t* out,
                             size_t cap, uint32_t* grid);
int dora_gpu_test_bar_write(int device, void* dst, const void* src, size_t bytes);
/* Test tools (host only) of the fill-flag protocol (FillFlag, 128 bytes, 64-byte aligned): the
 * completion test of epoch `epoch` (1: complete) and the sender's set-up of a fill the command
 * processor signals. */
int dora_gpu_test_fill_reached(const void* flag, uint64_t epoch);
int dora_gpu_test_cp_arm(void* flag, uint64_t epoch);
/* Test hook (microbenchmark): `n` single-segment AQL packs of `bytes` from rotating HBM sources,
 * round robin over `queues` of the device's AQL queues with at most `depth` outstanding per
 * queue; mode 0 completes them with the in-kernel fill signal, 1 with the packet's completion
 * signal (release fence none), 2 the same with an agent release fence, 3 and 4 as 0 and 1 without
 * the acquire fence, 5 as 1 with every wave waiting for its stores.  *us_per_msg = host time
 * per pack. */
int dora_gpu_test_aql_pipeline(int device, size_t bytes, int n, int mode, int queues, int depth,
                               double* us_per_msg);
void dora_gpu_test_bar_free(void* ptr);
/* Test hook (RCCL path of the fan-out): form a broadcast group of one rank on
 * `device` (unique id -> join(nranks 1) -> ncclBroadcast of `bytes` at `buf` in place on a fresh
 * stream -> close), reporting the rank count and rank the communicator holds.  The one-GPU
 * exercise of bcast_unique_id / bcast_join / bcast_enqueue / bcast_close. */
int dora_gpu_test_bcast_group(int device, void* buf, uint64_t bytes, int* nranks, int* rank);
/* Test tool (the fence probe's failing control): one 64-lane workgroup per CU reads 64 words of
 * BAR-written device memory, the host rewrites them through the BAR, and the same waves read
 * them again within the same dispatch; `mode` 0 plain (L1-cached) loads, 1 non-temporal, 2
 * agent-coherent (sc1).  Workgroups whose first read was wrong, whose second read was stale,
 * and the workgroups launched. */
int dora_gpu_test_l1_stale(int device, int mode, uint32_t* bad_first, uint32_t* stale,
                           uint32_t* blocks);
/* Test hooks of the inter-daemon wire, bincode of Timestamped<InterDaemonEvent> (replaces
 * bincode::serialize in binaries/daemon/src/inter_daemon.rs:66 and its deserialize at :156;
 * layouts in csrc/bincode.h): an Output event built from this library's type-info and parameter
 * encodings, an InputsClosed event of `n` (receiver, input) pairs, and a frame decoded into
 * JSON.  `hlc_id`: 16 bytes.  A buffer too small fails with *len set to the size needed. */
int dora_gpu_test_ide_output(const char* dataflow_id, const char* node_id, const char* output_id,
                             const uint8_t* type_info, size_t type_info_len, const uint8_t* params,
                             size_t params_len, uint64_t meta_ns, uint64_t event_ns,
                             const uint8_t* hlc_id, const uint8_t* data, size_t data_len,
                             int has_data, uint8_t* out, size_t cap, size_t* out_len);
int dora_gpu_test_ide_inputs_closed(const char* dataflow_id, const char* const* receivers,
                                    const char* const* inputs, size_t n, uint64_t event_ns,
                                    const uint8_t* hlc_id, uint8_t* out, size_t cap,
                                    size_t* out_len);
int dora_gpu_test_ide_decode(const uint8_t* frame, size_t len, char* json, size_t cap,
                             size_t* json_len);

#ifdef __cplusplus
}
#endif
#endif /* DORA_GPU_TESTING_H */
