/*
 * dora_gpu_testing.h — test and microbenchmark hooks of the device data plane, exported by
 * libdora_gpu_testing.so (dora_amd/csrc/testing/testing.cpp), which is built apart from the
 * shipped libdora_gpu.so and links against it.  The pack-tuning knobs of r01-r05 (variants,
 * grids, in-flight caps, queue counts) are gone with their variants (r06): the product carries no
 * code path only a microbenchmark selects.  No reference counterpart: tests/ and scripts/
 * use these to reach internals (the AQL backlog, the BAR, the fill-flag protocol, the RCCL group
 * path, the inter-daemon codec) that the product ABI (dora_gpu.h) does not expose.
 */
#ifndef DORA_GPU_TESTING_H
#define DORA_GPU_TESTING_H

#include "dora_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

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
/* Test hooks of the region-end stamp reduction (aql_stamp_reduce): how long it is waited for
 * (ns; 0 = the default 5 s) — a tiny value makes the wait time out while the packet still runs —
 * and the AQL argument slots left to reductions that timed out (never written again). */
int dora_gpu_test_reduce_timeout(uint64_t ns);
/* Experiment: `n` D2H copies of `bytes` from HBM into pinned host memory, `gap_ns` apart, each
 * timed call -> complete into out_ns[n]: mode 0 hipMemcpyAsync + hipStreamSynchronize on a
 * stream of its own, mode 1 hsa_amd_memory_async_copy + a busy wait on its signal. */
int dora_gpu_test_d2h_copy_probe(int device, int mode, uint64_t bytes, uint32_t n,
                                 uint64_t gap_ns, uint64_t* out_ns);
/* Experiment: per-message cost of ordering a sample written on a stream — `n` kernels writing
 * `bytes`, each followed by nothing (mode 0), hipStreamWriteValue64 into pinned host memory (1)
 * or an 8-byte kernel (2); out_ns[0] host enqueue, out_ns[1] enqueue + drain, ns per message. */
int dora_gpu_test_stream_order_probe(int device, int mode, uint64_t bytes, uint32_t n,
                                     uint64_t* out_ns);
int dora_gpu_test_abandoned_slots(int device, uint32_t* slots);
/* Test tool: empty packets the keep-awake thread of `device` has published in this process
 * (dora_gpu_set_keep_awake), and whether it is parked (no send for 100 ms). */
int dora_gpu_test_keep_awake_stats(int device, uint64_t* heartbeats, int* parked);
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
