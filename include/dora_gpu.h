/*
 * dora_gpu.h — C ABI of the MI355X device-resident message data plane for dora.
 *
 * Every entry point is `extern "C"`, takes plain pointers and sizes, and returns an int status
 * (0 = ok, < 0 = error) with a thread-local message in dora_gpu_last_error(), following the
 * reference C node API convention (apis/c/node/src/lib.rs:245-259: 0 / -1 + logged error).
 * Reference interfaces replaced are cited per function (paths relative to the dora v0.3.6 tree).
 *
 * Arrow arrays cross the boundary through the Arrow C Data Interface — the same ABI the
 * reference's operator plugins use (apis/rust/operator/types/src/lib.rs:104-135) and that the
 * Python node imports pyarrow arrays through (apis/python/node/src/lib.rs:157-185).
 */
#ifndef DORA_GPU_H
#define DORA_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------------------------------ */
/* Arrow C Data Interface + C Device Data Interface (public Arrow ABI, spec v1).              */
/* ------------------------------------------------------------------------------------------ */
#ifndef ARROW_C_DATA_INTERFACE
#define ARROW_C_DATA_INTERFACE
#define ARROW_FLAG_DICTIONARY_ORDERED 1
#define ARROW_FLAG_NULLABLE 2
#define ARROW_FLAG_MAP_KEYS_SORTED 4
struct ArrowSchema {
  const char* format;
  const char* name;
  const char* metadata;
  int64_t flags;
  int64_t n_children;
  struct ArrowSchema** children;
  struct ArrowSchema* dictionary;
  void (*release)(struct ArrowSchema*);
  void* private_data;
};
struct ArrowArray {
  int64_t length;
  int64_t null_count;
  int64_t offset;
  int64_t n_buffers;
  int64_t n_children;
  const void** buffers;
  struct ArrowArray** children;
  struct ArrowArray* dictionary;
  void (*release)(struct ArrowArray*);
  void* private_data;
};
#endif
#ifndef ARROW_C_DEVICE_DATA_INTERFACE
#define ARROW_C_DEVICE_DATA_INTERFACE
typedef int32_t ArrowDeviceType;
#define ARROW_DEVICE_CPU 1
#define ARROW_DEVICE_ROCM 10
#define ARROW_DEVICE_ROCM_HOST 11
struct ArrowDeviceArray {
  struct ArrowArray array;
  int64_t device_id;
  ArrowDeviceType device_type;
  void* sync_event;
  int64_t reserved[3];
};
#endif

/* ------------------------------------------------------------------------------------------ */
/* Status, errors, runtime plumbing                                                           */
/* ------------------------------------------------------------------------------------------ */
#define DORA_OK 0
#define DORA_ERR_INVALID (-1)      /* bad argument / unsupported type                       */
#define DORA_ERR_HIP (-2)          /* HIP runtime error                                     */
#define DORA_ERR_TOO_SMALL (-3)    /* target buffer too small (arrow_utils.rs:37-42 panic)  */
#define DORA_ERR_UNSUPPORTED (-4)  /* type outside the parity set (views, unions, ListView) */
#define DORA_ERR_CLOSED (-5)       /* channel / peer closed                                 */
#define DORA_ERR_TIMEOUT (-6)
#define DORA_ERR_NOT_FOUND (-7)    /* unknown output id / drop token                        */

typedef void* dora_stream_t; /* a hipStream_t; NULL = the device's null stream */

/* Thread-local message of the last failing call on this thread (never NULL). */
const char* dora_gpu_last_error(void);
/* Library version string "dora-gpu <semver> gfx950". */
const char* dora_gpu_version(void);
/* Diagnostics (no reference counterpart): this process's host time blocked on empty control
 * rings (node event/drop rings, the daemon's request rings) and spent spinning on producers'
 * fill flags, in ns since start.  Busy time = wall - idle locates a pipeline's bottleneck. */
int dora_gpu_busy_stats(uint64_t* idle_ns, uint64_t* fill_wait_ns);
/* Diagnostics (no reference counterpart): raw AQL packets this process dispatched on HIP device
 * `device`, per kernel of the embedded pack code object (min(cap, *n) entries written; *n = the
 * kernel count), and kernel k's symbol name ("" past the end).  The driver's smoke names the
 * kernels that packed its samples with these. */
int dora_gpu_aql_dispatch_counts(int device, uint64_t* counts, size_t cap, size_t* n);
const char* dora_gpu_aql_kernel_name(size_t k);
/* Diagnostics: batch packs dispatched on HIP device `device` by this process, the sends they
 * carried, and the sends that waited for queue capacity (aql.cpp: sends that find every AQL
 * queue busy leave together as one batch pack). */
int dora_gpu_aql_batch_stats(int device, uint64_t* batches, uint64_t* batched_msgs,
                             uint64_t* backlogged);
/* Diagnostics: packs on HIP device `device` whose fill the command processor signalled (the
 * packet's completion signal instead of the in-kernel flag store; mid-size single-segment packs
 * of 1-32 MiB, and synchronous single-segment sends from 1 MiB). */
int dora_gpu_aql_cp_signalled(int device, uint64_t* count);
/* Latency control (no reference counterpart): while this process sends device samples, a thread
 * per GPU publishes an empty AQL packet whenever nothing was dispatched for `period_us`, so the
 * command processor never idles long enough to need waking (~5.5 us per message otherwise, for
 * messages more than ~50 us apart); it parks 100 ms after the last send.  Default 25 us; 0 turns
 * it off (saves the thread's wake-ups); values below 5 are raised to 5.  Process-wide. */
int dora_gpu_set_keep_awake(double period_us);

int dora_gpu_device_count(int* count);
int dora_gpu_set_device(int ordinal);
int dora_gpu_get_device(int* ordinal);
int dora_gpu_stream_create(dora_stream_t* out);
int dora_gpu_stream_destroy(dora_stream_t stream);
int dora_gpu_stream_sync(dora_stream_t stream);
int dora_gpu_device_sync(void);
int dora_gpu_malloc(void** out, size_t nbytes);
int dora_gpu_free(void* ptr);
int dora_gpu_host_alloc(void** out, size_t nbytes); /* pinned host memory */
int dora_gpu_host_free(void* ptr);
/* Async copy on `stream` (direction inferred from the pointers, unified addressing). */
int dora_gpu_memcpy_async(void* dst, const void* src, size_t nbytes, dora_stream_t stream);
int dora_gpu_memset_async(void* dst, int value, size_t nbytes, dora_stream_t stream);

/* Timing on the stream the kernels run on (hipEvent pairs). */
typedef void* dora_event_t;
int dora_gpu_event_create(dora_event_t* out);
int dora_gpu_event_destroy(dora_event_t ev);
int dora_gpu_event_record(dora_event_t ev, dora_stream_t stream);
int dora_gpu_event_sync(dora_event_t ev);
int dora_gpu_event_elapsed_ms(dora_event_t start, dora_event_t stop, float* ms);

/* ------------------------------------------------------------------------------------------ */
/* Packing — replaces apis/rust/node/src/node/arrow_utils.rs:4-71                             */
/* ------------------------------------------------------------------------------------------ */
typedef struct dora_plan dora_plan;

/*
 * Host-side DFS over an Arrow array (a1, `required_data_size_inner`, arrow_utils.rs:9-21):
 * buffer lengths follow arrow-rs 53.2.0 FFI import, alignment follows arrow-data 53.2.0
 * `layout()`.  `device_type` says where the array's buffers live: ARROW_DEVICE_ROCM (HBM; the
 * pack is one HIP kernel) or ARROW_DEVICE_CPU (host memory; the pack is DMA into the slot).
 * Validity bitmaps and, for Utf8/Binary, the last offset are read to the host during planning
 * (the reference clones validity into metadata, arrow_utils.rs:66).
 * The array is borrowed: its buffers must stay valid until the pack completes on its stream.
 */
int dora_gpu_plan(const struct ArrowArray* array, const struct ArrowSchema* schema,
                  ArrowDeviceType device_type, dora_plan** out);
/*
 * Compacting plan (new capability; the reference copies sliced buffers whole and passes the
 * offset through): every node is reduced to its logical range — fixed-width values
 * sliced, Boolean bitmaps bit-shifted to bit 0, offsets rebased to 0 with the child / value
 * ranges they address sliced recursively, validity shifted for the type info — so the type info
 * has offset 0 everywhere and a slice moves only its own bytes.  Receivers are unchanged
 * (`into_arrow_array` yields a logically equal array).  Device-resident arrays only; run-end
 * encoded arrays are rejected.
 */
int dora_gpu_plan_compact(const struct ArrowArray* array, const struct ArrowSchema* schema,
                          ArrowDeviceType device_type, dora_plan** out);
/* Plan for `ArrowTypeInfo::byte_array(len)` over one contiguous buffer (metadata.rs:74-87):
 * what `send_output_raw`'s copy closure writes (node/mod.rs:180-196). */
int dora_gpu_plan_bytes(const void* src, size_t len, ArrowDeviceType device_type,
                        dora_plan** out);
void dora_gpu_plan_free(dora_plan* plan);
/* required_data_size (arrow_utils.rs:4-8). */
size_t dora_gpu_plan_size(const dora_plan* plan);
size_t dora_gpu_plan_num_segments(const dora_plan* plan);
/* Segment i: source pointer, destination offset in the sample, length. */
int dora_gpu_plan_segment(const dora_plan* plan, size_t i, const void** src, uint64_t* dst_off,
                          uint64_t* len);
/*
 * Serialized ArrowTypeInfo (libraries/message/src/metadata.rs:51-59), little endian:
 *   str data_type (u32 n + n bytes: the DataType as a schema tree — str format, str name,
 *   i64 flags, u8 has_meta [str meta], u32 n_children × tree, u8 has_dict [tree]),
 *   u64 len, u64 null_count,
 *   u8 has_validity [u64 n + n bytes], u64 offset, u32 n_buffers × (u64 offset, u64 len),
 *   u32 n_children × TypeInfo.
 * Call with buf = NULL to get the size.
 */
int dora_gpu_plan_type_info(const dora_plan* plan, uint8_t* buf, size_t cap, size_t* len);
/*
 * copy_array_into_sample (arrow_utils.rs:23-71): copy every buffer to its aligned offset in
 * `dst` (device memory, `dst_len` >= plan size) on `stream`; async.  Padding is not written.
 */
int dora_gpu_pack(const dora_plan* plan, void* dst, size_t dst_len, dora_stream_t stream);
/* ------------------------------------------------------------------------------------------ */
/* Device-resident Arrow arrays                                                               */
/* ------------------------------------------------------------------------------------------ */
/* Deep-copy a host Arrow array into HBM, same structure (offsets, lengths, children). The
 * result owns its device buffers; free with dora_gpu_array_release. */
int dora_gpu_array_upload(const struct ArrowArray* array, const struct ArrowSchema* schema,
                          struct ArrowArray* out);
/* Deep-copy a device Arrow array to host memory (for CPU consumers such as pyarrow). */
int dora_gpu_array_download(const struct ArrowArray* array, const struct ArrowSchema* schema,
                            struct ArrowArray* out);
/*
 * Receiver side of a sample — `RawData::into_arrow_array` / `buffer_into_arrow_array`
 * (apis/rust/node/src/event_stream/event.rs:35-91): a zero-copy device ArrowArray whose buffers
 * are slices of `sample` per BufferOffset (validity uploaded from the type info), plus its
 * ArrowSchema.  sample_len == 0 yields an empty array of the data type (event.rs:65-67).
 * `sample` must outlive the array.
 */
int dora_gpu_sample_import(const void* sample, size_t sample_len, const uint8_t* type_info,
                           size_t type_info_len, struct ArrowArray* out_array,
                           struct ArrowSchema* out_schema);
/* The DataType of a serialized ArrowTypeInfo as an ArrowSchema. */
int dora_gpu_type_info_schema(const uint8_t* type_info, size_t type_info_len,
                              struct ArrowSchema* out_schema);
void dora_gpu_array_release(struct ArrowArray* array);
void dora_gpu_schema_release(struct ArrowSchema* schema);

/* ------------------------------------------------------------------------------------------ */
/* Device checksums and payload generation (parity at full sizes; see oracle/checksum_ref.py) */
/* ------------------------------------------------------------------------------------------ */
/* csum64 of `len` device bytes; the result is written to device `out` (one u64), async. */
int dora_gpu_csum64(const void* data, size_t len, uint64_t* out_dev, dora_stream_t stream);
/* Blocking convenience: returns csum64 to the host. */
int dora_gpu_csum64_sync(const void* data, size_t len, dora_stream_t stream, uint64_t* out);
/* Fill `len` device bytes with the splitmix64 stream of `seed` (BASELINE.md §2 payloads). */
int dora_gpu_fill_splitmix(void* dst, size_t len, uint64_t seed, dora_stream_t stream);
/* ------------------------------------------------------------------------------------------ */
/* Node API — replaces DoraNode / EventStream (apis/rust/node/src/node/mod.rs:42-503,         */
/* apis/rust/node/src/event_stream/mod.rs:27-235) and the C node API (apis/c/node/node_api.h) */
/* ------------------------------------------------------------------------------------------ */
typedef struct dora_node dora_node;
typedef struct dora_sample dora_sample;
typedef struct dora_event dora_event;

enum {
  DORA_EVENT_STOP = 0,             /* Event::Stop                       (event.rs:12)     */
  DORA_EVENT_INPUT = 1,            /* Event::Input{id, metadata, data}  (event.rs:17-21)  */
  DORA_EVENT_INPUT_CLOSED = 2,     /* Event::InputClosed{id}            (event.rs:22-24)  */
  DORA_EVENT_ERROR = 3,            /* Event::Error                      (event.rs:25)     */
  DORA_EVENT_ALL_INPUTS_CLOSED = 4 /* end of the event stream (NodeEvent::AllInputsClosed) */
};

/* DoraNode::init (mod.rs:121-155): attach to the dataflow region `shm_name`, register as
 * `node_id` on GPU `device`, subscribe and wait for every node of the dataflow to be ready. */
int dora_node_init(const char* shm_name, const char* node_id, int device, dora_node** out);
/* DoraNode::init_from_env (mod.rs:65-76): DORA_GPU_DATAFLOW, DORA_NODE_ID, DORA_GPU_DEVICE. */
int dora_node_init_from_env(dora_node** out);
/* Drop for DoraNode (mod.rs:384-431): close outputs, wait <= 10 s for drop tokens, done. */
void dora_node_free(dora_node* node);
/* DoraNode::dataflow_id / id (mod.rs:373-382): the dataflow's id as its daemon names it (the
 * reference's DataflowId is a uuid; a name that is not one maps to the UUID the inter-daemon
 * wire carries, dora_amd/dataflow.py dataflow_uuid) and this node's id.  Owned by the node. */
const char* dora_node_dataflow_id(const dora_node* node);
const char* dora_node_id(const dora_node* node);
/* The node's HIP stream; consumers must run their kernels on it so the drop token is only
 * returned after they have read the sample.  Sends spread their fills over the node's fill
 * streams (three): a fill runs after the work queued on this stream
 * when the send is made, and the call orders every fill launched so far before the work the
 * caller queues on the returned stream next (a device source may be rewritten there). */
dora_stream_t dora_node_stream(dora_node* node);

/* allocate_data_sample (mod.rs:303-346): a device slot of `len` bytes (best-fit from the
 * node's cache of recycled slots, else a new exported hipMalloc slot); len 0 -> empty Vec.  A
 * host-only node (device < 0) gets the reference's samples instead: an inline Vec below 4096 B,
 * else a POSIX shared-memory region (DataMessage::SharedMemory, mod.rs:321-346) it writes with
 * the CPU; dora_sample_data is then a host pointer. */
int dora_node_allocate_data_sample(dora_node* node, size_t len, dora_sample** out);
void* dora_sample_data(dora_sample* sample); /* device pointer (slot) */
size_t dora_sample_len(const dora_sample* sample);
/* An unsent sample back to the node's cache.  A sample that was already sent or discarded is
 * left alone (dora_gpu_last_error says so). */
void dora_sample_discard(dora_node* node, dora_sample* sample);
/* send_output_sample (mod.rs:246-275): consumes `sample` (may be NULL = no data); a sample that
 * was already sent or discarded is refused with DORA_ERR_INVALID (the reference moves its
 * DataSample into the call).  The sample must be written before the call: on the host, or by
 * work queued on dora_node_stream() — receivers then wait for that work through the slot's fill
 * signal, the call does not — or on another stream the caller synchronized.  `params` is the encoded
 * MetadataParameters (u32 n, then per entry: u64 klen, key, u8 tag 0=bool 1=int 2=string,
 * value: u8 | i64 | u64 len + bytes). */
int dora_node_send_output_sample(dora_node* node, const char* output_id, const uint8_t* type_info,
                                 size_t type_info_len, const uint8_t* params, size_t params_len,
                                 dora_sample* sample);
/* send_output (mod.rs:198-215): plan + allocate + HIP pack + send.  `device_type` as in
 * dora_gpu_plan; a host-resident array whose sample is < 4096 B travels inline as the
 * reference's DataMessage::Vec (mod.rs:40,303-319: no slot, no GPU work).  Like the reference,
 * which copies the array inside the call
 * (arrow_utils.rs:48), the call returns once the sample no longer needs the source: for a
 * device source it waits (after the descriptor has left) until the pack kernel has read it, so
 * the caller may rewrite or free the source on any stream right away.  (A single-segment
 * sample of 1-192 MiB from a 16-byte-aligned source is packed read-first: the call returns
 * when every source byte is in the pack's registers, before its stores have drained.)  When
 * every receiver of the output runs without a GPU, a device sample <= 1 MiB is packed into
 * shared memory and a host sample >= 4096 B copied there by the CPU (DataMessage::SharedMemory,
 * complete when the call returns). */
int dora_node_send_output(dora_node* node, const char* output_id, const struct ArrowArray* array,
                          const struct ArrowSchema* schema, ArrowDeviceType device_type,
                          const uint8_t* params, size_t params_len);
/* send_output_raw / send_output_bytes (mod.rs:180-196, 217-228): `len` bytes as
 * ArrowTypeInfo::byte_array, copied into a device sample (kernel for HBM sources, DMA for host
 * sources); returns once the source has been read, as dora_node_send_output.  This is the
 * benchmark's send path (examples/benchmark/node/src/main.rs:46-48). */
int dora_node_send_output_bytes(dora_node* node, const char* output_id, const void* data,
                                size_t len, ArrowDeviceType device_type, const uint8_t* params,
                                size_t params_len);
/* Flags of the _ex variants (no reference counterpart). */
#define DORA_SEND_ASYNC 1u /* return before the pack has read a device source (below) */
/* dora_node_send_output / _bytes with `flags`.  With DORA_SEND_ASYNC a device-source send
 * returns as soon as its pack is queued: the caller must not write the source until the pack
 * has read it — i.e. until dora_node_sync(), or only by work queued on dora_node_stream()
 * fetched after the send (which orders every fill launched so far before it).  Senders that
 * never rewrite their sources (frame rings, the benchmark) overlap packs this way; a host
 * source is always safe to reuse on return. */
int dora_node_send_output_ex(dora_node* node, const char* output_id, const struct ArrowArray* array,
                             const struct ArrowSchema* schema, ArrowDeviceType device_type,
                             const uint8_t* params, size_t params_len, uint32_t flags);
int dora_node_send_output_bytes_ex(dora_node* node, const char* output_id, const void* data,
                                   size_t len, ArrowDeviceType device_type, const uint8_t* params,
                                   size_t params_len, uint32_t flags);
/* Make DORA_SEND_ASYNC the default of every send of this node (also DORA_GPU_SEND_ASYNC=1). */
int dora_node_set_async_sends(dora_node* node, int enable);
/* Event-stream thread (the reference's event_stream_loop, apis/rust/node/src/event_stream/
 * thread.rs:81-188; no counterpart in the C API): `enable` starts a thread that drains the
 * daemon's events into the node's input queue continuously and applies the drop-oldest policy
 * there (node_communication/mod.rs:320-359), so inputs keep arriving — broadcast receives posted,
 * tokens of dropped inputs returned — while the user thread is busy; dora_node_next_event then
 * takes events from that queue.  Nodes that receive over an RCCL broadcast group start it
 * themselves.  0 stops it. */
int dora_node_set_event_thread(dora_node* node, int enable);
/* Use compacting plans (dora_gpu_plan_compact) in dora_node_send_output for device arrays. */
int dora_node_set_compact(dora_node* node, int enable);
/* close_outputs (mod.rs:277-289). */
int dora_node_close_outputs(dora_node* node, const char* const* output_ids, size_t count);

/* EventStream::recv / recv_timeout (event_stream/mod.rs:121-140); timeout_us < 0 blocks.
 * Returns DORA_ERR_TIMEOUT on timeout and DORA_ERR_CLOSED after the stream ended. */
int dora_node_next_event(dora_node* node, int64_t timeout_us, dora_event** out);
int dora_event_type(const dora_event* ev);
const char* dora_event_id(const dora_event* ev);
const char* dora_event_error(const dora_event* ev);
/* Raw sample of an input: device pointer (mapped IPC slot) or host pointer for inline Vec data
 * and for a host-only receiver's shared-memory samples (dora_event_is_device says which).  An
 * input whose slot lives on another GPU, or a host-only producer's shared-memory sample at a
 * device receiver, is pulled into local HBM on the first call (complete on return; the
 * producer's token goes back at once; see dora_node_peer_stats). */
int dora_event_data(const dora_event* ev, const void** ptr, size_t* len);
int dora_event_is_device(const dora_event* ev);
/* Serialized ArrowTypeInfo / MetadataParameters / timestamp of the input's Metadata. */
int dora_event_type_info(const dora_event* ev, const uint8_t** type_info, size_t* len);
int dora_event_parameters(const dora_event* ev, const uint8_t** params, size_t* len);
uint64_t dora_event_timestamp_ns(const dora_event* ev);
/* RawData::into_arrow_array (event.rs:35-91): zero-copy device ArrowArray over the sample; it
 * keeps the input (and its drop token) alive until released.  An inline Vec sample (< 4096 B
 * from a host source) and a host-only receiver's shared-memory sample import as a host
 * ArrowArray over their bytes instead. */
int dora_event_array(const dora_event* ev, struct ArrowArray* out_array,
                     struct ArrowSchema* out_schema);
/* Drop the event; the drop token is reported once no array references the data any more. */
void dora_event_free(dora_event* ev);
/* Relay stage (new; a reference relay node does recv -> send_output_sample with a copy of the
 * data, apis/rust/node/src/node/mod.rs:180-275): send the input `ev` on `output_id` with its
 * ArrowTypeInfo and the given parameters.  The payload moves once: a cross-GPU input is copied
 * from the peer's slot straight into this node's new slot.  `ev` stays valid (free it after). */
int dora_node_forward(dora_node* node, const char* output_id, const dora_event* ev,
                      const uint8_t* params, size_t params_len);
/* A same-GPU device input is forwarded in place: the new message points at the producer's slot
 * under a token of this node, and the input (with the producer's token) is held until that token
 * returns — no copy, no new slot.  Cross-GPU inputs, broadcast-group inputs and
 * copy into a fresh slot instead.  Forwards done in place, and forwards
 * whose token has not returned yet. */
int dora_node_forward_stats(dora_node* node, uint64_t* in_place, uint64_t* held);

int dora_node_stats(dora_node* node, uint64_t* slots_created, uint64_t* cache_hits,
                    uint64_t* in_flight, uint64_t* dropped_inputs);
/* Counters of any node of this node's dataflow (new; diagnostics, read through the shared
 * control region): device slots it created, producers' slots it mapped with
 * hipIpcOpenMemHandle, and inputs its queue_size policy dropped.  A steady edge creates and maps
 * nothing: a benchmark reads them around a timed region to show it paid no set-up cost inside
 * and that every message it counts was delivered. */
int dora_node_dataflow_counters(dora_node* node, const char* node_id, uint64_t* slots_created,
                                uint64_t* ipc_opens, uint64_t* dropped_inputs);
/* Fills (packs of sends) by dispatch path: raw AQL packets on the process's HSA queue (device
 * sources of <= 8 segments) or hipLaunchKernel on
 * the node's fill streams (larger, host sources, compacting transforms, relays). */
int dora_node_fill_paths(dora_node* node, uint64_t* aql_packs, uint64_t* hip_packs);
/* The host side of the data plane (new; diagnostics): host-resident sources of 4096 B..2 MiB a
 * device node wrote into its slot with the CPU through the large BAR (the reference's memcpy
 * into its shared-memory sample, arrow_utils.rs:48: no GPU dispatch), and device samples a node
 * without a GPU (DORA_GPU_DEVICE < 0) staged into host memory on receipt (count, bytes): such a
 * receiver gets the reference's host ArrowData (event.rs:35-91); and samples this node put
 * straight into shared memory because every receiver of the output lacks a GPU (sent as the
 * reference's DataMessage::SharedMemory): device arrays <= 1 MiB packed there by the GPU, host
 * sources >= 4096 B copied there by the CPU.  Any pointer may be NULL. */
int dora_node_host_paths(dora_node* node, uint64_t* bar_fills, uint64_t* staged,
                         uint64_t* staged_bytes, uint64_t* host_packs);
/* The outputs of this node the daemon named host-bound in AllNodesReady (new; diagnostics):
 * every receiver is a running local node without a GPU and none is on another machine, so a
 * device node packs them into shared memory (above).  Newline-terminated names, sorted, NUL
 * after the last; *len (if not NULL) = their bytes without the NUL.  buf NULL: only *len;
 * cap < *len + 1: DORA_ERR_INVALID. */
int dora_node_host_bound_outputs(dora_node* node, char* buf, uint64_t cap, uint64_t* len);
/* dora_node_send_output of device arrays keeps the plans of recent sends that read no array
 * bytes (fixed-width and nested arrays with known null counts), keyed by everything such a plan
 * depends on (schema strings and flags, lengths, offsets, null counts, buffer addresses): a
 * sender re-sending the same buffers plans each once.  Sends served from it, plans kept. */
int dora_node_plan_cache_stats(dora_node* node, uint64_t* hits, uint64_t* entries);
/* Cross-GPU edges: an input whose slot lives on another GPU is pulled over xGMI
 * into a local receive slot on first access (dora_event_data / dora_event_array) and the
 * producer's token is returned at once; dora_node_forward pulls it straight into an outgoing
 * slot instead.  The pull is the pack kernel reading the peer's HBM (default) or the copy
 * engines (DORA_GPU_PEER_COPY=sdma).  Counts and bytes of such pulls.  DORA_GPU_EDGE_COPY=1
 * forces the path on same-GPU edges. */
int dora_node_peer_stats(dora_node* node, uint64_t* copies, uint64_t* bytes);
/* 1 -> N fan-out over RCCL (no reference counterpart: the reference has no GPU
 * transport).  A node started with DORA_GPU_FANOUT=rccl asks the daemon at init for a broadcast
 * group per output; the daemon admits one when each receiver of the output runs on its own GPU
 * and none on the producer's.  Sends on such an output broadcast the slot over the group
 * (ncclBroadcast rooted at the producer, on the node stream); receivers post the matching
 * receive into local HBM as the descriptor arrives and hand the input out once it completes.
 * Outputs without a group keep the per-receiver pulls.  Groups formed (as producer / as
 * receiver), samples broadcast / received, bytes received, and the last group error ("" if
 * none). */
int dora_node_bcast_stats(dora_node* node, uint64_t* groups_out, uint64_t* groups_in,
                          uint64_t* sent, uint64_t* received, uint64_t* received_bytes,
                          const char** error);
/* Ranks of this node's broadcast groups as RCCL formed them: the largest group's rank count
 * (producer included; 0 without a group). */
int dora_node_bcast_ranks(dora_node* node, uint64_t* max_ranks);
/* Pack-kernel timing: hipExtLaunchKernel start/stop stamps of every n-th pack launch
 * (dora_node_set_timing_period; 0 = the default, 8). */
int dora_node_set_profiling(dora_node* node, int enable);
int dora_node_set_timing_period(dora_node* node, uint64_t period);
int dora_node_pack_stats(dora_node* node, uint64_t* count, double* total_ms, uint64_t* bytes);
/* (start, stop) of each pack of the last timed region in ms after its earliest start, from the
 * packs' own stamps (below); without a region, of each event-stamped pack in ms after
 * profiling was enabled.  `cap` pairs at most (concurrent packs overlap: their union is the
 * pack busy time). */
int dora_node_pack_intervals(dora_node* node, double* out_ms, size_t cap, size_t* count);
/* Device span of a run of sends: every pack that signals its own fill also stamps its first
 * workgroup's start and its signal time (s_memrealtime, 100 MHz) into its fill flag's line;
 * the span is the earliest start to the latest signal over the packs sent between region_begin
 * and region_end (which waits for them).  Packs that cannot stamp (kernel signal off,
 * compacting transforms) fall back to HIP events: the first pack's start stamp to events
 * recorded after the last pack on every stream.  Packs and sample bytes timed. */
int dora_node_region_begin(dora_node* node);
/* Wait until every fill this node launched (AQL packets, fill streams) and the work on its node
 * stream have completed (new; the node-scoped counterpart of a device synchronise). */
int dora_node_sync(dora_node* node);
/* Record the region's stop events now (after the last send), without waiting; region_end then
 * waits for them.  Lets a caller close its clock before it waits on the device. */
int dora_node_region_mark(dora_node* node);
int dora_node_region_end(dora_node* node, double* span_ms, uint64_t* packs, uint64_t* bytes);
/* Mean host time (µs) per send phase since profiling was (re)enabled: [0] allocate incl.
 * backpressure, [1] pack launch, [2] fill event record / stream sync, [3] descriptor send. */
int dora_node_send_profile(dora_node* node, double* out_us, size_t n_out, uint64_t* count);

/* ------------------------------------------------------------------------------------------ */
/* Daemon — the data-plane part of binaries/daemon (send_out, drop tokens, input closing)     */
/* ------------------------------------------------------------------------------------------ */
typedef struct dora_daemon dora_daemon;
/* Create the dataflow region `shm_name` ("/name").  `spec` lines:
 *   node <id> | output <node> <output> | input <node> <input> <src_node> <src_output> <queue>
 * and, for dataflows spanning machines (InterDaemonEvent, libraries/message/src/
 * daemon_to_daemon.rs:9-21; the reference's `_unstable_deploy.machine`):
 *   dataflow <id>                      shared by the daemons of one dataflow
 *   listen <host> <port>               accept peer daemons (port 0: any free port)
 *   machine <name> <host> <port>       a peer daemon
 *   remote <node> <output> <machine>   this output has receivers under that machine's daemon:
 *                                      its messages are staged to the host and sent there
 *   proxy <node> <gpu>                 <node> runs on another machine and feeds local inputs:
 *                                      the daemon serves it, re-sending its messages locally
 *                                      (device samples on GPU <gpu>, -1: inline host samples) */
int dora_daemon_create(const char* shm_name, const char* spec, size_t ring_bytes,
                       dora_daemon** out);
/* Route until every node is done (0), or timeout_ms elapses (DORA_ERR_TIMEOUT). */
int dora_daemon_run(dora_daemon* daemon, int64_t timeout_ms);
/* Send Event::Stop to every node. */
int dora_daemon_request_stop(dora_daemon* daemon);
int dora_daemon_stats(dora_daemon* daemon, uint64_t* routed, uint64_t* pending_tokens);
/* The port peer daemons connect to (-1: the spec has no `listen` and no `proxy` line). */
int dora_daemon_listen_port(dora_daemon* daemon, int* port);
/* Messages forwarded to other machines, device bytes staged for them, messages received. */
int dora_daemon_remote_stats(dora_daemon* daemon, uint64_t* forwarded, uint64_t* staged_bytes,
                             uint64_t* received);
void dora_daemon_free(dora_daemon* daemon);

#ifdef __cplusplus
}
#endif
#endif /* DORA_GPU_H */
