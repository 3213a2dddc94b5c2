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

#ifdef __cplusplus
}
#endif
#endif /* DORA_GPU_H */
