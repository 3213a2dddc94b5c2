// Runtime plumbing of the C ABI: errors, devices, streams, events, memory.
#include <hip/hip_runtime_api.h>

#include <unistd.h>

#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "aql.h"
#include "bcast.h"
#include "shm.h"
#include "common.h"

namespace dora {

static thread_local char g_last_error[1024] = "no error";
static std::atomic<uint64_t> g_idle_ns{0}, g_fill_wait_ns{0};

void add_idle_ns(uint64_t ns) { g_idle_ns.fetch_add(ns, std::memory_order_relaxed); }
void add_fill_wait_ns(uint64_t ns) { g_fill_wait_ns.fetch_add(ns, std::memory_order_relaxed); }

void set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
  va_end(ap);
}

int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
  va_end(ap);
  return code;
}

void clear_error() { std::strcpy(g_last_error, "no error"); }


}  // namespace dora

extern "C" {

const char* dora_gpu_last_error(void) { return dora::g_last_error; }

const char* dora_gpu_version(void) { return "dora-gpu 0.3.6-mi355x gfx950"; }

int dora_gpu_busy_stats(uint64_t* idle_ns, uint64_t* fill_wait_ns) {
  if (idle_ns) *idle_ns = dora::g_idle_ns.load(std::memory_order_relaxed);
  if (fill_wait_ns) *fill_wait_ns = dora::g_fill_wait_ns.load(std::memory_order_relaxed);
  return DORA_OK;
}

int dora_gpu_aql_dispatch_counts(int device, uint64_t* counts, size_t cap, size_t* n) {
  const size_t k = dora::aql_kernel_count();
  if (n) *n = k;
  for (size_t i = 0; i < k && i < cap && counts; ++i) counts[i] = dora::aql_dispatched(device, i);
  return DORA_OK;
}

int dora_gpu_aql_cp_signalled(int device, uint64_t* count) {
  if (!count) return dora::fail(DORA_ERR_INVALID, "NULL count");
  *count = dora::aql_cp_signalled(device);
  return DORA_OK;
}

int dora_gpu_set_keep_awake(double period_us) {
  if (!(period_us >= 0)) return dora::fail(DORA_ERR_INVALID, "keep-awake period must be >= 0");
  dora::aql_keep_awake(period_us);
  return DORA_OK;
}

int dora_gpu_aql_batch_stats(int device, uint64_t* batches, uint64_t* batched_msgs,
                             uint64_t* backlogged) {
  uint64_t a = 0, b = 0, c = 0;
  dora::aql_batch_stats(device, &a, &b, &c);
  if (batches) *batches = a;
  if (batched_msgs) *batched_msgs = b;
  if (backlogged) *backlogged = c;
  return DORA_OK;
}

const char* dora_gpu_aql_kernel_name(size_t k) {
  const char* s = dora::aql_kernel_name(k);
  return s ? s : "";
}

int dora_gpu_device_count(int* count) {
  if (!count) return dora::fail(DORA_ERR_INVALID, "count is NULL");
  DORA_HIP(hipGetDeviceCount(count));
  return DORA_OK;
}

int dora_gpu_set_device(int ordinal) {
  DORA_HIP(hipSetDevice(ordinal));
  return DORA_OK;
}

int dora_gpu_get_device(int* ordinal) {
  if (!ordinal) return dora::fail(DORA_ERR_INVALID, "ordinal is NULL");
  DORA_HIP(hipGetDevice(ordinal));
  return DORA_OK;
}

int dora_gpu_stream_create(dora_stream_t* out) {
  if (!out) return dora::fail(DORA_ERR_INVALID, "out is NULL");
  hipStream_t s;
  DORA_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  *out = s;
  return DORA_OK;
}

int dora_gpu_stream_destroy(dora_stream_t stream) {
  DORA_HIP(hipStreamDestroy(static_cast<hipStream_t>(stream)));
  return DORA_OK;
}

int dora_gpu_stream_sync(dora_stream_t stream) {
  DORA_HIP(hipStreamSynchronize(static_cast<hipStream_t>(stream)));
  return DORA_OK;
}

int dora_gpu_device_sync(void) {
  DORA_HIP(hipDeviceSynchronize());
  return DORA_OK;
}

int dora_gpu_malloc(void** out, size_t nbytes) {
  if (!out) return dora::fail(DORA_ERR_INVALID, "out is NULL");
  DORA_HIP(hipMalloc(out, nbytes ? nbytes : 1));
  return DORA_OK;
}

int dora_gpu_free(void* ptr) {
  dora::aql_fence_all();  // packs dispatched on the AQL queues may still read `ptr`
  DORA_HIP(hipFree(ptr));
  return DORA_OK;
}

int dora_gpu_host_alloc(void** out, size_t nbytes) {
  if (!out) return dora::fail(DORA_ERR_INVALID, "out is NULL");
  DORA_HIP(hipHostMalloc(out, nbytes ? nbytes : 1, hipHostMallocDefault));
  return DORA_OK;
}

int dora_gpu_host_free(void* ptr) {
  DORA_HIP(hipHostFree(ptr));
  return DORA_OK;
}

int dora_gpu_memcpy_async(void* dst, const void* src, size_t nbytes, dora_stream_t stream) {
  if (!nbytes) return DORA_OK;
  DORA_HIP(hipMemcpyAsync(dst, src, nbytes, hipMemcpyDefault, static_cast<hipStream_t>(stream)));
  return DORA_OK;
}

int dora_gpu_memset_async(void* dst, int value, size_t nbytes, dora_stream_t stream) {
  if (!nbytes) return DORA_OK;
  DORA_HIP(hipMemsetAsync(dst, value, nbytes, static_cast<hipStream_t>(stream)));
  return DORA_OK;
}

int dora_gpu_event_create(dora_event_t* out) {
  if (!out) return dora::fail(DORA_ERR_INVALID, "out is NULL");
  hipEvent_t e;
  DORA_HIP(hipEventCreate(&e));
  *out = e;
  return DORA_OK;
}

int dora_gpu_event_destroy(dora_event_t ev) {
  DORA_HIP(hipEventDestroy(static_cast<hipEvent_t>(ev)));
  return DORA_OK;
}

int dora_gpu_event_record(dora_event_t ev, dora_stream_t stream) {
  DORA_HIP(hipEventRecord(static_cast<hipEvent_t>(ev), static_cast<hipStream_t>(stream)));
  return DORA_OK;
}

int dora_gpu_event_sync(dora_event_t ev) {
  DORA_HIP(hipEventSynchronize(static_cast<hipEvent_t>(ev)));
  return DORA_OK;
}

int dora_gpu_event_elapsed_ms(dora_event_t start, dora_event_t stop, float* ms) {
  if (!ms) return dora::fail(DORA_ERR_INVALID, "ms is NULL");
  DORA_HIP(hipEventElapsedTime(ms, static_cast<hipEvent_t>(start), static_cast<hipEvent_t>(stop)));
  return DORA_OK;
}

}  // extern "C"
