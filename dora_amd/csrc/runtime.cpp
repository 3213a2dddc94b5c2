// Runtime plumbing of the C ABI: errors, devices, streams, events, memory.
#include <hip/hip_runtime_api.h>

#include <execinfo.h>
#include <signal.h>
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

namespace {

struct sigaction g_prev_segv;

void on_segv(int sig, siginfo_t* info, void* ctx) {
  void* frames[64];
  const int n = backtrace(frames, 64);
  char head[128];
  const int k = std::snprintf(head, sizeof(head), "dora-gpu: signal %d at address %p, backtrace:\n",
                              sig, info ? info->si_addr : nullptr);
  if (k > 0) (void)!write(2, head, size_t(k));
  backtrace_symbols_fd(frames, n, 2);
  sigaction(SIGSEGV, &g_prev_segv, nullptr);  // then whatever handled it before (faulthandler)
  raise(sig);
}

// DORA_GPU_SEGV_TRACE=1: print a native backtrace on SIGSEGV (debugging aid on the GPU box,
// where no debugger may attach).
struct SegvTrace {
  SegvTrace() {
    const char* e = std::getenv("DORA_GPU_SEGV_TRACE");
    if (!e || *e != '1') return;
    struct sigaction sa;
    std::memset(&sa, 0, sizeof(sa));
    sa.sa_sigaction = on_segv;
    sa.sa_flags = SA_SIGINFO;
    sigaction(SIGSEGV, &sa, &g_prev_segv);
  }
} g_segv_trace;

}  // namespace

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

int dora_gpu_test_fill_reached(const void* flag, uint64_t epoch) {
  if (!flag || (reinterpret_cast<uintptr_t>(flag) & 63))
    return dora::fail(DORA_ERR_INVALID, "fill flag must be 64-byte aligned");
  return dora::fill_reached(static_cast<const std::atomic<uint64_t>*>(flag), epoch) ? 1 : 0;
}

int dora_gpu_test_cp_arm(void* flag, uint64_t epoch) {
  if (!flag || (reinterpret_cast<uintptr_t>(flag) & 63) || epoch == 0)
    return dora::fail(DORA_ERR_INVALID, "fill flag must be 64-byte aligned, epoch > 0");
  dora::cp_arm(static_cast<dora::FillFlag*>(flag), epoch);
  return DORA_OK;
}

int dora_gpu_aql_cp_signalled(int device, uint64_t* count) {
  if (!count) return dora::fail(DORA_ERR_INVALID, "NULL count");
  *count = dora::aql_cp_signalled(device);
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

int dora_gpu_test_aql_hold(int device, int hold) { return dora::aql_hold(device, hold != 0); }

int dora_gpu_test_bcast_group(int device, void* buf, uint64_t bytes, int* nranks, int* rank) {
  if (!buf || !nranks || !rank) return dora::fail(DORA_ERR_INVALID, "NULL argument");
  DORA_GUARD_BEGIN
  DORA_HIP(hipSetDevice(device));
  uint8_t uid[dora::kBcastIdBytes];
  int rc = dora::bcast_unique_id(uid);
  if (rc != DORA_OK) return rc;
  dora::BcastComm* c = nullptr;
  rc = dora::bcast_join(uid, 1, 0, 30000, &c);
  if (rc != DORA_OK) return rc;
  *nranks = dora::bcast_nranks(c);
  *rank = dora::bcast_rank(c);
  hipStream_t st = nullptr;
  if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) {
    dora::bcast_close(c, nullptr, 0);
    return dora::fail(DORA_ERR_HIP, "hipStreamCreate");
  }
  rc = dora::bcast_enqueue(c, buf, bytes, st);
  if (rc == DORA_OK && hipStreamSynchronize(st) != hipSuccess)
    rc = dora::fail(DORA_ERR_HIP, "broadcast stream: %s", hipGetErrorString(hipGetLastError()));
  dora::bcast_close(c, st, 10000);
  (void)hipStreamDestroy(st);
  return rc;
  DORA_GUARD_END
}

int dora_gpu_test_aql_pipeline(int device, size_t bytes, int n, int mode, int queues, int depth,
                               double* us_per_msg) {
  if (!us_per_msg) return dora::fail(DORA_ERR_INVALID, "us_per_msg is NULL");
  return dora::aql_pipeline_bench(device, bytes, n, mode, queues, depth, us_per_msg);
}

int dora_gpu_test_bar_alloc(int device, size_t bytes, void** out) {
  if (!out) return dora::fail(DORA_ERR_INVALID, "out is NULL");
  return dora::bar_alloc(device, bytes, out);
}

int dora_gpu_test_bar_write(int device, void* dst, const void* src, size_t bytes) {
  if ((!dst || !src) && bytes) return dora::fail(DORA_ERR_INVALID, "NULL argument");
  return dora::bar_write(device, dst, src, bytes);
}

void dora_gpu_test_bar_free(void* ptr) { dora::bar_free(ptr); }

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
