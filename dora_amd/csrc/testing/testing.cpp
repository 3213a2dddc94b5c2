// libdora_gpu_testing.so: the test and microbenchmark hooks of the data plane, built apart from
// the shipped library (dora_amd/build.py build_testing) and linked against it — the product's
// ABI (include/dora_gpu.h) carries none of them.  Declared in include/dora_gpu_testing.h; used by
// tests/ and scripts/ only.  Each hook calls into the library's internals (aql.cpp, kernels.hip,
// bincode.cpp, bcast.cpp, shm.h).
#include <hip/hip_runtime_api.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <sys/prctl.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "aql.h"
#include "bcast.h"
#include "bincode.h"
#include "common.h"
#include "dora_gpu.h"
#include "dora_gpu_testing.h"
#include "plan.h"
#include "shm.h"

namespace dora {
// kernels.hip
int build_aql_batch_args(const BatchItem* items, size_t n, uint8_t* out, size_t cap,
                         uint32_t* grid);
int launch_l2_touch(const void* p, size_t len, hipStream_t stream);
int l1_stale_probe(int device, int mode, uint32_t* bad_first, uint32_t* stale, uint32_t* blocks);
}  // namespace dora

namespace dora {
namespace {

int copy_out(const std::vector<uint8_t>& v, uint8_t* out, size_t cap, size_t* out_len) {
  if (out_len) *out_len = v.size();
  if (!out || cap < v.size())
    return dora::fail(DORA_ERR_INVALID, "buffer of %zu bytes, %zu needed", cap, v.size());
  std::memcpy(out, v.data(), v.size());
  return DORA_OK;
}

std::string hex(const uint8_t* p, size_t n) {
  static const char* d = "0123456789abcdef";
  std::string s;
  s.reserve(2 * n);
  for (size_t i = 0; i < n; ++i) {
    s.push_back(d[p[i] >> 4]);
    s.push_back(d[p[i] & 15]);
  }
  return s;
}

std::string jstr(const std::string& v) {
  std::string s = "\"";
  for (unsigned char c : v) {
    if (c == '"' || c == '\\') {
      s.push_back('\\');
      s.push_back(static_cast<char>(c));
    } else if (c < 0x20) {
      char b[8];
      std::snprintf(b, sizeof(b), "\\u%04x", c);
      s += b;
    } else {
      s.push_back(static_cast<char>(c));
    }
  }
  return s + "\"";
}

}  // namespace
}  // namespace dora


extern "C" {

int dora_gpu_test_batch_args(size_t n_msgs, const size_t* seg_counts, const uint64_t* segs,
                             const uint64_t* dsts, const uint64_t* dst_caps,
                             const uint64_t* flags, const uint64_t* epochs, uint8_t* out,
                             size_t cap, uint32_t* grid) {
  if (!n_msgs || !seg_counts || !segs || !dsts || !dst_caps || !flags || !epochs || !out || !grid)
    return dora::fail(DORA_ERR_INVALID, "NULL argument");
  if (n_msgs > 8) return dora::fail(DORA_ERR_INVALID, "batch of %zu messages", n_msgs);
  std::vector<std::vector<dora::Segment>> s(n_msgs);
  dora::BatchItem items[8];
  size_t k = 0;
  for (size_t m = 0; m < n_msgs; ++m) {
    for (size_t j = 0; j < seg_counts[m]; ++j, ++k)
      s[m].push_back({reinterpret_cast<const void*>(segs[3 * k]), segs[3 * k + 1], segs[3 * k + 2]});
    items[m] = {s[m].data(), s[m].size(), reinterpret_cast<uint8_t*>(dsts[m]),
                dora::FillSignal{reinterpret_cast<uint64_t*>(flags[m]), epochs[m], nullptr},
                dst_caps[m]};
  }
  return dora::build_aql_batch_args(items, n_msgs, out, cap, grid);
}

int dora_gpu_test_l2_touch(const void* data, size_t len, dora_stream_t stream) {
  if (!data && len) return dora::fail(DORA_ERR_INVALID, "data is NULL");
  return dora::launch_l2_touch(data, len, static_cast<hipStream_t>(stream));
}

int dora_gpu_test_l1_stale(int device, int mode, uint32_t* bad_first, uint32_t* stale,
                           uint32_t* blocks) {
  if (!bad_first || !stale || !blocks || mode < 0 || mode > 2)
    return dora::fail(DORA_ERR_INVALID, "bad l1 stale probe arguments");
  DORA_GUARD_BEGIN
  return dora::l1_stale_probe(device, mode, bad_first, stale, blocks);
  DORA_GUARD_END
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


int dora_gpu_test_aql_hold(int device, int hold) { return dora::aql_hold(device, hold != 0); }

namespace {
hsa_status_t find_cpu_agent(hsa_agent_t a, void* p) {
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) == HSA_STATUS_SUCCESS &&
      t == HSA_DEVICE_TYPE_CPU) {
    *static_cast<hsa_agent_t*>(p) = a;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}
}  // namespace

int dora_gpu_test_d2h_copy_probe(int device, int mode, uint64_t bytes, uint32_t n,
                                 uint64_t gap_ns, uint64_t* out_ns) {
  if (!out_ns || !n || !bytes) return dora::fail(DORA_ERR_INVALID, "copy probe: arguments");
  DORA_HIP(hipSetDevice(device));
  void* src = nullptr;
  void* dst = nullptr;
  hipStream_t st = nullptr;
  DORA_HIP(hipMalloc(&src, bytes));
  DORA_HIP(hipMemset(src, 0x5a, bytes));
  DORA_HIP(hipHostMalloc(&dst, bytes, 0));
  DORA_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  DORA_HIP(hipDeviceSynchronize());
  hsa_agent_t gpu{}, cpu{};
  hsa_signal_t sig{0};
  if (mode == 1) {
    hsa_amd_pointer_info_t pi{};
    pi.size = sizeof(pi);
    if (hsa_init() != HSA_STATUS_SUCCESS ||
        hsa_amd_pointer_info(src, &pi, nullptr, nullptr, nullptr) != HSA_STATUS_SUCCESS ||
        hsa_iterate_agents(find_cpu_agent, &cpu) != HSA_STATUS_INFO_BREAK ||
        hsa_signal_create(1, 0, nullptr, &sig) != HSA_STATUS_SUCCESS)
      return dora::fail(DORA_ERR_HIP, "copy probe: HSA setup");
    gpu = pi.agentOwner;
  }
  using clock = std::chrono::steady_clock;
  int rc = DORA_OK;
  for (uint32_t i = 0; i < n && rc == DORA_OK; ++i) {
    const auto until = clock::now() + std::chrono::nanoseconds(gap_ns);
    while (clock::now() < until) std::this_thread::yield();
    const auto t0 = clock::now();
    if (mode == 1) {
      hsa_signal_store_relaxed(sig, 1);
      if (hsa_amd_memory_async_copy(dst, cpu, src, gpu, bytes, 0, nullptr, sig) !=
          HSA_STATUS_SUCCESS) {
        rc = dora::fail(DORA_ERR_HIP, "hsa_amd_memory_async_copy");
        break;
      }
      while (hsa_signal_load_scacquire(sig) != 0) {
        __builtin_ia32_pause();
        if (clock::now() - t0 > std::chrono::seconds(2)) {
          rc = dora::fail(DORA_ERR_TIMEOUT, "copy probe: no completion");
          break;
        }
      }
    } else if (hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, st) != hipSuccess ||
               hipStreamSynchronize(st) != hipSuccess) {
      rc = dora::fail(DORA_ERR_HIP, "hipMemcpyAsync");
    }
    out_ns[i] = uint64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(clock::now() - t0).count());
  }
  if (rc == DORA_OK && static_cast<const uint8_t*>(dst)[bytes - 1] != 0x5a)
    rc = dora::fail(DORA_ERR_INVALID, "copy probe: wrong bytes");
  if (sig.handle && rc == DORA_OK) hsa_signal_destroy(sig);
  (void)hipStreamDestroy(st);
  (void)hipHostFree(dst);
  (void)hipFree(src);
  return rc;
}

// Experiment: what ordering a sample written on the node stream costs per message
// (dora_node_send_output_sample -> order_fill): `n` kernels writing `bytes` on one stream, each
// followed by nothing (mode 0), hipStreamWriteValue64 into pinned host memory like a fill flag
// (1), or a second 8-byte kernel (2).  out_ns[0] = host enqueue ns per message, out_ns[1] =
// enqueue + drain ns per message.
int dora_gpu_test_stream_order_probe(int device, int mode, uint64_t bytes, uint32_t n,
                                     uint64_t* out_ns) {
  if (!out_ns || !n || !bytes || mode < 0 || mode > 2)
    return dora::fail(DORA_ERR_INVALID, "stream order probe: arguments");
  DORA_HIP(hipSetDevice(device));
  void* buf = nullptr;
  void* tiny = nullptr;
  uint64_t* word = nullptr;
  hipStream_t st = nullptr;
  DORA_HIP(hipMalloc(&buf, bytes));
  DORA_HIP(hipMalloc(&tiny, 64));
  DORA_HIP(hipHostMalloc(reinterpret_cast<void**>(&word), 64, hipHostMallocMapped));
  DORA_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  DORA_HIP(hipDeviceSynchronize());
  int rc = DORA_OK;
  using clock = std::chrono::steady_clock;
  const auto t0 = clock::now();
  for (uint32_t i = 0; i < n && rc == DORA_OK; ++i) {
    rc = dora_gpu_fill_splitmix(buf, bytes, i, st);
    if (rc != DORA_OK) break;
    if (mode == 1 && hipStreamWriteValue64(st, word, i + 1, 0) != hipSuccess)
      rc = dora::fail(DORA_ERR_HIP, "hipStreamWriteValue64");
    if (mode == 2) rc = dora_gpu_fill_splitmix(tiny, 8, i, st);
  }
  const auto t1 = clock::now();
  if (hipStreamSynchronize(st) != hipSuccess && rc == DORA_OK)
    rc = dora::fail(DORA_ERR_HIP, "hipStreamSynchronize");
  const auto t2 = clock::now();
  out_ns[0] = uint64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(t1 - t0).count()) / n;
  out_ns[1] = uint64_t(std::chrono::duration_cast<std::chrono::nanoseconds>(t2 - t0).count()) / n;
  if (rc == DORA_OK && mode == 1 && *reinterpret_cast<volatile uint64_t*>(word) != n)
    rc = dora::fail(DORA_ERR_INVALID, "stream order probe: flag %llu", (unsigned long long)*word);
  (void)hipStreamDestroy(st);
  (void)hipHostFree(word);
  (void)hipFree(tiny);
  (void)hipFree(buf);
  return rc;
}

int dora_gpu_test_reduce_timeout(uint64_t ns) {
  dora::aql_reduce_timeout(ns);
  return DORA_OK;
}

int dora_gpu_test_abandoned_slots(int device, uint32_t* slots) {
  if (!slots) return dora::fail(DORA_ERR_INVALID, "NULL argument");
  *slots = dora::aql_abandoned_slots(device);
  return DORA_OK;
}

int dora_gpu_test_keep_awake_stats(int device, uint64_t* heartbeats, int* parked) {
  if (!heartbeats || !parked) return dora::fail(DORA_ERR_INVALID, "NULL argument");
  bool pk = false;
  *heartbeats = dora::aql_heartbeats(device, &pk);
  *parked = pk ? 1 : 0;
  return DORA_OK;
}

int dora_gpu_test_aql_ring_wc(int device, int* wc, int* where) {
  if (!wc) return dora::fail(DORA_ERR_INVALID, "NULL argument");
  bool b = false;
  const int rc = dora::aql_ring_write_combined(device, &b, where);
  *wc = b ? 1 : 0;
  return rc;
}

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

int dora_gpu_test_bar_alloc(int device, size_t bytes, void** out) {
  if (!out) return dora::fail(DORA_ERR_INVALID, "out is NULL");
  return dora::bar_alloc(device, bytes, out);
}

int dora_gpu_test_bar_write(int device, void* dst, const void* src, size_t bytes) {
  if ((!dst || !src) && bytes) return dora::fail(DORA_ERR_INVALID, "NULL argument");
  return dora::bar_write(device, dst, src, bytes);
}

void dora_gpu_test_bar_free(void* ptr) { dora::bar_free(ptr); }

int dora_gpu_test_ide_output(const char* dataflow_id, const char* node_id,
                                        const char* output_id, const uint8_t* type_info,
                                        size_t type_info_len, const uint8_t* params,
                                        size_t params_len, uint64_t meta_ns, uint64_t event_ns,
                                        const uint8_t* hlc_id, const uint8_t* data, size_t data_len,
                                        int has_data, uint8_t* out, size_t cap, size_t* out_len) {
  if (!dataflow_id || !node_id || !output_id || !type_info || !hlc_id || (params_len && !params) ||
      (data_len && !data))
    return dora::fail(DORA_ERR_INVALID, "NULL argument");
  dora::InterDaemonEvent e;
  e.kind = dora::IDE_OUTPUT;
  e.dataflow_id = dataflow_id;
  e.node_id = node_id;
  e.output_id = output_id;
  e.type_info.assign(type_info, type_info + type_info_len);
  if (params_len) e.parameters.assign(params, params + params_len);
  e.timestamp_ns = meta_ns;
  e.event_ns = event_ns;
  std::memcpy(e.hlc_id.data(), hlc_id, 16);
  e.has_data = has_data != 0;
  if (data_len) e.data.assign(data, data + data_len);
  std::vector<uint8_t> f;
  try {
    dora::encode_ide(e, f);
  } catch (const std::exception& ex) {
    return dora::fail(DORA_ERR_INVALID, "%s", ex.what());
  }
  return dora::copy_out(f, out, cap, out_len);
}

int dora_gpu_test_ide_inputs_closed(const char* dataflow_id,
                                               const char* const* receivers,
                                               const char* const* inputs, size_t n,
                                               uint64_t event_ns, const uint8_t* hlc_id,
                                               uint8_t* out, size_t cap, size_t* out_len) {
  if (!dataflow_id || !hlc_id || (n && (!receivers || !inputs)))
    return dora::fail(DORA_ERR_INVALID, "NULL argument");
  dora::InterDaemonEvent e;
  e.kind = dora::IDE_INPUTS_CLOSED;
  e.dataflow_id = dataflow_id;
  for (size_t i = 0; i < n; ++i) e.inputs.emplace_back(receivers[i], inputs[i]);
  e.event_ns = event_ns;
  std::memcpy(e.hlc_id.data(), hlc_id, 16);
  std::vector<uint8_t> f;
  try {
    dora::encode_ide(e, f);
  } catch (const std::exception& ex) {
    return dora::fail(DORA_ERR_INVALID, "%s", ex.what());
  }
  return dora::copy_out(f, out, cap, out_len);
}

int dora_gpu_test_ide_decode(const uint8_t* frame, size_t len, char* json, size_t cap,
                                        size_t* json_len) {
  if (!frame && len) return dora::fail(DORA_ERR_INVALID, "NULL argument");
  dora::InterDaemonEvent e;
  try {
    e = dora::decode_ide(frame, len);
  } catch (const std::exception& ex) {
    return dora::fail(DORA_ERR_INVALID, "%s", ex.what());
  }
  using dora::hex;
  using dora::jstr;
  std::string j = "{\"kind\": " + std::to_string(e.kind) + ", \"dataflow_uuid\": \"" +
                  hex(e.dataflow_uuid.data(), 16) + "\", \"event_ns\": " +
                  std::to_string(e.event_ns);
  if (e.kind == dora::IDE_OUTPUT) {
    j += ", \"node_id\": " + jstr(e.node_id) + ", \"output_id\": " + jstr(e.output_id) +
         ", \"metadata_version\": " + std::to_string(e.meta_version) +
         ", \"meta_ns\": " + std::to_string(e.timestamp_ns) + ", \"type_info\": \"" +
         hex(e.type_info.data(), e.type_info.size()) + "\", \"parameters\": \"" +
         hex(e.parameters.data(), e.parameters.size()) + "\", \"has_data\": " +
         (e.has_data ? "true" : "false") + ", \"data\": \"" + hex(e.data.data(), e.data.size()) +
         "\"";
  } else {
    j += ", \"inputs\": [";
    for (size_t i = 0; i < e.inputs.size(); ++i)
      j += (i ? ", [" : "[") + jstr(e.inputs[i].first) + ", " + jstr(e.inputs[i].second) + "]";
    j += "]";
  }
  j += "}";
  std::vector<uint8_t> v(j.begin(), j.end());
  v.push_back(0);
  return dora::copy_out(v, reinterpret_cast<uint8_t*>(json), cap, json_len);
}

}  // extern "C"
