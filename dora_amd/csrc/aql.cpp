// Direct AQL dispatch of signalling packs (see aql.h): one HSA queue per device per process,
// the pack kernels from the code object embedded in this library (aql_kernels.hip,
// aql_blob.S).  Multi-segment packs read their 272-byte arguments from a device-memory ring
// the host writes through the BAR (one HDP flush per dispatch); single-segment packs take their
// 56 bytes preloaded into SGPRs by the command processor, from a ring in host memory (no BAR
// write, no flush: profiles/r01_aql_preload_probe.jsonl, 0.15 vs 1.6 us of host time).
#include "aql.h"

#include <hip/hip_runtime_api.h>
#include <hsa/hsa.h>
#include <hsa/amd_hsa_signal.h>
#include <hsa/hsa_ext_amd.h>
#include <immintrin.h>
#include <pthread.h>
#include <sys/prctl.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "common.h"
#include "shm.h"

static_assert(offsetof(amd_signal_t, value) == offsetof(dora::CpSignal, value) &&
                  offsetof(amd_signal_t, event_mailbox_ptr) ==
                      offsetof(dora::CpSignal, event_mailbox_ptr) &&
                  offsetof(amd_signal_t, start_ts) == offsetof(dora::CpSignal, start_ts) &&
                  sizeof(amd_signal_t) == sizeof(dora::CpSignal),
              "CpSignal must be laid out as amd_signal_t");
#include "subprof.h"

extern "C" const char dora_aql_code_object[];
extern "C" const char dora_aql_code_object_end[];

namespace dora {

// kernels.hip: the AQL kernels' argument block for `n` segments (<= aql_max_segments()).
int build_aql_args(const Segment* segs, size_t n, uint8_t* dst, const FillSignal& sig,
                   uint8_t* out, size_t cap, uint32_t* grid, uint64_t dst_cap);
size_t aql_args_size();
int build_aql_args1(const Segment& sg, uint8_t* dst, const FillSignal& sig, uint8_t* out,
                    uint32_t* grid);
size_t aql_batch_args_size();
uint32_t aql_chunk_bytes(const Segment* segs, size_t n);
int build_aql_batch_args(const BatchItem* items, size_t n, uint8_t* out, size_t cap,
                         uint32_t* grid);

namespace {

constexpr uint32_t kQueuePackets = 4096;
constexpr uint32_t kRingSlots = 512;
constexpr uint32_t kSlotBytes = 1024;    // AqlPackArgs 272 B, AqlBatchArgs 640 B
constexpr uint32_t kArgs1Bytes = 56;    // preloaded arguments of the single-segment kernels
constexpr uint32_t kHostSlotBytes = 64;
constexpr uint32_t kProfileSignals = 4096;
constexpr uint32_t kProfilePrealloc = 2048;  // created when profiling is first enabled

struct Use {
  const std::atomic<uint64_t>* flag = nullptr;
  uint64_t epoch = 0;
  uint64_t seq = 0;  // the dispatch's number (AqlQueue::next when it was written)
};

constexpr size_t kMaxItemSegs = 8;   // segments of one message the AQL path takes
constexpr size_t kBatchMsgs = 8;     // pack_device.h kMaxBatchMsgs
constexpr size_t kBatchSegs = 16;    // pack_device.h kMaxBatchSegs

// A send waiting for queue capacity (the backlog) or being dispatched.
struct Pending {
  Segment segs[kMaxItemSegs];
  size_t n = 0;
  uint8_t* dst = nullptr;
  FillSignal sig{};
  const std::atomic<uint64_t>* flag_host = nullptr;
  uint64_t dst_cap = 0, bytes = 0;
  uint32_t chunk = 0;
  bool profile = false;
  bool cp = false;  // signalled by the command processor (aql_cp_candidate)
  bool lone = false;  // runs alone on the GPU (a synchronous send, or every queue idle)
  bool read = false;  // read-signalled (dora_aql_pack1r_u4): a synchronous send returns on its read word
  uint64_t* cp_stamps = nullptr;  // CP-signalled: the timed region's stamp area (device), or none
};

}  // namespace

constexpr int kMaxQueues = 8;

// The kernels of the embedded code object, in AqlQueue::kobj order.
constexpr int kKernels = 6;
constexpr int kMultiKernel = 0;   // multi-segment packs (nested arrays)
constexpr int kOneKernel = 1;     // single-segment packs behind the acquire fence
constexpr int kOneCohKernel = 2;  // single-segment packs with agent-coherent loads, no fence
constexpr int kBatchKernel = 3;
constexpr int kReduceKernel = 4;
constexpr int kReadKernel = 5;    // read-signalled synchronous packs (aql_kernels.hip)
constexpr uint32_t kReduceArgsBytes = 32;  // base, areas, out, n, area_words
constexpr uint32_t kReadArgsBytes = 64;    // dst, src, len, rflag, done, epoch, stamps, grid, per
constexpr const char* kKernelNames[kKernels] = {"dora_aql_pack_u4", "dora_aql_pack1_u4",
                                                "dora_aql_pack1c_u4", "dora_aql_packb_u4",
                                                "dora_aql_stamp_reduce", "dora_aql_pack1r_u4"};

// Dispatch policy (every figure below was measured against the alternative
// on MI355X, the alternatives are not built any more):
// * four HSA queues per process: 4 MB 2.4 -> 2.1 us per message, C3 2.09 -> 2.41 TB/s against
//   two (profiles/r01_aql_queues_ab.jsonl);
//   Three instead (one compute queue fewer per sending process): C3 0.74-0.75 ->
//   0.65-0.66, native 4 MB 1.35-1.41 -> 1.91 us per message (profiles/r06_queues_ab.jsonl);
constexpr int kQueues = 4;
// * packs of [1 MiB, 32 MiB) are signalled by the command processor (the packet's completion
//   signal, every wave waiting for its own stores), so consecutive packets of a queue overlap:
//   4 MB over 4 queues 1.95 -> 1.59-1.64 us each (profiles/r03_aql_pipeline_probe.jsonl), C3's
//   multi-segment clouds too (r04, profiles/r04_c3_ab.jsonl).  Larger packs only when they run
//   alone (a synchronous send): 40.96 MB 17.8-18.3 -> 14.05 us own time;
constexpr uint64_t kCpLo = uint64_t(1) << 20, kCpHi = uint64_t(32) << 20;
// * HBM-bound packs from 8 MiB run in order per queue (barrier bit) over four queues, three from
//   32 MiB: C3 0.68-0.70 -> 0.72-0.75 (profiles/r04_full_ab.jsonl), 40.96 MB 14.1-14.5 ->
//   12.9-13.0 us per pack (profiles/r02_aql_big_ab.jsonl);
constexpr uint64_t kBarrierBytes = uint64_t(8) << 20;
// * a queue holds at most two in-kernel-signalled packets (one running, one ready) and three
//   CP-signalled ones (they overlap: 4 MB 1.88 -> 1.66 us at depth 3, r03_cp_signal_ab.jsonl);
//   sends finding every queue that deep leave together as a batch pack of <= 32 MiB.
constexpr size_t kDepth = 2, kCpDepth = 3;
constexpr uint64_t kBatchBytes = uint64_t(32) << 20;

// Publish an AQL packet whose body is written: its header last, then the doorbell.  In the
// default packet ring (coherent system memory, x86 TSO) program order suffices.  A ring the
// runtime put in device memory behind the PCIe BAR (HSA_ALLOCATE_QUEUE_DEV_MEM=1) is
// write-combined, where x86 keeps no store order: fences put the body ahead of the header and
// the header ahead of the doorbell.  (That placement was measured and is not recommended: the
// synchronous 40.96 MB send gains ~1 us, pipelined sends lose 10-40 % to the fenced BAR writes,
// DESIGN §9.1.)
inline void publish_packet(hsa_queue_t* q, void* p, uint32_t header_setup, uint64_t idx,
                           bool wc_ring) {
  if (wc_ring) __builtin_ia32_sfence();
  __atomic_store_n(reinterpret_cast<uint32_t*>(p), header_setup, __ATOMIC_RELEASE);
  if (wc_ring) __builtin_ia32_sfence();
  hsa_signal_store_relaxed(q->doorbell_signal, hsa_signal_value_t(idx));
}

struct AqlQueue {
  std::mutex mu;
  hsa_agent_t gpu{};
  bool wc_ring = false;  // packet rings in device memory (write-combined): fenced publication
  int ring_where = 0;    // diagnostics: pointer type * 4 + owner (1 CPU agent, 2 this GPU, 3 other)
  // Packs rotate over these hardware queues: one queue overlaps consecutive packs only partly
  // (4 MB: 3.6 us per pack back to back on one queue, 1.9 on two; profiles/r01_aql_probe.jsonl),
  // and the command processor's per-queue dispatch rate bounds a pipeline of <= 8 messages in
  // flight (traces: ~12 us from dispatch to fill flag at 2 queues).  4 queues (kQueues):
  // 4 MB 2.4 -> 2.1 us per message, C3 2.09 -> 2.41 TB/s, the 40.96 MB
  // headline (HIP fill streams) unchanged (profiles/r01_aql_queues_ab.jsonl).
  hsa_queue_t* qs[kMaxQueues] = {};
  uint64_t rd[kMaxQueues] = {};  // last read index seen per queue (the CP writes it to host memory)
  int nq = 0;
  // kKernelNames order
  uint64_t kobj[kKernels] = {};
  uint32_t group[kKernels] = {}, priv[kKernels] = {};
  uint8_t* ring = nullptr;    // kRingSlots x kSlotBytes of device memory, host-mapped
  uint8_t* hring = nullptr;   // kRingSlots x kHostSlotBytes of host memory (single-segment packs)
  uint32_t* hdp = nullptr;    // HDP_MEM_FLUSH_CNTL
  uint64_t next = 0, next_big = 0;
  Use uses[kRingSlots];
  // argument slots left to a packet that may still run (a stamp reduction that timed out): never
  // written again (take_slot skips them)
  bool abandoned[kRingSlots] = {};
  uint32_t n_abandoned = 0;
  std::atomic<bool> failed{false};
  bool profiling = false;
  std::vector<hsa_signal_t> free_sigs, used_sigs;
  uint64_t ts_freq = 0;
  uint64_t dispatched[kKernels] = {};  // packets per kernel (kKernelNames order)
  // Batching (aql_pack): per queue, the packets dispatched and not yet seen complete (the fill
  // flag + epoch their last message signals); sends that find every queue `depth` packets deep
  // wait in the backlog and leave together, one batch pack per dispatch, when a queue drains.
  std::deque<Use> outq[kMaxQueues];
  std::deque<Pending> backlog;
  std::condition_variable cv;  // backlog non-empty (the dispatcher thread waits on it)
  bool dispatcher = false;
  bool hold = false;  // test tool (aql_hold): every batchable send waits in the backlog
  uint64_t batches = 0, batched_msgs = 0, backlogged = 0, cp_signalled = 0;
  // test tool (bar_alloc): the GPU's coarse-grained pool, host-accessible through the BAR
  hsa_agent_t cpu{};
  hsa_amd_memory_pool_t coarse{};
  bool coarse_ok = false;
  // HIP device of the queues, and the stream that takes sends a failed queue could not dispatch
  // (fallback_locked)
  int device = -1;
  hipStream_t fallback = nullptr;
  uint64_t fallbacks = 0;
  hsa_signal_t reduce_sig{0};  // completion of aql_stamp_reduce's dispatch
  // Keeping the dispatch side awake (warm_main): packets dispatched so far (written under mu),
  // and whether the warm thread is parked (no dispatch for kWarmWindow)
  std::atomic<uint64_t> activity{0};
  std::atomic<bool> warm_parked{false};
  std::atomic<bool> warm_stop{false};  // process exit (stop_warm_threads)
  std::thread warm_thread;
  std::atomic<uint64_t> heartbeats{0};  // empty packets published (aql_heartbeats)
  std::mutex warm_mu;
  std::condition_variable warm_cv;
};

namespace {

struct Agents {
  uint32_t bdf = 0, domain = 0;
  hsa_agent_t gpu{}, cpu{};
  bool gpu_ok = false, cpu_ok = false;
  int matches = 0;  // GPU agents at this PCI location (> 1: a partitioned GPU)
  hsa_amd_memory_pool_t pool{};
  bool pool_ok = false, pool_fine = false;
  hsa_amd_memory_pool_t kernarg{};  // host memory the command processor reads arguments from
  bool kernarg_ok = false;
};

hsa_status_t on_agent(hsa_agent_t a, void* p) {
  Agents* f = static_cast<Agents*>(p);
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS)
    return HSA_STATUS_SUCCESS;
  if (t == HSA_DEVICE_TYPE_GPU) {
    uint32_t bdf = 0, dom = 0;
    hsa_agent_get_info(a, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_BDFID), &bdf);
    hsa_agent_get_info(a, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_DOMAIN), &dom);
    if (bdf == f->bdf && dom == f->domain) {
      f->gpu = a;
      f->gpu_ok = true;
      ++f->matches;
    }
  } else if (t == HSA_DEVICE_TYPE_CPU && !f->cpu_ok) {
    f->cpu = a;
    f->cpu_ok = true;
  }
  return HSA_STATUS_SUCCESS;
}

hsa_status_t on_pool(hsa_amd_memory_pool_t pool, void* p) {
  Agents* f = static_cast<Agents*>(p);
  hsa_amd_segment_t seg;
  hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
  if (seg != HSA_AMD_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
  bool alloc = false;
  hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_RUNTIME_ALLOC_ALLOWED, &alloc);
  if (!alloc) return HSA_STATUS_SUCCESS;
  uint32_t flags = 0;
  hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
  const bool fine = flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_FINE_GRAINED;
  if (!f->pool_ok || (fine && !f->pool_fine)) {
    f->pool = pool;
    f->pool_ok = true;
    f->pool_fine = fine;
  }
  return HSA_STATUS_SUCCESS;
}

hsa_status_t on_coarse_pool(hsa_amd_memory_pool_t pool, void* p) {
  auto* out = static_cast<std::pair<hsa_amd_memory_pool_t, bool>*>(p);
  hsa_amd_segment_t seg;
  hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
  if (seg != HSA_AMD_SEGMENT_GLOBAL || out->second) return HSA_STATUS_SUCCESS;
  bool alloc = false;
  hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_RUNTIME_ALLOC_ALLOWED, &alloc);
  uint32_t flags = 0;
  hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
  if (alloc && (flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_COARSE_GRAINED)) {
    out->first = pool;
    out->second = true;
  }
  return HSA_STATUS_SUCCESS;
}

hsa_status_t on_cpu_pool(hsa_amd_memory_pool_t pool, void* p) {
  Agents* f = static_cast<Agents*>(p);
  hsa_amd_segment_t seg;
  hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
  if (seg != HSA_AMD_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
  uint32_t flags = 0;
  hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
  if ((flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_KERNARG_INIT) && !f->kernarg_ok) {
    f->kernarg = pool;
    f->kernarg_ok = true;
  }
  return HSA_STATUS_SUCCESS;
}

void on_queue_error(hsa_status_t st, hsa_queue_t*, void* data) {
  const char* m = nullptr;
  hsa_status_string(st, &m);
  std::fprintf(stderr, "dora-gpu: AQL pack queue error: %s\n", m ? m : "?");
  static_cast<AqlQueue*>(data)->failed.store(true);
}

// Set up the queue of HIP device `device`; nullptr (and a note on stderr when DORA_GPU_TRACE
// is set) when anything is missing.
AqlQueue* create(int device) {
  auto note = [&](const char* what) {
    if (std::getenv("DORA_GPU_TRACE"))
      std::fprintf(stderr, "dora-gpu: AQL dispatch off on device %d: %s\n", device, what);
    return nullptr;
  };
  int bus = 0, dev = 0, dom = 0;
  if (hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, device) != hipSuccess ||
      hipDeviceGetAttribute(&dev, hipDeviceAttributePciDeviceId, device) != hipSuccess ||
      hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, device) != hipSuccess)
    return note("PCI location");
  if (hsa_init() != HSA_STATUS_SUCCESS) return note("hsa_init");
  Agents f;
  f.bdf = (uint32_t(bus) << 8) | (uint32_t(dev) << 3);
  f.domain = uint32_t(dom);
  hsa_iterate_agents(on_agent, &f);
  if (!f.gpu_ok || !f.cpu_ok) return note("agent");
  // a partitioned GPU (several agents at one PCI location) cannot be told apart here
  if (f.matches != 1) return note("several GPU agents at the device's PCI location");
  hsa_amd_agent_iterate_memory_pools(f.gpu, on_pool, &f);
  if (!f.pool_ok) return note("device memory pool");
  auto* a = new AqlQueue();
  a->gpu = f.gpu;
  a->device = device;
  hsa_amd_hdp_flush_t hdp{};
  if (hsa_agent_get_info(f.gpu, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_HDP_FLUSH),
                         &hdp) != HSA_STATUS_SUCCESS ||
      !hdp.HDP_MEM_FLUSH_CNTL) {
    delete a;
    return note("HDP flush register");
  }
  a->hdp = hdp.HDP_MEM_FLUSH_CNTL;
  // code object
  hsa_code_object_reader_t reader;
  hsa_executable_t exe;
  const size_t co_size = size_t(dora_aql_code_object_end - dora_aql_code_object);
  if (hsa_code_object_reader_create_from_memory(dora_aql_code_object, co_size, &reader) !=
          HSA_STATUS_SUCCESS ||
      hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT,
                                nullptr, &exe) != HSA_STATUS_SUCCESS ||
      hsa_executable_load_agent_code_object(exe, f.gpu, reader, nullptr, nullptr) !=
          HSA_STATUS_SUCCESS ||
      hsa_executable_freeze(exe, nullptr) != HSA_STATUS_SUCCESS) {
    delete a;
    return note("code object");
  }
  for (int k = 0; k < kKernels; ++k) {
    hsa_executable_symbol_t sym;
    uint32_t ka = 0;
    const std::string sym_name = std::string(kKernelNames[k]) + ".kd";
    if (hsa_executable_get_symbol_by_name(exe, sym_name.c_str(), &f.gpu, &sym) != HSA_STATUS_SUCCESS ||
        hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT,
                                       &a->kobj[k]) != HSA_STATUS_SUCCESS ||
        hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE,
                                       &ka) != HSA_STATUS_SUCCESS ||
        hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE,
                                       &a->group[k]) != HSA_STATUS_SUCCESS ||
        hsa_executable_symbol_get_info(
            sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &a->priv[k]) !=
            HSA_STATUS_SUCCESS ||
        ka != (k == kMultiKernel    ? aql_args_size()
               : k == kBatchKernel  ? aql_batch_args_size()
               : k == kReduceKernel ? size_t(kReduceArgsBytes)
               : k == kReadKernel   ? size_t(kReadArgsBytes)
                                    : size_t(kArgs1Bytes)) ||
        ka > kSlotBytes) {
      delete a;
      return note("kernel symbol / argument size");  // no hidden arguments expected
    }
  }
  // argument ring: device memory the host writes through the BAR
  void* ring = nullptr;
  if (hsa_amd_memory_pool_allocate(f.pool, size_t(kRingSlots) * kSlotBytes, 0, &ring) !=
          HSA_STATUS_SUCCESS ||
      hsa_amd_agents_allow_access(1, &f.cpu, nullptr, ring) != HSA_STATUS_SUCCESS) {
    delete a;
    return note("argument ring");
  }
  a->ring = static_cast<uint8_t*>(ring);
  // every slot starts out as a valid no-op pack (no segments, no flag), made visible with a
  // read-back once: a dispatch can never see uninitialised arguments
  std::vector<uint8_t> zero(kSlotBytes, 0);
  for (uint32_t r = 0; r < kRingSlots; ++r)
    std::memcpy(a->ring + size_t(r) * kSlotBytes, zero.data(), kSlotBytes);
  __builtin_ia32_sfence();
  (void)*reinterpret_cast<volatile uint32_t*>(a->ring + size_t(kRingSlots - 1) * kSlotBytes);
  const int create_queues = std::min(kMaxQueues, kQueues);
  for (int i = 0; i < create_queues; ++i) {
    if (hsa_queue_create(f.gpu, kQueuePackets, HSA_QUEUE_TYPE_SINGLE, on_queue_error, a,
                         UINT32_MAX, UINT32_MAX, &a->qs[i]) != HSA_STATUS_SUCCESS)
      break;
    a->nq = i + 1;
  }
  // where the runtime put the packet rings: system memory unless HSA_ALLOCATE_QUEUE_DEV_MEM,
  // which allocates them from this GPU's memory (owner: the GPU agent)
  if (a->nq > 0) {
    hsa_amd_pointer_info_t pi{};
    pi.size = sizeof(pi);
    if (hsa_amd_pointer_info(a->qs[0]->base_address, &pi, nullptr, nullptr, nullptr) ==
        HSA_STATUS_SUCCESS) {
      const int owner = pi.agentOwner.handle == f.cpu.handle   ? 1
                        : pi.agentOwner.handle == f.gpu.handle ? 2
                        : pi.agentOwner.handle                  ? 3
                                                                : 0;
      a->ring_where = int(pi.type) * 4 + owner;
      a->wc_ring = owner == 2;
    }
  }
  if (a->nq == 0) {
    hsa_amd_memory_pool_free(ring);
    delete a;
    return note("queue");
  }
  // host-memory argument ring of the single-segment kernels (their arguments are preloaded once
  // per dispatch by the command processor, so no wave reads them over PCIe)
  hsa_amd_agent_iterate_memory_pools(f.cpu, on_cpu_pool, &f);
  void* hr = nullptr;
  if (f.kernarg_ok &&
      hsa_amd_memory_pool_allocate(f.kernarg, size_t(kRingSlots) * kHostSlotBytes, 0, &hr) ==
          HSA_STATUS_SUCCESS) {
    if (hsa_amd_agents_allow_access(1, &f.gpu, nullptr, hr) == HSA_STATUS_SUCCESS) {
      std::memset(hr, 0, size_t(kRingSlots) * kHostSlotBytes);
      a->hring = static_cast<uint8_t*>(hr);
    } else {
      hsa_amd_memory_pool_free(hr);
    }
  }
  hsa_system_get_info(HSA_SYSTEM_INFO_TIMESTAMP_FREQUENCY, &a->ts_freq);
  a->cpu = f.cpu;
  std::pair<hsa_amd_memory_pool_t, bool> coarse{{}, false};
  hsa_amd_agent_iterate_memory_pools(f.gpu, on_coarse_pool, &coarse);
  a->coarse = coarse.first;
  a->coarse_ok = coarse.second;
  return a;
}

}  // namespace

namespace {
void warm_main(AqlQueue* a);
void stop_warm_threads();
std::mutex g_queues_mu;
AqlQueue* g_queues[64] = {};
}  // namespace

AqlQueue* aql_queue(int device) {
  static std::mutex& mu = g_queues_mu;
  static AqlQueue** queues = g_queues;
  static bool tried[64] = {};
  if (device < 0 || device >= 64) return nullptr;
  std::lock_guard<std::mutex> g(mu);
  if (!tried[device]) {
    tried[device] = true;
    queues[device] = create(device);
    // the warm thread (warm_main) lives as long as the process, like the queues; it is stopped
    // and joined at exit, before HIP's and HSA's own teardown (registered earlier, so run later)
    if (queues[device]) {
      queues[device]->warm_thread = std::thread(warm_main, queues[device]);
      static std::once_flag once;
      std::call_once(once, [] {
        std::atexit(stop_warm_threads);
        // a forked child has no warm threads: it must not join its parent's
        pthread_atfork(nullptr, nullptr, [] {
          for (AqlQueue* q : g_queues)
            if (q && q->warm_thread.joinable()) {
              new (&q->warm_thread) std::thread();
              q->warm_stop.store(true);
            }
        });
      });
    }
  }
  AqlQueue* q = queues[device];
  return (q && !q->failed.load()) ? q : nullptr;
}

bool aql_usable(const AqlQueue* q) { return q && !q->failed.load(std::memory_order_relaxed); }

size_t aql_max_segments() { return 8; }

namespace {
// Wait (bounded) until the dispatcher has dispatched every backlogged send: their fill flags are
// in no argument slot before that.
void drain_backlog(AqlQueue* a, std::chrono::steady_clock::time_point t0,
                   std::chrono::steady_clock::duration limit) {
  for (;;) {
    {
      std::lock_guard<std::mutex> g(a->mu);
      if (a->backlog.empty() || a->failed.load()) return;
    }
    if (std::chrono::steady_clock::now() - t0 > limit) return;
    std::this_thread::yield();
  }
}
}  // namespace

void aql_fence_all() {
  AqlQueue* qs[64];
  {
    std::lock_guard<std::mutex> g(g_queues_mu);
    std::copy(g_queues, g_queues + 64, qs);
  }
  const auto t0 = std::chrono::steady_clock::now();
  for (AqlQueue* a : qs) {
    if (!a) continue;
    drain_backlog(a, t0, std::chrono::seconds(5));
    std::lock_guard<std::mutex> g(a->mu);
    // fills launched through HIP after a failed dispatch (fallback_locked) are in no Use
    if (a->fallback) (void)hipStreamSynchronize(a->fallback);
    for (Use& u : a->uses)
      while (u.flag && !fill_reached(u.flag, u.epoch) &&
             std::chrono::steady_clock::now() - t0 < std::chrono::seconds(5))
        __builtin_ia32_pause();
  }
}

void aql_forget_flags(int device, const void* base, size_t size) {
  AqlQueue* a = aql_queue(device);
  if (!a) return;
  const auto t0 = std::chrono::steady_clock::now();
  drain_backlog(a, t0, std::chrono::seconds(2));
  std::lock_guard<std::mutex> g(a->mu);
  // fallback fills (fallback_locked) write flags in no Use: the region must outlive them
  if (a->fallback) (void)hipStreamSynchronize(a->fallback);
  const auto* lo = static_cast<const uint8_t*>(base);
  // sends still backlogged after the bound: never dispatched, and their flags are about to go
  // away — drop them rather than let a later dispatch write into the unmapped region
  std::deque<Pending> keep_backlog;
  for (const Pending& p : a->backlog) {
    const auto* f = reinterpret_cast<const uint8_t*>(p.flag_host);
    if (f < lo || f >= lo + size) keep_backlog.push_back(p);
  }
  a->backlog.swap(keep_backlog);
  for (auto& o : a->outq) {  // outstanding entries pointing into the region go too
    std::deque<Use> keep;
    for (const Use& u : o) {
      const auto* f = reinterpret_cast<const uint8_t*>(u.flag);
      if (f < lo || f >= lo + size) keep.push_back(u);
    }
    o.swap(keep);
  }
  for (Use& u : a->uses) {
    const auto* f = reinterpret_cast<const uint8_t*>(u.flag);
    if (!u.flag || f < lo || f >= lo + size) continue;
    while (!fill_reached(u.flag, u.epoch) &&
           std::chrono::steady_clock::now() - t0 < std::chrono::seconds(2))
      __builtin_ia32_pause();
    u.flag = nullptr;  // the slot is free; the flag's region goes away
  }
}

namespace {

// Queues the barrier-bit packs of `bytes` spread over: three from 32 MiB (three concurrent 40 MB
// copies saturate HBM: 12.9-13.0 us per pack on three queues vs 13.2 on four,
// profiles/r02_aql_big_ab.jsonl), four below (C3's 13 MB clouds: 0.71-0.72 -> 0.75 of HBM over
// the 20-cloud burst, profiles/r04_full_ab.jsonl).
// Read-signalled packs (dora_aql_pack1r_u4): <= kReadLaneUnits (12) units of 16 B per lane
// (plan.h), <= kMaxSignalWgs workgroups (their done words), so up to 192 MiB; 1024
// workgroups unless that holds too little, and no more than give every lane 4 units: a
// synchronous 4 MiB send 8.4-8.7 -> 7.2-7.5 us against one unit per lane, 40.96 MB unchanged
// (profiles/r06_read_grid_ab.jsonl; 8 units per lane 7.2-7.4).
constexpr uint64_t kReadLaneMin = 4;
constexpr uint64_t kReadMaxUnits = uint64_t(kMaxSignalWgs) * 256 * kReadLaneUnits;
uint32_t read_grid(uint64_t units) {
  const uint64_t need = (units + 256 * kReadLaneUnits - 1) / (256 * kReadLaneUnits);
  const uint64_t fill =
      std::min<uint64_t>(1024, (units + 256 * kReadLaneMin - 1) / (256 * kReadLaneMin));
  return static_cast<uint32_t>(std::max<uint64_t>(std::max(need, fill), 1));
}
int big_queues(int nq, uint64_t bytes) {
  return std::min(nq, bytes >= (uint64_t(32) << 20) ? 3 : 4);
}

// The argument slot of dispatch number a->next (a->mu held), past any abandoned slot.
uint64_t take_slot(AqlQueue* a) {
  while (a->abandoned[a->next % kRingSlots]) ++a->next;
  return a->next % kRingSlots;
}

// The number of the oldest dispatch still in an outstanding list (a->next when none is).
uint64_t oldest_outstanding(const AqlQueue* a) {
  uint64_t m = a->next;
  for (int i = 0; i < a->nq; ++i)
    if (!a->outq[i].empty()) m = std::min(m, a->outq[i].front().seq);
  return m;
}

// Write and ring one packet on queue `qi` (a->mu held): one message with the single- or
// multi-segment kernels, or a batch of `n` > 1 messages with dora_aql_packb_u4.
void wake_warm(AqlQueue* a);

int dispatch_locked(AqlQueue* a, size_t qi, const Pending* items, size_t n, bool big) {
  const Pending& it0 = items[0];
  const Segment* segs = it0.segs;
  uint8_t* const dst = it0.dst;
  const FillSignal& sig = it0.sig;
  const bool profile = std::any_of(items, items + n, [](const Pending& x) { return x.profile; });
  // the argument slot of the dispatch kRingSlots back must have completed.  Every dispatch
  // sits in its queue's outstanding list until seen complete (prune) and the lists hold
  // dispatches in order, so one older than every list's front is complete: no load of its flag
  // line (which the GPU has written since: a cache miss per send)
  const uint64_t r = take_slot(a);
  Use& u = a->uses[r];
  if (u.flag && u.seq >= oldest_outstanding(a) && !fill_reached(u.flag, u.epoch)) {
    const auto t0 = std::chrono::steady_clock::now();
    while (!fill_reached(u.flag, u.epoch)) {
      __builtin_ia32_pause();
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(5)) {
        a->failed.store(true);  // a pack that never completes: stop dispatching here
        return fail(DORA_ERR_TIMEOUT, "AQL argument slot still in use after 5 s");
      }
    }
  }
  SubSpan sp_args(SP_AQL_ARGS);
  uint8_t args[kSlotBytes];
  uint32_t grid = 0;
  // one segment at sample offset 0: the preloaded kernels, arguments from host memory
  const bool batch = n > 1;
  const bool one = !batch && a->hring && it0.n == 1 && segs[0].dst_off == 0;
  // A mid-size pack, or a lone big single-segment one, signalled by the command processor
  // (aql_cp_candidate): no in-kernel flag, every wave waits for its own stores, the packet's
  // completion signal is the flag's CpSignal line (shm.h FillFlag)
  const bool cp = !batch && it0.cp && it0.flag_host;
  int rc;
  if (it0.read) {
    // dst, src, len, the flag line's read word, done words, epoch, stamp area, grid, units per
    // workgroup (read_grid)
    const uint64_t units = segs[0].len >> 4;
    grid = read_grid(units);
    const uint32_t per = static_cast<uint32_t>((units + grid - 1) / grid);
    const uint64_t w[7] = {reinterpret_cast<uintptr_t>(dst), reinterpret_cast<uintptr_t>(segs[0].src),
                           segs[0].len,
                           reinterpret_cast<uintptr_t>(sig.flag) + offsetof(FillFlag, read_epoch),
                           reinterpret_cast<uintptr_t>(sig.done), sig.epoch,
                           reinterpret_cast<uintptr_t>(it0.cp_stamps)};
    std::memcpy(args, w, sizeof(w));
    std::memcpy(args + 56, &grid, 4);
    std::memcpy(args + 60, &per, 4);
    rc = DORA_OK;
  } else if (batch) {
    BatchItem bi[kBatchMsgs];
    for (size_t m = 0; m < n; ++m)
      bi[m] = {items[m].segs, items[m].n, items[m].dst, items[m].sig, items[m].dst_cap};
    rc = build_aql_batch_args(bi, n, args, sizeof(args), &grid);
  } else if (cp) {
    // no flag, done words non-null: per-wave store waits; `epoch` carries the stamp area
    const FillSignal per_wave{nullptr, reinterpret_cast<uintptr_t>(it0.cp_stamps), sig.done};
    rc = one ? build_aql_args1(segs[0], dst, per_wave, args, &grid)
             : build_aql_args(segs, it0.n, dst, per_wave, args, sizeof(args), &grid, it0.dst_cap);
  } else if (one) {
    rc = build_aql_args1(segs[0], dst, sig, args, &grid);
  } else {
    rc = build_aql_args(segs, it0.n, dst, sig, args, sizeof(args), &grid, it0.dst_cap);
  }
  if (rc != DORA_OK) return rc;
  hsa_signal_t done{0};
  if (cp) {
    // set the flag up for this fill (its previous fill has completed: the slot was reused), then
    // name the epoch; the command processor's decrement completes it (fill_reached)
    static_assert(AMD_SIGNAL_KIND_USER == 1, "cp_arm's signal kind");
    cp_arm(reinterpret_cast<FillFlag*>(const_cast<std::atomic<uint64_t>*>(it0.flag_host)),
           sig.epoch);
    // the device address of the CpSignal line: the flag's device address + its offset
    done.handle = reinterpret_cast<uint64_t>(sig.flag) + offsetof(FillFlag, cp);
  } else if (profile && a->profiling) {
    if (a->free_sigs.empty() && a->used_sigs.size() < kProfileSignals) {
      hsa_signal_t s;
      if (hsa_signal_create(1, 0, nullptr, &s) == HSA_STATUS_SUCCESS) a->free_sigs.push_back(s);
    }
    if (!a->free_sigs.empty()) {
      done = a->free_sigs.back();
      a->free_sigs.pop_back();
      hsa_signal_store_relaxed(done, 1);
      a->used_sigs.push_back(done);
    }
  }
  uint8_t* slot;
  // A lone single-segment pack (nothing to overlap its dispatch with) takes its arguments from
  // the device ring like a multi-segment one: the command processor's preload then reads HBM, not
  // host memory over PCIe — 0.6-0.7 us less from doorbell to completion at any size
  // (aql_pipeline_bench modes 5 vs 7, profiles/r04_lone_dispatch_ab.jsonl).  Pipelined packs keep
  // the host ring: no HDP flush per send.
  const bool dev_args1 = (one && it0.lone) || it0.read;
  if (one && !dev_args1) {
    // coherent host memory: ordered before the packet header's release store (x86 TSO)
    slot = a->hring + r * kHostSlotBytes;
    std::memcpy(slot, args, kArgs1Bytes);
  } else {
    slot = a->ring + r * kSlotBytes;
    std::memcpy(slot, args, it0.read ? kReadArgsBytes
                            : one    ? kArgs1Bytes
                            : batch  ? aql_batch_args_size()
                                     : aql_args_size());
    // write-combined stores leave the CPU, the HDP flush makes them visible to the GPU; both
    // are posted writes ordered before the doorbell
    __builtin_ia32_sfence();
    *reinterpret_cast<volatile uint32_t*>(a->hdp) = 1;  // UC store: ordered before the packet
  }
  // HBM-bound packs (>= barrier_bytes) run in order per queue (barrier bit) over at most three
  // queues (aql_pack).  Smaller packs overlap freely on all queues.
  sp_args.stop();
  SubSpan sp_disp(SP_AQL_DISPATCH);
  hsa_queue_t* const q = a->qs[qi];
  // Wait for a free packet slot before reserving one: a reserved packet must be written, or the
  // command processor stalls at its INVALID header for good.  This process is the queue's only
  // producer (HSA_QUEUE_TYPE_SINGLE, under a->mu), so the write index cannot move meanwhile.  The
  // read index lives in host memory the CP writes: reload it (a cache miss) only when the last
  // value seen does not already prove a free slot.
  const uint64_t idx = hsa_queue_load_write_index_relaxed(q);
  if (idx - a->rd[qi] >= q->size) {
    const auto t0 = std::chrono::steady_clock::now();
    while (idx - (a->rd[qi] = hsa_queue_load_read_index_scacquire(q)) >= q->size) {
      __builtin_ia32_pause();
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(5)) {
        a->failed.store(true);  // a stuck queue: later sends take the HIP fill streams
        return fail(DORA_ERR_TIMEOUT, "AQL queue full for 5 s");
      }
    }
  }
  hsa_queue_store_write_index_relaxed(q, idx + 1);
  auto* p = static_cast<hsa_kernel_dispatch_packet_t*>(q->base_address) + (idx & (q->size - 1));
  // A CP-signalled single-segment pack inside the CP window (1-32 MiB), and a lone one, read
  // their source with agent-coherent loads (dora_aql_pack1c_u4: sc1 nt, bypassing the CU's L1 like
  // the fenced kernel's nt loads) and their packets carry no acquire fence: the packet's acquire is
  // a per-packet cost of the command processor (4 MB: 1.50-1.58 -> 1.37-1.46 us per message
  // pipelined; a lone pack's dispatch 0.1-0.2 us, r04_lone_dispatch_ab.jsonl), and a
  // pack whose every source load bypasses the CU's L1 has nothing for it to invalidate (DESIGN §8:
  // inside one dispatch only plain loads re-read stale words; across dispatches no configuration
  // ever read stale, test_gpu_fence.py rewrites the source between > 512 such packs).  Their
  // arguments come preloaded into SGPRs, or from the device ring behind the HDP flush (lone).
  // Pipelined packs outside the window and multi-segment packs keep the fence.
  const bool coh = it0.read || (one && ((cp && it0.bytes < kCpHi) || it0.lone));
  const int k = it0.read ? kReadKernel
                : batch  ? kBatchKernel
                : one    ? (coh ? kOneCohKernel : kOneKernel)
                         : kMultiKernel;
  p->workgroup_size_x = 256;
  p->workgroup_size_y = 1;
  p->workgroup_size_z = 1;
  p->reserved0 = 0;
  p->grid_size_x = grid * 256u;
  p->grid_size_y = 1;
  p->grid_size_z = 1;
  p->private_segment_size = a->priv[k];
  p->group_segment_size = a->group[k];
  p->kernel_object = a->kobj[k];
  p->kernarg_address = slot;
  p->reserved2 = 0;
  p->completion_signal = done;
  // agent-scope acquire: the pack reads device memory of this GPU; it publishes its sample
  // itself (write-through stores + fill flag), so no release.  Below the barrier size no barrier
  // bit, so packs of one queue overlap (ramps and signal tails hide behind each other); HBM-bound
  // packs at or above it run one at a time per queue, like HIP stream order (more concurrent
  // 40 MB copies only contend for HBM).  No release fence at the end of a pack: its sample, done
  // words and fill flag are all stored write-through (sc1 / system scope) and complete before the
  // flag is set, so the kernel-end L2 write-back has nothing of the pack's to publish — and costs
  // C3 ~8 % of its device time (5.18-5.41 -> 4.81-4.83 us per cloud, profiles/r02_release_ab.jsonl).
  const uint16_t header = (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                          (big ? (1 << HSA_PACKET_HEADER_BARRIER) : 0) |
                          ((coh ? HSA_FENCE_SCOPE_NONE : HSA_FENCE_SCOPE_AGENT)
                           << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                          (HSA_FENCE_SCOPE_NONE << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
  const uint16_t setup = 1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;
  publish_packet(q, p, header | (uint32_t(setup) << 16), idx, a->wc_ring);
  a->activity.store(a->next + 1, std::memory_order_relaxed);  // the warm thread's clock
  if (a->warm_parked.load(std::memory_order_relaxed)) wake_warm(a);
  // every message of a batch signals at its end: the last one's flag stands for the packet
  u.flag = items[n - 1].flag_host;
  u.epoch = items[n - 1].sig.epoch;
  u.seq = a->next;
  a->outq[qi].push_back(u);
  ++a->next;
  ++a->dispatched[k];
  if (cp) ++a->cp_signalled;
  if (batch) {
    ++a->batches;
    a->batched_msgs += n;
  }
  return DORA_OK;
}

// Drop the completed packets at the front of queue `i`'s outstanding list.
void prune(AqlQueue* a, int i) {
  auto& o = a->outq[i];
  while (!o.empty() && fill_reached(o.front().flag, o.front().epoch))
    o.pop_front();
}

// No queue has an outstanding packet (a pack dispatched now runs alone on the GPU).
bool queues_idle(AqlQueue* a) {
  if (!a->backlog.empty()) return false;
  for (int i = 0; i < a->nq; ++i) {
    prune(a, i);
    if (!a->outq[i].empty()) return false;
  }
  return true;
}

// The first queue in round-robin order, among the first `nq` (0: the first kQueues), with fewer than `depth`
// outstanding packets, or -1.  An idle queue is taken without loading anything; a busy one is
// pruned first (one load of its oldest packet's flag line, which the GPU has written since: a
// cache miss), and only as far as needed — r03 pruned all four queues on every send.
int pick_queue(AqlQueue* a, int nq = 0, size_t depth = 0) {
  if (a->hold) return -1;
  if (nq <= 0 || nq > a->nq) nq = std::min(a->nq, kQueues);
  const size_t d = depth ? depth : kDepth;
  for (int j = 0; j < nq; ++j) {
    const int i = int((a->next + uint64_t(j)) % uint64_t(nq));
    if (a->outq[i].size() >= d) prune(a, i);
    if (a->outq[i].size() < d) return i;
  }
  return -1;
}

// Sends that were accepted (aql_pack returned DORA_OK) but can no longer leave through the AQL
// queues — a dispatch failed and the queues are marked failed — are launched through HIP on
// the fallback stream instead, each signalling its own fill flag in-kernel (launch_pack), so
// no sender or receiver waits out a timeout for a fill that was never dispatched (a->mu held).
void fallback_locked(AqlQueue* a, const Pending* items, size_t n) {
  if (!n) return;
  int prev = -1;
  (void)hipGetDevice(&prev);
  if (prev != a->device) (void)hipSetDevice(a->device);
  if (!a->fallback && hipStreamCreateWithFlags(&a->fallback, hipStreamNonBlocking) != hipSuccess) {
    a->fallback = nullptr;
    std::fprintf(stderr, "dora-gpu: AQL fallback stream: %s; %zu fills lost\n",
                 hipGetErrorString(hipGetLastError()), n);
  }
  for (size_t k = 0; k < n && a->fallback; ++k) {
    const Pending& p = items[k];
    bool signalled = false;
    if (launch_pack(p.segs, p.n, ARROW_DEVICE_ROCM, p.dst, a->fallback, nullptr, nullptr, &p.sig,
                    &signalled, p.dst_cap) != DORA_OK ||
        !signalled)
      std::fprintf(stderr, "dora-gpu: AQL fallback launch failed: %s\n", dora_gpu_last_error());
    else
      ++a->fallbacks;
  }
  if (prev >= 0 && prev != a->device) (void)hipSetDevice(prev);
}

void fallback_backlog_locked(AqlQueue* a) {
  std::vector<Pending> rest(a->backlog.begin(), a->backlog.end());
  a->backlog.clear();
  fallback_locked(a, rest.data(), rest.size());
}

// Dispatch the backlog into queues with room, as batches of consecutive sends that share a
// chunk size (a->mu held).
void pump_locked(AqlQueue* a) {
  if (a->failed.load()) fallback_backlog_locked(a);
  while (!a->backlog.empty() && !a->failed.load()) {
    // the batch at the front of the backlog
    size_t n = 0, segs = 0;
    uint64_t bytes = 0;
    for (const Pending& p : a->backlog) {
      if (n == kBatchMsgs) break;
      if (n && (segs + p.n > kBatchSegs || p.chunk != a->backlog.front().chunk ||
                bytes + p.bytes > kBatchBytes))
        break;
      segs += p.n;
      bytes += p.bytes;
      ++n;
    }
    const int qi = pick_queue(a, 0, n == 1 && a->backlog.front().cp ? kCpDepth : 0);
    if (qi < 0) return;
    Pending batch[kBatchMsgs];
    for (size_t k = 0; k < n; ++k) {
      batch[k] = a->backlog.front();
      a->backlog.pop_front();
    }
    if (dispatch_locked(a, size_t(qi), batch, n, false) != DORA_OK) {
      // the queues are unusable from here on: these sends and the rest of the backlog leave
      // through HIP instead
      a->failed.store(true);
      fallback_locked(a, batch, n);
      fallback_backlog_locked(a);
      return;
    }
  }
}

// One empty barrier-AND packet (no dependencies, no completion signal) on the first queue
// (a->mu held); nothing if that queue's ring is full.
void heartbeat_locked(AqlQueue* a) {
  hsa_queue_t* const q = a->qs[0];
  const uint64_t idx = hsa_queue_load_write_index_relaxed(q);
  if (idx - a->rd[0] >= q->size && idx - (a->rd[0] = hsa_queue_load_read_index_scacquire(q)) >= q->size)
    return;
  hsa_queue_store_write_index_relaxed(q, idx + 1);
  auto* p = static_cast<hsa_barrier_and_packet_t*>(q->base_address) + (idx & (q->size - 1));
  std::memset(reinterpret_cast<uint8_t*>(p) + 4, 0, sizeof(*p) - 4);
  const uint16_t header = (HSA_PACKET_TYPE_BARRIER_AND << HSA_PACKET_HEADER_TYPE) |
                          (HSA_FENCE_SCOPE_NONE << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                          (HSA_FENCE_SCOPE_NONE << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
  publish_packet(q, p, header, idx, a->wc_ring);
  a->heartbeats.fetch_add(1, std::memory_order_relaxed);
}

// Keeping the dispatch side awake.  Once no packet of the process has reached the GPU for
// 50-200 us, the next one takes ~5.5 us longer from doorbell to completion: a device message 1 ms
// after the previous one arrives in 11.5-11.8 us instead of 5.6-6.1.  A resident
// sleeping wave does not prevent that, nor do PCIe reads or writes of device memory; an empty
// barrier-AND packet every 40 us does (5.4-5.9 us, profiles/r05_small_lat_heartbeat_zb.jsonl).
// So while the process is sending, this thread wakes every `period` and, when nothing was
// dispatched since its last wake, publishes one such packet; kWarmWindow after the last dispatch
// it parks until the next.  dora_gpu_set_keep_awake sets the period (default 25 us; 0: off).
constexpr auto kWarmWindow = std::chrono::milliseconds(100);
// A slow periodic sender — its last kSlowSends dispatches each came more than kSlowGap after the
// one before — would pay kSlowGap / period wake-ups per message for a wake-up of ~5.5 us
// (a 10 Hz sender never parked): its thread parks kSlowIdle after each dispatch
// instead (the command processor itself idles after 50-200 us), and one quicker dispatch brings
// the 100 ms window back.
constexpr auto kSlowGap = std::chrono::milliseconds(5);
constexpr auto kSlowIdle = std::chrono::microseconds(200);
constexpr int kSlowSends = 3;
std::atomic<int64_t> g_warm_period_ns{25000};

void warm_main(AqlQueue* a) {
  (void)prctl(PR_SET_TIMERSLACK, 1UL, 0, 0, 0);  // wake on time, not up to 50 us late
  using clock = std::chrono::steady_clock;
  uint64_t seen = a->activity.load(std::memory_order_relaxed);
  auto last_change = clock::now();
  auto next = last_change;
  int slow = 0;  // consecutive dispatches more than kSlowGap apart
  auto note_gap = [&](clock::time_point now) {
    slow = now - last_change > kSlowGap ? std::min(slow + 1, kSlowSends) : 0;
    last_change = now;
  };
  while (!a->failed.load(std::memory_order_relaxed) &&
         !a->warm_stop.load(std::memory_order_relaxed)) {
    const auto period = std::chrono::nanoseconds(g_warm_period_ns.load(std::memory_order_relaxed));
    if (period.count() <= 0) {  // off: look again every 10 ms
      std::this_thread::sleep_for(std::chrono::milliseconds(10));
      seen = a->activity.load(std::memory_order_relaxed);
      last_change = next = clock::now();
      continue;
    }
    next += period;
    std::this_thread::sleep_until(next);
    auto now = clock::now();
    if (next + period < now) next = now;  // descheduled: resume the beat, do not catch up
    const uint64_t c = a->activity.load(std::memory_order_relaxed);
    if (c != seen) {
      seen = c;
      note_gap(now);
      continue;
    }
    if (now - last_change > (slow >= kSlowSends ? std::chrono::duration_cast<clock::duration>(kSlowIdle)
                                                 : std::chrono::duration_cast<clock::duration>(kWarmWindow))) {
      // park; a dispatch wakes it (wake_warm).  The 10 ms bound covers a dispatch that raced
      // the parking.
      std::unique_lock<std::mutex> lk(a->warm_mu);
      a->warm_parked.store(true);
      while (a->warm_parked.load() && a->activity.load(std::memory_order_relaxed) == seen &&
             !a->failed.load(std::memory_order_relaxed) &&
             !a->warm_stop.load(std::memory_order_relaxed))
        a->warm_cv.wait_for(lk, std::chrono::milliseconds(10));
      a->warm_parked.store(false);
      seen = a->activity.load(std::memory_order_relaxed);
      note_gap(clock::now());  // woken by a dispatch (or the stop)
      next = last_change;
      continue;
    }
    if (a->mu.try_lock()) {  // busy: a send is being dispatched right now
      heartbeat_locked(a);
      a->mu.unlock();
    }
  }
}

// At exit: no empty packet may be written into a queue while HSA tears it down.
void stop_warm_threads() {
  for (AqlQueue* a : g_queues) {
    if (!a || !a->warm_thread.joinable()) continue;
    {
      std::lock_guard<std::mutex> g(a->warm_mu);
      a->warm_stop.store(true);
    }
    a->warm_cv.notify_all();
    a->warm_thread.join();
  }
}

void wake_warm(AqlQueue* a) {
  {
    std::lock_guard<std::mutex> g(a->warm_mu);
    a->warm_parked.store(false);
  }
  a->warm_cv.notify_one();
}

// The dispatcher thread: dispatches the backlog as queues drain while no send is being made.
void dispatcher_main(AqlQueue* a) {
  std::unique_lock<std::mutex> lk(a->mu);
  for (;;) {
    a->cv.wait(lk, [a] { return !a->backlog.empty(); });
    pump_locked(a);
    if (a->backlog.empty() || a->failed.load()) {
      if (a->failed.load()) fallback_backlog_locked(a);
      continue;
    }
    // every queue is full: wait (unlocked) for the oldest packet of any queue to complete
    Use front[kMaxQueues];
    for (int i = 0; i < a->nq; ++i) front[i] = a->outq[i].empty() ? Use{} : a->outq[i].front();
    lk.unlock();
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t spin = 0;; ++spin) {
      bool any = false;
      for (int i = 0; i < a->nq && !any; ++i)
        any = !front[i].flag || fill_reached(front[i].flag, front[i].epoch);
      if (any) break;
      if ((spin & 1023) == 1023) {
        const auto dt = std::chrono::steady_clock::now() - t0;
        if (dt > std::chrono::milliseconds(2)) break;  // re-check under the lock
        if (dt > std::chrono::microseconds(200)) std::this_thread::yield();
      }
      __builtin_ia32_pause();
    }
    lk.lock();
  }
}

}  // namespace

int aql_pack(AqlQueue* a, const Segment* segs, size_t n, uint8_t* dst, const FillSignal& sig,
             const std::atomic<uint64_t>* flag_host, bool profile, uint64_t dst_cap,
             uint64_t* cp_stamps, bool sync, bool* read_signalled) {
  if (read_signalled) *read_signalled = false;
  if (!a || a->failed.load()) return fail(DORA_ERR_HIP, "AQL queue unavailable");
  if (n == 0 || n > kMaxItemSegs) return fail(DORA_ERR_INVALID, "AQL pack: %zu segments", n);
  SubSpan sp_all(SP_AQL_PACK);
  Pending p;
  std::copy(segs, segs + n, p.segs);
  p.n = n;
  p.dst = dst;
  p.sig = sig;
  p.flag_host = flag_host;
  p.dst_cap = dst_cap;
  p.profile = profile;
  p.cp_stamps = cp_stamps;
  for (size_t i = 0; i < n; ++i) p.bytes += segs[i].len;
  std::lock_guard<std::mutex> g(a->mu);
  // lone: runs alone on the GPU (a synchronous send, or every queue idle): its arguments go to
  // the device ring and it reads without the acquire fence (dispatch_locked).  Signalled by the
  // command processor (inside a timed region only with a stamp area for the pack's own stamps):
  // a pack in the CP window, and a synchronous single-segment pack above it (aql.h).  An async
  // send that finds the queues idle usually opens a burst: given the whole GPU (3584 workgroups)
  // it delays the packs queued right behind it, so it keeps the in-kernel signal (the 20-step
  // headline 0.778 vs 0.786 mean over six interleaved rounds, profiles/r04_headline20_ab.jsonl).
  // (lone only shapes a single-segment pack — its argument ring and kernel — so a multi-segment
  // one skips the idle check, which loads a GPU-written flag line per queue)
  p.lone = sync || (n == 1 && segs[0].dst_off == 0 && queues_idle(a));
  p.cp = (!profile || cp_stamps) && flag_host && aql_cp_candidate(segs, n, sync);
  // a synchronous CP-signalled single-segment pack of aligned bytes up to what its workgroups
  // hold in VGPRs: read-signalled (dora_aql_pack1r_u4)
  p.read = sync && p.cp && n == 1 && segs[0].op == SEG_COPY &&
           segs[0].dst_off == 0 && sig.done && sig.flag && p.bytes >= kCpLo &&
           (p.bytes >> 4) <= kReadMaxUnits &&
           ((reinterpret_cast<uintptr_t>(segs[0].src) | reinterpret_cast<uintptr_t>(dst)) & 15) == 0;
  if (read_signalled) *read_signalled = p.read;
  // HBM-bound packs (>= kBarrierBytes) run in order per queue (barrier bit) over at most three
  // (four below 32 MiB) queues, big_queues: more concurrent 40 MB copies only contend (14.1-14.5
  // us per pack without the barrier, 12.9-13.0 with it; profiles/r02_aql_big_ab.jsonl).
  const bool big = p.bytes >= kBarrierBytes;
  if (big) {
    const size_t qi = size_t(a->next_big++ % uint64_t(big_queues(a->nq, p.bytes)));
    const int rc = dispatch_locked(a, qi, &p, 1, true);
    // pruning loads the oldest packet's flag line (a cache miss the GPU caused): only once the
    // queue holds more than the two it runs in turn
    if (a->outq[qi].size() > 2) prune(a, int(qi));
    return rc;
  }
  // Below that, a queue holds at most kDepth packets (one running, one ready): the command
  // processor runs a queue's packets one after another with a ~1-2 us gap, four queues at most
  // share the compute pipes, so a send that finds them all busy waits in the backlog
  // and leaves with the sends queued behind it as one batch pack — fewer, larger dispatches
  // instead of more queues.
  p.chunk = aql_chunk_bytes(segs, n);
  if (a->backlog.empty()) {
    const int qi = pick_queue(a, 0, p.cp ? kCpDepth : 0);
    if (qi >= 0) return dispatch_locked(a, size_t(qi), &p, 1, false);
  }
  a->backlog.push_back(p);
  ++a->backlogged;
  pump_locked(a);
  if (!a->backlog.empty()) {
    if (!a->dispatcher) {
      a->dispatcher = true;
      std::thread(dispatcher_main, a).detach();
    }
    a->cv.notify_one();
  }
  return DORA_OK;
}

uint64_t aql_heartbeats(int device, bool* parked) {
  if (device < 0 || device >= 64) return 0;
  AqlQueue* a;
  {
    std::lock_guard<std::mutex> g(g_queues_mu);
    a = g_queues[device];
  }
  if (!a) return 0;
  if (parked) *parked = a->warm_parked.load();
  return a->heartbeats.load();
}

void aql_keep_awake(double period_us) {
  g_warm_period_ns.store(period_us > 0 ? int64_t(std::max(period_us, 5.0) * 1000) : 0);
}

bool aql_cp_candidate(const Segment* segs, size_t n, bool lone) {
  if (n == 0) return false;
  const bool single = n == 1 && segs[0].dst_off == 0;
  uint64_t bytes = 0;
  for (size_t i = 0; i < n; ++i) bytes += segs[i].len;
  // a lone single-segment pack above the window is CP-signalled too (r04)
  return bytes >= kCpLo && (bytes < kCpHi || (lone && single));
}

int bar_alloc(int device, size_t bytes, void** out) {
  AqlQueue* a = aql_queue(device);
  if (!a || !a->coarse_ok) return fail(DORA_ERR_UNSUPPORTED, "no AQL queue / coarse-grained pool");
  void* p = nullptr;
  if (hsa_amd_memory_pool_allocate(a->coarse, bytes, 0, &p) != HSA_STATUS_SUCCESS)
    return fail(DORA_ERR_HIP, "hsa_amd_memory_pool_allocate");
  if (hsa_amd_agents_allow_access(1, &a->cpu, nullptr, p) != HSA_STATUS_SUCCESS) {
    hsa_amd_memory_pool_free(p);
    return fail(DORA_ERR_UNSUPPORTED, "host access to device memory (no large BAR)");
  }
  *out = p;
  return DORA_OK;
}

int bar_write(int device, void* dst, const void* src, size_t bytes) {
  AqlQueue* a = aql_queue(device);
  if (!a) return fail(DORA_ERR_UNSUPPORTED, "no AQL queue");
  std::memcpy(dst, src, bytes);
  __builtin_ia32_sfence();
  *reinterpret_cast<volatile uint32_t*>(a->hdp) = 1;
  // a read-back of the last line: the posted writes have reached the memory
  if (bytes) (void)*reinterpret_cast<volatile uint8_t*>(static_cast<uint8_t*>(dst) + bytes - 1);
  return DORA_OK;
}

void bar_free(void* p) {
  if (p) hsa_amd_memory_pool_free(p);
}

int bar_map(AqlQueue* q, void* p) {
  if (!aql_usable(q)) return fail(DORA_ERR_UNSUPPORTED, "no AQL queue");
  if (hsa_amd_agents_allow_access(1, &q->cpu, nullptr, p) != HSA_STATUS_SUCCESS)
    return fail(DORA_ERR_UNSUPPORTED, "host access to device memory (no large BAR)");
  return DORA_OK;
}

namespace {
// 32-B non-temporal stores for the aligned body: the BAR mapping is write-combined, and
// streaming stores leave the CPU in whole lines without a read for ownership (4 KB: 1.94 us vs
// 3.17 for memcpy, readback included, profiles/r06_host_path_probe.jsonl)
__attribute__((target("avx2"))) void stream_body(uint8_t* d, const uint8_t* s, size_t n) {
  size_t i = 0;
  for (; i + 128 <= n; i += 128) {
    const __m256i a = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i));
    const __m256i b = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i + 32));
    const __m256i c = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i + 64));
    const __m256i e = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i + 96));
    _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i), a);
    _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i + 32), b);
    _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i + 64), c);
    _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i + 96), e);
  }
  for (; i + 32 <= n; i += 32)
    _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i),
                        _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i)));
  if (i < n) std::memcpy(d + i, s + i, n - i);
}
}  // namespace

void bar_copy(void* dst, const void* src, size_t n) {
  auto* d = static_cast<uint8_t*>(dst);
  auto* s = static_cast<const uint8_t*>(src);
  const size_t head = std::min(n, size_t((32 - (reinterpret_cast<uintptr_t>(d) & 31)) & 31));
  if (head) std::memcpy(d, s, head);
  stream_body(d + head, s + head, n - head);
}

void bar_publish(AqlQueue* q, const void* last) {
  __builtin_ia32_sfence();
  *reinterpret_cast<volatile uint32_t*>(q->hdp) = 1;
  // a read (non-posted) behind the posted writes: once it returns, they have reached the memory,
  // whichever agent reads the sample next
  if (last) (void)*static_cast<const volatile uint8_t*>(last);
}

size_t aql_kernel_count() { return kKernels; }

const char* aql_kernel_name(size_t k) { return k < size_t(kKernels) ? kKernelNames[k] : nullptr; }

int aql_ring_write_combined(int device, bool* wc, int* where) {
  AqlQueue* a = aql_queue(device);
  if (!a) return fail(DORA_ERR_UNSUPPORTED, "no AQL queue on device %d", device);
  *wc = a->wc_ring;
  if (where) *where = a->ring_where;
  return DORA_OK;
}

int aql_hold(int device, bool hold) {
  AqlQueue* a = aql_queue(device);
  if (!a) return fail(DORA_ERR_UNSUPPORTED, "no AQL queue on device %d", device);
  std::lock_guard<std::mutex> g(a->mu);
  a->hold = hold;
  if (!hold) {
    pump_locked(a);
    if (!a->backlog.empty()) a->cv.notify_one();
  }
  return DORA_OK;
}

int aql_batch_stats(int device, uint64_t* batches, uint64_t* batched_msgs, uint64_t* backlogged) {
  *batches = *batched_msgs = *backlogged = 0;
  if (device < 0 || device >= 64) return DORA_OK;
  AqlQueue* a;
  {
    std::lock_guard<std::mutex> g(g_queues_mu);
    a = g_queues[device];
  }
  if (!a) return DORA_OK;
  std::lock_guard<std::mutex> g(a->mu);
  *batches = a->batches;
  *batched_msgs = a->batched_msgs;
  *backlogged = a->backlogged;
  return DORA_OK;
}

namespace {
hsa_status_t first_cpu_agent(hsa_agent_t a, void* p) {
  hsa_device_type_t t;
  if (hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t) == HSA_STATUS_SUCCESS &&
      t == HSA_DEVICE_TYPE_CPU) {
    *static_cast<hsa_agent_t*>(p) = a;
    return HSA_STATUS_INFO_BREAK;
  }
  return HSA_STATUS_SUCCESS;
}

// The GPU agent owning device memory `p` (this process's or IPC-imported), or none.
bool gpu_owner(const void* p, hsa_agent_t* out) {
  hsa_amd_pointer_info_t pi{};
  pi.size = sizeof(pi);
  hsa_device_type_t t{};
  if (hsa_amd_pointer_info(const_cast<void*>(p), &pi, nullptr, nullptr, nullptr) !=
          HSA_STATUS_SUCCESS ||
      (pi.type != HSA_EXT_POINTER_TYPE_HSA && pi.type != HSA_EXT_POINTER_TYPE_IPC) ||
      !pi.agentOwner.handle ||
      hsa_agent_get_info(pi.agentOwner, HSA_AGENT_INFO_DEVICE, &t) != HSA_STATUS_SUCCESS ||
      t != HSA_DEVICE_TYPE_GPU)
    return false;
  *out = pi.agentOwner;
  return true;
}
}  // namespace

int hsa_copy_host(void* dst, const void* src, uint64_t n, bool to_host) {
  static hsa_agent_t cpu{};
  static const bool ok = [] {
    return hsa_init() == HSA_STATUS_SUCCESS &&
           hsa_iterate_agents(first_cpu_agent, &cpu) == HSA_STATUS_INFO_BREAK;
  }();
  if (!ok) return fail(DORA_ERR_UNSUPPORTED, "no HSA CPU agent");
  hsa_agent_t gpu{};
  if (!gpu_owner(to_host ? src : dst, &gpu))
    return fail(DORA_ERR_UNSUPPORTED, "not device memory the runtime knows");
  // completion signals are pooled process-wide (any thread may stage or pull; a signal per
  // thread would leak with every short-lived one), and never destroyed: the pool is as large as
  // the most copies ever in flight at once
  // (never freed either: a thread still copying during exit finds them)
  static auto* pool_mu = new std::mutex;
  static auto* pool = new std::vector<hsa_signal_t>;
  hsa_signal_t sig{0};
  {
    std::lock_guard<std::mutex> g(*pool_mu);
    if (!pool->empty()) {
      sig = pool->back();
      pool->pop_back();
    }
  }
  if (!sig.handle && hsa_signal_create(1, 0, nullptr, &sig) != HSA_STATUS_SUCCESS)
    return fail(DORA_ERR_UNSUPPORTED, "hsa_signal_create");
  auto give_back = [&] {
    std::lock_guard<std::mutex> g(*pool_mu);
    pool->push_back(sig);
  };
  hsa_signal_store_relaxed(sig, 1);
  if (hsa_amd_memory_async_copy(dst, to_host ? cpu : gpu, src, to_host ? gpu : cpu, n, 0, nullptr,
                                sig) != HSA_STATUS_SUCCESS) {
    give_back();
    return fail(DORA_ERR_UNSUPPORTED, "hsa_amd_memory_async_copy refused the copy");
  }
  const auto t0 = std::chrono::steady_clock::now();
  for (uint32_t spin = 0; hsa_signal_load_scacquire(sig) != 0; ++spin) {
    __builtin_ia32_pause();
    if ((spin & 1023) == 1023) {
      const auto dt = std::chrono::steady_clock::now() - t0;
      if (dt > std::chrono::seconds(10))  // the copy may still complete: its signal is dropped
        return fail(DORA_ERR_TIMEOUT, "copy engine did not complete in 10 s");
      if (dt > std::chrono::microseconds(200)) std::this_thread::yield();
    }
  }
  give_back();
  return DORA_OK;
}

uint64_t aql_cp_signalled(int device) {
  if (device < 0 || device >= 64) return 0;
  AqlQueue* a;
  {
    std::lock_guard<std::mutex> g(g_queues_mu);
    a = g_queues[device];
  }
  if (!a) return 0;
  std::lock_guard<std::mutex> g(a->mu);
  return a->cp_signalled;
}

uint64_t aql_dispatched(int device, size_t k) {
  if (k >= size_t(kKernels) || device < 0 || device >= 64) return 0;
  AqlQueue* a;
  {
    std::lock_guard<std::mutex> g(g_queues_mu);
    a = g_queues[device];
  }
  if (!a) return 0;
  std::lock_guard<std::mutex> g(a->mu);
  return a->dispatched[k];
}


// How long a region end waits for its stamp reduction (test hook: aql_reduce_timeout), and how
// many abandoned argument slots retire a process's queues.
std::atomic<uint64_t> g_reduce_timeout_ns{uint64_t(5) * 1000000000ull};
constexpr uint32_t kMaxAbandoned = 8;

void aql_reduce_timeout(uint64_t ns) {
  g_reduce_timeout_ns.store(ns ? ns : uint64_t(5) * 1000000000ull);
}

uint32_t aql_abandoned_slots(int device) {
  AqlQueue* a = aql_queue(device);
  if (!a) return 0;
  std::lock_guard<std::mutex> g(a->mu);
  return a->n_abandoned;
}

int aql_stamp_reduce(int device, const uint64_t* base, uint32_t area_words,
                     const uint32_t* areas, uint32_t n, uint64_t* out) {
  AqlQueue* a = aql_queue(device);
  if (!a || !a->hring) return fail(DORA_ERR_UNSUPPORTED, "no AQL queue / host argument ring");
  if (n == 0) return DORA_OK;
  std::lock_guard<std::mutex> g(a->mu);
  if (!a->reduce_sig.handle && hsa_signal_create(1, 0, nullptr, &a->reduce_sig) != HSA_STATUS_SUCCESS) {
    a->reduce_sig.handle = 0;
    return fail(DORA_ERR_HIP, "hsa_signal_create");
  }
  // the host argument slot of the dispatch kRingSlots back must be free (as in dispatch_locked)
  const uint64_t r = take_slot(a);
  Use& u = a->uses[r];
  const auto t0 = std::chrono::steady_clock::now();
  while (u.flag && u.seq >= oldest_outstanding(a) && !fill_reached(u.flag, u.epoch)) {
    if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(5))
      return fail(DORA_ERR_TIMEOUT, "AQL argument slot still in use after 5 s");
    __builtin_ia32_pause();
  }
  uint8_t* slot = a->hring + r * kHostSlotBytes;
  const uint64_t w[3] = {reinterpret_cast<uintptr_t>(base), reinterpret_cast<uintptr_t>(areas),
                         reinterpret_cast<uintptr_t>(out)};
  std::memcpy(slot, w, sizeof(w));
  std::memcpy(slot + 24, &n, 4);
  std::memcpy(slot + 28, &area_words, 4);
  u = Use{nullptr, 0, a->next};
  ++a->next;
  hsa_signal_store_relaxed(a->reduce_sig, 1);
  hsa_queue_t* const q = a->qs[0];
  const uint64_t idx = hsa_queue_load_write_index_relaxed(q);
  while (idx - (a->rd[0] = hsa_queue_load_read_index_scacquire(q)) >= q->size) {
    if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(5))
      return fail(DORA_ERR_TIMEOUT, "AQL queue full for 5 s");
    __builtin_ia32_pause();
  }
  hsa_queue_store_write_index_relaxed(q, idx + 1);
  auto* p = static_cast<hsa_kernel_dispatch_packet_t*>(q->base_address) + (idx & (q->size - 1));
  const int k = kReduceKernel;
  p->workgroup_size_x = 256;
  p->workgroup_size_y = 1;
  p->workgroup_size_z = 1;
  p->reserved0 = 0;
  p->grid_size_x = n * 256u;
  p->grid_size_y = 1;
  p->grid_size_z = 1;
  p->private_segment_size = a->priv[k];
  p->group_segment_size = a->group[k];
  p->kernel_object = a->kobj[k];
  p->kernarg_address = slot;
  p->reserved2 = 0;
  p->completion_signal = a->reduce_sig;
  // barrier: after every packet of the queue; system-scope release: the host reads `out`
  const uint16_t header = (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                          (1 << HSA_PACKET_HEADER_BARRIER) |
                          (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                          (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
  const uint16_t setup = 1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;
  publish_packet(q, p, header | (uint32_t(setup) << 16), idx, a->wc_ring);
  ++a->dispatched[k];
  if (hsa_signal_wait_scacquire(a->reduce_sig, HSA_SIGNAL_CONDITION_LT, 1,
                                g_reduce_timeout_ns.load(std::memory_order_relaxed),
                                HSA_WAIT_STATE_ACTIVE) != 0) {
    // A diagnostic: the data-path queues stay in use.  The packet is still queued and may yet
    // run: its signal is abandoned (a later reduction makes its own), the caller must not free
    // or reuse `areas` / `out` (node.cpp leaks them and reads the areas through the BAR), and
    // its argument slot is never written again — a later pack's arguments there would be the
    // reduction's if it ran after them.  Queues that lose several stop dispatching.
    a->reduce_sig.handle = 0;
    a->abandoned[r] = true;
    if (++a->n_abandoned >= kMaxAbandoned) a->failed.store(true);
    return fail(DORA_ERR_TIMEOUT, "stamp reduction did not complete in time");
  }
  return DORA_OK;
}

uint64_t aql_gpu_tick_to_realtime_ns(int device, uint64_t tick) {
  AqlQueue* a = aql_queue(device);
  if (!a || !a->ts_freq) return 0;
  static std::once_flag once;
  static double off_ns = 0;  // CLOCK_REALTIME - HSA system clock, ns
  const double sys_ns = 1e9 / double(a->ts_freq);
  std::call_once(once, [&] {
    uint64_t best = ~uint64_t(0);
    for (int i = 0; i < 16; ++i) {
      uint64_t sys = 0;
      const uint64_t r0 = now_ns();
      hsa_system_get_info(HSA_SYSTEM_INFO_TIMESTAMP, &sys);
      const uint64_t r1 = now_ns();
      if (r1 - r0 < best) {
        best = r1 - r0;
        off_ns = double(r0 / 2 + r1 / 2) - double(sys) * sys_ns;
      }
    }
  });
  uint64_t sys = 0;
  if (hsa_amd_profiling_convert_tick_to_system_domain(a->gpu, tick, &sys) != HSA_STATUS_SUCCESS)
    return 0;
  return uint64_t(double(sys) * sys_ns + off_ns);
}

int aql_profile_enable(AqlQueue* a, bool on) {
  if (!a) return DORA_OK;
  std::lock_guard<std::mutex> g(a->mu);
  for (int i = 0; i < a->nq; ++i)
    if (hsa_amd_profiling_set_profiler_enabled(a->qs[i], on ? 1 : 0) != HSA_STATUS_SUCCESS)
      return fail(DORA_ERR_HIP, "hsa_amd_profiling_set_profiler_enabled");
  // completion signals are created here, not per dispatch inside a timed region
  while (on && a->free_sigs.size() + a->used_sigs.size() < kProfilePrealloc) {
    hsa_signal_t s;
    if (hsa_signal_create(1, 0, nullptr, &s) != HSA_STATUS_SUCCESS) break;
    a->free_sigs.push_back(s);
  }
  a->profiling = on;
  return DORA_OK;
}

int aql_profile_take(AqlQueue* a, uint64_t* first_start, uint64_t* last_end, uint64_t* count) {
  *first_start = *last_end = *count = 0;
  if (!a) return DORA_OK;
  std::lock_guard<std::mutex> g(a->mu);
  const double to_ns = a->ts_freq ? 1e9 / double(a->ts_freq) : 1.0;
  int rc = DORA_OK;
  for (hsa_signal_t s : a->used_sigs) {
    if (hsa_signal_wait_scacquire(s, HSA_SIGNAL_CONDITION_LT, 1, 10ull * 1000000000ull,
                                  HSA_WAIT_STATE_ACTIVE) != 0) {
      rc = fail(DORA_ERR_TIMEOUT, "profiled AQL pack did not complete");
      continue;
    }
    hsa_amd_profiling_dispatch_time_t t{};
    if (hsa_amd_profiling_get_dispatch_time(a->gpu, s, &t) == HSA_STATUS_SUCCESS) {
      const uint64_t st = uint64_t(double(t.start) * to_ns), en = uint64_t(double(t.end) * to_ns);
      if (*count == 0 || st < *first_start) *first_start = st;
      if (en > *last_end) *last_end = en;
      ++*count;
    }
    a->free_sigs.push_back(s);
  }
  a->used_sigs.clear();
  return rc;
}

}  // namespace dora
