// Node API of the device data plane — the MI355X counterpart of `DoraNode` + `EventStream`
// (apis/rust/node/src/node/mod.rs:42-503, apis/rust/node/src/event_stream/*).
//
// Sender (mod.rs:180-275, 303-371):
//   allocate_data_sample -> a device slot (hipMalloc, exported once with hipIpcGetMemHandle),
//   best-fit from a 20-entry cache of recycled slots exactly like `allocate_shared_memory`;
//   send_output -> plan + HIP pack kernel into the slot on the node's stream; the timestamp is
//   taken after the fill (mod.rs:258); the slot is kept in `sent_out` until its drop token
//   returns (mod.rs:269-272, 348-371).
// Receiver (event_stream/mod.rs:121-198, event.rs:35-126):
//   events are drained from the node's ring into a local queue with the daemon Listener's
//   drop-oldest-per-input policy (node_communication/mod.rs:320-359); a DeviceIpc sample is
//   mapped with hipIpcOpenMemHandle once per slot and cached (never per message); the drop token
//   is reported when the last reference to the input data is released, after the node's stream
//   has drained, so the owner can reuse the slot.
#include <hip/hip_runtime_api.h>
#include <pthread.h>
#include <unistd.h>
#include <x86intrin.h>

#include <algorithm>
#include <chrono>
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <memory_resource>
#include <mutex>
#include <new>
#include <thread>
#include <set>
#include <sstream>
#include <random>
#include <string>
#include <unordered_map>
#include <unordered_set>
#include <vector>

#include "aql.h"
#include "bcast.h"
#include "common.h"
#include "device_array.h"
#include "dora_gpu.h"
#include "plan.h"
#include "shm.h"
#include "stdout_capture.h"
#include "subprof.h"
#include "trace.h"
#include "wire.h"

namespace dora {

// HIP's current device is per thread, and the library acts on the node's GPU from whichever
// thread calls it — an EventStream moved to another thread (the reference's is Send), an async
// pump, the event-stream thread: slots, IPC mappings, events, streams and receive buffers are
// created on the current device.  Every place that creates one (or launches through HIP) makes
// the node's device current for that step and gives the caller's back afterwards.  The steady
// send and receive paths (cached slot, cached mapping, AQL dispatch) create nothing and take no
// scope: hipGetDevice alone costs ~54 ns per call (scripts/get_device_probe.cpp).
struct DeviceScope {
  int prev = -1;
  explicit DeviceScope(int device) {
    int cur = -1;
    if (device >= 0 && hipGetDevice(&cur) == hipSuccess && cur != device &&
        hipSetDevice(device) == hipSuccess)
      prev = cur;
  }
  ~DeviceScope() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
  DeviceScope(const DeviceScope&) = delete;
  DeviceScope& operator=(const DeviceScope&) = delete;
};

// A received slot's identity as a hash key without a heap allocation per lookup: the
// hipIpcMemHandle_t bytes plus the owner's pid and its process-unique slot id.  The handle alone
// is not enough: a freed slot's handle encoding can recur for a new allocation of the same size.
struct IpcKey {
  uint8_t b[64];
  int32_t pid;
  uint64_t slot;
  bool operator==(const IpcKey& o) const {
    return pid == o.pid && slot == o.slot && std::memcmp(b, o.b, 64) == 0;
  }
};
struct IpcKeyHash {
  size_t operator()(const IpcKey& k) const {
    uint64_t h = 0xcbf29ce484222325ull ^ k.slot ^ (uint64_t(uint32_t(k.pid)) << 40);
    for (size_t i = 0; i < 64; i += 8) {
      uint64_t w;
      std::memcpy(&w, k.b + i, 8);
      h = (h ^ w) * 0x100000001b3ull;
    }
    return static_cast<size_t>(h ^ (h >> 29));
  }
};

// One hipIpcOpenMemHandle mapping of a producer's slot.  Shared by the receiver's mapping cache
// and every input that points into it; closed when the last of them lets go, so evicting a
// mapping from the cache never unmaps memory an input still reads.
struct IpcMapping {
  void* base = nullptr;
  uint64_t last_use = 0;
  ~IpcMapping() {
    if (base) (void)hipIpcCloseMemHandle(base);
  }
};

// A host-only producer's shared-memory sample region as mapped here (DataMessage::SharedMemory),
// shared like IpcMapping.  A device receiver registers it with HIP once, so its pull into HBM is a
// DMA from pinned pages rather than a staged copy.
struct ShmMapping {
  void* base = nullptr;
  size_t len = 0;
  bool registered = false, reg_tried = false;  // pinned for DMA on the first pull (ensure_local)
  uint64_t last_use = 0;
  ~ShmMapping() {
    if (registered) (void)hipHostUnregister(base);
    shmem_unmap(base, len);
  }
};

// Mappings a receiver keeps open for reuse (LRU beyond this).  Producers recycle at most
// kMaxCacheSlots slots plus those in flight, so a steady edge stays within it; slots a producer
// has freed (size changes) age out instead of pinning the producer's memory for good.
constexpr size_t kMaxIpcMappings = 128;
// Shared-memory regions a device receiver keeps mapped and pinned while nothing holds them: at
// most this many bytes (the least recently used unheld ones are unpinned and unmapped first), so
// regions a producer has dropped do not stay page-locked in every receiver.
constexpr uint64_t kMaxCachedShmBytes = uint64_t(1) << 30;

namespace {

// A sender's slot cache (mod.rs:365: 20 entries).  Device slots are HBM, and freeing one costs
// the sender 0.5-1 ms of hipFree and the GPU a TLB invalidation while its packs run; a sender
// whose message sizes change (the bench's ladders, variable point clouds) evicted slots at every
// size change.  So the cache keeps the reference's 20 entries and more, up to kMaxCacheSlots, as
// long as they hold at most slot_cache_bytes() (DORA_GPU_SLOT_CACHE_BYTES, default 4 GiB of the
// GPU's 288 GB; 0: the reference's 20 entries); evicted slots are freed off the send path.
constexpr size_t kMaxCacheSize = 20;          // mod.rs:365
constexpr size_t kMaxCacheSlots = 64;
uint64_t slot_cache_bytes() {
  static const uint64_t v = [] {
    const char* e = std::getenv("DORA_GPU_SLOT_CACHE_BYTES");
    return e ? std::strtoull(e, nullptr, 10) : uint64_t(4) << 30;
  }();
  return v;
}
constexpr uint64_t kDropWaitNs = 10000000000;  // 10 s per token on drop (mod.rs:397-426)

struct Slot {
  void* ptr = nullptr;
  // bytes the slot holds (its whole 2 MiB-grain allocation): the cache's best-fit key.  The
  // reference keys on the requested length (Shmem::len); a slot's full capacity lets a 4 MiB
  // sample reuse a slot first made for 4,096,000 B (the ladder's next size created fresh slots,
  // hipMalloc + export + the receiver's mapping, for ~20 of its sends).
  uint64_t cap = 0;
  uint64_t id = 0;
  hipIpcMemHandle_t handle;
  int flag = -1;              // FillFlag index in the node's region entry (async sends)
  uint64_t fill_epoch = 0;    // epoch the last fill into this slot stores into `flag`
  uint64_t region_epoch = 0;  // that fill belongs to a timed region: harvest its stamps
  int region_cp_area = -1;    // ... its stamp area, if the command processor signalled it
  hipEvent_t done = nullptr;  // fallback: interprocess completion event of the last fill
  hipIpcEventHandle_t done_handle;
  // node-stream work on the slot with no fill flag (a broadcast group's pack + broadcast):
  // recorded after it, waited on before the slot is reused or freed
  hipEvent_t use_ev = nullptr;
  bool use_pending = false;
  // host-only node: a POSIX shared-memory region (DataMessage::SharedMemory) instead of HBM
  bool host = false;
  std::string shm_name;
  // a device node's shared-memory slot (host_bound_sample): page-locked and mapped for the GPU,
  // which packs into it
  bool registered = false;
  // device slot mapped for the CPU through the large BAR (host sources written in place,
  // host_bar_fill): tried once per slot
  bool bar = false, bar_tried = false;
};

// The memory of a slot no fill can still write (its events, its HBM or shared-memory region).
void release_slot_memory(Slot* s) {
  if (s->host) {
    if (s->registered) (void)hipHostUnregister(s->ptr);
    shmem_unmap(s->ptr, s->cap);
    shmem_unlink(s->shm_name);
  } else {
    if (s->done) (void)hipEventDestroy(s->done);
    if (s->use_ev) (void)hipEventDestroy(s->use_ev);
    (void)hipFree(s->ptr);
  }
  delete s;
}

// getpid() is a system call on current glibc; the descriptor path asks for it per message.
// Cached per process, refreshed in a forked child.
int self_pid() {
  static std::atomic<int> pid{0};
  static std::once_flag once;
  std::call_once(once, [] { pthread_atfork(nullptr, nullptr, [] { pid.store(0); }); });
  int p = pid.load(std::memory_order_relaxed);
  if (!p) {
    p = static_cast<int>(getpid());
    pid.store(p, std::memory_order_relaxed);
  }
  return p;
}

// Samples a node may have in flight (sent, token not yet back) before an allocation waits.
constexpr uint64_t kSmallInFlightBytes = 8ull << 20;

// Samples a sender may have in flight (sent, token not back) before it waits for a returned
// slot.  Below 8 MiB a message's life is dominated by the dispatch-to-fill-flag latency
// (~5-8 us for a 4 KB-4 MB pack over the AQL queues, scripts/trace_report.py), so the pipeline
// depth sets the rate: 11 there, 8 for larger samples, which are HBM-bound and lose to more
// concurrent packs (C3, 13 MB: -20 % at 12).  11 = the reference's default queue_size (10) + the
// input a receiver is handed: every input queued at a receiver is in flight, and the drop-oldest
// policy runs after next_event has taken its event (dora_node_next_event), so a default receiver
// drops nothing whenever it pauses.  (r03 applied the policy before taking the event: a
// receiver that paused between releasing one input and taking the next then had 11 ready and
// dropped one, 0-5 per bench run in the throughput ladders.  A cap of 10 instead cost 4 MB
// sends ~6 %: 1.56-1.63 vs 1.41-1.50 us, profiles/r04_cap_ab.jsonl.)  DORA_GPU_MAX_IN_FLIGHT=N
// sets both, `S:L` each.
size_t max_in_flight(uint64_t len) {
  static const std::pair<long, long> env = [] {
    const char* e = std::getenv("DORA_GPU_MAX_IN_FLIGHT");
    if (!e) return std::make_pair(0L, 0L);
    char* end = nullptr;
    const long a = std::strtol(e, &end, 10);
    const long b = (end && *end == ':') ? std::atol(end + 1) : a;
    return std::make_pair(a, b);
  }();
  const long v = len < kSmallInFlightBytes ? env.first : env.second;
  if (v > 0) return static_cast<size_t>(v);
  return len < kSmallInFlightBytes ? 11 : 8;
}


// Streams the HIP-launched fills of a node rotate over (host sources, compacting transforms,
// relays; device-source packs go to the AQL queues, aql.h).  Three (r01: HIP-launched device
// packs overlapped their ramps and tails over three hardware queues, 40.96 MB 17.1 -> 13.2 us per
// message, profiles/r01_stream_probe.jsonl) until r06: device packs have left for the AQL
// queues, and every HIP stream costs one of the GPU's 24 compute queues.
constexpr size_t kFillStreams = 1;

// DORA_GPU_PIN=0: leave the node's CPU affinity alone (shm.cpp pin_to_numa)
bool numa_pinning() {
  static const bool v = [] {
    const char* e = std::getenv("DORA_GPU_PIN");
    return !(e && *e == '0');
  }();
  return v;
}

// NUMA node of HIP device `device` (sysfs of its PCI function), -1 when unknown.
int gpu_numa_node(int device) {
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, sizeof(bus), device) != hipSuccess) return -1;
  for (char* p = bus; *p; ++p) *p = char(std::tolower(*p));
  const std::string path = std::string("/sys/bus/pci/devices/") + bus + "/numa_node";
  FILE* f = std::fopen(path.c_str(), "r");
  if (!f) return -1;
  int numa = -1;
  if (std::fscanf(f, "%d", &numa) != 1) numa = -1;
  std::fclose(f);
  return numa;
}

// With profiling on, every n-th pack launch is stamped with timing events (default period;
// dora_node_set_timing_period)
constexpr uint64_t kTimingPeriod = 8;

enum PeerCopyMode { PEER_KERNEL, PEER_SDMA };

// How cross-GPU samples are pulled: the pack kernel on the receiving GPU reading the peer's HBM
// (default) or the copy engines via hipMemcpyPeerAsync (DORA_GPU_PEER_COPY=sdma).
PeerCopyMode peer_copy_mode() {
  static const PeerCopyMode v = [] {
    const char* e = std::getenv("DORA_GPU_PEER_COPY");
    return (e && std::string(e) == "sdma") ? PEER_SDMA : PEER_KERNEL;
  }();
  return v;
}

// DORA_GPU_EDGE_COPY=1 (testing): the cross-GPU receive path on same-GPU edges, the one-GPU
// rehearsal of C4/C5 (tests, bench.py DORA_BENCH_GPUS).
bool edge_copy_forced() {
  static const bool v = [] {
    const char* e = std::getenv("DORA_GPU_EDGE_COPY");
    return e && *e && *e != '0';
  }();
  return v;
}

// DORA_GPU_FANOUT=rccl: this node's outputs with receivers on other GPUs form RCCL broadcast
// groups (bcast.h) instead of letting every receiver pull over its own link.
bool fanout_rccl() {
  static const bool v = [] {
    const char* e = std::getenv("DORA_GPU_FANOUT");
    return e && std::strcmp(e, "rccl") == 0;
  }();
  return v;
}

// How long an allocation waits for a returned token at the in-flight cap before it allocates
// anyway, as the reference would (a receiver may legitimately hold many inputs)
constexpr uint64_t kSlotWaitNs = 5000000;

// Slots of every node in this process by process-wide id: a sample whose owner is this process
// (another node here, or the node itself) is read in place — IPC handles cannot be opened in
// the process that exported them.
struct OwnSlots {
  std::mutex mu;
  std::unordered_map<uint64_t, void*> ptrs;
  std::atomic<uint64_t> next_id{1};
};

OwnSlots& own_slots() {
  static OwnSlots* o = new OwnSlots();  // never destroyed: nodes may outlive static teardown
  return *o;
}

std::vector<std::string> split(const char* s, char sep) {
  std::vector<std::string> out;
  std::string cur;
  for (const char* p = s; *p; ++p) {
    if (*p == sep) {
      if (!cur.empty()) out.push_back(cur);
      cur.clear();
    } else {
      cur += *p;
    }
  }
  if (!cur.empty()) out.push_back(cur);
  return out;
}

}  // namespace

// State shared between the node handle and input data that may outlive events.
struct NodeCore {
  std::unique_ptr<Region> region;
  int idx = -1;
  int device = 0;
  hipStream_t stream = nullptr;
  // Whether anything may be queued on `stream`: the caller once it has it (dora_node_stream), or
  // this library's own asynchronous node-stream work (pulls, forwards).  Until then a send needs
  // no query of the stream (~150 ns of hipStreamQuery per send and per released input).
  std::atomic<bool> stream_used{false};
  bool stream_busy() {
    return stream_used.load(std::memory_order_relaxed) && hipStreamQuery(stream) == hipErrorNotReady;
  }
  // Fill streams (kFillStreams): HIP-launched fills rotate over them.  Work already queued on the
  // node stream is ordered before a fill (node_ev), and fills are ordered before node-stream
  // work queued after dora_node_stream() hands the stream out (fence_fills).
  std::vector<hipStream_t> fill_streams;
  std::vector<hipEvent_t> fill_events;
  std::vector<uint8_t> fill_dirty;
  hipEvent_t node_ev = nullptr;
  hipEvent_t sync_ev = nullptr;  // dora_node_sync's marker
  size_t fill_next = 0;
  bool fill_streams_tried = false;
  // fills dispatched on the AQL queue and not yet seen complete (fence_fills waits for them)
  std::vector<std::pair<const std::atomic<uint64_t>*, uint64_t>> aql_pending;
  // every kernel-signalled fill not yet seen complete (AQL and fill streams): dora_node_sync
  // waits for their flags instead of synchronising streams
  std::vector<std::pair<const std::atomic<uint64_t>*, uint64_t>> flag_pending;
  std::vector<uint8_t> fill_unsignalled;  // per fill stream: work not covered by a fill flag

  // One entry per fill flag with the latest epoch ordered on it (a flag's epochs only grow, so
  // waiting for the latest covers the earlier ones).  Matching by pointer reads no flag: the
  // flags are host lines the GPU writes, and pruning by loading them cost a cache miss each
  // (64 per prune, ~0.4 us per send amortised over the two lists).  The list stays as long as
  // the node has slots with flags; only past 256 entries are completed ones pruned.
  static void note(std::vector<std::pair<const std::atomic<uint64_t>*, uint64_t>>& v,
                   const std::atomic<uint64_t>* f, uint64_t epoch) {
    for (auto& x : v)
      if (x.first == f) {
        x.second = std::max(x.second, epoch);
        return;
      }
    if (v.size() >= 256) {
      size_t k = 0;
      for (auto& x : v)
        if (!fill_reached(x.first, x.second)) v[k++] = x;
      v.resize(k);
    }
    v.push_back({f, epoch});
  }
  RingWriter req;
  RingReader ev;
  RingReader drops;
  std::mutex req_mu;
  std::mutex ipc_mu;
  // (handle, owner pid, slot id) -> open mapping; bounded LRU (kMaxIpcMappings)
  std::unordered_map<IpcKey, std::shared_ptr<IpcMapping>, IpcKeyHash> ipc_cache;
  uint64_t ipc_clock = 0;
  std::atomic<uint64_t> ipc_opens{0}, ipc_closes{0};

  // Drop the least recently used mappings that no input holds until the cache is within bound.
  void trim_ipc_cache() {
    while (ipc_cache.size() > kMaxIpcMappings) {
      auto victim = ipc_cache.end();
      for (auto it = ipc_cache.begin(); it != ipc_cache.end(); ++it)
        if (it->second.use_count() == 1 &&
            (victim == ipc_cache.end() || it->second->last_use < victim->second->last_use))
          victim = it;
      if (victim == ipc_cache.end()) return;  // every mapping is held by an input
      ipc_cache.erase(victim);
      ipc_closes.fetch_add(1, std::memory_order_relaxed);
    }
  }
  // shared-memory region name -> mapping (host-only producers' samples); bounded like ipc_cache
  std::unordered_map<std::string, std::shared_ptr<ShmMapping>> shm_cache;

  std::shared_ptr<ShmMapping> map_shmem(const std::string& name, uint64_t len, std::string* err) {
    std::lock_guard<std::mutex> g(ipc_mu);
    auto it = shm_cache.find(name);
    std::shared_ptr<ShmMapping> m;
    if (it != shm_cache.end()) {
      m = it->second;
    } else {
      m = std::make_shared<ShmMapping>();
      m->base = shmem_open(name, &m->len);
      if (!m->base) {
        *err = "shared-memory sample `" + name + "`: " + std::strerror(errno);
        return nullptr;
      }
      shm_cache.emplace(name, m);
      // bounded by count and by bytes; mappings an input still holds stay
      for (;;) {
        uint64_t bytes = 0;
        for (auto& kv : shm_cache) bytes += kv.second->len;
        if (shm_cache.size() <= kMaxIpcMappings && bytes <= kMaxCachedShmBytes) break;
        auto victim = shm_cache.end();
        for (auto v = shm_cache.begin(); v != shm_cache.end(); ++v)
          if (v->second != m && v->second.use_count() == 1 &&
              (victim == shm_cache.end() || v->second->last_use < victim->second->last_use))
            victim = v;
        if (victim == shm_cache.end()) break;
        shm_cache.erase(victim);
      }
    }
    if (len > m->len) {
      *err = "shared-memory sample `" + name + "` is shorter than its message";
      return nullptr;
    }
    m->last_use = ++ipc_clock;
    return m;
  }
  std::unordered_map<std::string, hipEvent_t> ipc_events;  // event handle bytes -> opened event
  // fill flags: the region is host-registered so the stream can write epochs into it
  uint8_t* region_dev = nullptr;
  uint32_t* fill_done = nullptr;  // device: per fill flag, kMaxSignalWgs workgroup done words
  dora::AqlQueue* aql = nullptr;  // this process's AQL queues of `device` (fill_sample)
  bool aql_tried = false;
  std::vector<uint32_t> free_flags;
  uint64_t epoch = 0;

  // Receive pool for cross-GPU edges: local HBM copies of remote samples, recycled by size.
  std::mutex pool_mu;
  std::multimap<uint64_t, void*> recv_pool;
  static constexpr size_t kMaxPooled = 16;
  std::set<int> peer_enabled;  // peer devices this node's device may access (under ipc_mu)
  std::atomic<uint64_t> peer_copies{0}, peer_bytes{0};  // cross-GPU samples pulled

  // RCCL broadcast groups this node receives on (input id -> communicator); every receive is
  // posted on bcast_stream in the order the daemon routed the samples
  std::map<std::string, BcastComm*> bcast_in;
  hipStream_t bcast_stream = nullptr;
  std::string bcast_error;
  uint64_t bcast_recvs = 0, bcast_bytes = 0;

  void* recv_pool_get(uint64_t len, uint64_t* cap) {
    {
      std::lock_guard<std::mutex> g(pool_mu);
      auto it = recv_pool.lower_bound(len);
      if (it != recv_pool.end() && it->first <= 2 * len + 4096) {
        void* p = it->second;
        *cap = it->first;
        recv_pool.erase(it);
        return p;
      }
    }
    void* p = nullptr;
    const uint64_t c = (len + 4095) / 4096 * 4096;
    DeviceScope ds(device);
    if (hipMalloc(&p, c) != hipSuccess) return nullptr;
    *cap = c;
    return p;
  }

  void recv_pool_put(void* p, uint64_t cap) {
    std::lock_guard<std::mutex> g(pool_mu);
    if (recv_pool.size() >= kMaxPooled) {
      auto it = recv_pool.begin();  // evict the smallest
      (void)hipFree(it->second);
      recv_pool.erase(it);
    }
    recv_pool.emplace(cap, p);
  }

  // Host-only receiver (device < 0): device samples are staged into pinned host memory (one DMA
  // per input, stage_to_host), recycled by size like the receive pool.  Pinned allocations cost
  // milliseconds at the large sizes, so a steady edge reuses its buffers.
  std::multimap<uint64_t, void*> host_pool;
  std::map<int, hipStream_t> stage_streams;  // per producer GPU (under pool_mu)
  std::atomic<uint64_t> host_staged{0}, host_staged_bytes{0};

  void* host_pool_get(uint64_t len, uint64_t* cap) {
    {
      std::lock_guard<std::mutex> g(pool_mu);
      auto it = host_pool.lower_bound(len);
      if (it != host_pool.end() && it->first <= 2 * len + 4096) {
        void* p = it->second;
        *cap = it->first;
        host_pool.erase(it);
        return p;
      }
    }
    void* p = nullptr;
    const uint64_t c = (len + 4095) / 4096 * 4096;
    if (hipHostMalloc(&p, c, hipHostMallocPortable | hipHostMallocMapped) != hipSuccess) {
      (void)hipGetLastError();
      return nullptr;
    }
    *cap = c;
    return p;
  }

  void host_pool_put(void* p, uint64_t cap) {
    std::lock_guard<std::mutex> g(pool_mu);
    if (host_pool.size() >= kMaxPooled) {
      auto it = host_pool.begin();  // evict the smallest
      (void)hipHostFree(it->second);
      host_pool.erase(it);
    }
    host_pool.emplace(cap, p);
  }

  // A private stream of GPU `src_device` for copies waited for alone (a host-only receiver's
  // staging, a device receiver's pulls); the current device must be it
  hipStream_t stage_stream(int src_device) {
    std::lock_guard<std::mutex> g(pool_mu);
    auto it = stage_streams.find(src_device);
    if (it != stage_streams.end()) return it->second;
    hipStream_t s = nullptr;
    if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) {
      (void)hipGetLastError();
      return nullptr;
    }
    stage_streams[src_device] = s;
    return s;
  }

  uint64_t* flag_dev(int idx) const {
    const uint8_t* host = reinterpret_cast<const uint8_t*>(&region->hdr()->nodes[this->idx].fill[idx]);
    return reinterpret_cast<uint64_t*>(region_dev + (host - region->base()));
  }

  // True when the daemon was asleep and had to be woken (the message trace notes it).
  bool ring_doorbell() {
    // the daemon sets `daemon_sleeping` before it reads the doorbell and re-checks the rings;
    // the fence orders the request's head store before our load of the flag (shm.cpp's ring
    // wake-up argument), so the doorbell is only bumped for a sleeping daemon
    RegionHdr* h = region->hdr();
    std::atomic_thread_fence(std::memory_order_seq_cst);
    if (h->daemon_sleeping.load(std::memory_order_relaxed)) {
      h->doorbell.fetch_add(1, std::memory_order_seq_cst);
      futex_wake(&h->doorbell);
      return true;
    }
    return false;
  }
  bool last_rang = false;  // the last request woke the daemon (trace only)

  int request(uint32_t kind, const std::vector<uint8_t>& payload) {
    return request(kind, payload.data(), payload.size());
  }
  int request(uint32_t kind, const uint8_t* payload, size_t len) {
    {
      std::lock_guard<std::mutex> g(req_mu);
      if (!req.fits(len))
        return fail(DORA_ERR_INVALID, "message of %zu bytes exceeds the control ring", len);
      if (!req.push(kind, payload, len, 30000000))
        return fail(DORA_ERR_TIMEOUT, "daemon did not drain the request ring for 30 s");
    }
    last_rang = ring_doorbell();
    return DORA_OK;
  }

  void report_drop_token(const DropToken& t) {
    // count (u32) + token, encoded on the stack: released inputs allocate nothing
    uint8_t b[4 + sizeof(DropToken)];
    const uint32_t one = 1;
    std::memcpy(b, &one, 4);
    std::memcpy(b + 4, &t, sizeof(DropToken));
    (void)request(REQ_REPORT_DROP_TOKENS, b, sizeof(b));
  }

  // The stream the next fill runs on (round robin), ordered after the node stream's queued work.
  void ensure_fill_streams() {
    if (!fill_streams.empty() || fill_streams_tried) return;
    fill_streams_tried = true;
    DeviceScope ds(device);
    if (hipEventCreateWithFlags(&node_ev, hipEventDisableTiming) == hipSuccess) {
      for (size_t i = 0; i < kFillStreams; ++i) {
        hipStream_t s = nullptr;
        hipEvent_t e = nullptr;
        if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) break;
        if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) {
          (void)hipStreamDestroy(s);
          break;
        }
        fill_streams.push_back(s);
        fill_events.push_back(e);
      }
      fill_dirty.assign(fill_streams.size(), 0);
      fill_unsignalled.assign(fill_streams.size(), 0);
    }
    (void)hipGetLastError();
  }

  // Order stream `s` after the work queued on the node stream so far (producer kernels of a source).
  void order_after_node_stream(hipStream_t s) {
    if (stream_busy()) {
      if (!node_ev) {
        DeviceScope ds(device);
        (void)hipEventCreateWithFlags(&node_ev, hipEventDisableTiming);
      }
      if (node_ev && hipEventRecord(node_ev, stream) == hipSuccess) (void)hipStreamWaitEvent(s, node_ev, 0);
    }
    (void)hipGetLastError();
  }

  hipStream_t next_fill_stream() {
    ensure_fill_streams();
    if (fill_streams.empty()) {
      stream_used.store(true, std::memory_order_relaxed);  // fills on the node stream itself
      return stream;
    }
    const size_t i = fill_next++ % fill_streams.size();
    hipStream_t s = fill_streams[i];
    if (stream_busy()) {
      // producer kernels of the source may still run on the node stream
      if (hipEventRecord(node_ev, stream) == hipSuccess) (void)hipStreamWaitEvent(s, node_ev, 0);
    }
    (void)hipGetLastError();
    fill_dirty[i] = 1;
    return s;
  }

  const std::atomic<uint64_t>* flag_host(int i) const {
    return &region->hdr()->nodes[idx].fill[i].epoch;
  }

  void note_aql_fill(const std::atomic<uint64_t>* f, uint64_t epoch) {
    note(aql_pending, f, epoch);
    note(flag_pending, f, epoch);
  }

  // Order every fill launched so far before work queued on the node stream from now on.
  void fence_fills() {
    // AQL fills are on no HIP stream: wait for their flags on the host
    const uint64_t t0 = mono_ns();
    for (auto& x : aql_pending)
      while (!fill_reached(x.first, x.second) && mono_ns() - t0 < 10000000000ull)
        __builtin_ia32_pause();
    aql_pending.clear();
    for (size_t i = 0; i < fill_streams.size(); ++i) {
      if (!fill_dirty[i]) continue;
      fill_dirty[i] = 0;
      if (hipStreamQuery(fill_streams[i]) == hipSuccess) continue;  // already drained
      if (hipEventRecord(fill_events[i], fill_streams[i]) == hipSuccess)
        (void)hipStreamWaitEvent(stream, fill_events[i], 0);
    }
    (void)hipGetLastError();
  }

  ~NodeCore() {
    for (auto& kv : bcast_in) bcast_close(kv.second, bcast_stream, 10000);
    if (bcast_stream) (void)hipStreamDestroy(bcast_stream);
    // AQL argument slots must not keep pointing at this region's fill flags once it is unmapped
    if (device >= 0 && region) aql_forget_flags(device, region->base(), region->size());
    for (auto& kv : ipc_events) (void)hipEventDestroy(kv.second);
    ipc_cache.clear();
    for (hipStream_t s : fill_streams) {
      (void)hipStreamSynchronize(s);
      (void)hipStreamDestroy(s);
    }
    for (hipEvent_t e : fill_events) (void)hipEventDestroy(e);
    if (node_ev) (void)hipEventDestroy(node_ev);
    if (sync_ev) (void)hipEventDestroy(sync_ev);
    if (stream) (void)hipStreamSynchronize(stream);
    for (auto& kv : recv_pool) (void)hipFree(kv.second);
    for (auto& kv : stage_streams) {
      (void)hipStreamSynchronize(kv.second);
      (void)hipStreamDestroy(kv.second);
    }
    for (auto& kv : host_pool) (void)hipHostFree(kv.second);
    if (fill_done) (void)hipFree(fill_done);
    if (region_dev) (void)hipHostUnregister(region->base());
    if (stream) (void)hipStreamDestroy(stream);
  }
};

// The received sample of one input; reports the drop token when the last owner releases it.
struct InputData {
  std::shared_ptr<NodeCore> core;
  const void* ptr = nullptr;
  uint64_t len = 0;
  uint64_t ext_len = 0;       // bytes of the sample incl. its validity tail (>= len)
  bool has_token = false;
  DropToken token{};
  std::vector<uint8_t> vec;   // inline (Vec) samples stay on the host
  std::shared_ptr<IpcMapping> mapping;  // the producer's slot as mapped here (IPC edges)
  void* local = nullptr;      // cross-GPU edge: local copy in this node's receive pool
  uint64_t local_cap = 0;
  int remote_device = -1;     // >= 0: `ptr` is a peer GPU's slot not yet pulled (ensure_local)
  hipEvent_t bcast_ev = nullptr;  // broadcast group input: completion of its receive into `local`
  std::shared_ptr<ShmMapping> shm;  // a host-only producer's shared-memory sample, mapped here
  bool host_mem = false;   // host receiver: `ptr` is host memory (shared memory read in place,
                           // or a device sample staged into `host_local`)
  bool host_pull = false;  // device receiver: `ptr` is shared memory not yet pulled into HBM
  void* host_local = nullptr;  // host-only receiver: pinned copy of a device sample (stage_to_host)
  uint64_t host_local_cap = 0;
  ~InputData() {
    if (!core) return;
    if (bcast_ev) {
      (void)hipEventSynchronize(bcast_ev);
      (void)hipEventDestroy(bcast_ev);
    }
    if (has_token || local) {
      // consumer reads on the node stream must be complete before the memory is reused
      SubSpan sq(SP_STREAM_QUERY);
      if (core->stream && core->stream_used.load(std::memory_order_relaxed) &&
          hipStreamQuery(core->stream) != hipSuccess)
        (void)hipStreamSynchronize(core->stream);
    }
    if (has_token) {
      SubSpan sp(SP_RECV_RELEASE);
      core->report_drop_token(token);
      trace(TP_RELEASED, token);
    }
    if (local) core->recv_pool_put(local, local_cap);
    if (host_local) core->host_pool_put(host_local, host_local_cap);
  }
};

}  // namespace dora

struct dora_sample {
  dora::Slot* slot = nullptr;
  std::vector<uint8_t> vec;  // zero-length samples (Vec path)
  uint64_t len = 0;
  uint64_t ext_len = 0;      // slot bytes filled: len + the validity tail (0: len)
  uint8_t fill = dora::FILL_DONE;  // how the receiver learns the fill completed
  uint64_t epoch = 0;
  bool stamped = false;  // the pack kernel stamps its start / signal time into the flag line
  bool read_signalled = false;  // its pack raises the flag line's read word (aql.h aql_pack)
};

namespace dora {
// Kernel-duration stamps of async packs (hipExtLaunchKernel start/stop), harvested lazily.
struct TimingPair {
  hipEvent_t start = nullptr, stop = nullptr;
  uint64_t bytes = 0;
  bool pending = false;
};
}  // namespace dora

struct dora_event {
  int type = 0;
  std::string id;
  dora::Metadata meta;
  std::shared_ptr<dora::InputData> data;
  std::string error;
  bool pending = false;  // device input not yet completed (fill wait / cross-GPU pull)
  uint64_t arrived_ns = 0;  // mono_ns when the descriptor was drained (transit age bound)
  dora::DeviceIpc ipc{};
  // dora_event_type_info's reference (inline-validity) form, built on first request when the
  // type info points into the sample's validity tail
  mutable bool ti_checked = false;
  mutable std::vector<uint8_t> ti_inline;
};

struct dora_node {
  std::shared_ptr<dora::NodeCore> core;
  std::string id;
  std::set<std::string> outputs;
  std::map<std::string, uint32_t> queue_size;
  size_t min_queue_size = 0;  // smallest value of queue_size
  std::deque<dora::Slot*> cache;
  // samples sent, by drop token (map nodes from a pool: no malloc per send)
  std::pmr::unsynchronized_pool_resource sent_pool;
  std::pmr::unordered_map<dora::DropToken, dora::Slot*, dora::DropTokenHash> sent_out{&sent_pool};
  dora::WBuf send_buf;                 // request encoding scratch of send_sample, reused
  std::vector<uint8_t> ti_buf;         // type-info scratch of pack_and_send, reused
  dora_plan bytes_plan;                // send_output_bytes: the one-buffer plan, re-pointed
  std::vector<uint8_t> bytes_ti;       // ... and its type info for a sample of bytes_ti_len
  uint64_t bytes_ti_len = 0;
  std::deque<std::unique_ptr<dora_event>> queue;
  bool ended = false;
  // samples dora_node_allocate_data_sample handed out and not yet sent or discarded
  std::unordered_set<dora_sample*> samples_live;
  // Event-stream thread (dora_node_set_event_thread; started by every node that joins an RCCL
  // broadcast group as a receiver): the reference's event_stream_loop (event_stream/thread.rs:
  // 81-188) — it drains the daemon's ring into `queue` continuously and applies the drop-oldest
  // policy there (node_communication/mod.rs:320-359), so inputs keep arriving, their broadcast
  // receives are posted and the tokens of dropped inputs go back while the user thread is busy
  // elsewhere.  `qmu` guards `queue` and `ended` while it runs.
  std::thread pump;
  std::mutex qmu;
  std::condition_variable qcv;
  std::atomic<bool> pump_on{false}, pump_stop{false};
  bool want_pump = false;  // a broadcast group was joined: start the thread at the next chance
  bool pin_pending = false;  // host-only node not yet in the dataflow's L3 domain (pin_host_node)
  // profiling of the pack kernel on the node stream
  bool profile = false;
  std::vector<dora::TimingPair> timing;  // ring of kTimingPairs
  size_t timing_next = 0;
  uint64_t timing_seq = 0;
  uint64_t timing_period = 0;            // stamp every n-th pack (0: kTimingPeriod)
  hipEvent_t timing_ref = nullptr;       // recorded when profiling is (re)enabled
  std::vector<double> intervals;         // (start, stop) ms after timing_ref per stamped pack
  // Timed region (dora_node_region_begin/end): the first pack after begin stamps its start;
  // end records a stop event on every fill stream once the packs queued there have finished.
  bool region_armed = false, region_started = false, region_marked = false;
  uint64_t region_aql = 0;  // packs of the region dispatched on the AQL queue
  // kernel stamps (s_memrealtime ticks) of the region's packs, harvested from their flag lines
  uint64_t region_stamped = 0, region_unstamped = 0, region_tmin = 0, region_tmax = 0;
  std::vector<uint64_t> region_ticks;  // (start, end) stamps of the region's packs
  // stamp areas of a region's CP-signalled packs (aql.h aql_pack `cp_stamps`): device memory the
  // host reads through the BAR (stamps written to host memory held every pack's end for their
  // PCIe writes: C3 0.44-0.52 of HBM), made and zeroed at the node's first send (ensure_cp_stamps).
  // No HIP work around a
  // region: a memset or copy on a HIP stream right before a region made its first send take
  // 25-45 us instead of 4 (profiles/r03_cp_signal_ab.jsonl, first_send_ab).  Areas are never
  // re-zeroed: an area's stale words are an earlier pack's, older than the current pack's own.
  uint64_t* region_cp_stamps = nullptr;  // coarse-grained device memory, host-mapped (aql.h bar_alloc)
  // region end: the used areas' indices and their (start, end) pairs, pinned host memory the
  // stamp reduction (aql_stamp_reduce) reads and writes
  uint32_t* region_reduce_idx = nullptr;
  uint64_t* region_reduce_out = nullptr;
  uint32_t region_cp_next = 0;
  std::vector<uint32_t> region_cp_used;
  uint64_t aql_packs = 0, hip_packs = 0;  // fills by dispatch path
  uint64_t bar_fills = 0;  // host sources written into their slot by the CPU (host_bar_fill)
  // outputs whose every receiver has no GPU (the daemon's AllNodesReady): device sources up to
  // kHostPackMax are packed straight into shared memory for them (host_bound_sample)
  std::set<std::string, std::less<>> host_bound;
  // samples put straight into shared memory for such outputs: device arrays packed there by the
  // GPU (host_bound_sample), host sources copied there by the CPU
  uint64_t host_packs = 0, host_copies = 0;
  bool aql_ready = false;  // the process's AQL queues were set up (first non-empty sample)
  hipEvent_t region_start = nullptr;
  std::vector<hipEvent_t> region_stop;
  uint64_t region_packs = 0, region_bytes = 0;
  uint64_t pack_count = 0, pack_bytes = 0;
  double pack_ms = 0;
  uint64_t slots_created = 0, cache_hits = 0, dropped_inputs = 0;
  // host time per send phase: allocate (incl. backpressure), launch, fill sync/record, send
  std::vector<uint8_t> drop_buf;  // payload buffer of handle_finished_drop_tokens
  std::vector<uint8_t> ev_buf;    // payload buffer of drain_events
  uint64_t phase_ns[4] = {0, 0, 0, 0};
  uint64_t phase_count = 0;
  bool compact = false;                     // send_output uses compacting plans
  // DORA_SEND_ASYNC for every send (DORA_GPU_SEND_ASYNC=1): device-source sends return before
  // their pack has read the source
  bool async_default = false;
  // Plans of recent device-array sends by plan_key (a sender re-sending the same buffers, e.g. a
  // ring of preallocated frames, plans each once): the plan and its serialized type info
  struct CachedPlan {
    std::vector<uint64_t> key;
    dora_plan* plan = nullptr;
    std::vector<uint8_t> ti;
    uint64_t last_use = 0;
  };
  std::vector<CachedPlan> plan_cache;
  std::unordered_map<uint64_t, size_t> plan_index;  // hash of a key -> its plan_cache entry
  std::vector<uint64_t> plan_key_buf;
  uint64_t plan_clock = 0, plan_hits = 0;
  // RCCL broadcast groups of this node's fan-out outputs (rank 0 of each), DORA_GPU_FANOUT=rccl.
  // Each output packs and broadcasts on a stream of its own: a rank that stalls the collective
  // holds up that output only (its slots, then its in-flight cap), not the node stream nor the
  // node's other outputs.
  struct BcastOut {
    dora::BcastComm* comm = nullptr;
    hipStream_t stream = nullptr;
  };
  std::map<std::string, BcastOut> bcast_out;
  uint64_t bcast_seq = 0;
  dora::StdoutCapture* stdout_capture = nullptr;  // send_stdout_as (DORA_GPU_SEND_STDOUT_AS)
  // zero-copy forwards: the input re-sent in place, kept (and its producer's token held) until
  // the forward's own token returns
  std::unordered_map<dora::DropToken, std::shared_ptr<dora::InputData>, dora::DropTokenHash>
      forwarded;
  uint64_t zero_copy_forwards = 0;
};

namespace dora {
namespace {

// The stamps of a timed region's pack, read from its flag line before the slot's next fill
// overwrites them (the flag must already show the pack's epoch).
void harvest_region_stamp(dora_node* n, Slot* s) {
  if (!s->region_epoch || s->flag < 0) return;
  const FillFlag& ff = n->core->region->hdr()->nodes[n->core->idx].fill[s->flag];
  if (s->region_cp_area >= 0 && ff.epoch.load(std::memory_order_acquire) != s->region_epoch &&
      ff.cp_epoch.load(std::memory_order_acquire) == s->region_epoch) {
    n->region_cp_used.push_back(uint32_t(s->region_cp_area));  // resolved at region_end
  } else if (ff.epoch.load(std::memory_order_acquire) == s->region_epoch) {
    // an in-kernel-signalled fill (its workgroup 0 stamps the line)
    const uint64_t a = ff.t_start, b = ff.t_end;
    if (b >= a && a) {
      if (!n->region_stamped || a < n->region_tmin) n->region_tmin = a;
      if (!n->region_stamped || b > n->region_tmax) n->region_tmax = b;
      ++n->region_stamped;
      if (n->region_ticks.size() < 2 * (1u << 16)) {
        n->region_ticks.push_back(a);
        n->region_ticks.push_back(b);
      }
    }
  }
  s->region_epoch = 0;
  s->region_cp_area = -1;
}

// A returned drop token does not prove that the slot's last fill has completed: the daemon
// returns the token at once for an output without receivers, a receiver's drop-oldest queue
// releases inputs it never waited on, and a finished receiver's tokens are released for it.
// Before a slot is refilled or freed, wait for its last fill (normally long complete: one load).
// False when the fill did not complete within `timeout_ns` — the slot must then be neither
// reused nor freed (a kernel may still write it).
bool wait_slot_idle(dora_node* n, Slot* s, uint64_t timeout_ns = 10000000000ull) {
  const uint64_t t0 = mono_ns();
  if (s->flag >= 0 && s->fill_epoch) {
    const std::atomic<uint64_t>* f = n->core->flag_host(s->flag);
    while (!fill_reached(f, s->fill_epoch)) {
      if (mono_ns() - t0 > timeout_ns) return false;
      __builtin_ia32_pause();
    }
    harvest_region_stamp(n, s);
  }
  if (s->done && hipEventQuery(s->done) == hipErrorNotReady &&
      hipEventSynchronize(s->done) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  if (s->use_pending) {
    if (hipEventSynchronize(s->use_ev) != hipSuccess) {
      (void)hipGetLastError();
      return false;
    }
    s->use_pending = false;
  }
  return true;
}

void free_slot(dora_node* n, Slot* s) {
  if (!s) return;
  {
    std::lock_guard<std::mutex> g(own_slots().mu);
    own_slots().ptrs.erase(s->id);
  }
  if (!wait_slot_idle(n, s)) {
    // a fill that never completed may still write the slot (and its flag's done words): leak
    // both rather than hand them to another allocation
    std::fprintf(stderr, "dora-gpu: slot %llu: last fill did not complete; not freed\n",
                 (unsigned long long)s->id);
    return;
  }
  if (s->flag >= 0) n->core->free_flags.push_back(static_cast<uint32_t>(s->flag));
  release_slot_memory(s);
}

// Slots evicted from a sender's cache are freed by a process-wide thread, not on the send path:
// hipFree of a 40.96 MB slot took 0.5-1 ms inside the first send after a size change (the
// eviction happens when returned tokens are handled in alloc_sample), which made one message in
// two hundred cost a millisecond — the slow mode of bench.py's 40.96 MB ladder step
// (first_send 0.5-1.0 ms, alloc_us, in profiles/r04_py40_first_send.jsonl).  Freed off the send
// path, the packs running meanwhile still slowed by ~0.3 us each (the unmapping), hence the
// larger cache above.  The sender still
// waits for the slot's last fill and takes back its fill flag; the thread only destroys the
// slot's events and frees its memory.  dora_node_free and exit drain it.
struct SlotReaper {
  std::mutex mu;
  std::condition_variable cv, idle;
  std::deque<std::pair<int, Slot*>> q;
  size_t busy = 0;
  bool started = false;

  void push(int device, Slot* s) {
    std::unique_lock<std::mutex> g(mu);
    if (!started) {
      started = true;
      std::thread([this] { run(); }).detach();
      std::atexit([] { reaper().drain(); });  // before HIP's own teardown (registered earlier)
      // a forked child has no reaper thread: it starts its own, and forgets the parent's queue
      pthread_atfork(nullptr, nullptr, [] {
        SlotReaper& r = reaper();
        new (&r.mu) std::mutex();
        new (&r.cv) std::condition_variable();
        new (&r.idle) std::condition_variable();
        r.q.clear();
        r.busy = 0;
        r.started = false;
      });
    }
    q.emplace_back(device, s);
    cv.notify_one();
  }
  void run() {
    std::unique_lock<std::mutex> g(mu);
    for (;;) {
      cv.wait(g, [this] { return !q.empty(); });
      auto [dev, s] = q.front();
      q.pop_front();
      ++busy;
      g.unlock();
      int prev = -1;
      (void)hipGetDevice(&prev);
      if (dev >= 0 && prev != dev) (void)hipSetDevice(dev);
      release_slot_memory(s);
      (void)hipGetLastError();
      g.lock();
      --busy;
      if (q.empty() && !busy) idle.notify_all();
    }
  }
  void drain() {
    std::unique_lock<std::mutex> g(mu);
    idle.wait(g, [this] { return q.empty() && !busy; });
  }
  static SlotReaper& reaper() {
    static SlotReaper* r = new SlotReaper();  // never destroyed: its thread is detached
    return *r;
  }
};

void free_slot_deferred(dora_node* n, Slot* s) {
  if (!s) return;
  {
    std::lock_guard<std::mutex> g(own_slots().mu);
    own_slots().ptrs.erase(s->id);
  }
  if (!wait_slot_idle(n, s)) {  // as free_slot: a fill that never completed keeps its slot
    std::fprintf(stderr, "dora-gpu: slot %llu: last fill did not complete; not freed\n",
                 (unsigned long long)s->id);
    return;
  }
  if (s->flag >= 0) n->core->free_flags.push_back(static_cast<uint32_t>(s->flag));
  s->flag = -1;
  SlotReaper::reaper().push(n->core->device, s);
}

void add_to_cache(dora_node* n, Slot* s) {  // mod.rs:364-371
  n->cache.push_back(s);
  auto over = [n] {
    if (n->cache.size() <= kMaxCacheSize) return false;
    if (n->cache.size() > kMaxCacheSlots) return true;
    uint64_t bytes = 0;
    for (const Slot* c : n->cache) bytes += c->cap;
    return bytes > slot_cache_bytes();
  };
  while (over()) {
    Slot* old = n->cache.front();
    n->cache.pop_front();
    free_slot_deferred(n, old);
  }
}

void on_token(dora_node* n, const DropToken& t) {
  trace(TP_TOKEN_BACK, t);
  auto f = n->forwarded.find(t);
  if (f != n->forwarded.end()) {  // a zero-copy forward: release the input it re-sent
    n->forwarded.erase(f);
    return;
  }
  auto it = n->sent_out.find(t);
  if (it == n->sent_out.end()) return;  // "received unknown finished drop token"
  Slot* s = it->second;
  n->sent_out.erase(it);
  // the slot's fill flag line was last written by the GPU: start pulling it in now, so the
  // last-fill check of its reuse (allocate_slot, oldest first) finds it in cache
  if (s->flag >= 0) _mm_prefetch(reinterpret_cast<const char*>(n->core->flag_host(s->flag)), _MM_HINT_T0);
  add_to_cache(n, s);
}

int handle_finished_drop_tokens(dora_node* n) {  // mod.rs:348-362
  uint32_t kind;
  std::vector<uint8_t>& p = n->drop_buf;  // reused: popping a token allocates nothing
  while (n->core->drops.try_pop(&kind, &p)) {
    if (kind != DROP_OUTPUT_DROPPED) continue;
    RBuf r(p);
    on_token(n, r.token());
  }
  return DORA_OK;
}

// Slots are whole 2 MiB allocations: HIP sub-allocates smaller hipMallocs from shared blocks,
// and an IPC import of such a slot failed ("invalid device pointer") when the exporting process
// freed other memory of the block meanwhile (two nodes in one process, r01).
uint64_t slot_bytes(uint64_t len) {
  constexpr uint64_t kSlotGrain = 2ull << 20;
  return (std::max<uint64_t>(len, 1) + kSlotGrain - 1) / kSlotGrain * kSlotGrain;
}

// Best fit among cached slots (mod.rs:321-346 `.rev()...min_by_key`); among slots of equal
// capacity the oldest returned one, whose last fill has had the longest to complete and whose
// flag line on_token has prefetched (the reference takes the newest; any fit is equivalent).
// `need`: the smallest capacity a new slot of `len` would have (an exact fit ends the search).
// `host`: a shared-memory slot is wanted (a device node caches both kinds).
int best_fit(dora_node* n, uint64_t len, uint64_t need, bool host) {
  int best = -1;
  for (int i = 0; i < static_cast<int>(n->cache.size()); ++i) {
    Slot* s = n->cache[static_cast<size_t>(i)];
    if (s->host != host) continue;
    if (s->cap >= len && (best < 0 || s->cap < n->cache[static_cast<size_t>(best)]->cap)) {
      best = i;
      if (s->cap == need) break;  // an exact fit: no later slot fits better
    }
  }
  return best;
}

int allocate_slot(dora_node* n, uint64_t len, Slot** out) {  // mod.rs:321-346
  const int best = best_fit(n, len, slot_bytes(len), false);
  if (best >= 0) {
    Slot* s = n->cache[static_cast<size_t>(best)];
    n->cache.erase(n->cache.begin() + best);
    SubSpan sp_flag(SP_SLOT_FLAG);
    const bool idle = wait_slot_idle(n, s);
    sp_flag.stop();
    if (idle) {
      *out = s;
      ++n->cache_hits;
      return DORA_OK;
    }
    // its last fill never completed: leak the slot (a kernel may still write it), take a new one
    std::fprintf(stderr, "dora-gpu: slot %llu: last fill did not complete; not reused\n",
                 (unsigned long long)s->id);
    std::lock_guard<std::mutex> g(own_slots().mu);
    own_slots().ptrs.erase(s->id);
  }
  auto* s = new Slot();
  s->cap = slot_bytes(len);
  s->id = own_slots().next_id.fetch_add(1);
  DeviceScope ds(n->core->device);
  hipError_t e = hipMalloc(&s->ptr, slot_bytes(len));
  if (e == hipSuccess) e = hipIpcGetMemHandle(&s->handle, s->ptr);
  if (e == hipSuccess) {
    if (n->core->region_dev && !n->core->free_flags.empty()) {
      s->flag = static_cast<int>(n->core->free_flags.back());
      n->core->free_flags.pop_back();
    } else {
      e = hipEventCreateWithFlags(&s->done, hipEventInterprocess | hipEventDisableTiming);
      if (e == hipSuccess) e = hipIpcGetEventHandle(&s->done_handle, s->done);
    }
  }
  if (e != hipSuccess) {
    if (s->flag >= 0) n->core->free_flags.push_back(static_cast<uint32_t>(s->flag));
    if (s->done) (void)hipEventDestroy(s->done);
    if (s->ptr) (void)hipFree(s->ptr);
    delete s;
    return fail(DORA_ERR_HIP, "device slot of %llu bytes: %s", (unsigned long long)len,
                hipGetErrorString(e));
  }
  {
    std::lock_guard<std::mutex> g(own_slots().mu);
    own_slots().ptrs[s->id] = s->ptr;
  }
  ++n->slots_created;
  n->core->region->hdr()->nodes[n->core->idx].slots_created.fetch_add(1, std::memory_order_relaxed);
  *out = s;
  return DORA_OK;
}

// A host-only node's sample >= 4096 B (mod.rs:321-346): best fit from the slot cache, else a
// new POSIX shared-memory region of whole pages.  The node writes it with the CPU (as the
// reference's copy_array_into_sample); device receivers pull it into HBM by DMA.
int allocate_host_slot(dora_node* n, uint64_t len, Slot** out) {
  constexpr uint64_t kPage = 4096;
  const uint64_t need = (std::max<uint64_t>(len, 1) + kPage - 1) / kPage * kPage;
  const int best = best_fit(n, len, need, true);
  if (best >= 0) {
    *out = n->cache[static_cast<size_t>(best)];
    n->cache.erase(n->cache.begin() + best);
    ++n->cache_hits;
    return DORA_OK;
  }
  auto* s = new Slot();
  s->host = true;
  s->cap = need;
  s->id = own_slots().next_id.fetch_add(1);
  // pid + a per-process nonce + slot id: a receiver's cached mapping of a region is keyed by its
  // name, so a later process that got the same pid must not produce the same names
  static const uint32_t nonce = [] {
    std::random_device rd;
    return static_cast<uint32_t>(rd());
  }();
  char nbuf[16];
  std::snprintf(nbuf, sizeof(nbuf), "%08x", nonce);
  s->shm_name = "/dora-gpu-s-" + std::to_string(self_pid()) + "-" + nbuf + "-" + std::to_string(s->id);
  s->ptr = shmem_create(s->shm_name, s->cap);
  if (!s->ptr) {
    const int err = errno;
    delete s;
    return fail(DORA_ERR_INVALID, "shared-memory sample of %llu bytes: %s",
                (unsigned long long)len, std::strerror(err));
  }
  ++n->slots_created;
  n->core->region->hdr()->nodes[n->core->idx].slots_created.fetch_add(1, std::memory_order_relaxed);
  *out = s;
  return DORA_OK;
}

// EV_BCAST_JOIN: become rank `rank` of the producer's broadcast group for input `input`.
void join_bcast_group(dora_node* n, const std::string& input, const uint8_t* uid, uint32_t nranks,
                      uint32_t rank) {
  NodeCore* c = n->core.get();
  if (c->device < 0) {
    c->bcast_error = "host-only node cannot join a broadcast group";
    return;
  }
  DeviceScope ds(c->device);
  if (!c->bcast_stream && hipStreamCreateWithFlags(&c->bcast_stream, hipStreamNonBlocking) != hipSuccess) {
    (void)hipGetLastError();
    c->bcast_stream = nullptr;
    c->bcast_error = "broadcast receive stream";
    return;
  }
  BcastComm* comm = nullptr;
  if (bcast_join(uid, static_cast<int>(nranks), static_cast<int>(rank), 30000, &comm) != DORA_OK) {
    c->bcast_error = dora_gpu_last_error();
    return;
  }
  auto it = c->bcast_in.find(input);
  if (it != c->bcast_in.end()) bcast_close(it->second, c->bcast_stream, 10000);
  c->bcast_in[input] = comm;
  // a rank that stops polling must not stall the collective for the others: post receives
  // from the event-stream thread (started by the user thread when it next returns from the
  // event loop, dora_node_next_event / init)
  n->want_pump = true;
}

// A FILL_BCAST sample: post this rank's receive of the producer's broadcast into the receive
// pool right away (at drain time, so every rank issues the group's broadcasts in routing order,
// whether or not the input is later dropped); the input is complete when `bcast_ev` fires.
int post_bcast_receive(NodeCore* c, InputData* in, const std::string& input) {
  auto it = c->bcast_in.find(input);
  if (it == c->bcast_in.end())
    return fail(DORA_ERR_INVALID, "input `%s`: broadcast sample but no group joined (%s)",
                input.c_str(), c->bcast_error.c_str());
  DeviceScope ds(c->device);
  uint64_t cap = 0;
  void* local = c->recv_pool_get(in->ext_len, &cap);
  if (!local)
    return fail(DORA_ERR_HIP, "receive slot of %llu bytes", (unsigned long long)in->ext_len);
  int rc = bcast_enqueue(it->second, local, in->ext_len, c->bcast_stream);
  hipEvent_t e = nullptr;
  if (rc == DORA_OK) {
    hipError_t he = hipEventCreateWithFlags(&e, hipEventDisableTiming);
    if (he == hipSuccess) he = hipEventRecord(e, c->bcast_stream);
    if (he != hipSuccess) {
      // the receive is queued: wait for it here rather than lose track of it
      (void)hipStreamSynchronize(c->bcast_stream);
      if (e) (void)hipEventDestroy(e);
      e = nullptr;
    }
  }
  if (rc != DORA_OK) {
    c->recv_pool_put(local, cap);
    return rc;
  }
  in->local = local;
  in->local_cap = cap;
  in->ptr = local;
  in->bcast_ev = e;
  ++c->bcast_recvs;
  c->bcast_bytes += in->ext_len;
  return DORA_OK;
}

void encode_event(dora_node* n, uint32_t kind, const std::vector<uint8_t>& p) {
  SubSpan sp(SP_RECV_ENCODE);
  auto ev = std::make_unique<dora_event>();
  RBuf r(p);
  switch (kind) {
    case EV_INPUT: {
      ev->type = DORA_EVENT_INPUT;
      ev->arrived_ns = mono_ns();
      ev->id = r.str();
      const uint64_t meta_len = r.u64();
      r.need(meta_len);
      RBuf mr(r.ptr(), meta_len);  // parsed in place: no copy of the metadata bytes
      ev->meta = mr.metadata();
      r.skip(meta_len);
      DataMsg d = r.data();
      auto in = std::make_shared<InputData>();
      in->core = n->core;
      const bool woke = ring_take_woke();
      if (d.kind != DATA_DEVICE_IPC && trace_enabled())
        trace(woke ? TP_POPPED_WOKE : TP_POPPED, ts_key(ev->meta.timestamp_ns));
      if (d.kind == DATA_VEC) {
        in->vec = std::move(d.vec);
        in->ptr = in->vec.data();
        in->len = in->vec.size();
        in->ext_len = in->len;
      } else if (d.kind == DATA_SHMEM) {
        // a host-only node's sample: read in place by a host receiver, pulled into HBM by DMA
        // on first access by a device receiver (ensure_local)
        in->has_token = true;
        in->token = d.shm.token;
        in->len = in->ext_len = d.shm.len;
        std::string err;
        in->shm = n->core->map_shmem(d.shm.name, d.shm.len, &err);
        if (!in->shm) {
          ev->type = DORA_EVENT_ERROR;
          ev->error = err;
        } else {
          in->ptr = in->shm->base;
          (n->core->device >= 0 ? in->host_pull : in->host_mem) = true;
        }
      } else if (d.kind == DATA_DEVICE_IPC) {
        in->has_token = true;  // set first: a mapping failure still returns the token
        in->token = d.ipc.token;
        trace(woke ? TP_POPPED_WOKE : TP_POPPED, in->token);
        in->len = d.ipc.len;
        in->ext_len = std::max(d.ipc.ext_len, d.ipc.len);
        void* base = nullptr;
        if (d.ipc.fill == FILL_BCAST) {
          // the sample arrives through the output's RCCL group, not the producer's slot
          if (post_bcast_receive(n->core.get(), in.get(), ev->id) != DORA_OK) {
            ev->type = DORA_EVENT_ERROR;
            ev->error = dora_gpu_last_error();
            in->ptr = nullptr;
          }
        } else if (d.ipc.owner_pid == self_pid()) {
          std::lock_guard<std::mutex> g(own_slots().mu);
          auto it = own_slots().ptrs.find(d.ipc.slot_id);
          if (it != own_slots().ptrs.end()) base = it->second;
        } else {
          IpcKey key;
          std::memcpy(key.b, d.ipc.handle, 64);
          key.pid = d.ipc.owner_pid;
          key.slot = d.ipc.slot_id;
          NodeCore* c = n->core.get();
          std::lock_guard<std::mutex> g(c->ipc_mu);
          auto it = c->ipc_cache.find(key);
          if (it != c->ipc_cache.end()) {
            in->mapping = it->second;
          } else {
            hipIpcMemHandle_t h;
            std::memcpy(&h, d.ipc.handle, sizeof(h));
            // a host-only receiver maps the slot on its producer's GPU, whose copy engine stages
            // it to host memory (stage_to_host)
            DeviceScope ds(c->device >= 0 ? c->device : int(d.ipc.device));
            hipError_t e = hipIpcOpenMemHandle(&base, h, hipIpcMemLazyEnablePeerAccess);
            if (e != hipSuccess) {
              ev->type = DORA_EVENT_ERROR;
              ev->error = std::string("hipIpcOpenMemHandle: ") + hipGetErrorString(e) +
                          " (slot " + std::to_string(d.ipc.slot_id) + " of pid " +
                          std::to_string(d.ipc.owner_pid) + " on GPU " +
                          std::to_string(d.ipc.device) + ", " + std::to_string(d.ipc.len) + " B)";
              base = nullptr;
            } else {
              in->mapping = std::make_shared<IpcMapping>();
              in->mapping->base = base;
              c->ipc_cache.emplace(key, in->mapping);
              c->ipc_opens.fetch_add(1, std::memory_order_relaxed);
              n->core->region->hdr()->nodes[c->idx].ipc_opens.fetch_add(1, std::memory_order_relaxed);
              c->trim_ipc_cache();
            }
          }
          if (in->mapping) {
            in->mapping->last_use = ++c->ipc_clock;
            base = in->mapping->base;
          }
        }
        if (base) in->ptr = static_cast<uint8_t*>(base) + d.ipc.offset;
        // the fill wait and a cross-GPU pull happen when the event is handed out
        // (finish_input), so draining a burst never serialises on later fills
        ev->pending = true;
        ev->ipc = d.ipc;
      }
      ev->data = std::move(in);
      break;
    }
    case EV_INPUT_CLOSED:
      ev->type = DORA_EVENT_INPUT_CLOSED;
      ev->id = r.str();
      break;
    case EV_ALL_INPUTS_CLOSED:
      ev->type = DORA_EVENT_ALL_INPUTS_CLOSED;
      break;
    case EV_STOP:
      ev->type = DORA_EVENT_STOP;
      break;
    case EV_BCAST_JOIN: {
      const std::string input = r.str();
      uint8_t uid[kBcastIdBytes];
      r.raw(uid, sizeof(uid));
      const uint32_t nranks = r.u32();
      const uint32_t rank = r.u32();
      join_bcast_group(n, input, uid, nranks, rank);
      return;  // internal: no event for the user
    }
    default:
      return;  // EV_READY after init is ignored
  }
  n->queue.push_back(std::move(ev));
}

// A device sample delivered to a node without a GPU (DORA_GPU_DEVICE < 0): one DMA by the
// producer GPU's copy engines into pinned host memory the input owns (recycled, host_pool), then
// the producer's token goes back at once and the input is a host input like a shared-memory one
// (the reference's receivers always get host ArrowData, event_stream/event.rs:35-91; a Python
// receiver a pyarrow array, apis/python/operator/src/lib.rs:135-144).  The copy is issued to the
// copy engines through HSA and its signal polled (aql.h hsa_copy_host): 4 KB in 6.9 us where
// hipMemcpyAsync + hipStreamSynchronize took 17 (scripts/d2h_copy_probe.py,
// profiles/r06_d2h_copy_probe.jsonl); a 4 KB message to such a receiver beside a device one,
// send call to receipt, 15.5-16.5 us p50 / 19-21 p99 against 20.9-21.9 / 37-38 with HIP's copy
// (profiles/r06_stage_copy_ab.txt, five interleaved rounds); HIP's copy stays the fallback.  40.96 MB: 56 GB/s on an
// MI355X box (profiles/r06_host_path_probe.jsonl, d2h_pinned).  The pack kernel writing pinned
// host memory from one raw AQL packet of the receiver was slower at every size tried, 23 / 27 /
// 30 us against 18 / 16 / 20 at 4 KB / 64 KB / 256 KB (profiles/r06_d2h_stage_ab.jsonl).
int stage_to_host(InputData* in, int src_device) {
  NodeCore* c = in->core.get();
  if (in->ext_len) {
    DeviceScope ds(src_device);
    uint64_t cap = 0;
    void* h = c->host_pool_get(in->ext_len, &cap);
    if (!h)
      return fail(DORA_ERR_HIP, "pinned staging buffer of %llu bytes",
                  (unsigned long long)in->ext_len);
    hipError_t e = hipSuccess;
    const int hrc = hsa_copy_host(h, in->ptr, in->ext_len, true);
    if (hrc == DORA_ERR_TIMEOUT) return hrc;  // the buffer is not reused: the copy may still land
    if (hrc != DORA_OK) {
      static std::atomic<bool> noted{false};
      if (std::getenv("DORA_GPU_TRACE") && !noted.exchange(true))
        std::fprintf(stderr, "dora-gpu: staging through HIP's copy: %s\n", dora_gpu_last_error());
      clear_error();
      hipStream_t st = c->stage_stream(src_device);
      e = st ? hipMemcpyAsync(h, in->ptr, in->ext_len, hipMemcpyDeviceToHost, st)
             : hipErrorInvalidResourceHandle;
      if (e == hipSuccess) e = hipStreamSynchronize(st);
    }
    if (e != hipSuccess) {
      (void)hipGetLastError();
      c->host_pool_put(h, cap);
      return fail(DORA_ERR_HIP, "staging a device sample to host memory: %s",
                  hipGetErrorString(e));
    }
    in->host_local = h;
    in->host_local_cap = cap;
    c->host_staged.fetch_add(1, std::memory_order_relaxed);
    c->host_staged_bytes.fetch_add(in->ext_len, std::memory_order_relaxed);
  }
  in->ptr = in->host_local;
  in->host_mem = true;
  in->mapping.reset();
  if (in->has_token) {
    c->report_drop_token(in->token);
    trace(TP_RELEASED, in->token);
    in->has_token = false;
  }
  return DORA_OK;
}

// Complete a queued device input right before it is handed to the user: wait for the
// producer's fill (flag or interprocess event) and, for a slot on another GPU, pull it into a
// local receive slot with one peer copy and return the producer's token at once.
void finish_input(dora_node* n, dora_event* ev) {
  if (!ev->pending) return;
  SubSpan sp(SP_RECV_FINISH);
  ev->pending = false;
  InputData* in = ev->data.get();
  const DeviceIpc& d = ev->ipc;
  if (!in || !in->ptr) return;
  if (d.fill == FILL_BCAST) {
    // the receive was posted at drain time; hand the input out once it has completed
    hipError_t e = in->bcast_ev ? hipEventQuery(in->bcast_ev) : hipSuccess;
    const uint64_t t0 = mono_ns();
    while (e == hipErrorNotReady && mono_ns() - t0 < 60000000000ull) {
      if (mono_ns() - t0 > uint64_t(spin_budget_us()) * 1000) usleep(20);
      else __builtin_ia32_pause();
      e = hipEventQuery(in->bcast_ev);
    }
    if (e != hipSuccess) {
      ev->type = DORA_EVENT_ERROR;
      ev->error = e == hipErrorNotReady ? "broadcast receive did not complete within 60 s"
                                        : std::string("broadcast receive: ") + hipGetErrorString(e);
      in->ptr = nullptr;
      return;
    }
    trace(TP_FILLED, in->token);
    return;
  }
  if (d.fill == FILL_FLAG) {
    // the producer's stream writes the epoch into its fill flag after the pack: poll it
    RegionHdr* h = n->core->region->hdr();
    if (d.flag_node >= h->n_nodes || d.flag_index >= kFillFlags) {
      ev->type = DORA_EVENT_ERROR;
      ev->error = "fill flag out of range";
      in->ptr = nullptr;
      return;
    }
    const std::atomic<uint64_t>& f = h->nodes[d.flag_node].fill[d.flag_index].epoch;
    const uint64_t t0 = mono_ns();
    unsigned spins = 0;
    while (!fill_reached(&f, d.epoch)) {
      if (++spins < 4096) {
        __builtin_ia32_pause();
        continue;
      }
      spins = 0;
      if (mono_ns() - t0 > 60000000000ull) {
        ev->type = DORA_EVENT_ERROR;
        ev->error = "the producer's fill did not complete within 60 s";
        in->ptr = nullptr;
        return;
      }
      if (mono_ns() - t0 > uint64_t(spin_budget_us()) * 1000) usleep(20);
    }
    add_fill_wait_ns(mono_ns() - t0);
    if (trace_enabled()) {
      // the pack's own stamps (s_memrealtime), for the GPU side of a message's latency: only an
      // in-kernel-signalled fill of exactly this epoch writes them (a CP-signalled fill writes
      // none, and the line may already carry a later fill's stamps if the slot was refilled)
      const FillFlag& ff = h->nodes[d.flag_node].fill[d.flag_index];
      if (ff.epoch.load(std::memory_order_acquire) == d.epoch &&
          ff.cp_epoch.load(std::memory_order_acquire) != d.epoch) {
        // on the host's clock when the HSA runtime can map GPU ticks (aql.h), else GPU ns
        const uint64_t s0 = aql_gpu_tick_to_realtime_ns(n->core->device, ff.t_start);
        const uint64_t s1 = aql_gpu_tick_to_realtime_ns(n->core->device, ff.t_end);
        const double ns_per_tick = 1e9 / kRealtimeHz;
        trace_at(TP_GPU_START, in->token, s0 ? s0 : uint64_t(double(ff.t_start) * ns_per_tick));
        trace_at(TP_GPU_SIGNAL, in->token, s1 ? s1 : uint64_t(double(ff.t_end) * ns_per_tick));
      }
    }
  } else if (d.fill == FILL_EVENT) {
    // the producer's fill completes when its interprocess event fires
    hipEvent_t fill = nullptr;
    std::string key(reinterpret_cast<const char*>(d.event), 64);
    {
      std::lock_guard<std::mutex> g(n->core->ipc_mu);
      auto it = n->core->ipc_events.find(key);
      if (it != n->core->ipc_events.end()) {
        fill = it->second;
      } else {
        hipIpcEventHandle_t h;
        std::memcpy(&h, d.event, sizeof(h));
        DeviceScope ds(n->core->device);
        if (hipIpcOpenEventHandle(&fill, h) == hipSuccess) n->core->ipc_events[key] = fill;
        else fill = nullptr;
      }
    }
    // spin on the event (hipEventSynchronize sleeps in ~1 ms quanta on interprocess events
    // that are not yet complete), then fall back to the blocking wait
    hipError_t e = fill ? hipEventQuery(fill) : hipErrorInvalidHandle;
    const uint64_t t0 = mono_ns();
    while (e == hipErrorNotReady && mono_ns() - t0 < 20000000ull) {
      __builtin_ia32_pause();
      e = hipEventQuery(fill);
    }
    if (e == hipErrorNotReady) e = hipEventSynchronize(fill);
    if (e != hipSuccess) {
      ev->type = DORA_EVENT_ERROR;
      ev->error = std::string("waiting for the producer's fill event: ") + hipGetErrorString(e);
      in->ptr = nullptr;
      return;
    }
  }
  trace(TP_FILLED, in->token);
  if (n->core->device < 0) {
    // a receiver without a GPU gets the reference's host ArrowData (event.rs:35-91): the sample
    // is staged to host memory now and the producer's token goes back at once
    if (stage_to_host(in, int(d.device)) != DORA_OK) {
      ev->type = DORA_EVENT_ERROR;
      ev->error = dora_gpu_last_error();
      in->ptr = nullptr;
    }
    return;
  }
  if (in->len && (d.device != n->core->device || edge_copy_forced())) {
    // Cross-GPU edge: the sample is pulled over xGMI on first access to its data
    // (ensure_local), or straight into an outgoing slot by dora_node_forward.
    in->remote_device = d.device;
  }
}

// Enqueue one copy of `len` bytes from a slot on `src_device` (IPC-mapped) into local HBM on
// the node stream: the pack kernel reading the peer's HBM over xGMI (default), or the copy
// engines (DORA_GPU_PEER_COPY=sdma).
int ensure_peer_access(NodeCore* c, int src_device) {
  if (src_device == c->device) return DORA_OK;
  std::lock_guard<std::mutex> g(c->ipc_mu);
  if (c->peer_enabled.count(src_device)) return DORA_OK;
  hipError_t e = hipDeviceEnablePeerAccess(src_device, 0);
  if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled)
    return fail(DORA_ERR_HIP, "enable peer access %d -> %d: %s", c->device, src_device,
                hipGetErrorString(e));
  (void)hipGetLastError();
  c->peer_enabled.insert(src_device);
  return DORA_OK;
}

int enqueue_peer_copy(NodeCore* c, void* dst, const void* src, int src_device, uint64_t len) {
  int rc = ensure_peer_access(c, src_device);
  if (rc != DORA_OK) return rc;
  c->stream_used.store(true, std::memory_order_relaxed);
  if (peer_copy_mode() == PEER_SDMA) {
    hipError_t e = hipMemcpyPeerAsync(dst, c->device, src, src_device, len, c->stream);
    if (e != hipSuccess) return fail(DORA_ERR_HIP, "hipMemcpyPeerAsync: %s", hipGetErrorString(e));
    return DORA_OK;
  }
  Segment seg{src, 0, len};
  return launch_pack(&seg, 1, ARROW_DEVICE_ROCM, static_cast<uint8_t*>(dst), c->stream, nullptr,
                     nullptr);
}

// Pull a cross-GPU input into this node's receive pool (complete on return) and hand the
// producer its slot back at once.
int ensure_local(InputData* in) {
  if (!in || (in->remote_device < 0 && !in->host_pull)) return DORA_OK;
  NodeCore* c = in->core.get();
  DeviceScope ds(c->device);
  uint64_t cap = 0;
  void* local = c->recv_pool_get(in->ext_len, &cap);
  if (!local)
    return fail(DORA_ERR_HIP, "receive slot of %llu bytes", (unsigned long long)in->ext_len);
  // The pull runs on a stream of its own and is waited for alone: on the node stream it would
  // queue behind (and its wait would wait for) every consumer kernel already there.
  // The pulled copy is complete on return, so any stream may read it.
  hipStream_t ps = c->stage_stream(c->device);
  if (!ps) ps = c->stream;
  int rc = DORA_OK;
  if (in->host_pull) {
    // a host-only producer's shared memory: pinned once per region on its first pull (not at
    // drain time, which may hold the event queue's lock), then one DMA into HBM
    {
      std::lock_guard<std::mutex> g(c->ipc_mu);
      if (!in->shm->reg_tried) {
        in->shm->reg_tried = true;
        in->shm->registered =
            hipHostRegister(in->shm->base, in->shm->len, hipHostRegisterDefault) == hipSuccess;
        (void)hipGetLastError();
      }
    }
    // the copy engines through HSA, its signal polled (as stage_to_host), once the region is
    // pinned; else HIP's copy.  Host-only 4 KB to a device receiver, send call to receipt:
    // 10.8-14.3 us p50 / 23-32 p99 against 17.5-20.3 / 45-58 (profiles/r06_pull_copy_ab.txt)
    rc = in->shm->registered ? hsa_copy_host(local, in->ptr, in->ext_len, false)
                             : int(DORA_ERR_UNSUPPORTED);
    if (rc == DORA_ERR_TIMEOUT) return rc;  // the receive slot is not reused: the copy may land
    if (rc != DORA_OK) {
      clear_error();
      rc = DORA_OK;
      hipError_t e = hipMemcpyAsync(local, in->ptr, in->ext_len, hipMemcpyHostToDevice, ps);
      if (e == hipSuccess) e = hipStreamSynchronize(ps);
      if (e != hipSuccess) rc = fail(DORA_ERR_HIP, "shared-memory pull: %s", hipGetErrorString(e));
    }
  } else if (peer_copy_mode() == PEER_SDMA) {
    rc = ensure_peer_access(c, in->remote_device);
    if (rc == DORA_OK) {
      hipError_t e =
          hipMemcpyPeerAsync(local, c->device, in->ptr, in->remote_device, in->ext_len, ps);
      if (e == hipSuccess) e = hipStreamSynchronize(ps);
      if (e != hipSuccess) rc = fail(DORA_ERR_HIP, "cross-GPU pull: %s", hipGetErrorString(e));
    }
  } else {
    // the pack kernel reads the peer's HBM over xGMI; wait on its own completion flag
    rc = ensure_peer_access(c, in->remote_device);
    Segment seg{in->ptr, 0, in->ext_len};
    if (rc == DORA_OK) rc = launch_pack_wait(&seg, 1, static_cast<uint8_t*>(local), ps);
  }
  if (rc != DORA_OK) {
    c->recv_pool_put(local, cap);
    return rc;
  }
  in->local = local;
  in->local_cap = cap;
  in->ptr = local;
  c->report_drop_token(in->token);
  trace(TP_RELEASED, in->token);
  in->has_token = false;
  if (in->host_pull) {
    in->host_pull = false;
    in->shm.reset();
    return DORA_OK;
  }
  in->remote_device = -1;
  c->peer_copies.fetch_add(1, std::memory_order_relaxed);
  c->peer_bytes.fetch_add(in->ext_len, std::memory_order_relaxed);
  return DORA_OK;
}

// An input whose producer's fill is still running.  In the reference the sample is filled before
// the message leaves the sender (send_output returns after the copy), so such an input would not
// be queued here yet: the queue_size policy neither counts nor drops it.  Without this, an
// async sender with more samples in flight than a receiver's queue_size (12 vs the default 10)
// made the receiver drop inputs whenever it waited on the GPU: 20-25 % of a 1-4 MB burst from
// the Python node (scripts/py_tp.py), inputs the reference would have delivered.
// How long an input may sit in the queue uncounted because its producer's fill has not
// signalled: past 2 s the drop-oldest policy counts it again, so a fill that never completes (a
// lost queue, a GPU fault) cannot grow the queue beyond its queue_size.
constexpr uint64_t kTransitLimitNs = 2000000000ull;

bool fill_in_transit(dora_node* n, const dora_event* e) {
  if (!e->pending || e->ipc.fill != FILL_FLAG) return false;
  RegionHdr* h = n->core->region->hdr();
  if (e->ipc.flag_node >= h->n_nodes || e->ipc.flag_index >= kFillFlags) return false;
  if (fill_reached(&h->nodes[e->ipc.flag_node].fill[e->ipc.flag_index].epoch, e->ipc.epoch))
    return false;
  return mono_ns() - e->arrived_ns < kTransitLimitNs;
}

// drop_oldest_inputs (node_communication/mod.rs:320-359): newest first, keep queue_size per input.
// `held_front`: the queue's first event counts as taken (the event-stream thread's: the one the
// reference's thread holds in its channel, event_stream/thread.rs:139-157).
void drop_oldest_inputs(dora_node* n, bool held_front = false) {
  // no input can exceed its queue size while the whole queue holds no more events than the
  // smallest one (the common case of a receiver keeping up): nothing to count
  const size_t held = held_front ? 1 : 0;
  if (n->queue_size.empty() || n->queue.size() <= n->min_queue_size + held) return;
  SubSpan sp(SP_RECV_DROPOLD);
  std::map<std::string, uint32_t> remaining = n->queue_size;
  for (auto it = n->queue.rbegin(); it != n->queue.rend() - std::ptrdiff_t(held); ++it) {
    dora_event* e = it->get();
    if (!e || e->type != DORA_EVENT_INPUT) continue;
    auto q = remaining.find(e->id);
    if (q == remaining.end()) continue;
    if (fill_in_transit(n, e)) continue;
    if (q->second == 0) {
      it->reset();  // releases the InputData -> drop token reported
      ++n->dropped_inputs;
      n->core->region->hdr()->nodes[n->core->idx].dropped_inputs.fetch_add(
          1, std::memory_order_relaxed);
    } else {
      --q->second;
    }
  }
  n->queue.erase(std::remove_if(n->queue.begin(), n->queue.end(),
                                [](const std::unique_ptr<dora_event>& e) { return !e; }),
                 n->queue.end());
}

// Move every event the daemon has delivered into the node's queue; true when any arrived.
bool drain_events(dora_node* n) {
  uint32_t kind;
  std::vector<uint8_t>& p = n->ev_buf;  // reused across events
  SubSpan sp(SP_RECV_DRAIN);
  bool got = false;
  while (n->core->ev.try_pop(&kind, &p)) {
    encode_event(n, kind, p);
    got = true;
  }
  return got;
}

// A host-only node joins the L3 domain the dataflow's GPU nodes chose, once one has (it may
// start before them): its control-ring lines then move inside one L3 like theirs.
void pin_host_node(dora_node* n) {
  RegionHdr* rh = n->core->region->hdr();
  const int32_t numa = rh->numa_hint.load(std::memory_order_acquire);
  if (numa < 0 || rh->l3_cpu.load(std::memory_order_acquire) < 0) return;
  n->pin_pending = false;
  (void)pin_to_numa(numa, -1, &rh->l3_cpu, int(rh->n_nodes) + 1);
}

// The event-stream thread (dora_node::pump): drain, apply drop-oldest, wake the user thread.
// Draining allocates receive slots, opens IPC mappings, creates events and posts broadcast
// receives, all on the current HIP device of the calling thread: this thread's is the node's.
void pump_main(dora_node* n) {
  if (n->core->device >= 0) (void)hipSetDevice(n->core->device);
  while (!n->pump_stop.load(std::memory_order_acquire)) {
    bool got;
    {
      std::lock_guard<std::mutex> g(n->qmu);
      got = drain_events(n);
      if (got) drop_oldest_inputs(n, /*held_front=*/true);
    }
    if (got) n->qcv.notify_all();
    else n->core->ev.wait(10000);  // bounded: notices pump_stop
  }
}

void start_pump(dora_node* n) {
  if (n->pump_on.load()) return;
  n->pump_stop.store(false);
  n->pump_on.store(true);
  n->pump = std::thread(pump_main, n);
}

void stop_pump(dora_node* n) {
  if (!n->pump_on.load()) return;
  n->pump_stop.store(true, std::memory_order_release);
  if (n->pump.joinable()) n->pump.join();
  n->pump_on.store(false);
}

// The Metadata of a send as WBuf::bytes(WBuf::metadata(m)) would write it, straight into `w`
// (no Metadata copy of the type info and parameters per send).
void put_metadata(WBuf& w, const std::vector<uint8_t>& ti, const uint8_t* params,
                  size_t params_len, uint64_t ts) {
  const uint64_t n = 2 + 8 + 8 + ti.size() + 8 + (params ? params_len : 0);
  w.u64(n);
  w.u16(0);  // metadata version
  w.u64(ts);
  w.bytes(ti.data(), ti.size());
  w.bytes(params, params ? params_len : 0);
}

int send_sample(dora_node* n, const char* output_id, const std::vector<uint8_t>& ti,
                const uint8_t* params, size_t params_len, dora_sample* sample,
                DropToken* token_out = nullptr, uint64_t ts_override = 0) {
  {
    SubSpan sp(SP_SEND_TOKENS);
    handle_finished_drop_tokens(n);
  }
  SubSpan sp_lookup(SP_SEND_LOOKUP);
  if (!n->outputs.count(output_id)) {
    delete sample;  // the sample is consumed either way
    return fail(DORA_ERR_NOT_FOUND,
                "unknown dora node output `%s` called by `send_output`. Double-check if this "
                "output is defined within your dataflow YAML file.",
                output_id);
  }
  // Metadata::from_parameters(clock.new_timestamp(), ..) mod.rs:258; a proxy of a remote
  // node keeps the producer's timestamp (the inter-daemon message's metadata)
  sp_lookup.stop();
  SubSpan sp_req(SP_SEND_REQUEST);
  const uint64_t ts = ts_override ? ts_override : now_ns();
  DataMsg d;
  Slot* slot = nullptr;
  if (sample) {
    if (sample->slot && sample->slot->host) {
      slot = sample->slot;
      d.kind = DATA_SHMEM;
      d.shm.name = slot->shm_name;
      d.shm.len = sample->len;
      d.shm.token = generate_drop_token();
    } else if (sample->slot) {
      slot = sample->slot;
      d.kind = DATA_DEVICE_IPC;
      std::memcpy(d.ipc.handle, &slot->handle, 64);
      d.ipc.device = n->core->device;
      d.ipc.owner_pid = self_pid();
      d.ipc.slot_id = slot->id;
      d.ipc.offset = 0;
      d.ipc.len = sample->len;
      d.ipc.ext_len = std::max(sample->len, sample->ext_len);
      d.ipc.token = generate_drop_token();
      d.ipc.fill = sample->fill;
      auto g = n->bcast_out.find(output_id);
      if (g != n->bcast_out.end()) {
        // fan-out over the output's RCCL group: broadcast the slot on the output's stream, after
        // its pack there (pack_and_send), or — a sample the user filled — after the work queued on
        // the node stream and every fill so far
        hipStream_t bs = g->second.stream;
        DeviceScope ds(n->core->device);
        if (sample->fill != FILL_DONE) n->core->fence_fills();
        n->core->order_after_node_stream(bs);
        int rc = bcast_enqueue(g->second.comm, slot->ptr, d.ipc.ext_len, bs);
        // the broadcast reads the slot on its stream: the slot is idle after it
        if (!slot->use_ev && hipEventCreateWithFlags(&slot->use_ev, hipEventDisableTiming) != hipSuccess)
          slot->use_ev = nullptr;
        if (slot->use_ev && hipEventRecord(slot->use_ev, bs) == hipSuccess)
          slot->use_pending = true;
        else
          (void)hipStreamSynchronize(bs);
        (void)hipGetLastError();
        if (rc != DORA_OK) {
          add_to_cache(n, slot);
          delete sample;
          return rc;
        }
        d.ipc.fill = FILL_BCAST;
        d.ipc.epoch = ++n->bcast_seq;
      } else if (sample->fill == FILL_FLAG) {
        d.ipc.flag_node = static_cast<uint32_t>(n->core->idx);
        d.ipc.flag_index = static_cast<uint32_t>(slot->flag);
        d.ipc.epoch = sample->epoch;
      }
      if (d.ipc.fill == FILL_EVENT) std::memcpy(d.ipc.event, &slot->done_handle, 64);
    } else {
      d.kind = DATA_VEC;
      d.vec = std::move(sample->vec);
    }
    delete sample;
  }
  WBuf& w = n->send_buf;
  w.clear();
  w.str(output_id);
  put_metadata(w, ti, params, params_len, ts);
  w.data(d);
  int rc = n->core->request(REQ_SEND_MESSAGE, w.data(), w.size());
  sp_req.stop();
  if (rc != DORA_OK) {
    if (slot) add_to_cache(n, slot);
    return rc;
  }
  SubSpan sp_track(SP_SEND_TRACK);
  if (slot && d.kind == DATA_SHMEM) {
    n->sent_out[d.shm.token] = slot;
    if (token_out) *token_out = d.shm.token;
  } else if (slot) {
    n->sent_out[d.ipc.token] = slot;
    if (token_out) *token_out = d.ipc.token;
    trace(n->core->last_rang ? TP_SENT_RANG : TP_SENT, d.ipc.token);
  } else if (trace_enabled()) {
    trace(n->core->last_rang ? TP_SENT_RANG : TP_SENT, ts_key(ts));  // an inline sample
  }
  return DORA_OK;
}

constexpr uint64_t kZeroCopyThreshold = 4096;  // mod.rs:40

// `ext_len` > len: the slot also holds a validity tail (plans with in-sample bitmaps).
// Stamp areas of a timed region's CP-signalled packs: [0] start, [1 + k mod kCpStampWgs] the
// latest end of the workgroups k mapping there.
constexpr uint32_t kRegionCpAreas = 256;
constexpr size_t kCpAreaWords = 1 + kCpStampWgs;

// Stamp areas for timed regions' CP-signalled packs (dora_node_region_begin), made and zeroed with
// the node's AQL queues at its first send, never inside or just before a region (without them,
// e.g. no large BAR, such packs signal in-kernel inside regions).
void ensure_cp_stamps(dora_node* n) {
  if (n->region_cp_stamps || n->core->device < 0) return;
  const size_t bytes = size_t(kRegionCpAreas) * kCpAreaWords * 8;
  void* d = nullptr;
  if (bar_alloc(n->core->device, bytes, &d) != DORA_OK) {
    clear_error();
    return;  // no large BAR: a region's packs signal in-kernel
  }
  const std::vector<uint8_t> zero(bytes, 0);
  if (bar_write(n->core->device, d, zero.data(), bytes) != DORA_OK) {
    bar_free(d);
    clear_error();
    return;
  }
  n->region_cp_stamps = static_cast<uint64_t*>(d);
  void* idx = nullptr;
  void* out = nullptr;
  if (hipHostMalloc(&idx, kRegionCpAreas * 4, hipHostMallocCoherent) == hipSuccess &&
      hipHostMalloc(&out, kRegionCpAreas * 16, hipHostMallocCoherent) == hipSuccess) {
    n->region_reduce_idx = static_cast<uint32_t*>(idx);
    n->region_reduce_out = static_cast<uint64_t*>(out);
  } else {
    (void)hipGetLastError();  // region ends read the areas through the BAR
    if (idx) (void)hipHostFree(idx);
  }
}

// `host_inline`: the sample will be written by the host (a host-resident source), so below the
// zero-copy threshold it takes the reference's inline `DataMessage::Vec` (mod.rs:303-319) on a
// device node too: no slot, no H2D copy, no fill signal.
int alloc_sample(dora_node* n, uint64_t len, dora_sample** out, uint64_t ext_len = 0,
                 bool host_inline = false) {  // mod.rs:303-319
  if (n->core->device < 0 && len >= kZeroCopyThreshold) {
    // host-only node: a POSIX shared-memory slot (the reference's allocate_shared_memory)
    auto* s = new dora_sample();
    s->len = len;
    handle_finished_drop_tokens(n);
    int rc = allocate_host_slot(n, len, &s->slot);
    if (rc != DORA_OK) {
      delete s;
      return rc;
    }
    *out = s;
    return DORA_OK;
  }
  if (n->core->device < 0 || (host_inline && std::max(len, ext_len) < kZeroCopyThreshold)) {
    auto* s = new dora_sample();
    s->len = len;
    s->vec.assign(len, 0);  // AVec::__from_elem(128, 0, len)
    *out = s;
    return DORA_OK;
  }
  SubSpan sp_new(SP_SAMPLE_NEW);
  auto* s = new dora_sample();
  s->len = len;
  sp_new.stop();
  if (len > 0) {
    if (!n->aql_ready) {
      // the first non-empty sample of this node sets up the process's AQL queues and loads the
      // pack code object (~20 ms), whatever its size: a later small send then finds them ready
      // instead of paying that inside its latency (nodes that never send data create none)
      n->aql_ready = true;
      if (aql_queue(n->core->device)) ensure_cp_stamps(n);
    }
    SubSpan sp_tok(SP_ALLOC_TOKENS);
    handle_finished_drop_tokens(n);
    sp_tok.stop();
    // Sends run ahead of the GPU; bound the samples in flight so the sender waits for a
    // returned slot instead of hipMalloc-ing new ones (a device slot costs far more to create
    // than a shm region).  After kSlotWaitNs without a returned token the slot is allocated
    // anyway, as the reference would (a receiver may legitimately hold many inputs).
    SubSpan sp_wait(SP_ALLOC_WAIT);
    const uint64_t t0 = mono_ns();
    while (n->sent_out.size() >= max_in_flight(len) && mono_ns() - t0 < kSlotWaitNs) {
      n->core->drops.wait(1000);
      handle_finished_drop_tokens(n);
      if (n->core->region->hdr()->nodes[n->core->idx].state.load() == 2) break;
    }
    sp_wait.stop();
    s->ext_len = std::max(len, ext_len);
    SubSpan sp_slot(SP_ALLOC_SLOT);
    int rc = allocate_slot(n, s->ext_len, &s->slot);
    if (rc != DORA_OK) {
      delete s;
      return rc;
    }
  }
  *out = s;
  return DORA_OK;
}

// Device-resident samples up to this size for an output whose receivers all lack a GPU are
// packed by the GPU straight into a shared-memory region (host_bound_sample): one dispatch on
// the sender's warm queues instead of a slot in HBM that each receiver copies out with a HIP copy
// of its own (stage_to_host, ~13 us of runtime overhead at any small size).  Larger samples keep
// that path: the copy engines move them at the box's DMA rate and leave the CUs free, where a
// pack writing over PCIe would hold its workgroups for the whole transfer.
constexpr uint64_t kHostPackMax = 1ull << 20;

// A sample for such an output: a shared-memory slot of this node (the reference's
// DataMessage::SharedMemory, which its receivers map), page-locked and mapped for the GPU once,
// with a fill flag for the pack to signal.  Null, with no error, when one cannot be made (no
// free fill flag, registration refused): the caller takes an HBM slot.
dora_sample* host_bound_sample(dora_node* n, uint64_t len, uint64_t ext_len) {
  NodeCore* c = n->core.get();
  if (!c->region_dev || !c->fill_done) return nullptr;
  handle_finished_drop_tokens(n);
  const uint64_t t0 = mono_ns();
  while (n->sent_out.size() >= max_in_flight(len) && mono_ns() - t0 < kSlotWaitNs) {
    c->drops.wait(1000);
    handle_finished_drop_tokens(n);
    if (c->region->hdr()->nodes[c->idx].state.load() == 2) break;
  }
  Slot* slot = nullptr;
  const uint64_t ext = std::max(len, ext_len);
  if (allocate_host_slot(n, ext, &slot) != DORA_OK) {
    clear_error();
    return nullptr;
  }
  if (!slot->registered) {
    DeviceScope ds(c->device);
    void* dp = nullptr;
    if (hipHostRegister(slot->ptr, slot->cap, hipHostRegisterMapped | hipHostRegisterPortable) !=
        hipSuccess) {
      (void)hipGetLastError();
      release_slot_memory(slot);
      return nullptr;
    }
    slot->registered = true;
    // the pack writes through the host address (one address space for host and GPU)
    if (hipHostGetDevicePointer(&dp, slot->ptr, 0) != hipSuccess || dp != slot->ptr) {
      (void)hipGetLastError();
      release_slot_memory(slot);
      return nullptr;
    }
  }
  if (slot->flag < 0) {
    if (c->free_flags.empty()) {
      add_to_cache(n, slot);
      return nullptr;
    }
    slot->flag = static_cast<int>(c->free_flags.back());
    c->free_flags.pop_back();
  }
  auto* s = new dora_sample();
  s->len = len;
  s->ext_len = ext;
  s->slot = slot;
  return s;
}

// An unsent sample back to the node: its slot to the cache (an inline Vec is just freed).
void discard_sample(dora_node* n, dora_sample* s) {
  if (!s) return;
  if (s->slot) add_to_cache(n, s->slot);
  delete s;
}

constexpr size_t kTimingPairs = 64;
constexpr size_t kMaxIntervals = 1 << 16;  // stamped packs whose (start, stop) are kept

void harvest(dora_node* n, TimingPair& p) {
  if (!p.pending) return;
  float ms = 0;
  if (hipEventSynchronize(p.stop) == hipSuccess &&
      hipEventElapsedTime(&ms, p.start, p.stop) == hipSuccess) {
    n->pack_ms += ms;
    ++n->pack_count;
    n->pack_bytes += p.bytes;
    float a = 0, b = 0;
    if (n->timing_ref && n->intervals.size() < 2 * kMaxIntervals &&
        hipEventElapsedTime(&a, n->timing_ref, p.start) == hipSuccess &&
        hipEventElapsedTime(&b, n->timing_ref, p.stop) == hipSuccess) {
      n->intervals.push_back(a);
      n->intervals.push_back(b);
    }
  }
  (void)hipGetLastError();
  p.pending = false;
}

void harvest_all(dora_node* n) {
  for (auto& p : n->timing) harvest(n, p);
}

int ensure_timing(dora_node* n) {
  if (!n->timing.empty()) return DORA_OK;
  DeviceScope ds(n->core->device);
  DORA_HIP(hipEventCreate(&n->timing_ref));
  n->timing.resize(kTimingPairs);
  for (auto& p : n->timing) {
    DORA_HIP(hipEventCreate(&p.start));
    DORA_HIP(hipEventCreate(&p.stop));
  }
  return DORA_OK;
}

TimingPair* next_timing_pair(dora_node* n, uint64_t bytes) {
  if (n->timing.empty()) return nullptr;
  TimingPair& p = n->timing[n->timing_next++ % n->timing.size()];
  harvest(n, p);  // normally long complete
  p.bytes = bytes;
  p.pending = true;
  return &p;
}

// Tell receivers when the fill enqueued on stream `st` is complete.
hipError_t order_fill(dora_node* n, dora_sample* s, hipStream_t st) {
  if (s->slot->flag >= 0) {
    // async: the stream writes the send epoch into the slot's fill flag once the fill has
    // completed; the receiver polls it, the sender moves on
    s->epoch = ++n->core->epoch;
    s->fill = FILL_FLAG;
    s->slot->fill_epoch = s->epoch;
    return hipStreamWriteValue64(st, n->core->flag_dev(s->slot->flag), s->epoch, 0);
  }
  if (s->slot->done) {
    // async fallback: interprocess event
    s->fill = FILL_EVENT;
    return hipEventRecord(s->slot->done, st);
  }
  // sync: the sample must be complete before its descriptor leaves the process
  return hipStreamSynchronize(st);
}

// Launch the fill of sample `s` (segments into its slot) on stream `st` and order its
// completion signal.
int fill_sample(dora_node* n, dora_sample* s, const Segment* segs, size_t nseg,
                ArrowDeviceType dev, hipStream_t st, hipEvent_t t_start, hipEvent_t t_stop,
                bool signal = true, bool sync = false) {
  if (!signal) {
    // the caller orders what follows on `st` (a broadcast-group send): no fill flag
    DeviceScope ds(n->core->device);
    ++n->hip_packs;
    return launch_pack(segs, nseg, dev, static_cast<uint8_t*>(s->slot->ptr), st, t_start, t_stop,
                       nullptr, nullptr, slot_bytes(s->slot->cap));
  }
  FillSignal sig{};
  const FillSignal* sp = nullptr;
  if (s->slot->flag >= 0 && n->core->fill_done) {
    sig.flag = n->core->flag_dev(s->slot->flag);
    sig.epoch = ++n->core->epoch;
    sig.done = n->core->fill_done + size_t(s->slot->flag) * kMaxSignalWgs;
    sp = &sig;
  }
  if (sp && !st && !t_start && !t_stop && dev == ARROW_DEVICE_ROCM &&
      nseg <= aql_max_segments() &&
      std::all_of(segs, segs + nseg, [](const Segment& g) { return g.op == SEG_COPY; }) &&
      [&] {
        SubSpan sq(SP_STREAM_QUERY);
        return !n->core->stream_busy();
      }()) {
    // host-bound size: one raw AQL packet instead of hipLaunchKernel (aql.h)
    if (!n->core->aql_tried) {  // looked up once (a global lock), then kept
      n->core->aql_tried = true;
      n->core->aql = aql_queue(n->core->device);
    }
    if (AqlQueue* q = aql_usable(n->core->aql) ? n->core->aql : nullptr) {
      const std::atomic<uint64_t>* fh = n->core->flag_host(s->slot->flag);
      // a timed region's pack may be signalled by the command processor if it has a stamp area
      int area = -1;
      uint64_t* stamps = nullptr;
      // (only a pack aql_pack will CP-signal takes one: a region has kRegionCpAreas of them)
      if (n->region_armed && n->region_cp_stamps && n->region_cp_next < kRegionCpAreas &&
          aql_cp_candidate(segs, nseg, sync)) {
        area = int(n->region_cp_next++);
        stamps = n->region_cp_stamps + size_t(area) * kCpAreaWords;
      }
      s->slot->region_cp_area = area;
      bool read = false;
      if (aql_pack(q, segs, nseg, static_cast<uint8_t*>(s->slot->ptr), sig, fh,
                   n->region_armed, s->slot->host ? s->slot->cap : slot_bytes(s->slot->cap),
                   stamps, sync, &read) == DORA_OK) {
        s->read_signalled = read;
        n->core->note_aql_fill(fh, sig.epoch);
        if (n->region_armed) ++n->region_aql;
        ++n->aql_packs;
        s->epoch = sig.epoch;
        s->fill = FILL_FLAG;
        s->slot->fill_epoch = sig.epoch;
        s->stamped = true;
        return DORA_OK;
      }
    }
  }
  DeviceScope ds(n->core->device);  // HIP launches and event records below
  if (!st) st = n->core->next_fill_stream();
  ++n->hip_packs;
  bool signalled = false;
  int rc = launch_pack(segs, nseg, dev, static_cast<uint8_t*>(s->slot->ptr), st, t_start,
                       t_stop, sp, &signalled,
                       s->slot->host ? s->slot->cap : slot_bytes(s->slot->cap));
  if (rc != DORA_OK) return rc;
  if (signalled) {
    s->epoch = sig.epoch;
    s->fill = FILL_FLAG;
    s->slot->fill_epoch = sig.epoch;
    s->stamped = true;
    NodeCore::note(n->core->flag_pending, n->core->flag_host(s->slot->flag), sig.epoch);
    return DORA_OK;
  }
  for (size_t i = 0; i < n->core->fill_streams.size(); ++i)
    if (n->core->fill_streams[i] == st) n->core->fill_unsignalled[i] = 1;
  hipError_t e = order_fill(n, s, st);
  if (e != hipSuccess) return fail(DORA_ERR_HIP, "fill signal: %s", hipGetErrorString(e));
  return DORA_OK;
}

// Re-send a received input on an output with its type info (a relay stage): one copy into a
// fresh slot of this node — for a cross-GPU input straight from the peer's slot over xGMI, so
// a pipeline hop moves the payload once.

// A same-GPU device input re-sent in place: the descriptor points at the producer's slot (its
// fill is complete: the input was handed out), under a token of this node; the input — and with
// it the producer's token — is held until that token returns.  No copy, no new slot.
int forward_in_place(dora_node* n, const char* output_id, const dora_event* ev,
                     const uint8_t* params, size_t params_len) {
  handle_finished_drop_tokens(n);
  if (!n->outputs.count(output_id))
    return fail(DORA_ERR_NOT_FOUND, "unknown dora node output `%s`", output_id);
  DataMsg d;
  d.kind = DATA_DEVICE_IPC;
  d.ipc = ev->ipc;
  d.ipc.token = generate_drop_token();
  d.ipc.fill = FILL_DONE;
  d.ipc.flag_node = d.ipc.flag_index = 0;
  d.ipc.epoch = 0;
  WBuf& w = n->send_buf;
  w.clear();
  w.str(output_id);
  put_metadata(w, ev->meta.type_info, params, params_len, now_ns());
  w.data(d);
  int rc = n->core->request(REQ_SEND_MESSAGE, w.data(), w.size());
  if (rc != DORA_OK) return rc;
  n->forwarded[d.ipc.token] = ev->data;
  ++n->zero_copy_forwards;
  trace(TP_SENT, d.ipc.token);
  return DORA_OK;
}

int forward_input(dora_node* n, const char* output_id, const dora_event* ev, const uint8_t* params,
                  size_t params_len) {
  InputData* in = ev->data.get();
  if (in->host_pull) {  // a shared-memory input of a device receiver: into HBM first
    int rc = ensure_local(in);
    if (rc != DORA_OK) return rc;
  }
  if (in->has_token && !in->local && in->remote_device < 0 && in->len && !in->host_mem &&
      ev->ipc.device == n->core->device && ev->ipc.fill != FILL_BCAST && !edge_copy_forced() &&
      !n->bcast_out.count(output_id))
    return forward_in_place(n, output_id, ev, params, params_len);
  const uint64_t len = in->len;
  const uint64_t ext = std::max(in->ext_len, len);  // the validity tail travels along
  const bool device_src = (in->has_token || in->local) && !in->host_mem;
  dora_sample* s = nullptr;
  int rc = alloc_sample(n, len, &s, ext, !device_src);
  if (rc != DORA_OK) return rc;
  if (len && (!s->slot || s->slot->host)) {
    if (device_src) {
      discard_sample(n, s);
      return fail(DORA_ERR_INVALID, "host-only node cannot forward device-resident data");
    }
    std::memcpy(s->slot ? s->slot->ptr : s->vec.data(), in->ptr, len);
  } else if (len) {
    Segment seg{in->ptr, 0, ext};
    if (in->remote_device >= 0 && peer_copy_mode() == PEER_SDMA) {
      rc = enqueue_peer_copy(n->core.get(), s->slot->ptr, in->ptr, in->remote_device, ext);
      hipError_t e = rc == DORA_OK ? order_fill(n, s, n->core->stream) : hipSuccess;
      if (rc == DORA_OK && e != hipSuccess)
        rc = fail(DORA_ERR_HIP, "forward: %s", hipGetErrorString(e));
    } else {
      // the pack kernel, reading the peer's HBM over xGMI for a cross-GPU input; on the node
      // stream, which the input's destructor drains before its token goes back
      rc = in->remote_device >= 0 ? ensure_peer_access(n->core.get(), in->remote_device)
                                  : DORA_OK;
      n->core->stream_used.store(true, std::memory_order_relaxed);
      if (rc == DORA_OK)
        rc = fill_sample(n, s, &seg, 1, device_src ? ARROW_DEVICE_ROCM : ARROW_DEVICE_CPU,
                         n->core->stream, nullptr, nullptr);
    }
    if (rc == DORA_OK && in->remote_device >= 0) {
      n->core->peer_copies.fetch_add(1, std::memory_order_relaxed);
      n->core->peer_bytes.fetch_add(ext, std::memory_order_relaxed);
    }
    if (rc != DORA_OK) {
      add_to_cache(n, s->slot);
      delete s;
      return rc;
    }
  }
  // the input keeps the producer's token until this node's stream has passed the copy
  // (InputData's destructor), so the producer cannot refill the slot under it
  return send_sample(n, output_id, ev->meta.type_info, params, params_len, s);
}

// DORA_GPU_FANOUT=rccl, at init: ask the daemon for a broadcast group per output and, when it
// admits one (receivers each on their own GPU, none on ours), form the communicator as rank 0.
// Outputs without a group keep the pull path.  Every wait is bounded.
void form_bcast_groups(dora_node* n) {
  NodeCore* c = n->core.get();
  DeviceScope ds(c->device);  // the groups' streams and communicators belong to the node's GPU
  std::string why;
  if (!bcast_available(&why)) {
    c->bcast_error = why;
    return;
  }
  for (const std::string& o : n->outputs) {
    uint8_t uid[kBcastIdBytes];
    if (bcast_unique_id(uid) != DORA_OK) {
      c->bcast_error = dora_gpu_last_error();
      return;
    }
    WBuf w;
    w.str(o);
    w.raw(uid, sizeof(uid));
    if (c->request(REQ_BCAST_GROUP, w.data(), w.size()) != DORA_OK) return;
    uint32_t nranks = 0;
    bool answered = false;
    const uint64_t t0 = mono_ns();
    while (!answered && mono_ns() - t0 < 10000000000ull) {
      uint32_t kind;
      std::vector<uint8_t> p;
      if (!c->drops.try_pop(&kind, &p)) {
        c->drops.wait(10000);
        continue;
      }
      RBuf r(p);
      if (kind == DROP_OUTPUT_DROPPED) {
        on_token(n, r.token());
      } else if (kind == DROP_BCAST_GROUP && r.str() == o) {
        nranks = r.u32();
        answered = true;
      }
    }
    if (nranks < 2) {
      c->bcast_error = "output `" + o + "`: the daemon admitted no broadcast group (each receiver "
                       "must run on its own GPU, none on the producer's); receivers pull";
      continue;
    }
    BcastComm* comm = nullptr;
    hipStream_t st = nullptr;
    if (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess) {
      (void)hipGetLastError();
      c->bcast_error = "broadcast stream of output `" + o + "`";
      continue;
    }
    if (bcast_join(uid, static_cast<int>(nranks), 0, 30000, &comm) == DORA_OK) {
      n->bcast_out[o] = {comm, st};
    } else {
      c->bcast_error = dora_gpu_last_error();
      (void)hipStreamDestroy(st);
    }
  }
}

// What a synchronous send of a device source waits for: the pack has read the whole source.
struct SourceWait {
  uint8_t kind = FILL_DONE;  // FILL_FLAG: flag >= epoch; FILL_EVENT: event; FILL_BCAST: stream
  bool read = false;  // FILL_FLAG of a read-signalled pack: its read word >= epoch suffices
  hipStream_t stream = nullptr;  // FILL_BCAST: the output's broadcast stream
  const std::atomic<uint64_t>* flag = nullptr;
  uint64_t epoch = 0;
  hipEvent_t event = nullptr;
};

// The reference copies a source inside send_output (arrow_utils.rs:48, node/mod.rs:206-209), so
// its caller may rewrite the source as soon as the call returns.  A device source is read by the
// pack kernel after the call has queued it; without DORA_SEND_ASYNC the call waits for that pack
// (spin, then yield; bounded) — after the descriptor has left, so receivers are not delayed.
int wait_source_read(dora_node* n, const SourceWait& w) {
  SubSpan sp(SP_SEND_SOURCE_WAIT);
  if (w.kind == FILL_FLAG && w.flag) {
    const uint64_t t0 = mono_ns();
    uint32_t spins = 0;
    const auto* ff = reinterpret_cast<const FillFlag*>(w.flag);
    while (!(w.read && ff->read_epoch.load(std::memory_order_acquire) >= w.epoch) &&
           !fill_reached(w.flag, w.epoch)) {
      if (++spins < 4096) {
        __builtin_ia32_pause();
        continue;
      }
      const uint64_t dt = mono_ns() - t0;
      if (dt > 10000000000ull) return fail(DORA_ERR_TIMEOUT, "pack did not read its source in 10 s");
      if (dt > 200000) std::this_thread::yield();
    }
  } else if (w.kind == FILL_EVENT && w.event) {
    DORA_HIP(hipEventSynchronize(w.event));
  } else if (w.kind == FILL_BCAST && w.stream) {
    DORA_HIP(hipStreamSynchronize(w.stream));
  }
  return DORA_OK;
}

// Host-resident sources up to this size are written into their device slot by the CPU through
// the large BAR (host_bar_fill); larger ones are DMA'd by HIP.  On an MI355X box the BAR path
// delivers 4 KB in 1.9 us and 1 MiB in 30 us (35 GB/s), HIP's copy takes 13-14 us up to 64 KB,
// 52 us at 1 MiB and wins from ~2 MiB (4 MiB: 89 vs 140 us; 40.96 MB: 56 GB/s)
// (profiles/r06_host_path_probe.jsonl).
constexpr uint64_t kBarFillMax = 2ull << 20;

// The reference copies a host source into its shared-memory sample on the CPU inside
// send_output (arrow_utils.rs:48, node/mod.rs:180-215).  A device node does the same into its
// HBM slot: the slot is mapped for the CPU once, the segments are written with streaming stores,
// and one HDP flush + read-back makes them visible before the descriptor leaves, so the sample
// is complete when the call returns (FILL_DONE: no GPU dispatch, no fill flag).  False when the
// slot cannot be mapped (no large BAR, no HSA): the caller takes the HIP copy.
bool host_bar_fill(dora_node* n, dora_sample* s, const std::vector<Segment>& segs) {
  Slot* slot = s->slot;
  if (!slot || slot->host || s->ext_len > kBarFillMax) return false;
  if (!n->core->aql_tried) {
    n->core->aql_tried = true;
    n->core->aql = aql_queue(n->core->device);
  }
  AqlQueue* q = aql_usable(n->core->aql) ? n->core->aql : nullptr;
  if (!q) return false;
  if (!slot->bar_tried) {
    slot->bar_tried = true;
    slot->bar = bar_map(q, slot->ptr) == DORA_OK;
    if (!slot->bar) clear_error();
  }
  if (!slot->bar) return false;
  for (const Segment& g : segs)
    if (g.op != SEG_COPY) return false;
  auto* dst = static_cast<uint8_t*>(slot->ptr);
  const uint8_t* last = nullptr;
  for (const Segment& g : segs) {
    if (!g.len) continue;
    bar_copy(dst + g.dst_off, g.src, g.len);
    last = dst + g.dst_off + g.len - 1;
  }
  bar_publish(q, last);
  s->fill = FILL_DONE;
  ++n->bar_fills;
  return true;
}

int pack_and_send(dora_node* n, const char* output_id, const dora_plan* plan, const uint8_t* params,
                  size_t params_len, const std::vector<uint8_t>* ti_pre = nullptr,
                  uint32_t flags = 0) {
  dora_sample* s = nullptr;
  const uint64_t t0 = mono_ns();
  // a host-resident array below the zero-copy threshold goes inline, as in the reference
  const bool host_src = plan->dev != ARROW_DEVICE_ROCM;
  // a device array for receivers that all lack a GPU: packed into shared memory
  // (host_bound_sample; not inside a timed region, whose stamps live in HBM slots' flags, and
  // not a plan whose validity bitmaps travel in a tail past the sample: a SharedMemory message
  // has no room to name one)
  const bool host_bound = plan->size && plan->fill_size() == plan->size && !n->host_bound.empty() &&
                          !n->region_armed && n->core->device >= 0 &&
                          n->host_bound.count(output_id) && !n->bcast_out.count(output_id);
  if (host_bound && !host_src && plan->size <= kHostPackMax) {
    s = host_bound_sample(n, plan->size, plan->size);
  } else if (host_bound && host_src && plan->size >= kZeroCopyThreshold) {
    // a host source for them: the CPU copies it into shared memory, as a node without a GPU
    // does (the reference's copy_array_into_sample) — no HBM slot for each receiver to copy out
    handle_finished_drop_tokens(n);
    Slot* slot = nullptr;
    if (allocate_host_slot(n, plan->size, &slot) == DORA_OK) {
      s = new dora_sample();
      s->len = plan->size;
      s->slot = slot;
      ++n->host_copies;
    } else {
      clear_error();
    }
  }
  int rc = s ? DORA_OK : alloc_sample(n, plan->size, &s, plan->fill_size(), host_src);
  if (rc != DORA_OK) return rc;
  const uint64_t t1 = mono_ns();
  uint64_t t2 = t1, t3 = t1;
  if (plan->size && (!s->slot || (s->slot->host && (host_src || !s->slot->registered)))) {
    // an inline Vec or a host-only node's shared-memory slot: the host copies the buffers
    // (copy_array_into_sample, arrow_utils.rs:48)
    if (!host_src) {
      discard_sample(n, s);
      return fail(DORA_ERR_INVALID, "host-only node cannot send device-resident data");
    }
    uint8_t* dst = s->slot ? static_cast<uint8_t*>(s->slot->ptr) : s->vec.data();
    for (const Segment& g : plan->segs) std::memcpy(dst + g.dst_off, g.src, g.len);
    t2 = t3 = mono_ns();
  } else if (plan->size && host_src && plan->dev == ARROW_DEVICE_CPU &&
             host_bar_fill(n, s, plan->segs)) {
    t2 = t3 = mono_ns();
  } else if (plan->size) {
    // Kernel stamps cost host time and a timestamp packet on each side of the dispatch, so only
    // every n-th pack is stamped (dora_node_set_timing_period, default kTimingPeriod).
    const uint64_t period = n->timing_period ? n->timing_period : kTimingPeriod;
    const bool timed = n->profile && plan->dev != ARROW_DEVICE_CPU &&
                       (n->timing_seq++ % period) == 0;
    TimingPair* tp = timed ? next_timing_pair(n, plan->size) : nullptr;
    hipEvent_t t_start = tp ? tp->start : nullptr, t_stop = tp ? tp->stop : nullptr;
    // Timed region: packs that signal their own fill stamp their device time into the flag
    // line; only packs that cannot (kernel signal off, transforms) need timing events
    const bool stampable = n->core->fill_done && !plan->compact;
    if (n->region_armed && plan->dev != ARROW_DEVICE_CPU) {
      if (!stampable && !n->region_started && !tp) {  // its start is the fallback's origin
        t_start = n->region_start;
        n->region_started = true;
      }
      ++n->region_packs;
      n->region_bytes += plan->size;
    }
    // a broadcast-group output packs on its own stream, where its broadcast follows
    auto bo = n->bcast_out.find(output_id);
    const bool bcast = bo != n->bcast_out.end();
    if (bcast) n->core->order_after_node_stream(bo->second.stream);
    const bool sync = plan->dev == ARROW_DEVICE_ROCM &&
                      !((flags & DORA_SEND_ASYNC) || n->async_default);
    rc = fill_sample(n, s, plan->segs.data(), plan->segs.size(), plan->dev,
                     bcast ? bo->second.stream : nullptr, t_start, t_stop, !bcast, sync);
    if (rc != DORA_OK) {
      if (tp) tp->pending = false;
      add_to_cache(n, s->slot);
      delete s;
      return rc;
    }
    if (n->region_armed && plan->dev != ARROW_DEVICE_CPU) {
      if (s->stamped) s->slot->region_epoch = s->epoch;
      else ++n->region_unstamped;
    }
    if (s->slot->host) {
      // packed into shared memory: its receivers read it on the host when it arrives (the
      // reference's SharedMemory sample is complete when sent), so the pack completes first
      SourceWait w;
      w.kind = s->fill;
      w.epoch = s->epoch;
      if (s->fill == FILL_FLAG) w.flag = n->core->flag_host(s->slot->flag);
      rc = wait_source_read(n, w);
      if (rc != DORA_OK) {
        delete s;  // a pack that may still write the region: its slot is not reused
        return rc;
      }
      s->fill = FILL_DONE;
      ++n->host_packs;
    }
    t2 = t3 = mono_ns();
  }
  SubSpan sp_ti(SP_SEND_TI);
  if (!ti_pre) {
    n->ti_buf.clear();
    serialize_type_info(plan->root, n->ti_buf);
  }
  const std::vector<uint8_t>& ti = ti_pre ? *ti_pre : n->ti_buf;
  sp_ti.stop();
  DropToken tok{};
  const bool traced = trace_enabled() && s->slot;
  SourceWait wait;
  const bool sync_src = plan->dev == ARROW_DEVICE_ROCM && s->slot && plan->size &&
                        !((flags & DORA_SEND_ASYNC) || n->async_default);
  if (sync_src) {
    auto bo = n->bcast_out.find(output_id);
    wait.kind = bo != n->bcast_out.end() ? uint8_t(FILL_BCAST) : s->fill;
    if (bo != n->bcast_out.end()) wait.stream = bo->second.stream;
    wait.epoch = s->epoch;
    wait.read = s->read_signalled;
    if (s->fill == FILL_FLAG) wait.flag = n->core->flag_host(s->slot->flag);
    if (s->fill == FILL_EVENT) wait.event = s->slot->done;
  }
  rc = send_sample(n, output_id, ti, params, params_len, s, &tok);
  if (rc == DORA_OK && sync_src) rc = wait_source_read(n, wait);
  const uint64_t t4 = mono_ns();
  if (traced && rc == DORA_OK) {
    const uint64_t off = now_ns() - mono_ns();  // mono -> realtime for the trace
    trace_at(TP_ALLOC_BEGIN, tok, t0 + off);
    trace_at(TP_ALLOC_END, tok, t1 + off);
    trace_at(TP_LAUNCHED, tok, t2 + off);
    trace_at(TP_FILL_ORDERED, tok, t3 + off);
  }
  n->phase_ns[0] += t1 - t0;
  n->phase_ns[1] += t2 - t1;
  n->phase_ns[2] += t3 - t2;
  n->phase_ns[3] += t4 - t3;
  ++n->phase_count;
  return rc;
}

}  // namespace

// An inline Vec sample holding `len` host bytes: a remote node's small message, delivered as the
// reference's receiving daemon delivers remote data (`data.map(DataMessage::Vec)`,
// binaries/daemon/src/lib.rs:567), with no slot and no upload.
dora_sample* vec_sample(const uint8_t* p, size_t len) {
  auto* s = new dora_sample();
  s->len = len;
  s->vec.assign(p, p + len);
  return s;
}

// A remote node's message re-sent by its proxy (interdaemon.cpp): the metadata keeps the
// producer's timestamp.
int proxy_send(dora_node* n, const char* output_id, const uint8_t* ti, size_t ti_len,
               const uint8_t* params, size_t params_len, dora_sample* sample, uint64_t ts) {
  DORA_GUARD_BEGIN
  n->samples_live.erase(sample);  // consumed here (an allocate_data_sample sample or inline)
  std::vector<uint8_t> t(ti, ti + ti_len);
  return send_sample(n, output_id, t, params, params_len, sample, nullptr, ts);
  DORA_GUARD_END
}

}  // namespace dora

extern "C" {

int dora_node_init(const char* shm_name, const char* node_id, int device, dora_node** out) {
  if (!shm_name || !node_id || !out) return dora::fail(DORA_ERR_INVALID, "NULL argument");
  *out = nullptr;
  DORA_GUARD_BEGIN
  auto core = std::make_shared<dora::NodeCore>();
  try {
    core->region.reset(dora::Region::attach(shm_name));
  } catch (const std::exception& e) {
    return dora::fail(DORA_ERR_INVALID, "attach dataflow: %s", e.what());
  }
  core->idx = core->region->node_index(node_id);
  if (core->idx < 0)
    return dora::fail(DORA_ERR_NOT_FOUND, "node `%s` is not part of the dataflow", node_id);
  dora::NodeEntry& e = core->region->hdr()->nodes[core->idx];
  int32_t expected = 0;
  if (!e.pid.compare_exchange_strong(expected, static_cast<int32_t>(getpid())))
    return dora::fail(DORA_ERR_INVALID, "node `%s` is already running (pid %d)", node_id,
                      expected);
  core->req = dora::RingWriter(core->region.get(), &e.requests);
  core->ev = dora::RingReader(core->region.get(), &e.events);
  core->drops = dora::RingReader(core->region.get(), &e.drops);
  core->device = device;
  e.device.store(device < 0 ? -1 : device);
  dora::trace_set_name(node_id);
  if (device >= 0) {  // device < 0: host-only node (control plane + inline Vec samples only)
    DORA_HIP(hipSetDevice(device));
    // NUMA placement: the send/receive path writes the GPU's BAR (AQL arguments, doorbells)
    // and polls host memory the GPU writes (fill flags); keep this thread next to its GPU and
    // tell the daemon where that is (DORA_GPU_PIN=0: leave the affinity alone)
    if (dora::numa_pinning()) {
      const int numa = dora::gpu_numa_node(device);
      if (numa >= 0) {
        dora::RegionHdr* rh = core->region->hdr();
        (void)dora::pin_to_numa(numa, device, &rh->l3_cpu, int(rh->n_nodes) + 1);
        int32_t none = -1;
        core->region->hdr()->numa_hint.compare_exchange_strong(none, numa);
      }
    }
    DORA_HIP(hipStreamCreateWithFlags(&core->stream, hipStreamNonBlocking));
    // Fill streams are created on first use: device-source packs go to the AQL queues, so only
    // host sources, compacting transforms and node-stream-ordered fills need them, and a node
    // that never sends such a pack holds one HIP hardware queue, not four.
    {
      // host-register the control region so this node's stream can write fill epochs into it
      void* dev = nullptr;
      if (hipHostRegister(core->region->base(), core->region->size(), hipHostRegisterMapped) ==
              hipSuccess &&
          hipHostGetDevicePointer(&dev, core->region->base(), 0) == hipSuccess) {
        core->region_dev = static_cast<uint8_t*>(dev);
        for (uint32_t k = dora::kFillFlags; k-- > 0;) core->free_flags.push_back(k);
        const size_t cb = size_t(dora::kFillFlags) * dora::kMaxSignalWgs * sizeof(uint32_t);
        if (hipMalloc(&core->fill_done, cb) != hipSuccess ||
            hipMemset(core->fill_done, 0, cb) != hipSuccess ||
            hipDeviceSynchronize() != hipSuccess) {
          (void)hipGetLastError();  // the stream write-value packet signals instead
          if (core->fill_done) (void)hipFree(core->fill_done);
          core->fill_done = nullptr;
        }
      } else {
        (void)hipGetLastError();  // fall back to interprocess events
      }
    }
  }

  auto* n = new dora_node();
  n->pin_pending = device < 0 && dora::numa_pinning();
  if (const char* e = std::getenv("DORA_GPU_SEND_ASYNC")) n->async_default = *e == '1';
  n->core = core;
  n->id = node_id;
  for (auto& o : dora::split(e.outputs, ',')) n->outputs.insert(o);
  for (auto& kv : dora::split(e.inputs, ',')) {
    auto eq = kv.find('=');
    n->queue_size[kv.substr(0, eq)] = static_cast<uint32_t>(std::stoul(kv.substr(eq + 1)));
  }
  n->min_queue_size = SIZE_MAX;
  for (auto& kv : n->queue_size) n->min_queue_size = std::min<size_t>(n->min_queue_size, kv.second);
  // Subscribe and wait for AllNodesReady (event_stream/mod.rs:37-118, daemon PendingNodes)
  int rc = core->request(dora::REQ_SUBSCRIBE, {});
  if (rc != DORA_OK) {
    delete n;
    return rc;
  }
  const uint64_t t0 = dora::mono_ns();
  for (;;) {
    uint32_t kind;
    std::vector<uint8_t> p;
    if (core->ev.try_pop(&kind, &p)) {
      if (kind == dora::EV_READY) {
        // the outputs whose receivers all lack a GPU (daemon.cpp ready_payload); kept on a
        // host-only node too, for dora_node_host_bound_outputs, though only a device node packs
        if (p.size() >= 4) {
          dora::RBuf r(p);
          for (uint32_t k = r.u32(); k > 0; --k) n->host_bound.insert(r.str());
        }
        break;
      }
      dora::encode_event(n, kind, p);
      continue;
    }
    if (dora::mono_ns() - t0 > 60000000000ull) {
      delete n;
      return dora::fail(DORA_ERR_TIMEOUT, "no AllNodesReady from the daemon within 60 s");
    }
    core->ev.wait(100000);
  }
  if (device >= 0 && dora::fanout_rccl() && !n->outputs.empty()) dora::form_bcast_groups(n);
  if (n->want_pump) dora::start_pump(n);  // a broadcast group joined during init
  // send_stdout_as (spawn.rs:280-437): the descriptor names one of this node's outputs
  if (const char* so = std::getenv("DORA_GPU_SEND_STDOUT_AS")) {
    if (!n->outputs.count(so)) {
      delete n;
      return dora::fail(DORA_ERR_NOT_FOUND, "send_stdout_as names `%s`, not an output of `%s`",
                        so, node_id);
    }
    std::weak_ptr<dora::NodeCore> wc = core;
    n->stdout_capture = dora::stdout_capture_start(
        so, [wc](uint32_t kind, const std::vector<uint8_t>& p) {
          auto c = wc.lock();
          return c ? c->request(kind, p) : DORA_ERR_CLOSED;
        });
  }
  *out = n;
  return DORA_OK;
  DORA_GUARD_END
}

int dora_node_init_from_env(dora_node** out) {
  const char* shm = std::getenv("DORA_GPU_DATAFLOW");
  const char* id = std::getenv("DORA_NODE_ID");
  const char* dev = std::getenv("DORA_GPU_DEVICE");
  if (!shm || !id)
    return dora::fail(DORA_ERR_INVALID,
                      "env variables DORA_GPU_DATAFLOW and DORA_NODE_ID must be set. Are you sure "
                      "the node was started by the dataflow launcher?");
  return dora_node_init(shm, id, dev ? std::atoi(dev) : 0, out);
}

void dora_node_free(dora_node* n) {  // Drop for DoraNode (mod.rs:384-431)
  if (!n) return;
  struct Flush {
    ~Flush() { dora::trace_flush(); }
  } flush_trace_at_end;
  dora::stdout_capture_stop(n->stdout_capture);  // the last lines go out before the outputs close
  n->stdout_capture = nullptr;
  dora::stop_pump(n);  // the event-stream thread first: the queue is this thread's again
  std::vector<std::string> outs(n->outputs.begin(), n->outputs.end());
  dora::WBuf w;
  w.u32(static_cast<uint32_t>(outs.size()));
  for (auto& o : outs) w.str(o);
  (void)n->core->request(dora::REQ_CLOSE_OUTPUTS, w.data(), w.size());
  n->queue.clear();  // releases undelivered inputs (tokens reported)
  uint64_t t0 = dora::mono_ns();
  while (!n->sent_out.empty() || !n->forwarded.empty()) {
    dora::handle_finished_drop_tokens(n);
    if (n->sent_out.empty() && n->forwarded.empty()) break;
    if (dora::mono_ns() - t0 > dora::kDropWaitNs) break;  // "timeout while waiting for drop tokens"
    n->core->drops.wait(10000);
    if (n->core->region->hdr()->nodes[n->core->idx].state.load() == 2) break;
  }
  n->forwarded.clear();  // inputs still held by unanswered forwards: their tokens go back
  (void)n->core->request(dora::REQ_OUTPUTS_DONE, {});
  // broadcasts read the slots: the groups go (after their streams drain, bounded) first
  for (auto& kv : n->bcast_out) {
    dora::bcast_close(kv.second.comm, kv.second.stream, 10000);
    (void)hipStreamDestroy(kv.second.stream);
  }
  n->bcast_out.clear();
  for (dora_sample* s : n->samples_live) dora::discard_sample(n, s);  // allocated, never sent
  n->samples_live.clear();
  for (auto& kv : n->sent_out) dora::free_slot(n, kv.second);
  for (auto* s : n->cache) dora::free_slot(n, s);
  dora::SlotReaper::reaper().drain();  // evicted slots: freed before the node's state goes
  for (auto& e : n->plan_cache) delete e.plan;
  n->plan_cache.clear();
  n->plan_index.clear();
  dora::harvest_all(n);
  for (auto& p : n->timing) {
    (void)hipEventDestroy(p.start);
    (void)hipEventDestroy(p.stop);
  }
  if (n->timing_ref) (void)hipEventDestroy(n->timing_ref);
  if (n->region_start) (void)hipEventDestroy(n->region_start);
  for (hipEvent_t e : n->region_stop) (void)hipEventDestroy(e);
  if (n->region_cp_stamps) {
    dora::aql_fence_all();  // no pack of this node may still write its stamps
    dora::bar_free(n->region_cp_stamps);
  }
  if (n->region_reduce_idx) (void)hipHostFree(n->region_reduce_idx);
  if (n->region_reduce_out) (void)hipHostFree(n->region_reduce_out);
  delete n;
}

int dora_node_sync(dora_node* n) {
  if (!n) return dora::fail(DORA_ERR_INVALID, "NULL node");
  if (n->core->device < 0) return DORA_OK;
  dora::DeviceScope ds(n->core->device);
  dora::NodeCore* c = n->core.get();
  // Kernel-signalled fills (AQL and fill streams): their flags.  A stream query or synchronise
  // would wait for HIP to notice the kernels' completion, ~100-200 us after the flags are up.
  const uint64_t t0 = dora::mono_ns();
  for (auto* v : {&c->aql_pending, &c->flag_pending}) {
    for (auto& x : *v)
      while (!dora::fill_reached(x.first, x.second)) {
        if (dora::mono_ns() - t0 > 10000000000ull)
          return dora::fail(DORA_ERR_TIMEOUT, "a fill did not complete within 10 s");
        __builtin_ia32_pause();
      }
    v->clear();
  }
  // work no flag covers: fills signalled by the stream (kernel signal off, transforms, host
  // sources) and whatever the caller queued on the node stream
  for (size_t i = 0; i < c->fill_streams.size(); ++i) {
    if (!c->fill_unsignalled[i]) continue;
    DORA_HIP(hipStreamSynchronize(c->fill_streams[i]));
    c->fill_unsignalled[i] = 0;
  }
  if (hipStreamQuery(c->stream) == hipErrorNotReady) DORA_HIP(hipStreamSynchronize(c->stream));
  (void)hipGetLastError();
  return DORA_OK;
}

dora_stream_t dora_node_stream(dora_node* n) {
  if (!n) return nullptr;
  n->core->stream_used.store(true, std::memory_order_relaxed);
  n->core->fence_fills();  // work the caller queues next runs after every fill so far
  return n->core->stream;
}

int dora_node_allocate_data_sample(dora_node* n, size_t len, dora_sample** out) {
  if (!n || !out) return dora::fail(DORA_ERR_INVALID, "NULL argument");
  DORA_GUARD_BEGIN
  const int rc = dora::alloc_sample(n, len, out);
  if (rc == DORA_OK) n->samples_live.insert(*out);
  return rc;
  DORA_GUARD_END
}

void* dora_sample_data(dora_sample* s) {
  if (!s) return nullptr;
  return s->slot ? s->slot->ptr : s->vec.data();
}

size_t dora_sample_len(const dora_sample* s) { return s ? s->len : 0; }

void dora_sample_discard(dora_node* n, dora_sample* s) {
  if (!s || !n) return;
  // only a sample this node handed out and nobody consumed yet (a second discard, or a discard
  // after the send, would free it twice)
  if (!n->samples_live.erase(s)) {
    dora::fail(DORA_ERR_INVALID, "sample was already sent or discarded");
    return;
  }
  dora::discard_sample(n, s);
}

int dora_node_send_output_sample(dora_node* n, const char* output_id, const uint8_t* type_info,
                                 size_t type_info_len, const uint8_t* params, size_t params_len,
                                 dora_sample* sample) {
  if (!n || !output_id || (!type_info && type_info_len))
    return dora::fail(DORA_ERR_INVALID, "NULL argument");
  // the reference's DataSample is moved into send_output_sample (mod.rs:246-275): a C caller
  // may hold on to the pointer, so a sample that was already sent or discarded is refused
  if (sample && !n->samples_live.erase(sample))
    return dora::fail(DORA_ERR_INVALID,
                      "sample was already sent or discarded (or belongs to another node)");
  DORA_GUARD_BEGIN
  if (sample && sample->slot && !sample->slot->host && sample->len &&
      n->core->stream_used.load(std::memory_order_relaxed)) {
    // a sample written by kernels on the node stream (dora_node_stream): receivers wait for
    // that work through the slot's fill flag, the sender does not (no host synchronisation)
    dora::DeviceScope ds(n->core->device);
    const hipError_t e = dora::order_fill(n, sample, n->core->stream);
    if (e != hipSuccess) {
      (void)hipGetLastError();
      dora::discard_sample(n, sample);
      return dora::fail(DORA_ERR_HIP, "ordering the sample after the node stream: %s",
                        hipGetErrorString(e));
    }
  }
  std::vector<uint8_t> ti(type_info, type_info + type_info_len);
  return dora::send_sample(n, output_id, ti, params, params_len, sample);
  DORA_GUARD_END
}

int dora_node_send_output(dora_node* n, const char* output_id, const struct ArrowArray* array,
                          const struct ArrowSchema* schema, ArrowDeviceType device_type,
                          const uint8_t* params, size_t params_len) {
  return dora_node_send_output_ex(n, output_id, array, schema, device_type, params, params_len, 0);
}

int dora_node_send_output_ex(dora_node* n, const char* output_id, const struct ArrowArray* array,
                             const struct ArrowSchema* schema, ArrowDeviceType device_type,
                             const uint8_t* params, size_t params_len, uint32_t flags) {
  if (!n || !output_id) return dora::fail(DORA_ERR_INVALID, "NULL argument");
  DORA_GUARD_BEGIN
  const bool device = device_type == ARROW_DEVICE_ROCM && n->core->device >= 0;
  const bool cacheable = device && !n->compact && array && schema;
  uint64_t h = 0;
  bool keyed = false;
  if (cacheable && dora::plan_key(array, schema, n->plan_key_buf)) {
    keyed = true;
    h = 0xcbf29ce484222325ull;
    for (uint64_t w : n->plan_key_buf) h = (h ^ w) * 0x100000001b3ull;
    auto it = n->plan_index.find(h);
    if (it != n->plan_index.end()) {
      auto& e = n->plan_cache[it->second];
      if (e.key == n->plan_key_buf) {
        e.last_use = ++n->plan_clock;
        ++n->plan_hits;
        return dora::pack_and_send(n, output_id, e.plan, params, params_len, &e.ti, flags);
      }
      keyed = false;  // a hash collision: plan this one afresh, uncached
    }
  }
  dora_plan* plan = nullptr;
  int rc = (n->compact && device_type == ARROW_DEVICE_ROCM)
               ? dora::build_plan_compact(array, schema, device_type, &plan)
               : dora::build_plan(array, schema, device_type, &plan,
                                  device);
  if (rc != DORA_OK) return rc;
  if (keyed && !plan->read_device) {
    // keep it: a later send of the same buffers reuses plan and type info.  64 entries cover a
    // sender rotating over a few dozen preallocated arrays (C3 bench: 24)
    constexpr size_t kPlanCache = 64;
    size_t slot = n->plan_cache.size();
    if (slot >= kPlanCache) {
      slot = 0;
      for (size_t k = 1; k < n->plan_cache.size(); ++k)
        if (n->plan_cache[k].last_use < n->plan_cache[slot].last_use) slot = k;
      auto& old = n->plan_cache[slot];
      uint64_t oh = 0xcbf29ce484222325ull;
      for (uint64_t w : old.key) oh = (oh ^ w) * 0x100000001b3ull;
      n->plan_index.erase(oh);
      delete old.plan;
      old = dora_node::CachedPlan();
    } else {
      n->plan_cache.emplace_back();
    }
    auto& e = n->plan_cache[slot];
    e.key = n->plan_key_buf;
    e.plan = plan;
    dora::serialize_type_info(plan->root, e.ti);
    e.last_use = ++n->plan_clock;
    n->plan_index[h] = slot;
    return dora::pack_and_send(n, output_id, e.plan, params, params_len, &e.ti, flags);
  }
  rc = dora::pack_and_send(n, output_id, plan, params, params_len, nullptr, flags);
  delete plan;
  return rc;
  DORA_GUARD_END
}

int dora_node_send_output_bytes_ex(dora_node* n, const char* output_id, const void* data,
                                   size_t len, ArrowDeviceType device_type, const uint8_t* params,
                                   size_t params_len, uint32_t flags) {
  if (!n || !output_id || (!data && len)) return dora::fail(DORA_ERR_INVALID, "NULL argument");
  DORA_GUARD_BEGIN
  dora::SubSpan sp(dora::SP_SEND_PLAN);
  // one UInt8 buffer: the plan and its type info are built once per node and re-pointed per send
  dora_plan& plan = n->bytes_plan;
  if (n->bytes_ti.empty()) {
    ArrowSchema u8{};
    u8.format = "C";
    dora::serialize_schema(&u8, true, plan.root.schema);
    plan.root.bufs.assign(1, {0, 0});
  }
  plan.dev = device_type;
  plan.size = len;
  plan.root.len = len;
  plan.root.bufs[0] = {0, len};
  plan.segs.clear();
  if (len) plan.segs.push_back({data, 0, len});
  // the type info depends on len only through the buffer length: re-serialize when it changes
  if (n->bytes_ti.empty() || n->bytes_ti_len != len) {
    n->bytes_ti.clear();
    dora::serialize_type_info(plan.root, n->bytes_ti);
    n->bytes_ti_len = len;
  }
  sp.stop();
  return dora::pack_and_send(n, output_id, &plan, params, params_len, &n->bytes_ti, flags);
  DORA_GUARD_END
}

int dora_node_send_output_bytes(dora_node* n, const char* output_id, const void* data, size_t len,
                                ArrowDeviceType device_type, const uint8_t* params,
                                size_t params_len) {
  return dora_node_send_output_bytes_ex(n, output_id, data, len, device_type, params, params_len,
                                        0);
}

int dora_node_set_async_sends(dora_node* n, int enable) {
  if (!n) return dora::fail(DORA_ERR_INVALID, "NULL node");
  n->async_default = enable != 0;
  return DORA_OK;
}

int dora_node_set_event_thread(dora_node* n, int enable) {
  if (!n) return dora::fail(DORA_ERR_INVALID, "NULL node");
  DORA_GUARD_BEGIN
  if (enable) dora::start_pump(n);
  else dora::stop_pump(n);
  return DORA_OK;
  DORA_GUARD_END
}

int dora_node_set_compact(dora_node* n, int enable) {
  if (!n) return dora::fail(DORA_ERR_INVALID, "NULL node");
  n->compact = enable != 0;
  return DORA_OK;
}

int dora_node_close_outputs(dora_node* n, const char* const* ids, size_t count) {
  if (!n || (!ids && count)) return dora::fail(DORA_ERR_INVALID, "NULL argument");
  DORA_GUARD_BEGIN
  for (size_t i = 0; i < count; ++i)
    if (!n->outputs.count(ids[i])) return dora::fail(DORA_ERR_NOT_FOUND, "unknown output %s", ids[i]);
  dora::WBuf w;
  w.u32(static_cast<uint32_t>(count));
  for (size_t i = 0; i < count; ++i) {
    n->outputs.erase(ids[i]);
    w.str(ids[i]);
  }
  return n->core->request(dora::REQ_CLOSE_OUTPUTS, w.data(), w.size());
  DORA_GUARD_END
}

int dora_node_next_event(dora_node* n, int64_t timeout_us, dora_event** out) {
  if (!n || !out) return dora::fail(DORA_ERR_INVALID, "NULL argument");
  *out = nullptr;
  DORA_GUARD_BEGIN
  if (n->pin_pending) dora::pin_host_node(n);
  const uint64_t t0 = dora::mono_ns();
  if (n->want_pump && !n->pump_on.load()) dora::start_pump(n);
  if (n->pump_on.load()) {
    // the event-stream thread fills the queue: take its oldest event
    std::unique_lock<std::mutex> g(n->qmu);
    for (;;) {
      if (!n->queue.empty()) {
        *out = n->queue.front().release();
        n->queue.pop_front();
        if ((*out)->type == DORA_EVENT_ALL_INPUTS_CLOSED) n->ended = true;
        g.unlock();
        dora::finish_input(n, *out);
        return DORA_OK;
      }
      if (n->ended) return dora::fail(DORA_ERR_CLOSED, "event stream closed");
      if (timeout_us < 0) {
        n->qcv.wait_for(g, std::chrono::milliseconds(100));
        continue;
      }
      const int64_t left = timeout_us - int64_t(dora::mono_ns() - t0) / 1000;
      if (left <= 0) return dora::fail(DORA_ERR_TIMEOUT, "no event within timeout");
      n->qcv.wait_for(g, std::chrono::microseconds(left));
    }
  }
  for (;;) {
    const bool got = dora::drain_events(n);
    if (n->want_pump && !n->pump_on.load()) {
      // a broadcast group was joined while draining: the thread takes over from here
      dora::start_pump(n);
      return dora_node_next_event(n, timeout_us < 0 ? -1
                                     : std::max<int64_t>(0, timeout_us - int64_t(dora::mono_ns() - t0) / 1000), out);
    }
    if (!n->queue.empty()) {
      // The event handed over now is the node's, like the one the reference's event-stream
      // thread holds (event_stream/thread.rs:139-157: taken from the daemon's queue, in its
      // channel): the drop-oldest policy keeps queue_size inputs per input id among the rest.
      // So a sender with queue_size + 1 samples in flight (node.cpp max_in_flight) never makes
      // a default receiver drop, whenever that receiver pauses.
      *out = n->queue.front().release();
      n->queue.pop_front();
      if ((*out)->type == DORA_EVENT_ALL_INPUTS_CLOSED) n->ended = true;
      if (got) dora::drop_oldest_inputs(n);
      dora::finish_input(n, *out);
      return DORA_OK;
    }
    if (n->ended) return dora::fail(DORA_ERR_CLOSED, "event stream closed");
    int64_t left = -1;
    if (timeout_us >= 0) {
      left = timeout_us - int64_t(dora::mono_ns() - t0) / 1000;
      if (left <= 0) return dora::fail(DORA_ERR_TIMEOUT, "no event within timeout");
    }
    n->core->ev.wait(left < 0 ? 1000000 : left);
  }
  DORA_GUARD_END
}

int dora_event_type(const dora_event* e) { return e ? e->type : DORA_EVENT_ERROR; }

const char* dora_event_id(const dora_event* e) { return e ? e->id.c_str() : ""; }

const char* dora_event_error(const dora_event* e) { return e ? e->error.c_str() : ""; }

int dora_event_data(const dora_event* e, const void** ptr, size_t* len) {
  if (!e || !ptr || !len) return dora::fail(DORA_ERR_INVALID, "NULL argument");
  if (!e->data) return dora::fail(DORA_ERR_INVALID, "event has no data");
  DORA_GUARD_BEGIN
  int rc = dora::ensure_local(e->data.get());
  if (rc != DORA_OK) return rc;
  DORA_GUARD_END
  *ptr = e->data->ptr;
  *len = e->data->len;
  return DORA_OK;
}

int dora_event_is_device(const dora_event* e) {
  return e && e->data && (e->data->has_token || e->data->local) && !e->data->host_mem;
}

int dora_event_type_info(const dora_event* e, const uint8_t** ti, size_t* len) {
  if (!e || !ti || !len) return dora::fail(DORA_ERR_INVALID, "NULL argument");
  if (!e->ti_checked && e->type == DORA_EVENT_INPUT && e->data && e->data->ext_len > e->data->len) {
    // bitmaps in the sample's tail: restore the reference's inline ArrowTypeInfo bytes
    DORA_GUARD_BEGIN
    int rc = dora::ensure_local(e->data.get());
    if (rc != DORA_OK) return rc;
    bool changed = false;
    rc = dora::inline_type_info(e->meta.type_info.data(), e->meta.type_info.size(),
                                e->data->ptr, e->data->ext_len, &e->ti_inline, &changed,
                                e->data->host_mem);
    if (rc != DORA_OK) return rc;
    DORA_GUARD_END
  }
  e->ti_checked = true;
  const std::vector<uint8_t>& t = e->ti_inline.empty() ? e->meta.type_info : e->ti_inline;
  *ti = t.data();
  *len = t.size();
  return DORA_OK;
}

int dora_event_parameters(const dora_event* e, const uint8_t** p, size_t* len) {
  if (!e || !p || !len) return dora::fail(DORA_ERR_INVALID, "NULL argument");
  *p = e->meta.parameters.data();
  *len = e->meta.parameters.size();
  return DORA_OK;
}

uint64_t dora_event_timestamp_ns(const dora_event* e) { return e ? e->meta.timestamp_ns : 0; }

int dora_event_array(const dora_event* e, struct ArrowArray* out_array,
                     struct ArrowSchema* out_schema) {
  if (!e || !out_array || !out_schema) return dora::fail(DORA_ERR_INVALID, "NULL argument");
  if (e->type != DORA_EVENT_INPUT || !e->data)
    return dora::fail(DORA_ERR_INVALID, "not an input event");
  if (!e->data->ptr && e->data->len)
    return dora::fail(DORA_ERR_INVALID, "input data is not mapped: %s", e->error.c_str());
  DORA_GUARD_BEGIN
  int rc = dora::ensure_local(e->data.get());
  if (rc != DORA_OK) return rc;
  DORA_GUARD_END
  std::shared_ptr<void> keep = e->data;
  // an inline Vec sample, shared memory read in place or a device sample staged to host memory:
  // a host array over its bytes (a staged sample keeps its validity tail)
  if (e->data->host_mem || (!e->data->has_token && !e->data->local))
    return dora::import_sample(e->data->ptr, e->data->len, e->meta.type_info.data(),
                               e->meta.type_info.size(), keep, out_array, out_schema,
                               e->data->ext_len, true);
  return dora::import_sample(e->data->ptr, e->data->len, e->meta.type_info.data(),
                             e->meta.type_info.size(), keep, out_array, out_schema,
                             e->data->ext_len);
}

void dora_event_free(dora_event* e) { delete e; }

int dora_node_forward(dora_node* n, const char* output_id, const dora_event* ev,
                      const uint8_t* params, size_t params_len) {
  if (!n || !output_id || !ev) return dora::fail(DORA_ERR_INVALID, "NULL argument");
  if (ev->type != DORA_EVENT_INPUT || !ev->data)
    return dora::fail(DORA_ERR_INVALID, "only input events can be forwarded");
  if (!ev->data->ptr && ev->data->len)
    return dora::fail(DORA_ERR_INVALID, "input data is not mapped: %s", ev->error.c_str());
  dora::DeviceScope ds(n->core->device);
  DORA_GUARD_BEGIN
  return dora::forward_input(n, output_id, ev, params, params_len);
  DORA_GUARD_END
}

const char* dora_node_dataflow_id(const dora_node* n) {
  return n ? n->core->region->hdr()->dataflow_id : "";
}

const char* dora_node_id(const dora_node* n) { return n ? n->id.c_str() : ""; }

int dora_node_stats(dora_node* n, uint64_t* slots_created, uint64_t* cache_hits,
                    uint64_t* in_flight, uint64_t* dropped_inputs) {
  if (!n) return dora::fail(DORA_ERR_INVALID, "NULL node");
  if (slots_created) *slots_created = n->slots_created;
  if (cache_hits) *cache_hits = n->cache_hits;
  if (in_flight) *in_flight = n->sent_out.size();
  if (dropped_inputs) *dropped_inputs = n->dropped_inputs;
  return DORA_OK;
}

int dora_node_pack_stats(dora_node* n, uint64_t* count, double* total_ms, uint64_t* bytes) {
  if (!n) return dora::fail(DORA_ERR_INVALID, "NULL node");
  dora::harvest_all(n);  // waits for the stamps of packs still in flight
  if (count) *count = n->pack_count;
  if (total_ms) *total_ms = n->pack_ms;
  if (bytes) *bytes = n->pack_bytes;
  return DORA_OK;
}

int dora_node_dataflow_counters(dora_node* n, const char* node_id, uint64_t* slots_created,
                                uint64_t* ipc_opens, uint64_t* dropped_inputs) {
  if (!n || !node_id) return dora::fail(DORA_ERR_INVALID, "NULL argument");
  const int i = n->core->region->node_index(node_id);
  if (i < 0) return dora::fail(DORA_ERR_NOT_FOUND, "node `%s` is not part of the dataflow", node_id);
  const dora::NodeEntry& e = n->core->region->hdr()->nodes[i];
  if (slots_created) *slots_created = e.slots_created.load(std::memory_order_relaxed);
  if (ipc_opens) *ipc_opens = e.ipc_opens.load(std::memory_order_relaxed);
  if (dropped_inputs) *dropped_inputs = e.dropped_inputs.load(std::memory_order_relaxed);
  return DORA_OK;
}

int dora_node_plan_cache_stats(dora_node* n, uint64_t* hits, uint64_t* entries) {
  if (!n) return dora::fail(DORA_ERR_INVALID, "NULL node");
  if (hits) *hits = n->plan_hits;
  if (entries) *entries = n->plan_cache.size();
  return DORA_OK;
}

int dora_node_fill_paths(dora_node* n, uint64_t* aql_packs, uint64_t* hip_packs) {
  if (!n) return dora::fail(DORA_ERR_INVALID, "NULL node");
  if (aql_packs) *aql_packs = n->aql_packs;
  if (hip_packs) *hip_packs = n->hip_packs;
  return DORA_OK;
}

int dora_node_host_paths(dora_node* n, uint64_t* bar_fills, uint64_t* staged,
                         uint64_t* staged_bytes, uint64_t* host_packs) {
  if (!n) return dora::fail(DORA_ERR_INVALID, "NULL node");
  if (bar_fills) *bar_fills = n->bar_fills;
  if (host_packs) *host_packs = n->host_packs + n->host_copies;
  if (staged) *staged = n->core->host_staged.load();
  if (staged_bytes) *staged_bytes = n->core->host_staged_bytes.load();
  return DORA_OK;
}

int dora_node_host_bound_outputs(dora_node* n, char* buf, uint64_t cap, uint64_t* len) {
  if (!n) return dora::fail(DORA_ERR_INVALID, "NULL node");
  std::string all;
  for (const auto& o : n->host_bound) all += o + "\n";
  if (len) *len = all.size();
  if (!buf) return DORA_OK;
  if (cap < all.size() + 1) return dora::fail(DORA_ERR_INVALID, "buffer too small");
  std::memcpy(buf, all.c_str(), all.size() + 1);
  return DORA_OK;
}

int dora_node_set_timing_period(dora_node* n, uint64_t period) {
  if (!n) return dora::fail(DORA_ERR_INVALID, "NULL node");
  n->timing_period = period;
  return DORA_OK;
}

int dora_node_region_begin(dora_node* n) {
  if (!n) return dora::fail(DORA_ERR_INVALID, "NULL node");
  if (n->core->device < 0) return dora::fail(DORA_ERR_INVALID, "host-only node");
  dora::DeviceScope ds(n->core->device);
  if (!n->region_start) DORA_HIP(hipEventCreate(&n->region_start));
  n->region_cp_next = 0;
  n->region_cp_used.clear();
  n->region_armed = true;
  n->region_started = false;
  n->region_packs = n->region_bytes = n->region_aql = 0;
  n->region_stamped = n->region_unstamped = n->region_tmin = n->region_tmax = 0;
  n->region_ticks.clear();
  return DORA_OK;
}

namespace dora {
namespace {
// Record the region's stop events: one after the last pack queued on each fill stream and on
// the node stream.  No wait.
int region_record_stops(dora_node* n) {
  DeviceScope ds(n->core->device);
  std::vector<hipStream_t> ss = n->core->fill_streams;
  ss.push_back(n->core->stream);
  while (n->region_stop.size() < ss.size()) {  // fill streams are created lazily
    hipEvent_t e = nullptr;
    DORA_HIP(hipEventCreate(&e));
    n->region_stop.push_back(e);
  }
  for (size_t i = 0; i < ss.size(); ++i) DORA_HIP(hipEventRecord(n->region_stop[i], ss[i]));
  n->region_marked = true;
  return DORA_OK;
}
}  // namespace
}  // namespace dora

int dora_node_region_mark(dora_node* n) {
  if (!n) return dora::fail(DORA_ERR_INVALID, "NULL node");
  if (!n->region_armed) return dora::fail(DORA_ERR_INVALID, "no region begun");
  if (!n->region_started || !n->region_unstamped) return DORA_OK;  // stamped packs need none
  return dora::region_record_stops(n);
}

int dora_node_region_end(dora_node* n, double* span_ms, uint64_t* packs, uint64_t* bytes) {
  if (!n || !span_ms) return dora::fail(DORA_ERR_INVALID, "NULL argument");
  if (!n->region_armed) return dora::fail(DORA_ERR_INVALID, "no region begun");
  dora::DeviceScope ds(n->core->device);
  n->region_armed = false;
  const bool marked = n->region_marked;
  n->region_marked = false;
  *span_ms = 0;
  if (packs) *packs = n->region_packs;
  if (bytes) *bytes = n->region_bytes;
  if (!n->region_unstamped) {
    // every pack stamped its own device time: first workgroup start of the earliest to the
    // signal of the last (s_memrealtime); harvest the stamps not yet read at slot reuse
    std::vector<dora::Slot*> live(n->cache.begin(), n->cache.end());
    for (auto& kv : n->sent_out) live.push_back(kv.second);
    for (dora::Slot* s : live)
      if (s->region_epoch && !dora::wait_slot_idle(n, s))
        return dora::fail(DORA_ERR_TIMEOUT, "a timed pack did not complete within 10 s");
    if (n->region_cp_next) {
      // CP-signalled packs: their first workgroup's start and their last workgroup's end, read
      // from the stamp areas through the BAR (written through by the packs, all of which have
      // completed).  An area's other words are older packs' (earlier regions), never the max.
      n->region_cp_next = 0;
      // one AQL dispatch reduces every used area to (start, latest end) in host memory; the
      // BAR read is the fallback (~0.3 ms of uncached reads per area)
      const uint32_t na = uint32_t(std::min<size_t>(n->region_cp_used.size(), dora::kRegionCpAreas));
      bool reduced = false;
      if (na && n->region_reduce_idx) {
        std::copy(n->region_cp_used.begin(), n->region_cp_used.begin() + na, n->region_reduce_idx);
        std::fill(n->region_reduce_out, n->region_reduce_out + 2 * na, uint64_t(0));
        const int rrc = dora::aql_stamp_reduce(n->core->device, n->region_cp_stamps,
                                               uint32_t(dora::kCpAreaWords), n->region_reduce_idx,
                                               na, n->region_reduce_out);
        reduced = rrc == DORA_OK;
        if (rrc == DORA_ERR_TIMEOUT) {
          // the reduction may still run and write them: leak both (later regions read the BAR)
          n->region_reduce_idx = nullptr;
          n->region_reduce_out = nullptr;
        }
        if (!reduced) dora::clear_error();
      }
      std::vector<uint64_t> w(1 + dora::kCpStampWgs);
      for (uint32_t j = 0; j < n->region_cp_used.size(); ++j) {
        const uint32_t area = n->region_cp_used[j];
        uint64_t a, b;
        if (reduced && j < na) {
          a = __atomic_load_n(n->region_reduce_out + 2 * j, __ATOMIC_ACQUIRE);
          b = __atomic_load_n(n->region_reduce_out + 2 * j + 1, __ATOMIC_ACQUIRE);
        } else {
          std::memcpy(w.data(), n->region_cp_stamps + size_t(area) * dora::kCpAreaWords,
                      w.size() * 8);
          a = w[0];
          b = *std::max_element(w.begin() + 1, w.end());
        }
        if (!a || b < a) continue;
        if (!n->region_stamped || a < n->region_tmin) n->region_tmin = a;
        if (!n->region_stamped || b > n->region_tmax) n->region_tmax = b;
        ++n->region_stamped;
        if (n->region_ticks.size() < 2 * (1u << 16)) {
          n->region_ticks.push_back(a);
          n->region_ticks.push_back(b);
        }
      }
      n->region_cp_used.clear();
    }
    if (n->region_stamped)
      *span_ms = double(n->region_tmax - n->region_tmin) / dora::kRealtimeHz * 1e3;
    if (packs) *packs = n->region_stamped;
    if (bytes && n->region_packs) *bytes = n->region_bytes / n->region_packs * n->region_stamped;
    return DORA_OK;
  }
  if (!n->region_started) return DORA_OK;
  // fallback (packs without kernel stamps): the first pack's start event to events recorded
  // after the last pack on each fill stream and the node stream, by dora_node_region_mark right
  // after the last send, or now
  if (!marked) {
    int rc = dora::region_record_stops(n);
    if (rc != DORA_OK) return rc;
    n->region_marked = false;
  }
  const size_t ns = n->core->fill_streams.size() + 1;
  for (size_t i = 0; i < ns && i < n->region_stop.size(); ++i) {
    DORA_HIP(hipEventSynchronize(n->region_stop[i]));
    float ms = 0;
    DORA_HIP(hipEventElapsedTime(&ms, n->region_start, n->region_stop[i]));
    *span_ms = std::max<double>(*span_ms, ms);
  }
  return DORA_OK;
}

int dora_node_pack_intervals(dora_node* n, double* out_ms, size_t cap, size_t* count) {
  if (!n || !count || (!out_ms && cap)) return dora::fail(DORA_ERR_INVALID, "NULL argument");
  if (!n->region_ticks.empty()) {
    // the last timed region's packs, from their own stamps, ms after the earliest start
    const size_t pairs = n->region_ticks.size() / 2;
    *count = pairs;
    for (size_t i = 0; i < 2 * std::min(cap, pairs); ++i)
      out_ms[i] = double(n->region_ticks[i] - n->region_tmin) / dora::kRealtimeHz * 1e3;
    return DORA_OK;
  }
  dora::harvest_all(n);
  const size_t pairs = n->intervals.size() / 2;
  *count = pairs;
  for (size_t i = 0; i < 2 * std::min(cap, pairs); ++i) out_ms[i] = n->intervals[i];
  return DORA_OK;
}

int dora_node_forward_stats(dora_node* n, uint64_t* in_place, uint64_t* held) {
  if (!n) return dora::fail(DORA_ERR_INVALID, "NULL node");
  if (in_place) *in_place = n->zero_copy_forwards;
  if (held) *held = n->forwarded.size();
  return DORA_OK;
}

int dora_node_peer_stats(dora_node* n, uint64_t* copies, uint64_t* bytes) {
  if (!n) return dora::fail(DORA_ERR_INVALID, "NULL node");
  if (copies) *copies = n->core->peer_copies.load();
  if (bytes) *bytes = n->core->peer_bytes.load();
  return DORA_OK;
}

int dora_node_bcast_stats(dora_node* n, uint64_t* groups_out, uint64_t* groups_in,
                          uint64_t* sent, uint64_t* received, uint64_t* received_bytes,
                          const char** error) {
  if (!n) return dora::fail(DORA_ERR_INVALID, "NULL node");
  if (groups_out) *groups_out = n->bcast_out.size();
  if (groups_in) *groups_in = n->core->bcast_in.size();
  if (sent) *sent = n->bcast_seq;
  if (received) *received = n->core->bcast_recvs;
  if (received_bytes) *received_bytes = n->core->bcast_bytes;
  if (error) *error = n->core->bcast_error.c_str();
  return DORA_OK;
}

int dora_node_bcast_ranks(dora_node* n, uint64_t* max_ranks) {
  if (!n || !max_ranks) return dora::fail(DORA_ERR_INVALID, "NULL argument");
  *max_ranks = 0;
  for (const auto& kv : n->bcast_out)
    *max_ranks = std::max<uint64_t>(*max_ranks, uint64_t(dora::bcast_nranks(kv.second.comm)));
  return DORA_OK;
}

int dora_node_send_profile(dora_node* n, double* out_us, size_t n_out, uint64_t* count) {
  if (!n) return dora::fail(DORA_ERR_INVALID, "NULL node");
  const double c = n->phase_count ? double(n->phase_count) : 1.0;
  for (size_t i = 0; i < n_out && i < 4; ++i) out_us[i] = double(n->phase_ns[i]) / c / 1000.0;
  if (count) *count = n->phase_count;
  return DORA_OK;
}

int dora_node_set_profiling(dora_node* n, int enable) {
  if (!n) return dora::fail(DORA_ERR_INVALID, "NULL node");
  if (enable) {
    if (n->core->device < 0) return dora::fail(DORA_ERR_INVALID, "host-only node");
    int rc = dora::ensure_timing(n);
    if (rc != DORA_OK) return rc;
  }
  dora::harvest_all(n);
  n->profile = enable != 0;
  n->intervals.clear();
  if (enable) {
    // time origin of dora_node_pack_intervals
    DORA_HIP(hipEventRecord(n->timing_ref, n->core->stream));
    DORA_HIP(hipEventSynchronize(n->timing_ref));
  }
  for (auto& x : n->phase_ns) x = 0;
  n->phase_count = 0;
  n->pack_count = 0;
  n->timing_seq = 0;
  n->pack_ms = 0;
  n->pack_bytes = 0;
  return DORA_OK;
}

}  // extern "C"
