// Shared-memory control plane of a local dataflow: one POSIX shm region created by the daemon,
// holding, per node, three single-producer/single-consumer byte rings:
//   requests  node   -> daemon  (DaemonRequest: SendMessage, ReportDropTokens, CloseOutputs ...)
//   events    daemon -> node    (NodeEvent: Input, InputClosed, AllInputsClosed, Stop, Ready)
//   drops     daemon -> node    (NodeDropEvent::OutputDropped)
// It replaces the reference's per-node TCP/UDS/4 KiB-shmem request-reply channels
// (apis/rust/node/src/daemon_connection/*, binaries/daemon/src/node_communication/*,
// libraries/shared-memory-server/src/channel.rs) with rings that never block the producer on a
// reply (SendMessage expects no reply in the reference either, node_to_daemon.rs:36-41) and are
// sized for the type info of large nested arrays (the 4 KiB mailbox limit, F5, is gone).
// Waiting: spin for a bounded time, then futex-wait on a sequence word.
#pragma once

#include <atomic>
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace dora {

constexpr uint64_t kRegionMagic = 0x444f5241474d5358ull;  // "DORAGMSX"
constexpr uint32_t kRegionVersion = 5;  // 5: FillFlag carries a CP completion signal
// Upper bound on the nodes of one dataflow.  The region holds only the `n_nodes` entries in use
// (region_header_bytes), so the bound costs nothing.
constexpr uint32_t kMaxNodes = 4096;
constexpr size_t kIdLen = 64;

struct RingHdr {
  alignas(64) std::atomic<uint64_t> head;  // bytes written (producer)
  alignas(64) std::atomic<uint64_t> tail;  // bytes consumed (consumer)
  alignas(64) std::atomic<uint32_t> seq;   // futex word, bumped on every publish
  std::atomic<uint32_t> waiters;
  uint64_t data_off;  // from region base
  uint64_t cap;       // power of two
};

constexpr size_t kListLen = 2048;
constexpr uint32_t kFillFlags = 64;  // per node: one per live device slot

// A fill-completion word: the pack kernel that filled the slot stores the send epoch here (into
// the host-registered region) once every workgroup's stores are complete; receivers poll it with
// plain loads.  The same line carries the pack's first workgroup's start and its signal time
// (s_memrealtime, 100 MHz ticks): device timing of the fill without profiling the queue.  One
// cache line each.
//
// Mid-size single-segment packs (aql.cpp, cp_signal_window) are signalled by the command
// processor instead: the packet's completion signal is the `cp` line below, laid out as the
// runtime's amd_signal_t (hsa/amd_hsa_signal.h: the CP decrements `value` once the dispatch's
// last wave has ended; no mailbox, so no interrupt), and every wave of the pack waits for its
// own write-through stores before it ends.  Before such a dispatch the sender stores
// cp.value = 1, epoch = e - 1 and then cp_epoch = e (release): the fill of epoch e is complete
// once cp_epoch == e and cp.value has reached 0.  fill_reached() is the one completion test.
struct alignas(64) CpSignal {
  int64_t kind;                  // AMD_SIGNAL_KIND_USER
  std::atomic<int64_t> value;    // 1 while the dispatch runs, 0 after
  uint64_t event_mailbox_ptr;    // 0: no interrupt
  uint32_t event_id, reserved1;
  uint64_t start_ts, end_ts;     // written by the CP when the queue is profiled
  uint64_t queue_ptr;
  uint32_t reserved3[2];
};
static_assert(sizeof(CpSignal) == 64, "amd_signal_t layout");

struct FillFlag {
  alignas(64) std::atomic<uint64_t> epoch;
  uint64_t t_start, t_end;
  std::atomic<uint64_t> cp_epoch;  // epoch of the CP-signalled fill `cp` reports
  // the latest fill whose every source byte has been read (a read-signalled pack, aql.h): its
  // synchronous send may return while the pack's stores drain
  std::atomic<uint64_t> read_epoch;
  uint64_t pad_[3];
  CpSignal cp;
};
static_assert(offsetof(FillFlag, cp) == 64 && sizeof(FillFlag) == 128, "FillFlag layout");
constexpr double kRealtimeHz = 100e6;  // s_memrealtime

// Has the fill of epoch `e` into the flag whose `epoch` word `f` points at completed?  In-kernel
// signals store the epoch (epochs of a flag only grow); a CP-signalled fill is the one cp_epoch
// names, complete when the CP's decrement has brought cp.value to 0.  A sender sets a flag up for
// a new fill only after its previous fill has completed (slot reuse waits for it).
inline bool fill_reached(const std::atomic<uint64_t>* f, uint64_t e) {
  if (f->load(std::memory_order_acquire) >= e) return true;
  const FillFlag* ff = reinterpret_cast<const FillFlag*>(f);
  return ff->cp_epoch.load(std::memory_order_acquire) == e &&
         ff->cp.value.load(std::memory_order_acquire) <= 0;
}

// Set flag `ff` up for the CP-signalled fill of epoch `e` (the sender, before the dispatch; the
// flag's previous fill has completed).  The epoch word first, so that a check of an earlier
// epoch of this flag never sees it incomplete; cp_epoch last, with release.
inline void cp_arm(FillFlag* ff, uint64_t e) {
  ff->cp.kind = 1;  // AMD_SIGNAL_KIND_USER
  ff->cp.event_mailbox_ptr = 0;
  ff->cp.event_id = 0;
  ff->cp.queue_ptr = 0;
  if (ff->epoch.load(std::memory_order_relaxed) < e - 1)
    ff->epoch.store(e - 1, std::memory_order_relaxed);
  ff->cp.value.store(1, std::memory_order_relaxed);
  ff->cp_epoch.store(e, std::memory_order_release);
}

struct NodeEntry {
  FillFlag fill[kFillFlags];
  char id[kIdLen];
  char outputs[kListLen];  // "out1,out2"           (NodeRunConfig.outputs)
  char inputs[kListLen];   // "in1=10,in2=1"        (input id = queue_size)
  std::atomic<int32_t> pid;
  std::atomic<uint32_t> state;  // 0 idle, 1 subscribed, 2 done
  std::atomic<int32_t> device;  // GPU ordinal of the running node (-1 host-only, -2 not started)
  // diagnostics any process of the dataflow may read (bench: set-up work inside a timed region)
  std::atomic<uint64_t> slots_created;  // device slots this node allocated (hipMalloc + export)
  std::atomic<uint64_t> ipc_opens;      // producers' slots this node mapped (hipIpcOpenMemHandle)
  std::atomic<uint64_t> dropped_inputs; // inputs its queue_size policy dropped (drop_oldest)
  RingHdr requests;
  RingHdr events;
  RingHdr drops;
};

struct RegionHdr {
  uint64_t magic;
  uint32_t version;
  uint32_t n_nodes;
  uint64_t ring_cap;
  uint64_t total_size;
  alignas(64) std::atomic<uint32_t> doorbell;  // futex word the daemon sleeps on
  std::atomic<uint32_t> daemon_sleeping;
  std::atomic<uint32_t> shutdown;
  // NUMA node of the first GPU node to start (-1: none yet): the daemon moves next to it
  std::atomic<int32_t> numa_hint;
  // first CPU of the L3 cache domain the dataflow's processes share (-1: none chosen yet)
  std::atomic<int32_t> l3_cpu;
  char dataflow_id[kIdLen];
  NodeEntry nodes[kMaxNodes];  // only the first n_nodes exist in the mapping
};

// Bytes of the header of a region with `n` nodes (the node entries in use, nothing more).
size_t region_header_bytes(size_t n);

// A mapped region (creator or attacher).
class Region {
 public:
  ~Region();
  static Region* create(const std::string& name, const std::vector<std::string>& node_ids,
                        uint64_t ring_cap, const std::string& dataflow_id);
  static Region* attach(const std::string& name);
  RegionHdr* hdr() const { return hdr_; }
  uint8_t* base() const { return reinterpret_cast<uint8_t*>(hdr_); }
  int node_index(const std::string& id) const;
  void unlink();
  size_t size() const { return size_; }
  const std::string& name() const { return name_; }

 private:
  Region() = default;
  RegionHdr* hdr_ = nullptr;
  size_t size_ = 0;
  std::string name_;
  bool owner_ = false;
};

// Producer / consumer views of one ring.  Records: [u32 rec_len][u32 kind][u64 n][payload],
// 8-B aligned; a record of kind 0xFFFFFFFF pads to the end of the ring.
class RingWriter {
 public:
  RingWriter() = default;
  RingWriter(Region* r, RingHdr* h) : r_(r), h_(h) {}
  // Publish one record; returns false if it does not fit right now (caller retries / queues).
  bool try_push(uint32_t kind, const uint8_t* payload, size_t n);
  // Blocking push (spins, then sleeps) until space is available or `timeout_us` elapses.
  bool push(uint32_t kind, const uint8_t* payload, size_t n, int64_t timeout_us = -1);
  bool fits(size_t n) const;
  RingHdr* hdr() const { return h_; }

 private:
  Region* r_ = nullptr;
  RingHdr* h_ = nullptr;
};

// How long a waiter spins before it sleeps on a futex.  A futex wake-up on a shared host can take
// milliseconds (the woken thread waits for a CPU a neighbour holds): on one MI355X box the
// latency ladder's p99 (1000 messages 1 ms apart per size) was 0.2-3.2 ms with every waiter
// sleeping after 200 us of spinning, and 4-73 us when they spun through the gap
// (profiles/r02_lat_tail_ab.jsonl).  So a waiter spins through its recent idle gaps when they
// are short: budget = max(base, 2 x a fast-down / slow-up mean of the idle gaps that ended with
// data) while that is within the cap, else the base.  A stream slower than the cap allows (e.g. 30 Hz
// cameras) costs no more CPU than before; streams at >= ~400 Hz keep their waiters on-CPU.
// The base is 200 us, the cap 5 ms.
class AdaptiveSpin {
 public:
  int64_t budget_us() const;
  void observe(uint64_t idle_ns);  // an idle gap that ended because data arrived

 private:
  uint64_t mean_ns_ = 0;
};

// The daemon's estimate of the spacing of data messages alone (REQ_SEND_MESSAGE arrivals): a
// plain moving average, so the drop-token report that follows each device message a few
// microseconds later — a short gap of the daemon's other traffic, which AdaptiveSpin follows
// down at once — does not put the daemon to sleep before the next message of a 1 ms stream
// (each such message paid a ~2 us futex wake, 11-13 us from an idle core).
class MessageSpin {
 public:
  void arrived(uint64_t now_ns);
  int64_t budget_us() const;  // 0 when messages are too far apart to spin through

 private:
  uint64_t last_ns_ = 0, mean_ns_ = 0;
};

class RingReader {
 public:
  RingReader() = default;
  RingReader(Region* r, RingHdr* h) : r_(r), h_(h) {}
  // Pop one record into (kind, payload).  Returns false if empty.
  bool try_pop(uint32_t* kind, std::vector<uint8_t>* payload);
  // Wait until a record is available or timeout (us; <0 = forever).  Returns false on timeout.
  bool wait(int64_t timeout_us, const std::atomic<uint32_t>* abort_flag = nullptr);
  bool empty() const;
  RingHdr* hdr() const { return h_; }

 private:
  Region* r_ = nullptr;
  RingHdr* h_ = nullptr;
  AdaptiveSpin spin_;
  uint64_t idle_from_ = 0;    // start of the current idle gap (0: none)
  uint64_t last_return_ = 0;  // when wait() last returned
};

// Sample regions of host-only nodes: DataMessage::SharedMemory, the reference's
// `ShmemConf::new().size(len).create()` (apis/rust/node/src/node/mod.rs:321-346).  POSIX shm
// mapped shared read-write; the creator unlinks it when the slot is freed.
void* shmem_create(const std::string& name, size_t len);  // nullptr on failure (errno)
void* shmem_open(const std::string& name, size_t* len);   // the whole region; nullptr on failure
void shmem_unmap(void* p, size_t len);
void shmem_unlink(const std::string& name);
// The first `len` bytes of region `name` (the inter-daemon forwarder's copy).
bool read_shmem(const std::string& name, uint64_t len, std::vector<uint8_t>* out);

// A spinning thread that saw the clock jump by more than this between two passes was off the
// CPU meanwhile: that time does not count against its spin budget (shm.cpp, daemon.cpp).
constexpr uint64_t kOffCpuNs = 50000;

// futex helpers on shared (non-private) words
void futex_wait(std::atomic<uint32_t>* w, uint32_t expected, int64_t timeout_us);
void futex_wake(std::atomic<uint32_t>* w);
int64_t spin_budget_us();      // the base budget (200 us)
int64_t spin_max_us();         // the adaptive cap (5 ms)
uint64_t now_ns();          // CLOCK_REALTIME (timestamps that cross processes)
uint64_t mono_ns();          // CLOCK_MONOTONIC
// Restrict the calling thread (and threads it starts later) to the CPUs of NUMA node `numa`
// within its current affinity; false when that would leave none or changes nothing.
// Move the calling thread onto NUMA node `numa`'s CPUs (within its current affinity) and, when
// `l3_cpu` is given and the node's L3 domains have room for `procs` processes, onto the one L3
// domain the dataflow shares (DORA_GPU_PIN=numa: NUMA node only).
bool pin_to_numa(int numa, int device = -1, std::atomic<int32_t>* l3_cpu = nullptr,
                 int procs = 0);

}  // namespace dora
