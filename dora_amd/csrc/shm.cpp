// Shared-memory region + SPSC rings + futex waits (see shm.h).
#include "common.h"
#include "shm.h"
#include "trace.h"

#include <cstddef>

#include <fcntl.h>
#include <linux/futex.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <stdexcept>
#include <vector>

namespace dora {

namespace {
constexpr uint32_t kPadKind = 0xFFFFFFFFu;
constexpr uint64_t kPage = 4096;

uint64_t round_up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }

void init_ring(RingHdr& h, uint64_t off, uint64_t cap) {
  new (&h.head) std::atomic<uint64_t>(0);
  new (&h.tail) std::atomic<uint64_t>(0);
  new (&h.seq) std::atomic<uint32_t>(0);
  new (&h.waiters) std::atomic<uint32_t>(0);
  h.data_off = off;
  h.cap = cap;
}
}  // namespace

uint64_t now_ns() {
  timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  return uint64_t(ts.tv_sec) * 1000000000ull + uint64_t(ts.tv_nsec);
}

uint64_t mono_ns() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return uint64_t(ts.tv_sec) * 1000000000ull + uint64_t(ts.tv_nsec);
}

namespace {

// "0-63,128-191" -> set
void parse_cpulist(const char* path, cpu_set_t* out) {
  CPU_ZERO(out);
  FILE* f = std::fopen(path, "r");
  if (!f) return;
  char buf[4096];
  const size_t n = std::fread(buf, 1, sizeof(buf) - 1, f);
  std::fclose(f);
  buf[n] = 0;
  for (char* p = buf; *p;) {
    char* end = nullptr;
    const long a = std::strtol(p, &end, 10);
    if (end == p) break;
    long b = a;
    p = end;
    if (*p == '-') b = std::strtol(p + 1, &p, 10);
    for (long c = a; c <= b && c < CPU_SETSIZE; ++c) CPU_SET(int(c), out);
    while (*p == ',' || *p == '\n' || *p == ' ') ++p;
  }
}

// DORA_GPU_PIN (node.cpp numa_pinning: 0 = off): "numa" = NUMA node only; "fixed" = the L3
// domain by GPU ordinal (r03); default = the least busy L3 domain.
int l3_placement_mode() {
  static const int v = [] {
    const char* e = std::getenv("DORA_GPU_PIN");
    if (e && std::strcmp(e, "numa") == 0) return 0;
    if (e && std::strcmp(e, "fixed") == 0) return 1;
    return 2;
  }();
  return v;
}
bool l3_placement() { return l3_placement_mode() > 0; }

// Busy and total jiffies per CPU from /proc/stat.
void cpu_times(std::vector<std::pair<uint64_t, uint64_t>>* out) {
  out->assign(CPU_SETSIZE, {0, 0});
  FILE* f = std::fopen("/proc/stat", "r");
  if (!f) return;
  char line[512];
  while (std::fgets(line, sizeof(line), f)) {
    int cpu = -1;
    unsigned long long v[10] = {};
    if (std::sscanf(line, "cpu%d %llu %llu %llu %llu %llu %llu %llu %llu", &cpu, &v[0], &v[1],
                    &v[2], &v[3], &v[4], &v[5], &v[6], &v[7]) < 5 ||
        cpu < 0 || cpu >= CPU_SETSIZE)
      continue;
    const uint64_t idle = v[3] + v[4];
    const uint64_t total = v[0] + v[1] + v[2] + v[3] + v[4] + v[5] + v[6] + v[7];
    (*out)[size_t(cpu)] = {total - idle, total};
  }
  std::fclose(f);
}

}  // namespace

bool pin_to_numa(int numa, int device, std::atomic<int32_t>* l3_cpu, int procs) {
  if (numa < 0) return false;
  char path[128];
  std::snprintf(path, sizeof(path), "/sys/devices/system/node/node%d/cpulist", numa);
  cpu_set_t want, cur, both;
  parse_cpulist(path, &want);
  if (sched_getaffinity(0, sizeof(cur), &cur) != 0) return false;
  CPU_AND(&both, &want, &cur);
  if (CPU_COUNT(&both) == 0) return false;
  if (l3_cpu && procs > 0 && l3_placement()) {
    // One L3 cache domain (a CCD) for the dataflow's processes on this NUMA node: every message
    // hands control-ring cache lines sender -> daemon -> receiver and back, and a line moved
    // between CCDs costs several times one moved inside an L3.  The first process picks the
    // domain (GPU ordinal modulo the domains, so co-located dataflows spread out), the others
    // follow its choice; a domain without two CPUs per process is not used.
    std::vector<cpu_set_t> groups;
    cpu_set_t seen;
    CPU_ZERO(&seen);
    for (int c = 0; c < CPU_SETSIZE; ++c) {
      if (!CPU_ISSET(c, &both) || CPU_ISSET(c, &seen)) continue;
      std::snprintf(path, sizeof(path),
                    "/sys/devices/system/cpu/cpu%d/cache/index3/shared_cpu_list", c);
      cpu_set_t g, gb;
      parse_cpulist(path, &g);
      if (CPU_COUNT(&g) == 0) CPU_SET(c, &g);
      CPU_AND(&gb, &g, &both);
      CPU_OR(&seen, &seen, &gb);
      if (CPU_COUNT(&gb) > 0) groups.push_back(gb);
    }
    int pick = -1;
    const int hint = l3_cpu->load(std::memory_order_acquire);
    for (size_t i = 0; i < groups.size() && hint >= 0; ++i)
      if (hint < CPU_SETSIZE && CPU_ISSET(hint, &groups[i])) pick = int(i);
    if (pick < 0 && groups.size() > 1) {
      pick = device >= 0 ? device % int(groups.size()) : 0;
      if (l3_placement_mode() == 2) {
        // the domain whose CPUs were idlest over 20 ms (ties: the ordinal's): the dataflow's
        // processes spin, and a domain shared with busy threads of other processes left r04's
        // sender or sink off-CPU for tens of microseconds mid-burst (C3 bursts at 0.40-0.66)
        std::vector<std::pair<uint64_t, uint64_t>> t0, t1;
        cpu_times(&t0);
        usleep(20000);
        cpu_times(&t1);
        std::vector<double> idle(groups.size(), -1.0);  // idle CPUs per eligible domain
        int best = -1;
        for (size_t i = 0; i < groups.size(); ++i) {
          if (CPU_COUNT(&groups[i]) < 2 * procs) continue;
          idle[i] = 0;
          for (int c = 0; c < CPU_SETSIZE; ++c) {
            if (!CPU_ISSET(c, &groups[i])) continue;
            const uint64_t dt = t1[size_t(c)].second - t0[size_t(c)].second;
            const uint64_t db = t1[size_t(c)].first - t0[size_t(c)].first;
            idle[i] += dt ? 1.0 - double(db) / double(dt) : 1.0;
          }
          if (best < 0 || idle[i] > idle[size_t(best)]) best = int(i);
        }
        // the ordinal's domain unless another has at least half a CPU more idle
        if (best >= 0 && !(idle[size_t(pick)] >= 0 && idle[size_t(pick)] + 0.5 > idle[size_t(best)]))
          pick = best;
      }
      int first = 0;
      while (!CPU_ISSET(first, &groups[size_t(pick)])) ++first;
      int32_t none = -1;
      l3_cpu->compare_exchange_strong(none, first);
    }
    if (pick >= 0 && groups.size() > 1 && CPU_COUNT(&groups[size_t(pick)]) >= 2 * procs)
      both = groups[size_t(pick)];
  }
  if (CPU_EQUAL(&both, &cur)) return false;
  return sched_setaffinity(0, sizeof(both), &both) == 0;
}

int64_t spin_budget_us() { return 200; }

int64_t spin_max_us() { return 5000; }

int64_t AdaptiveSpin::budget_us() const {
  const int64_t base = spin_budget_us(), cap = spin_max_us();
  const int64_t want = int64_t(2 * mean_ns_ / 1000);
  return want <= cap && want > base ? want : base;
}

void AdaptiveSpin::observe(uint64_t idle_ns) {
  // Fast down, slow up: a gap shorter than the mean replaces it (after a pause, the next short
  // gap turns spinning back on at once — with a plain running mean the first ~16 messages of a
  // 1 ms ladder after a 20 ms pause still slept, p99 4.2 ms at that size); a longer gap moves it
  // 1/4 of the way (a 1 ms stream after a burst spins through its gaps from the 3rd message).
  // Gaps are clamped to 4 x the cap.
  const uint64_t lim = uint64_t(std::max<int64_t>(spin_max_us(), 0)) * 4000;
  if (idle_ns > lim) idle_ns = lim;
  mean_ns_ = idle_ns <= mean_ns_ || !mean_ns_ ? idle_ns : mean_ns_ + (idle_ns - mean_ns_) / 4;
}

void MessageSpin::arrived(uint64_t now_ns) {
  if (last_ns_) {
    // gaps beyond 4 x the cap count as the cap's 4 x (a pause ends a stream's estimate quickly
    // without one outlier dominating it); 1/8 weight per message
    const uint64_t lim = uint64_t(spin_max_us()) * 4000;
    const uint64_t g = std::min<uint64_t>(now_ns - last_ns_, lim);
    mean_ns_ = mean_ns_ ? mean_ns_ - mean_ns_ / 8 + g / 8 : g;
  }
  last_ns_ = now_ns;
}

int64_t MessageSpin::budget_us() const {
  const int64_t want = int64_t(2 * mean_ns_ / 1000);
  return mean_ns_ && want <= spin_max_us() ? want : 0;
}

void futex_wait(std::atomic<uint32_t>* w, uint32_t expected, int64_t timeout_us) {
  timespec ts, *tp = nullptr;
  if (timeout_us >= 0) {
    ts.tv_sec = timeout_us / 1000000;
    ts.tv_nsec = (timeout_us % 1000000) * 1000;
    tp = &ts;
  }
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(w), FUTEX_WAIT, expected, tp, nullptr, 0);
}

void futex_wake(std::atomic<uint32_t>* w) {
  syscall(SYS_futex, reinterpret_cast<uint32_t*>(w), FUTEX_WAKE, INT32_MAX, nullptr, nullptr, 0);
}

Region::~Region() {
  if (hdr_) munmap(hdr_, size_);
  if (owner_) shm_unlink(name_.c_str());
}

void Region::unlink() {
  if (owner_) {
    shm_unlink(name_.c_str());
    owner_ = false;
  }
}

void* shmem_create(const std::string& name, size_t len) {
  const int fd = ::shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
  if (fd < 0) return nullptr;
  void* p = MAP_FAILED;
  if (::ftruncate(fd, off_t(len)) == 0)
    p = ::mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  const int err = errno;
  ::close(fd);
  if (p == MAP_FAILED) {
    ::shm_unlink(name.c_str());
    errno = err;
    return nullptr;
  }
  return p;
}

void* shmem_open(const std::string& name, size_t* len) {
  const int fd = ::shm_open(name.c_str(), O_RDWR, 0);
  if (fd < 0) return nullptr;
  struct stat st {};
  void* p = MAP_FAILED;
  if (::fstat(fd, &st) == 0 && st.st_size > 0)
    p = ::mmap(nullptr, size_t(st.st_size), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  const int err = errno;
  ::close(fd);
  if (p == MAP_FAILED) {
    errno = err;
    return nullptr;
  }
  *len = size_t(st.st_size);
  return p;
}

void shmem_unmap(void* p, size_t len) {
  if (p) ::munmap(p, len);
}

void shmem_unlink(const std::string& name) { ::shm_unlink(name.c_str()); }

bool read_shmem(const std::string& name, uint64_t len, std::vector<uint8_t>* out) {
  size_t cap = 0;
  void* p = shmem_open(name, &cap);
  if (!p) return false;
  const bool ok = len <= cap;
  if (ok) out->assign(static_cast<const uint8_t*>(p), static_cast<const uint8_t*>(p) + len);
  shmem_unmap(p, cap);
  return ok;
}

size_t region_header_bytes(size_t n) {
  return offsetof(RegionHdr, nodes) + n * sizeof(NodeEntry);
}

Region* Region::create(const std::string& name, const std::vector<std::string>& node_ids,
                       uint64_t ring_cap, const std::string& dataflow_id) {
  if (node_ids.size() > kMaxNodes) throw std::invalid_argument("too many nodes");
  if (ring_cap < 4096 || (ring_cap & (ring_cap - 1)))
    throw std::invalid_argument("ring capacity must be a power of two >= 4096");
  const uint64_t hdr = round_up(region_header_bytes(node_ids.size()), kPage);
  const uint64_t total = hdr + 3 * ring_cap * node_ids.size();
  int fd = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
  if (fd < 0) throw std::runtime_error("shm_open(" + name + "): " + std::strerror(errno));
  if (ftruncate(fd, static_cast<off_t>(total)) != 0) {
    close(fd);
    shm_unlink(name.c_str());
    throw std::runtime_error(std::string("ftruncate: ") + std::strerror(errno));
  }
  void* p = mmap(nullptr, total, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) {
    shm_unlink(name.c_str());
    throw std::runtime_error(std::string("mmap: ") + std::strerror(errno));
  }
  auto* r = new Region();
  r->hdr_ = static_cast<RegionHdr*>(p);
  r->size_ = total;
  r->name_ = name;
  r->owner_ = true;
  RegionHdr* h = r->hdr_;
  std::memset(static_cast<void*>(h), 0, region_header_bytes(node_ids.size()));
  h->version = kRegionVersion;
  h->n_nodes = static_cast<uint32_t>(node_ids.size());
  h->numa_hint.store(-1);
  new (&h->l3_cpu) std::atomic<int32_t>(-1);
  h->ring_cap = ring_cap;
  h->total_size = total;
  new (&h->doorbell) std::atomic<uint32_t>(0);
  new (&h->daemon_sleeping) std::atomic<uint32_t>(0);
  new (&h->shutdown) std::atomic<uint32_t>(0);
  std::strncpy(h->dataflow_id, dataflow_id.c_str(), kIdLen - 1);
  uint64_t off = hdr;
  for (size_t i = 0; i < node_ids.size(); ++i) {
    NodeEntry& n = h->nodes[i];
    std::strncpy(n.id, node_ids[i].c_str(), kIdLen - 1);
    new (&n.pid) std::atomic<int32_t>(0);
    new (&n.state) std::atomic<uint32_t>(0);
    new (&n.device) std::atomic<int32_t>(-2);
    new (&n.slots_created) std::atomic<uint64_t>(0);
    new (&n.ipc_opens) std::atomic<uint64_t>(0);
    new (&n.dropped_inputs) std::atomic<uint64_t>(0);
    for (auto& f : n.fill) new (&f.epoch) std::atomic<uint64_t>(0);
    init_ring(n.requests, off, ring_cap);
    off += ring_cap;
    init_ring(n.events, off, ring_cap);
    off += ring_cap;
    init_ring(n.drops, off, ring_cap);
    off += ring_cap;
  }
  std::atomic_thread_fence(std::memory_order_release);
  h->magic = kRegionMagic;
  return r;
}

Region* Region::attach(const std::string& name) {
  int fd = shm_open(name.c_str(), O_RDWR, 0600);
  if (fd < 0) throw std::runtime_error("shm_open(" + name + "): " + std::strerror(errno));
  struct stat st;
  if (fstat(fd, &st) != 0) {
    close(fd);
    throw std::runtime_error("fstat failed");
  }
  void* p = mmap(nullptr, static_cast<size_t>(st.st_size), PROT_READ | PROT_WRITE, MAP_SHARED,
                 fd, 0);
  close(fd);
  if (p == MAP_FAILED) throw std::runtime_error(std::string("mmap: ") + std::strerror(errno));
  auto* r = new Region();
  r->hdr_ = static_cast<RegionHdr*>(p);
  r->size_ = static_cast<size_t>(st.st_size);
  r->name_ = name;
  if (r->size_ < offsetof(RegionHdr, nodes) || r->hdr_->magic != kRegionMagic ||
      r->hdr_->version != kRegionVersion || r->hdr_->n_nodes > kMaxNodes ||
      region_header_bytes(r->hdr_->n_nodes) > r->size_) {
    delete r;
    throw std::runtime_error("shm region " + name + " is not a dora-gpu dataflow region");
  }
  return r;
}

int Region::node_index(const std::string& id) const {
  for (uint32_t i = 0; i < hdr_->n_nodes; ++i)
    if (id == hdr_->nodes[i].id) return static_cast<int>(i);
  return -1;
}

// ------------------------------------------------------------------------------------------
bool RingWriter::fits(size_t n) const {
  const uint64_t rec = round_up(16 + n, 8);
  return rec <= h_->cap / 2;
}

bool RingWriter::try_push(uint32_t kind, const uint8_t* payload, size_t n) {
  const uint64_t cap = h_->cap;
  const uint64_t rec = round_up(16 + n, 8);
  if (rec > cap / 2) throw std::length_error("record larger than half the ring");
  uint64_t head = h_->head.load(std::memory_order_relaxed);
  const uint64_t tail = h_->tail.load(std::memory_order_acquire);
  uint64_t off = head & (cap - 1);
  uint64_t need = rec;
  if (off + rec > cap) need += cap - off;
  if (cap - (head - tail) < need) return false;
  uint8_t* data = r_->base() + h_->data_off;
  if (off + rec > cap) {
    const uint32_t pad = static_cast<uint32_t>(cap - off);
    std::memcpy(data + off, &pad, 4);
    std::memcpy(data + off + 4, &kPadKind, 4);
    head += pad;
    off = 0;
  }
  const uint32_t len = static_cast<uint32_t>(rec);
  std::memcpy(data + off, &len, 4);
  std::memcpy(data + off + 4, &kind, 4);
  const uint64_t n64 = n;
  std::memcpy(data + off + 8, &n64, 8);
  if (n) std::memcpy(data + off + 16, payload, n);
  h_->head.store(head + rec, std::memory_order_release);
  // Wake only a reader that sleeps: it announces itself in `waiters` before it reads `seq` and
  // re-checks for data, and the fence orders our head store before the `waiters` load, so
  // either we see it or it sees the record (no seq bump, no shared RMW, on the common path).
  std::atomic_thread_fence(std::memory_order_seq_cst);
  if (h_->waiters.load(std::memory_order_relaxed)) {
    h_->seq.fetch_add(1, std::memory_order_seq_cst);
    futex_wake(&h_->seq);
  }
  return true;
}

bool RingWriter::push(uint32_t kind, const uint8_t* payload, size_t n, int64_t timeout_us) {
  const uint64_t t0 = mono_ns();
  unsigned backoff = 1;
  while (!try_push(kind, payload, n)) {
    if (timeout_us >= 0 && int64_t(mono_ns() - t0) / 1000 > timeout_us) return false;
    usleep(backoff);
    backoff = backoff < 200 ? backoff * 2 : 200;
  }
  return true;
}

bool RingReader::empty() const {
  return h_->tail.load(std::memory_order_relaxed) == h_->head.load(std::memory_order_acquire);
}

bool RingReader::try_pop(uint32_t* kind, std::vector<uint8_t>* payload) {
  const uint64_t cap = h_->cap;
  uint8_t* data = r_->base() + h_->data_off;
  for (;;) {
    uint64_t tail = h_->tail.load(std::memory_order_relaxed);
    const uint64_t head = h_->head.load(std::memory_order_acquire);
    if (tail == head) return false;
    const uint64_t off = tail & (cap - 1);
    uint32_t len, k;
    std::memcpy(&len, data + off, 4);
    std::memcpy(&k, data + off + 4, 4);
    if (k == kPadKind) {
      h_->tail.store(tail + len, std::memory_order_release);
      continue;
    }
    *kind = k;
    uint64_t n;
    std::memcpy(&n, data + off + 8, 8);
    payload->assign(data + off + 16, data + off + 16 + n);
    h_->tail.store(tail + len, std::memory_order_release);
    return true;
  }
}

namespace {
thread_local bool tl_wait_slept = false;  // the thread's last wait slept in the futex
}  // namespace

bool ring_take_woke() {
  const bool v = tl_wait_slept;
  tl_wait_slept = false;
  return v;
}

bool RingReader::wait(int64_t timeout_us, const std::atomic<uint32_t>* abort_flag) {
  const uint64_t t0 = mono_ns();
  tl_wait_slept = false;
  // One idle gap may span several calls that time out (a sender polling for drop tokens every
  // 1 ms): the gap — for the spin budget and the adaptive mean — runs from the first of them,
  // unless the caller did other work for a while in between.
  // one emptiness check decides both the gap's start and Idle::was_empty: data arriving between
  // two checks left idle_from_ set for a call that then measured nothing
  const bool was_empty = empty();
  if (was_empty) {
    if (!idle_from_ || t0 - last_return_ > 100000) idle_from_ = t0;
  } else {
    idle_from_ = 0;
  }
  const uint64_t gap0 = idle_from_ ? idle_from_ : t0;
  const int64_t spin = spin_.budget_us();
  struct Idle {
    RingReader* r;
    uint64_t t0;
    bool was_empty;
    bool got = false;
    ~Idle() {
      const uint64_t now = mono_ns();
      r->last_return_ = now;
      if (!was_empty) return;
      add_idle_ns(now - t0);
      if (got) {
        r->spin_.observe(now - r->idle_from_);
        r->idle_from_ = 0;
      }
    }
  } idle{this, t0, was_empty};
  uint64_t spin_from = gap0, prev = t0;
  bool sleeping = false;  // past the spin: futex slices until a record comes
  while (empty()) {
    const uint64_t now = mono_ns();
    const int64_t el = int64_t(now - t0) / 1000;
    if (timeout_us >= 0 && el >= timeout_us) return false;
    if (abort_flag && abort_flag->load(std::memory_order_relaxed)) return false;
    if (!sleeping) {
      // time off the CPU is not spinning: the window moves by it (as the daemon's, daemon.cpp)
      if (now - prev > kOffCpuNs) spin_from += now - prev;
      prev = now;
      if (int64_t(now - spin_from) / 1000 < spin) {
        __builtin_ia32_pause();
        continue;
      }
      sleeping = true;
    }
    h_->waiters.fetch_add(1, std::memory_order_seq_cst);
    const uint32_t s = h_->seq.load(std::memory_order_seq_cst);
    if (empty()) {
      int64_t slice = 20000;  // re-check abort flags periodically
      if (timeout_us >= 0) slice = std::min<int64_t>(slice, timeout_us - el);
      if (slice > 0) {
        tl_wait_slept = true;
        futex_wait(&h_->seq, s, slice);
      }
    }
    h_->waiters.fetch_sub(1, std::memory_order_seq_cst);
  }
  idle.got = true;
  return true;
}

}  // namespace dora
