// Inter-daemon data path: wire format, TCP transport, Forwarder (staging of device samples for
// remote receivers) and Gateway (proxy nodes re-sending remote outputs locally).  See
// interdaemon.h for the protocol; reference: libraries/message/src/daemon_to_daemon.rs:9-21,
// binaries/daemon/src/lib.rs:955-1000 (send_out's remote branch), inter_daemon.rs (TCP framing).
#include "interdaemon.h"

#include <arpa/inet.h>
#include <hip/hip_runtime_api.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sys/socket.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>

#include "bincode.h"
#include "common.h"
#include "device_array.h"
#include "dora_gpu.h"

namespace dora {

// node.cpp: send a sample with the producer's original timestamp (the remote message's).
int proxy_send(dora_node* n, const char* output_id, const uint8_t* ti, size_t ti_len,
               const uint8_t* params, size_t params_len, dora_sample* sample, uint64_t ts);
dora_sample* vec_sample(const uint8_t* p, size_t len);

namespace {

bool send_all(int fd, const uint8_t* p, size_t n) {
  while (n) {
    const ssize_t k = ::send(fd, p, n, MSG_NOSIGNAL);
    if (k <= 0) {
      if (k < 0 && errno == EINTR) continue;
      return false;
    }
    p += k;
    n -= size_t(k);
  }
  return true;
}

bool recv_all(int fd, uint8_t* p, size_t n) {
  while (n) {
    const ssize_t k = ::recv(fd, p, n, 0);
    if (k <= 0) {
      if (k < 0 && errno == EINTR) continue;
      return false;
    }
    p += k;
    n -= size_t(k);
  }
  return true;
}

// TCP connection to host:port, retried for `timeout_ms` (the peer daemon may start later).
int connect_peer(const PeerAddr& a, int timeout_ms) {
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    addrinfo hints{}, *res = nullptr;
    hints.ai_family = AF_INET;
    hints.ai_socktype = SOCK_STREAM;
    const std::string port = std::to_string(a.port);
    if (getaddrinfo(a.host.c_str(), port.c_str(), &hints, &res) == 0) {
      for (addrinfo* ai = res; ai; ai = ai->ai_next) {
        int fd = ::socket(ai->ai_family, ai->ai_socktype, ai->ai_protocol);
        if (fd < 0) continue;
        if (::connect(fd, ai->ai_addr, ai->ai_addrlen) == 0) {
          int one = 1;
          setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
          freeaddrinfo(res);
          return fd;
        }
        ::close(fd);
      }
      freeaddrinfo(res);
    }
    if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(timeout_ms)) return -1;
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
  }
}

std::string ipc_key(const DeviceIpc& d) {
  std::string k(reinterpret_cast<const char*>(d.handle), 64);
  k.append(reinterpret_cast<const char*>(&d.owner_pid), 4);
  k.append(reinterpret_cast<const char*>(&d.slot_id), 8);
  return k;
}

}  // namespace

// ------------------------------------------------------------------------------------------
// Forwarder
// ------------------------------------------------------------------------------------------
Forwarder::Forwarder(Region* region, std::string dataflow_id,
                     std::map<std::string, PeerAddr> peers)
    : region_(region), dataflow_id_(std::move(dataflow_id)), peers_(std::move(peers)) {
  // a random uhlc ID, as uhlc's HLC::default() draws one (non-zero: ID wraps a NonZeroU128)
  const DropToken t = generate_drop_token();
  std::memcpy(hlc_id_.data(), t.b, 16);
  hlc_id_[0] |= 1;
  th_ = std::thread([this] { loop(); });
}

Forwarder::~Forwarder() {
  {
    std::lock_guard<std::mutex> g(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  if (th_.joinable()) th_.join();
  for (auto& kv : socks_) ::close(kv.second);
  for (auto& kv : maps_) (void)hipIpcCloseMemHandle(kv.second);
  if (pinned_) (void)hipHostFree(pinned_);
}

void Forwarder::push(ForwardJob job) {
  {
    std::lock_guard<std::mutex> g(mu_);
    q_.push_back(std::move(job));
  }
  cv_.notify_one();
}

void Forwarder::take_released(std::vector<DropToken>* out) {
  std::lock_guard<std::mutex> g(mu_);
  out->insert(out->end(), released_.begin(), released_.end());
  released_.clear();
}

bool Forwarder::idle() {
  std::lock_guard<std::mutex> g(mu_);
  return q_.empty() && !busy_ && released_.empty();
}

void Forwarder::loop() {
  for (;;) {
    ForwardJob job;
    {
      std::unique_lock<std::mutex> g(mu_);
      cv_.wait(g, [this] { return stop_ || !q_.empty(); });
      if (q_.empty()) return;  // stop_ with nothing left
      job = std::move(q_.front());
      q_.pop_front();
      busy_ = true;
    }
    handle(job);
    std::lock_guard<std::mutex> g(mu_);
    busy_ = false;
  }
}

// Copy a device sample to the host once its producer's fill has completed; its validity tail
// (type info tag 2) becomes inline bytes.  The producer's token is released by the caller.
bool Forwarder::stage(const ForwardJob& job, std::vector<uint8_t>* bytes,
                      std::vector<uint8_t>* ti) {
  const DeviceIpc& d = job.data.ipc;
  if (d.fill == FILL_FLAG) {
    RegionHdr* h = region_->hdr();
    if (d.flag_node >= h->n_nodes || d.flag_index >= kFillFlags) return false;
    const std::atomic<uint64_t>& f = h->nodes[d.flag_node].fill[d.flag_index].epoch;
    const auto t0 = std::chrono::steady_clock::now();
    while (!fill_reached(&f, d.epoch)) {
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60)) return false;
      std::this_thread::sleep_for(std::chrono::microseconds(5));
    }
  } else if (d.fill == FILL_BCAST) {
    return false;  // groups are not formed for outputs with remote receivers (daemon.cpp)
  }
  if (hipSetDevice(d.device) != hipSuccess) return false;
  if (d.fill == FILL_EVENT) {
    hipIpcEventHandle_t eh;
    std::memcpy(&eh, d.event, sizeof(eh));
    hipEvent_t ev = nullptr;
    if (hipIpcOpenEventHandle(&ev, eh) != hipSuccess) return false;
    const hipError_t e = hipEventSynchronize(ev);
    (void)hipEventDestroy(ev);
    if (e != hipSuccess) return false;
  }
  const std::string key = ipc_key(d);
  auto it = maps_.find(key);
  void* base = nullptr;
  if (it != maps_.end()) {
    base = it->second;
  } else {
    if (maps_.size() >= 64) {  // bounded: a staging copy is synchronous, nothing else holds them
      for (auto& kv : maps_) (void)hipIpcCloseMemHandle(kv.second);
      maps_.clear();
    }
    hipIpcMemHandle_t h;
    std::memcpy(&h, d.handle, sizeof(h));
    if (hipIpcOpenMemHandle(&base, h, hipIpcMemLazyEnablePeerAccess) != hipSuccess) return false;
    maps_[key] = base;
  }
  const uint64_t n = std::max(d.ext_len, d.len);
  if (pinned_cap_ < n) {
    if (pinned_) (void)hipHostFree(pinned_);
    pinned_ = nullptr;
    pinned_cap_ = 0;
    if (hipHostMalloc(reinterpret_cast<void**>(&pinned_), n) != hipSuccess) return false;
    pinned_cap_ = n;
  }
  if (n && hipMemcpy(pinned_, static_cast<uint8_t*>(base) + d.offset, n, hipMemcpyDeviceToHost) !=
               hipSuccess)
    return false;
  bytes->assign(pinned_, pinned_ + d.len);
  bool changed = false;
  std::vector<uint8_t> inl;
  if (inline_type_info(ti->data(), ti->size(), pinned_, n, &inl, &changed, true) != DORA_OK)
    return false;
  if (changed) ti->swap(inl);
  staged_bytes_.fetch_add(n, std::memory_order_relaxed);
  return true;
}

// Largest inter-daemon frame (DORA_GPU_MAX_FRAME_BYTES; default 64 GiB + 1 MiB of metadata,
// above any sample a slot holds, so every output the local path delivers also crosses machines).
// A gateway reading a longer length prefix takes the frame as corrupt or hostile and drops that
// connection; a forwarder refuses to send one (that message only, with an error naming it), so
// a message the peer would refuse never severs the link for the messages behind it.
uint64_t max_frame_bytes() {
  static const uint64_t v = [] {
    const char* e = std::getenv("DORA_GPU_MAX_FRAME_BYTES");
    const uint64_t x = e ? std::strtoull(e, nullptr, 10) : 0;
    return x ? x : (uint64_t(64) << 30) + (uint64_t(1) << 20);
  }();
  return v;
}

bool Forwarder::send_to(const std::string& machine, const std::vector<uint8_t>& frame) {
  auto p = peers_.find(machine);
  if (p == peers_.end()) {
    std::fprintf(stderr, "dora-gpu daemon: no address for machine `%s`\n", machine.c_str());
    return false;
  }
  const uint64_t now = mono_ns();
  auto d = down_until_.find(machine);
  if (d != down_until_.end() && now < d->second) return false;  // unreachable a moment ago
  for (int attempt = 0; attempt < 2; ++attempt) {
    auto s = socks_.find(machine);
    int fd = s != socks_.end() ? s->second : -1;
    if (fd < 0) {
      // the first connection waits for a peer that starts later; a reconnection does not
      fd = connect_peer(p->second, down_until_.count(machine) ? 1000 : 30000);
      if (fd < 0) {
        std::fprintf(stderr, "dora-gpu daemon: cannot connect to machine `%s` (%s:%d)\n",
                     machine.c_str(), p->second.host.c_str(), p->second.port);
        down_until_[machine] = mono_ns() + 5000000000ull;  // its messages are dropped for 5 s
        return false;
      }
      down_until_[machine] = 0;
      socks_[machine] = fd;
    }
    const uint64_t len = frame.size();
    if (send_all(fd, reinterpret_cast<const uint8_t*>(&len), 8) &&
        send_all(fd, frame.data(), frame.size()))
      return true;
    ::close(fd);  // broken connection: reconnect once
    socks_.erase(machine);
  }
  return false;
}

void Forwarder::handle(ForwardJob& job) {
  InterDaemonEvent e;
  e.dataflow_id = dataflow_id_;
  e.hlc_id = hlc_id_;
  e.event_ns = now_ns();
  e.node_id = job.node_id;
  if (job.closed) {
    // InputsClosed per machine, naming its receivers' inputs (lib.rs:1418-1440)
    e.kind = IDE_INPUTS_CLOSED;
    for (const auto& kv : job.closed_inputs) {
      e.inputs = kv.second;
      std::vector<uint8_t> frame;
      try {
        encode_ide(e, frame);
      } catch (const std::exception& ex) {
        std::fprintf(stderr, "dora-gpu daemon: forwarding: %s\n", ex.what());
        continue;
      }
      send_to(kv.first, frame);
    }
    forwarded_.fetch_add(1, std::memory_order_relaxed);
    return;
  } else {
    e.kind = IDE_OUTPUT;
    e.output_id = job.output_id;
    try {
      RBuf r(job.tail.data(), job.tail.size());
      const uint64_t ml = r.u64();
      r.need(ml);
      RBuf mr(r.ptr(), ml);
      Metadata m = mr.metadata();
      e.meta_version = m.version;
      e.timestamp_ns = m.timestamp_ns;
      e.type_info = std::move(m.type_info);
      e.parameters = std::move(m.parameters);
    } catch (const std::exception& ex) {
      std::fprintf(stderr, "dora-gpu daemon: forwarding: bad message: %s\n", ex.what());
    }
    if (job.data.kind == DATA_VEC) {
      e.has_data = true;
      e.data = std::move(job.data.vec);
    } else if (job.data.kind == DATA_SHMEM) {
      // a host-only node's shared-memory sample: copied out, then the token goes back
      e.has_data = true;
      const bool ok = read_shmem(job.data.shm.name, job.data.shm.len, &e.data);
      {
        std::lock_guard<std::mutex> g(mu_);
        released_.push_back(job.data.shm.token);
      }
      if (!ok) {
        std::fprintf(stderr, "dora-gpu daemon: could not read shared-memory sample `%s` of "
                             "`%s/%s` for remote receivers; dropped\n",
                     job.data.shm.name.c_str(), job.node_id.c_str(), job.output_id.c_str());
        return;
      }
    } else if (job.data.kind == DATA_DEVICE_IPC) {
      e.has_data = true;
      const bool ok = stage(job, &e.data, &e.type_info);
      (void)hipGetLastError();
      {
        std::lock_guard<std::mutex> g(mu_);
        released_.push_back(job.data.ipc.token);  // the producer may refill its slot now
      }
      if (!ok) {
        std::fprintf(stderr, "dora-gpu daemon: could not stage a device sample of `%s/%s` for "
                             "remote receivers; dropped\n",
                     job.node_id.c_str(), job.output_id.c_str());
        return;
      }
    }
  }
  std::vector<uint8_t> frame;
  try {
    encode_ide(e, frame);
  } catch (const std::exception& ex) {
    std::fprintf(stderr, "dora-gpu daemon: forwarding `%s/%s`: %s; dropped\n", job.node_id.c_str(),
                 job.output_id.c_str(), ex.what());
    return;
  }
  if (frame.size() > max_frame_bytes()) {
    std::fprintf(stderr,
                 "dora-gpu daemon: forwarding `%s/%s`: a %llu-byte frame exceeds the inter-daemon "
                 "frame limit (%llu bytes, DORA_GPU_MAX_FRAME_BYTES); dropped\n",
                 job.node_id.c_str(), job.output_id.c_str(),
                 static_cast<unsigned long long>(frame.size()),
                 static_cast<unsigned long long>(max_frame_bytes()));
    return;
  }
  for (const auto& m : job.machines) send_to(m, frame);
  forwarded_.fetch_add(1, std::memory_order_relaxed);
}

// ------------------------------------------------------------------------------------------
// Gateway
// ------------------------------------------------------------------------------------------
Gateway::Gateway(std::string shm_name, std::string dataflow_id, std::string listen_host,
                 int listen_port, std::vector<ProxySpec> proxies, InputSources input_src)
    : shm_(std::move(shm_name)),
      dataflow_id_(std::move(dataflow_id)),
      dataflow_uuid_(dataflow_uuid(dataflow_id_)),
      input_src_(std::move(input_src)) {
  listen_fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
  if (listen_fd_ < 0) throw std::runtime_error("gateway: socket");
  int one = 1;
  setsockopt(listen_fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons(static_cast<uint16_t>(listen_port));
  if (inet_pton(AF_INET, listen_host.c_str(), &a.sin_addr) != 1)
    throw std::invalid_argument("gateway: listen address " + listen_host);
  if (::bind(listen_fd_, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0 ||
      ::listen(listen_fd_, 16) != 0) {
    ::close(listen_fd_);
    throw std::runtime_error("gateway: cannot listen on " + listen_host + ":" +
                             std::to_string(listen_port) + ": " + std::strerror(errno));
  }
  socklen_t al = sizeof(a);
  getsockname(listen_fd_, reinterpret_cast<sockaddr*>(&a), &al);
  port_ = ntohs(a.sin_port);
  for (auto& ps : proxies) {
    auto p = std::make_unique<Proxy>();
    p->spec = ps;
    proxies_[ps.node_id] = std::move(p);
  }
  for (auto& kv : proxies_) {
    Proxy* p = kv.second.get();
    p->th = std::thread([this, p] { proxy_loop(p); });
  }
  accept_th_ = std::thread([this] { accept_loop(); });
}

Gateway::~Gateway() {
  stop_ = true;
  for (auto& kv : proxies_) kv.second->cv.notify_all();
  if (accept_th_.joinable()) accept_th_.join();
  {
    // only connections still open: a reader removes its fd under this lock before it closes
    // it, so no number here can belong to a later, unrelated socket
    std::lock_guard<std::mutex> g(readers_mu_);
    for (int fd : reader_fds_)
      if (fd >= 0) ::shutdown(fd, SHUT_RDWR);
  }
  for (auto& t : readers_)
    if (t.joinable()) t.join();
  for (auto& kv : proxies_)
    if (kv.second->th.joinable()) kv.second->th.join();
  if (listen_fd_ >= 0) ::close(listen_fd_);
}

bool Gateway::peers_gone() const {
  static const uint64_t grace_ns = [] {
    const char* e = std::getenv("DORA_GPU_PEER_GRACE_MS");
    return uint64_t(e ? std::strtoull(e, nullptr, 10) : 10000) * 1000000ull;
  }();
  return ever_connected_.load() && conns_.load() == 0 &&
         mono_ns() - last_disconnect_ns_.load() > grace_ns;
}

void Gateway::accept_loop() {
  while (!stop_) {
    pollfd pf{listen_fd_, POLLIN, 0};
    if (::poll(&pf, 1, 100) <= 0) continue;
    const int fd = ::accept(listen_fd_, nullptr, nullptr);
    if (fd < 0) continue;
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
    std::lock_guard<std::mutex> g(readers_mu_);
    conns_.fetch_add(1);
    ever_connected_.store(true);
    reader_fds_.push_back(fd);
    readers_.emplace_back([this, fd] { read_loop(fd); });
  }
}

void Gateway::read_loop(int fd) {
  std::vector<uint8_t> buf;
  while (!stop_) {
    uint64_t len = 0;
    if (!recv_all(fd, reinterpret_cast<uint8_t*>(&len), 8)) break;
    if (len > max_frame_bytes()) {  // a corrupt frame: drop this connection only
      std::fprintf(stderr, "dora-gpu daemon: inter-daemon frame of %llu bytes refused\n",
                   static_cast<unsigned long long>(len));
      break;
    }
    // The buffer grows as the bytes arrive, in steps of at most 64 MiB: a length prefix alone
    // (an unauthenticated peer's 8 bytes) commits no memory beyond the first step.
    constexpr uint64_t kStep = uint64_t(64) << 20;
    buf.clear();
    bool ok = true;
    try {
      while (ok && buf.size() < len) {
        const size_t at = buf.size();
        const size_t n = size_t(std::min<uint64_t>(kStep, len - at));
        buf.resize(at + n);
        ok = recv_all(fd, buf.data() + at, n);
      }
    } catch (const std::bad_alloc&) {
      std::fprintf(stderr, "dora-gpu daemon: no memory for a %llu-byte inter-daemon frame\n",
                   static_cast<unsigned long long>(len));
      break;
    }
    if (!ok) break;
    InterDaemonEvent e;
    try {
      e = decode_ide(buf.data(), buf.size());
    } catch (const std::exception& ex) {
      std::fprintf(stderr, "dora-gpu daemon: bad inter-daemon frame: %s\n", ex.what());
      break;
    }
    if (e.dataflow_uuid != dataflow_uuid_) {
      std::fprintf(stderr, "dora-gpu daemon: event of another dataflow (this is `%s`) ignored\n",
                   dataflow_id_.c_str());
      continue;
    }
    auto deliver = [this](const std::string& node, InterDaemonEvent&& ev) {
      auto it = proxies_.find(node);
      if (it == proxies_.end()) return;  // no local receiver of that node
      Proxy* p = it->second.get();
      {
        std::lock_guard<std::mutex> g(p->mu);
        p->q.push_back(std::move(ev));
      }
      p->cv.notify_one();
    };
    received_.fetch_add(1, std::memory_order_relaxed);
    if (e.kind == IDE_INPUTS_CLOSED) {
      // the closed inputs -> the proxy outputs feeding them (lib.rs:581-592 closes the inputs;
      // here the proxy closes its output, which closes every local input it feeds)
      std::map<std::string, std::vector<std::string>> by_src;
      for (const auto& in : e.inputs) {
        auto s = input_src_.find(in);
        if (s != input_src_.end()) by_src[s->second.first].push_back(s->second.second);
      }
      for (auto& kv : by_src) {
        InterDaemonEvent c;
        c.kind = IDE_PROXY_CLOSE;
        c.outputs = std::move(kv.second);
        deliver(kv.first, std::move(c));
      }
      continue;
    }
    const std::string node = e.node_id;
    deliver(node, std::move(e));
  }
  {
    std::lock_guard<std::mutex> g(readers_mu_);
    for (int& r : reader_fds_)
      if (r == fd) r = -1;
  }
  ::close(fd);
  last_disconnect_ns_.store(mono_ns());
  conns_.fetch_sub(1);
}

void Gateway::proxy_loop(Proxy* p) {
  dora_node* n = nullptr;
  if (dora_node_init(shm_.c_str(), p->spec.node_id.c_str(), p->spec.device, &n) != DORA_OK) {
    std::fprintf(stderr, "dora-gpu daemon: proxy `%s`: %s\n", p->spec.node_id.c_str(),
                 dora_gpu_last_error());
    return;
  }
  std::vector<std::string> open(p->spec.outputs.begin(), p->spec.outputs.end());
  while (!open.empty()) {
    InterDaemonEvent e;
    {
      std::unique_lock<std::mutex> g(p->mu);
      p->cv.wait_for(g, std::chrono::milliseconds(100), [&] { return stop_ || !p->q.empty(); });
      if (p->q.empty()) {
        if (stop_) break;
        if (peers_gone()) {
          // the remote node's daemon went away without closing its outputs: close them here
          std::fprintf(stderr, "dora-gpu daemon: peers of proxy `%s` gone; closing its outputs\n",
                       p->spec.node_id.c_str());
          e.kind = IDE_PROXY_CLOSE;
          e.outputs = open;
        } else {
          continue;
        }
      } else {
        e = std::move(p->q.front());
        p->q.pop_front();
      }
    }

    if (e.kind == IDE_PROXY_CLOSE) {
      std::vector<const char*> ids;
      for (const auto& o : e.outputs) {
        auto k = std::find(open.begin(), open.end(), o);
        if (k == open.end()) continue;
        ids.push_back(k->c_str());
      }
      if (!ids.empty() && dora_node_close_outputs(n, ids.data(), ids.size()) != DORA_OK)
        std::fprintf(stderr, "dora-gpu daemon: proxy `%s`: %s\n", p->spec.node_id.c_str(),
                     dora_gpu_last_error());
      for (const auto& o : e.outputs)
        open.erase(std::remove(open.begin(), open.end(), o), open.end());
      continue;
    }
    dora_sample* s = nullptr;
    int rc = DORA_OK;
    if (e.has_data && !e.data.empty() && e.data.size() < 4096) {
      s = vec_sample(e.data.data(), e.data.size());  // below the zero-copy threshold: inline
    } else if (e.has_data && !e.data.empty()) {
      rc = dora_node_allocate_data_sample(n, e.data.size(), &s);
      if (rc == DORA_OK) {
        void* dst = dora_sample_data(s);
        if (p->spec.device >= 0) {
          const hipError_t he = hipMemcpy(dst, e.data.data(), e.data.size(), hipMemcpyHostToDevice);
          if (he != hipSuccess) rc = fail(DORA_ERR_HIP, "upload: %s", hipGetErrorString(he));
        } else {
          std::memcpy(dst, e.data.data(), e.data.size());
        }
      }
    }
    if (rc == DORA_OK)
      rc = proxy_send(n, e.output_id.c_str(), e.type_info.data(), e.type_info.size(),
                      e.parameters.data(), e.parameters.size(), s, e.timestamp_ns);
    else if (s)
      dora_sample_discard(n, s);
    if (rc != DORA_OK)
      std::fprintf(stderr, "dora-gpu daemon: proxy `%s` output `%s`: %s\n",
                   p->spec.node_id.c_str(), e.output_id.c_str(), dora_gpu_last_error());
  }
  dora_node_free(n);
}

}  // namespace dora
