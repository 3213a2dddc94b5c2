// Inter-daemon data path: outputs whose receivers run under another machine's
// daemon, the counterpart of `InterDaemonEvent` (libraries/message/src/daemon_to_daemon.rs:9-21)
// and of the forwarding in `send_out` (binaries/daemon/src/lib.rs:955-1000).
//
// Sending side (Forwarder): the daemon hands every message of such an output to one forwarder
// thread, in routing order.  A device sample is staged to the host there — wait for the
// producer's fill (flag / event), map the slot (IPC, cached), one D2H copy — its validity
// tail folded back into the inline ArrowTypeInfo, and the producer's drop token released
// once the copy is done.  The message then leaves over a TCP connection per peer machine.
// The daemon's routing thread never waits on any of this.
//
// Receiving side (Gateway): a listener accepts peer daemons; every remote source node that
// feeds a local input has a proxy node in the local region, served by a thread of the gateway:
// it re-sends each remote message on the proxy's output (a device sample uploaded H2D for GPU
// proxies, an inline sample for host-only ones), so local receivers see an ordinary input;
// InputsClosed closes the proxy outputs feeding the named inputs and, once all are closed,
// finishes the proxy.
//
// Wire: the reference's — one frame = u64 little-endian length + bincode of
// Timestamped<InterDaemonEvent> (bincode.h); InputsClosed names the receivers' inputs on the
// machine it is sent to (lib.rs:1398-1440), which the receiving daemon maps to the proxy outputs
// feeding them.
#pragma once

#include <array>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "shm.h"
#include "wire.h"

namespace dora {

// InterDaemonEvent variants (wire indices), and the gateway's own close request to a proxy
enum : uint8_t { IDE_OUTPUT = 0, IDE_INPUTS_CLOSED = 1, IDE_PROXY_CLOSE = 2 };

struct InterDaemonEvent {
  uint8_t kind = IDE_OUTPUT;
  std::string dataflow_id;                  // sending: this dataflow's id (bincode.h dataflow_uuid)
  std::array<uint8_t, 16> dataflow_uuid{};  // received
  std::string node_id, output_id;           // Output
  std::vector<std::pair<std::string, std::string>> inputs;  // InputsClosed: (receiver, input)
  std::vector<std::string> outputs;         // IDE_PROXY_CLOSE: the proxy outputs to close
  uint16_t meta_version = 0;
  uint64_t timestamp_ns = 0;                // Metadata.timestamp (UNIX ns)
  uint64_t event_ns = 0;                    // Timestamped.timestamp (UNIX ns)
  std::array<uint8_t, 16> hlc_id{};         // the sending daemon's uhlc ID (non-zero)
  std::vector<uint8_t> type_info, parameters;
  bool has_data = false;
  std::vector<uint8_t> data;
};

struct PeerAddr {
  std::string host;
  int port = 0;
};

// One message of a local output with remote receivers, as the daemon routed it.
struct ForwardJob {
  std::vector<std::string> machines;
  std::string node_id, output_id;
  std::vector<uint8_t> tail;  // the request's metadata + data bytes (REQ_SEND_MESSAGE tail)
  DataMsg data;
  bool closed = false;  // InputsClosed instead of a message: per machine, its inputs to close
  std::map<std::string, std::vector<std::pair<std::string, std::string>>> closed_inputs;
};

class Forwarder {
 public:
  Forwarder(Region* region, std::string dataflow_id, std::map<std::string, PeerAddr> peers);
  ~Forwarder();
  void push(ForwardJob job);
  // Drop tokens whose staging is done (the daemon releases the forwarder's hold on them).
  void take_released(std::vector<DropToken>* out);
  bool idle();  // queue empty and nothing in progress
  uint64_t forwarded() const { return forwarded_.load(); }
  uint64_t staged_bytes() const { return staged_bytes_.load(); }

 private:
  void loop();
  void handle(ForwardJob& job);
  bool stage(const ForwardJob& job, std::vector<uint8_t>* bytes, std::vector<uint8_t>* ti);
  bool send_to(const std::string& machine, const std::vector<uint8_t>& frame);

  Region* region_;
  std::string dataflow_id_;
  std::map<std::string, PeerAddr> peers_;
  std::map<std::string, int> socks_;
  std::map<std::string, uint64_t> down_until_;  // a peer that refused us: skip it until then
  std::array<uint8_t, 16> hlc_id_{};             // this daemon's uhlc ID (random, non-zero)
  std::mutex mu_;
  std::condition_variable cv_;
  std::deque<ForwardJob> q_;
  std::vector<DropToken> released_;
  bool busy_ = false, stop_ = false;
  std::atomic<uint64_t> forwarded_{0}, staged_bytes_{0};
  // staging: IPC mappings of producers' slots, a pinned host buffer
  std::map<std::string, void*> maps_;
  uint8_t* pinned_ = nullptr;
  uint64_t pinned_cap_ = 0;
  std::thread th_;
};

// A remote source node served locally: its id, the local GPU its re-sent samples go to (-1:
// host-only) and its outputs.
struct ProxySpec {
  std::string node_id;
  int device = -1;
  std::vector<std::string> outputs;
};

class Gateway {
 public:
  // `input_src`: the local inputs fed by remote nodes, (receiver, input) -> (source, output)
  using InputSources =
      std::map<std::pair<std::string, std::string>, std::pair<std::string, std::string>>;
  Gateway(std::string shm_name, std::string dataflow_id, std::string listen_host, int listen_port,
          std::vector<ProxySpec> proxies, InputSources input_src);
  ~Gateway();
  int port() const { return port_; }
  uint64_t received() const { return received_.load(); }

 private:
  struct Proxy {
    ProxySpec spec;
    std::mutex mu;
    std::condition_variable cv;
    std::deque<InterDaemonEvent> q;
    std::thread th;
  };
  void accept_loop();
  void read_loop(int fd);
  void proxy_loop(Proxy* p);

  std::string shm_, dataflow_id_;
  std::array<uint8_t, 16> dataflow_uuid_{};
  InputSources input_src_;
  int listen_fd_ = -1, port_ = 0;
  std::atomic<bool> stop_{false};
  // peer connections: once every peer that connected has gone for longer than the grace period
  // (DORA_GPU_PEER_GRACE_MS, default 10 s) the proxies close their outputs — a crashed remote
  // daemon never sends InputsClosed, and the local dataflow must still finish
  std::atomic<int> conns_{0};
  std::atomic<bool> ever_connected_{false};
  std::atomic<uint64_t> last_disconnect_ns_{0};
  bool peers_gone() const;
  std::map<std::string, std::unique_ptr<Proxy>> proxies_;
  std::thread accept_th_;
  std::mutex readers_mu_;
  std::vector<std::thread> readers_;
  std::vector<int> reader_fds_;
  std::atomic<uint64_t> received_{0};
};

}  // namespace dora
