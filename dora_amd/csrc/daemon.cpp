// Local daemon: routes sample descriptors and drop tokens between the nodes of one dataflow.
//
// Restates the reference daemon's data-plane duties (binaries/daemon/src/lib.rs):
//   * send_out / send_output_to_local_receivers (:955-1003, :1314-1390): clone the Input event
//     (id, metadata, data) to every mapped receiver and register the receiver as pending on the
//     sample's drop token;
//   * ReportDrop (:890-917) + check_drop_token (:1642-1672): when no receiver is pending any
//     more, send NodeDropEvent::OutputDropped to the owner;
//   * CloseOutputs / OutputsDone -> InputClosed / AllInputsClosed;
//   * PendingNodes: nodes get Ready once every node of the dataflow has subscribed.
// Unlike the reference (F8, lib.rs:1361-1376) it never opens or copies a sample: device samples
// are routed as IPC handles, so the routing thread touches no payload bytes at all.  Outputs
// with receivers under another machine's daemon go through interdaemon.h: a forwarder thread
// stages them to the host and sends InterDaemonEvent::Output (lib.rs:976-1000); remote nodes
// feeding local inputs are proxy nodes of the gateway, which re-sends their messages here.
#include <signal.h>
#include <sys/types.h>

#include <cerrno>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <memory_resource>
#include <set>
#include <sstream>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

#include "bcast.h"
#include "common.h"
#include "interdaemon.h"
#include "dora_gpu.h"
#include "shm.h"
#include "subprof.h"
#include "trace.h"
#include "wire.h"

namespace dora {
namespace {

struct Receiver {
  int node;
  std::string input;
};

struct DNode {
  std::string id;
  std::set<std::string> outputs;
  std::map<std::string, uint32_t> queue_size;  // input -> queue size
  std::set<std::string> open_inputs;
  bool subscribed = false;
  bool done = false;
  bool all_closed_sent = false;
  std::deque<std::pair<uint32_t, std::vector<uint8_t>>> ev_overflow;    // events not yet in ring
  std::deque<std::pair<uint32_t, std::vector<uint8_t>>> drop_overflow;
};

// A sample's drop token: its owner and the receivers still holding it, with the number of
// inputs each was delivered (a node may map one output under several input ids: each delivery
// is released on its own, so the token returns only after the last one).  Up to kInline
// receivers live in the entry itself (C4's 1 -> 7 fan-out included), so routing a message
// allocates nothing for the refcount; wider fan-outs spill into `more`.
struct TokenInfo {
  static constexpr int kInline = 8;
  struct Hold {
    int32_t node;
    uint32_t count;
  };
  int owner = -1;
  uint32_t n = 0;  // entries of `inl` in use
  Hold inl[kInline];
  std::vector<Hold> more;

  Hold* find(int node) {
    for (uint32_t k = 0; k < n; ++k)
      if (inl[k].node == node) return &inl[k];
    for (Hold& h : more)
      if (h.node == node) return &h;
    return nullptr;
  }
  void add(int node) {
    if (Hold* h = find(node)) {
      ++h->count;
    } else if (n < kInline) {
      inl[n++] = {node, 1};
    } else {
      more.push_back({node, 1});
    }
  }
  void erase(Hold* h) {
    if (h >= inl && h < inl + n) {
      *h = inl[--n];
      if (!more.empty()) {  // keep the inline entries dense
        inl[n++] = more.back();
        more.pop_back();
      }
    } else {
      *h = more.back();
      more.pop_back();
    }
  }
  // One delivery to `node` released; false when `node` held none.
  bool release(int node) {
    Hold* h = find(node);
    if (!h) return false;
    if (--h->count == 0) erase(h);
    return true;
  }
  // Every delivery to `node` released (the node finished); false when it held none.
  bool release_all(int node) {
    Hold* h = find(node);
    if (!h) return false;
    erase(h);
    return true;
  }
  bool pending() const { return n != 0 || !more.empty(); }
};

}  // namespace

class Daemon {
 public:
  Daemon(const std::string& shm, const std::string& spec, uint64_t ring_cap) {
    parse(spec);
    std::vector<std::string> ids;
    for (auto& n : nodes_) ids.push_back(n.id);
    region_.reset(Region::create(shm, ids, ring_cap, dataflow_id_));
    for (size_t i = 0; i < nodes_.size(); ++i) {
      NodeEntry& e = region_->hdr()->nodes[i];
      std::string outs, ins;
      for (auto& o : nodes_[i].outputs) outs += (outs.empty() ? "" : ",") + o;
      for (auto& q : nodes_[i].queue_size)
        ins += (ins.empty() ? "" : ",") + q.first + "=" + std::to_string(q.second);
      if (outs.size() >= kListLen || ins.size() >= kListLen)
        throw std::invalid_argument("too many inputs/outputs on node " + nodes_[i].id);
      std::strncpy(e.outputs, outs.c_str(), kListLen - 1);
      std::strncpy(e.inputs, ins.c_str(), kListLen - 1);
      req_.emplace_back(region_.get(), &e.requests);
      ev_.emplace_back(region_.get(), &e.events);
      drop_.emplace_back(region_.get(), &e.drops);
    }
    bool any_remote = false;
    for (auto& m : remote_) any_remote |= !m.empty();
    if (any_remote) fwd_.reset(new Forwarder(region_.get(), dataflow_id_, peers_));
    if (listen_port_ >= 0 || !proxies_.empty())
      gw_.reset(new Gateway(shm, dataflow_id_, listen_host_, listen_port_ < 0 ? 0 : listen_port_,
                            proxies_, input_src_));
  }

  ~Daemon() {
    gw_.reset();  // proxies finish first (their outputs close), then the forwarder drains
    fwd_.reset();
  }

  int listen_port() const { return gw_ ? gw_->port() : -1; }
  uint64_t forwarded() const { return fwd_ ? fwd_->forwarded() : 0; }
  uint64_t staged_bytes() const { return fwd_ ? fwd_->staged_bytes() : 0; }
  uint64_t remote_received() const { return gw_ ? gw_->received() : 0; }

  // Returns 0 when every node is done, DORA_ERR_TIMEOUT after timeout_ms (<0: no timeout).
  int run(int64_t timeout_ms) {
    const uint64_t t0 = mono_ns();
    // The idle bookkeeping and the spin estimate persist across calls: the daemon binary calls
    // run() in 200 ms slices, and a fresh estimate (mean 0: the 200 us base budget) each slice
    // put the daemon to sleep before the next message of a 1 ms stream every 200 ms — ~1 % of
    // them then paid a futex wake, 11-13 us (the host 8 B p99, profiles/r06_inline_tail_*.json)
    uint64_t& idle_since = idle_since_;
    uint64_t& idle_from = idle_from_;
    uint64_t& last_liveness = last_liveness_;
    AdaptiveSpin& spin = spin_;  // spins through short idle gaps instead of sleeping (shm.h)
    uint64_t& last_spin = last_spin_;  // the previous spinning pass (0: not spinning)
    if (!idle_since) idle_since = t0;
    std::vector<uint8_t>& payload = payload_;
    RegionHdr* h = region_->hdr();
    bool placed = false;
    for (;;) {
      if (!placed) {  // move next to the GPU of the first node that started (numa_hint)
        const int32_t numa = h->numa_hint.load(std::memory_order_relaxed);
        if (numa >= 0) {
          placed = true;
          (void)pin_to_numa(numa, -1, &h->l3_cpu, int(h->n_nodes) + 1);
        }
      }
      bool work = false;
      for (size_t i = 0; i < nodes_.size(); ++i) {
        uint32_t kind;
        int budget = 64;
        while (budget-- > 0 && req_[i].try_pop(&kind, &payload)) {
          if (kind == REQ_SEND_MESSAGE) msg_spin_.arrived(mono_ns());
          handle(static_cast<int>(i), kind, payload);
          work = true;
        }
      }
      work |= flush_overflow();
      if (fwd_) {
        released_.clear();
        fwd_->take_released(&released_);
        for (const DropToken& t : released_) {
          auto it = tokens_.find(t);
          if (it != tokens_.end() && it->second.release(kForwarder)) check_drop_token(t);
        }
        work |= !released_.empty();
      }
      const uint64_t now = mono_ns();
      // idle time is accounted up to a slice's end once (idle_counted_), while the gap the spin
      // estimate observes runs on from idle_from across slices
      auto leave = [&](int rc) {
        if (idle_from && !work) {
          add_idle_ns(now - std::max(idle_from, idle_counted_));
          idle_counted_ = now;
        }
        return rc;
      };
      if (all_done()) return leave(DORA_OK);
      if (h->shutdown.load()) return leave(DORA_ERR_CLOSED);
      if (timeout_ms >= 0 && int64_t(now - t0) / 1000000 > timeout_ms)
        return leave(DORA_ERR_TIMEOUT);
      if (now - last_liveness > 200000000ull) {  // 200 ms: reap nodes whose process died
        check_liveness();
        last_liveness = now;
      }
      woke_ = false;  // only the pass right after a sleep routes "woken"
      if (work) {
        last_spin = 0;
        if (idle_from) {  // the spin/sleep that preceded this work
          add_idle_ns(now - std::max(idle_from, idle_counted_));
          spin.observe(now - idle_from);
        }
        idle_from = 0;
        idle_since = now;
        continue;
      }
      if (!idle_from) idle_from = now;
      // Time this thread spent off the CPU (descheduled) is not spinning: the window moves by
      // it, so being preempted does not put the daemon to sleep before the next message
      if (last_spin && now - last_spin > kOffCpuNs) idle_since += now - last_spin;
      last_spin = now;
      if (int64_t(now - idle_since) / 1000 < std::max(spin.budget_us(), msg_spin_.budget_us())) {
        __builtin_ia32_pause();
        continue;
      }
      last_spin = 0;
      h->daemon_sleeping.store(1, std::memory_order_seq_cst);
      std::atomic_thread_fence(std::memory_order_seq_cst);  // pairs with ring_doorbell's fence
      const uint32_t bell = h->doorbell.load(std::memory_order_seq_cst);
      bool empty = true;
      for (auto& r : req_) empty &= r.empty();
      if (empty) {
        futex_wait(&h->doorbell, bell, 20000);
        woke_ = true;
      }
      h->daemon_sleeping.store(0, std::memory_order_seq_cst);
      idle_since = mono_ns();
    }
  }

  void request_stop() {
    for (size_t i = 0; i < nodes_.size(); ++i) push_event(static_cast<int>(i), EV_STOP, {});
    flush_overflow();
  }

  uint64_t routed() const { return routed_; }
  uint64_t pending_tokens() const { return tokens_.size(); }

 private:
  void parse(const std::string& spec) {
    // Lines: "node <id>" | "output <node> <output>" |
    //        "input <node> <input> <src_node> <src_output> <queue_size>"
    std::istringstream in(spec);
    std::string line;
    std::map<std::string, int> idx;
    struct In {
      std::string node, input, src, out;
      uint32_t q;
    };
    std::vector<In> inputs;
    struct Remote {
      std::string node, out, machine;
      std::vector<std::pair<std::string, std::string>> inputs;  // receiver/input over there
    };
    std::vector<Remote> remote_lines;
    while (std::getline(in, line)) {
      std::istringstream ls(line);
      std::string kw;
      if (!(ls >> kw) || kw[0] == '#') continue;
      if (kw == "node") {
        DNode n;
        ls >> n.id;
        if (n.id.empty() || idx.count(n.id)) throw std::invalid_argument("bad node line: " + line);
        if (nodes_.size() >= kMaxNodes)
          throw std::invalid_argument("more than " + std::to_string(kMaxNodes) + " nodes");
        idx[n.id] = static_cast<int>(nodes_.size());
        nodes_.push_back(n);
        outputs_.emplace_back();
      } else if (kw == "output") {
        std::string node, out;
        ls >> node >> out;
        if (!idx.count(node)) throw std::invalid_argument("unknown node in: " + line);
        nodes_[idx[node]].outputs.insert(out);
      } else if (kw == "input") {
        In x;
        ls >> x.node >> x.input >> x.src >> x.out >> x.q;
        if (ls.fail()) throw std::invalid_argument("bad input line: " + line);
        inputs.push_back(x);
      } else if (kw == "dataflow") {
        ls >> dataflow_id_;
      } else if (kw == "listen") {  // listen <host> <port>: peer daemons connect here
        ls >> listen_host_ >> listen_port_;
        if (ls.fail()) throw std::invalid_argument("bad listen line: " + line);
      } else if (kw == "machine") {  // machine <name> <host> <port>: a peer daemon
        std::string name;
        PeerAddr a;
        ls >> name >> a.host >> a.port;
        if (ls.fail()) throw std::invalid_argument("bad machine line: " + line);
        peers_[name] = a;
      } else if (kw == "remote") {
        // remote <node> <output> <machine> <receiver>/<input>...: receivers over there
        Remote r;
        ls >> r.node >> r.out >> r.machine;
        if (ls.fail()) throw std::invalid_argument("bad remote line: " + line);
        std::string ri;
        while (ls >> ri) {
          const size_t slash = ri.find('/');
          if (slash == std::string::npos || slash == 0 || slash + 1 == ri.size())
            throw std::invalid_argument("bad remote input `" + ri + "` in: " + line);
          r.inputs.emplace_back(ri.substr(0, slash), ri.substr(slash + 1));
        }
        // without its receivers' inputs the output's close could name nothing for the peer
        // (InputsClosed), and the peer's proxies would never close
        if (r.inputs.empty())
          throw std::invalid_argument("remote line names no receiver/input: " + line);
        remote_lines.push_back(std::move(r));
      } else if (kw == "proxy") {  // proxy <node> <gpu>: a remote node feeding local inputs
        ProxySpec p;
        ls >> p.node_id >> p.device;
        if (ls.fail()) throw std::invalid_argument("bad proxy line: " + line);
        proxies_.push_back(p);
      } else {
        throw std::invalid_argument("unknown spec keyword: " + kw);
      }
    }
    for (auto& x : inputs) {
      if (!idx.count(x.node) || !idx.count(x.src))
        throw std::invalid_argument("input refers to unknown node: " + x.node + "/" + x.input);
      DNode& n = nodes_[idx[x.node]];
      n.queue_size[x.input] = x.q;
      n.open_inputs.insert(x.input);
      if (!nodes_[idx[x.src]].outputs.count(x.out))
        throw std::invalid_argument("input " + x.node + "/" + x.input + " maps unknown output " +
                                    x.src + "/" + x.out);
      outputs_[idx[x.src]][x.out].push_back({idx[x.node], x.input});
    }
    remote_.resize(nodes_.size());
    for (auto& r : remote_lines) {
      if (!idx.count(r.node) || !nodes_[idx[r.node]].outputs.count(r.out))
        throw std::invalid_argument("remote line names unknown output " + r.node + "/" + r.out);
      if (!peers_.count(r.machine))
        throw std::invalid_argument("remote line names unknown machine " + r.machine);
      remote_[idx[r.node]][r.out].push_back(r.machine);
      auto& ri = remote_inputs_[{r.node, r.out}][r.machine];
      ri.insert(ri.end(), r.inputs.begin(), r.inputs.end());
    }
    // local inputs fed by proxies (remote nodes): what an InputsClosed from their machine closes
    for (auto& x : inputs) {
      for (auto& p : proxies_)
        if (p.node_id == x.src) input_src_[{x.node, x.input}] = {x.src, x.out};
    }
    for (auto& p : proxies_) {
      if (!idx.count(p.node_id)) throw std::invalid_argument("proxy of unknown node " + p.node_id);
      const auto& outs = nodes_[idx[p.node_id]].outputs;
      p.outputs.assign(outs.begin(), outs.end());
    }
  }

  bool all_done() const {
    for (auto& n : nodes_)
      if (!n.done) return false;
    // messages still being staged / sent to other machines keep the daemon up
    return !nodes_.empty() && (!fwd_ || fwd_->idle());
  }

  void push_event(int node, uint32_t kind, std::vector<uint8_t> payload) {
    push_event_raw(node, kind, payload.data(), payload.size());
  }

  // Straight into the node's ring; copied only when the ring is full (overflow queue).
  void push_event_raw(int node, uint32_t kind, const uint8_t* p, size_t n) {
    DNode& d = nodes_[node];
    if (d.done) return;
    if (d.ev_overflow.empty() && ev_[node].try_push(kind, p, n)) return;
    d.ev_overflow.emplace_back(kind, std::vector<uint8_t>(p, p + n));
  }

  void push_drop(int node, const DropToken& t) {
    DNode& n = nodes_[node];
    if (n.done) return;
    if (n.drop_overflow.empty() && drop_[node].try_push(DROP_OUTPUT_DROPPED, t.b, sizeof(t.b)))
      return;
    n.drop_overflow.emplace_back(DROP_OUTPUT_DROPPED, std::vector<uint8_t>(t.b, t.b + sizeof(t.b)));
  }

  void push_drop_record(int node, uint32_t kind, std::vector<uint8_t> payload) {
    DNode& n = nodes_[node];
    if (n.done) return;
    if (n.drop_overflow.empty() && drop_[node].try_push(kind, payload.data(), payload.size()))
      return;
    n.drop_overflow.emplace_back(kind, std::move(payload));
  }

  bool flush_overflow() {
    bool any = false;
    for (size_t i = 0; i < nodes_.size(); ++i) {
      DNode& n = nodes_[i];
      while (!n.ev_overflow.empty()) {
        auto& f = n.ev_overflow.front();
        if (!ev_[i].try_push(f.first, f.second.data(), f.second.size())) break;
        n.ev_overflow.pop_front();
        any = true;
      }
      while (!n.drop_overflow.empty()) {
        auto& f = n.drop_overflow.front();
        if (!drop_[i].try_push(f.first, f.second.data(), f.second.size())) break;
        n.drop_overflow.pop_front();
        any = true;
      }
    }
    return any;
  }

  void handle(int i, uint32_t kind, const std::vector<uint8_t>& payload) {
    SubSpan sp(SP_DAEMON_ROUTE);
    RBuf r(payload);
    switch (kind) {
      case REQ_SUBSCRIBE:
        nodes_[i].subscribed = true;
        region_->hdr()->nodes[i].state.store(1);
        if (ready_sent_) {
          push_event(i, EV_READY, ready_payload(i));
        } else {
          bool all = true;
          for (auto& n : nodes_) all &= n.subscribed || n.done;
          if (all) send_ready();
        }
        break;
      case REQ_SEND_MESSAGE: {
        // [str output][bytes metadata][data]: the event a receiver gets is [str input] + the
        // same metadata and data bytes, forwarded verbatim
        const uint64_t olen = r.u64();
        r.need(olen);
        const std::string_view output(reinterpret_cast<const char*>(r.ptr()), olen);
        r.skip(olen);
        const size_t tail = r.pos();
        r.skip(r.u64());  // metadata
        const DataMsg data = r.data();
        send_out(i, output, payload.data() + tail, payload.size() - tail, data);
        break;
      }
      case REQ_REPORT_DROP_TOKENS: {
        const uint32_t n = r.u32();
        for (uint32_t k = 0; k < n; ++k) {
          const DropToken t = r.token();
          auto it = tokens_.find(t);
          if (it == tokens_.end()) continue;  // unknown drop token (warned in the reference)
          if (it->second.release(i)) check_drop_token(t);
        }
        break;
      }
      case REQ_CLOSE_OUTPUTS: {
        const uint32_t n = r.u32();
        for (uint32_t k = 0; k < n; ++k) close_output(i, r.str());
        break;
      }
      case REQ_OUTPUTS_DONE:
        node_done(i);
        break;
      case REQ_BCAST_GROUP: {
        const std::string output = r.str();
        uint8_t uid[kBcastIdBytes];
        r.raw(uid, sizeof(uid));
        bcast_group(i, output, uid);
        break;
      }
      default:
        break;
    }
  }

  // send_output_to_local_receivers (lib.rs:1314-1390), minus the F8 payload copy.
  // `tail`: the message's metadata + data bytes as the sender encoded them.
  void send_out(int i, std::string_view output, const uint8_t* tail, size_t tail_len,
                const DataMsg& data) {
    ++routed_;
    TokenInfo* ti = nullptr;
    if (data.has_token()) {  // inserted even with no local receivers
      ti = &tokens_[data.token()];
      ti->owner = i;
    }
    auto it = outputs_[i].find(output);
    if (it != outputs_[i].end()) {
      for (const Receiver& rc : it->second) {
        DNode& rn = nodes_[rc.node];
        if (!rn.subscribed || rn.done || !rn.open_inputs.count(rc.input)) continue;
        ev_buf_.clear();
        ev_buf_.str(rc.input);
        ev_buf_.raw(tail, tail_len);
        push_event_raw(rc.node, EV_INPUT, ev_buf_.data(), ev_buf_.size());
        if (ti) {
          trace(woke_ ? TP_ROUTED_WOKE : TP_ROUTED, data.token());
          ti->add(rc.node);
        } else if (trace_enabled() && tail_len >= 18) {
          uint64_t ts;  // an inline sample: keyed by its metadata timestamp (u64 len, u16, u64)
          std::memcpy(&ts, tail + 10, 8);
          trace(woke_ ? TP_ROUTED_WOKE : TP_ROUTED, ts_key(ts));
        }
      }
    }
    auto rit = remote_[i].find(output);
    if (fwd_ && rit != remote_[i].end()) {
      // receivers under other daemons (lib.rs:976-1000): the forwarder stages and sends it;
      // it holds the token until its copy is done
      ForwardJob job;
      job.machines = rit->second;
      job.node_id = nodes_[i].id;
      job.output_id = std::string(output);
      job.tail.assign(tail, tail + tail_len);
      job.data = data;
      if (ti) ti->add(kForwarder);
      fwd_->push(std::move(job));
    }
    if (ti) check_drop_token(data.token());
  }

  // REQ_BCAST_GROUP (bcast.h): admit an RCCL group for output `output` of node `i` when every
  // receiver runs on its own GPU and none on the producer's (one rank per device), then tell the
  // receivers their ranks and the producer the group size (0: no group, receivers pull).
  void bcast_group(int i, const std::string& output, const uint8_t* uid) {
    RegionHdr* h = region_->hdr();
    const int32_t root_dev = h->nodes[i].device.load();
    std::set<int32_t> devs{root_dev};
    std::vector<Receiver> members;
    // outputs with receivers on other machines stay on pulls: their forwarder reads the slot
    bool ok = root_dev >= 0 && nodes_[i].outputs.count(output) && !remote_[i].count(output);
    auto it = outputs_[i].find(output);
    if (ok && it != outputs_[i].end()) {
      for (const Receiver& rc : it->second) {
        const DNode& rn = nodes_[rc.node];
        const int32_t d = h->nodes[rc.node].device.load();
        if (!rn.subscribed || rn.done || !rn.open_inputs.count(rc.input) || d < 0 ||
            !devs.insert(d).second) {
          ok = false;
          break;
        }
        members.push_back(rc);
      }
    }
    ok = ok && !members.empty();
    const uint32_t nranks = ok ? static_cast<uint32_t>(members.size() + 1) : 0;
    for (uint32_t k = 0; ok && k < members.size(); ++k) {
      WBuf w;
      w.str(members[k].input);
      w.raw(uid, kBcastIdBytes);
      w.u32(nranks);
      w.u32(k + 1);
      push_event(members[k].node, EV_BCAST_JOIN, w.take());
    }
    WBuf a;
    a.str(output);
    a.u32(nranks);
    push_drop_record(i, DROP_BCAST_GROUP, a.take());
  }

  void check_drop_token(const DropToken& t) {
    auto it = tokens_.find(t);
    if (it == tokens_.end() || it->second.pending()) return;
    const int owner = it->second.owner;
    tokens_.erase(it);
    push_drop(owner, t);
    trace(TP_TOKEN_DONE, t);
  }

  void close_output(int i, const std::string& output) {
    if (!nodes_[i].outputs.erase(output)) return;
    auto rit = remote_[i].find(output);
    if (fwd_ && rit != remote_[i].end()) {
      ForwardJob job;
      job.machines = rit->second;
      job.node_id = nodes_[i].id;
      job.closed = true;
      auto ri = remote_inputs_.find({nodes_[i].id, output});
      if (ri != remote_inputs_.end()) job.closed_inputs = ri->second;
      fwd_->push(std::move(job));
    }
    auto it = outputs_[i].find(output);
    if (it == outputs_[i].end()) return;
    for (const Receiver& rc : it->second) {
      DNode& rn = nodes_[rc.node];
      if (!rn.open_inputs.erase(rc.input)) continue;
      WBuf w;
      w.str(rc.input);
      push_event(rc.node, EV_INPUT_CLOSED, w.take());
      if (rn.open_inputs.empty() && !rn.all_closed_sent) {
        rn.all_closed_sent = true;
        push_event(rc.node, EV_ALL_INPUTS_CLOSED, {});
      }
    }
  }

  void node_done(int i) {
    std::vector<std::string> outs(nodes_[i].outputs.begin(), nodes_[i].outputs.end());
    for (auto& o : outs) close_output(i, o);
    nodes_[i].done = true;
    nodes_[i].ev_overflow.clear();
    nodes_[i].drop_overflow.clear();
    region_->hdr()->nodes[i].state.store(2);
    // a finished receiver holds nothing any more: release its pending tokens
    std::vector<DropToken> touched;
    for (auto& kv : tokens_)
      if (kv.second.release_all(i)) touched.push_back(kv.first);
    for (auto& t : touched) check_drop_token(t);
    if (!ready_sent_) {  // a node that exits before subscribing must not stall the others
      bool all = true;
      for (auto& n : nodes_) all &= n.subscribed || n.done;
      if (all) send_ready();
    }
  }

  // AllNodesReady (the reference's PendingNodes, daemon pending.rs): every node has subscribed
  // (or exited), so every node's GPU is known.
  void send_ready() {
    ready_sent_ = true;
    for (size_t k = 0; k < nodes_.size(); ++k)
      push_event(static_cast<int>(k), EV_READY, ready_payload(static_cast<int>(k)));
  }

  // EV_READY's payload for node i: its outputs whose every receiver is a running local node
  // without a GPU (DORA_GPU_DEVICE < 0) — such samples are wanted in host memory only, so the
  // producer packs them straight into shared memory (node.cpp pack_and_send) instead of into
  // an HBM slot each receiver would copy out.  [u32 n][str output] x n.
  std::vector<uint8_t> ready_payload(int i) {
    std::vector<const std::string*> outs;
    for (const auto& kv : outputs_[size_t(i)]) {
      if (remote_[size_t(i)].count(kv.first)) continue;
      size_t live = 0;
      bool host = true;
      for (const Receiver& rc : kv.second) {
        if (nodes_[size_t(rc.node)].done) continue;
        ++live;
        host &= region_->hdr()->nodes[rc.node].device.load() == -1;
      }
      if (live && host) outs.push_back(&kv.first);
    }
    if (outs.empty()) return {};
    WBuf w;
    w.u32(static_cast<uint32_t>(outs.size()));
    for (const std::string* o : outs) w.str(*o);
    return w.take();
  }

  void check_liveness() {
    for (size_t i = 0; i < nodes_.size(); ++i) {
      if (nodes_[i].done) continue;
      const int32_t pid = region_->hdr()->nodes[i].pid.load();
      if (pid > 0 && kill(pid, 0) != 0 && errno == ESRCH) node_done(static_cast<int>(i));
    }
  }

  std::unique_ptr<Region> region_;
  std::vector<DNode> nodes_;
  // per node: output -> receivers (heterogeneous lookup: no string built per message)
  std::vector<std::map<std::string, std::vector<Receiver>, std::less<>>> outputs_;
  // tokens in flight; nodes come from a pool (no malloc per routed message)
  std::pmr::unsynchronized_pool_resource token_pool_;
  std::pmr::unordered_map<DropToken, TokenInfo, DropTokenHash> tokens_{&token_pool_};
  WBuf ev_buf_;  // event encoding scratch, reused
  // inter-daemon (interdaemon.h): per node, output -> machines with receivers; peers; proxies
  static constexpr int kForwarder = -2;  // the forwarder's hold on a drop token
  std::vector<std::map<std::string, std::vector<std::string>, std::less<>>> remote_;
  // (node, output) -> machine -> its receivers' (node, input): InputsClosed when it closes
  std::map<std::pair<std::string, std::string>,
           std::map<std::string, std::vector<std::pair<std::string, std::string>>>>
      remote_inputs_;
  Gateway::InputSources input_src_;
  std::map<std::string, PeerAddr> peers_;
  std::vector<ProxySpec> proxies_;
  std::string dataflow_id_ = "local", listen_host_ = "127.0.0.1";
  bool woke_ = false;  // this loop pass follows a futex sleep (message trace)
  // run()'s loop state, kept between calls
  uint64_t idle_since_ = 0, idle_from_ = 0, last_liveness_ = 0, last_spin_ = 0, idle_counted_ = 0;
  AdaptiveSpin spin_;
  MessageSpin msg_spin_;  // data messages' spacing alone (shm.h)
  std::vector<uint8_t> payload_;
  int listen_port_ = -1;
  std::unique_ptr<Forwarder> fwd_;
  std::unique_ptr<Gateway> gw_;
  std::vector<DropToken> released_;
  std::vector<RingReader> req_;
  std::vector<RingWriter> ev_, drop_;
  bool ready_sent_ = false;
  uint64_t routed_ = 0;
};

}  // namespace dora

struct dora_daemon {
  std::unique_ptr<dora::Daemon> d;
};

extern "C" {

int dora_daemon_create(const char* shm_name, const char* spec, size_t ring_bytes,
                       dora_daemon** out) {
  if (!shm_name || !spec || !out) return dora::fail(DORA_ERR_INVALID, "NULL argument");
  DORA_GUARD_BEGIN
  auto* d = new dora_daemon();
  d->d.reset(new dora::Daemon(shm_name, spec, ring_bytes ? ring_bytes : (4u << 20)));
  dora::trace_set_name("daemon");
  *out = d;
  return DORA_OK;
  DORA_GUARD_END
}

int dora_daemon_run(dora_daemon* d, int64_t timeout_ms) {
  if (!d) return dora::fail(DORA_ERR_INVALID, "NULL daemon");
  DORA_GUARD_BEGIN
  int rc = d->d->run(timeout_ms);
  if (rc == DORA_ERR_TIMEOUT) return dora::fail(rc, "daemon run timed out");
  return rc;
  DORA_GUARD_END
}

int dora_daemon_request_stop(dora_daemon* d) {
  if (!d) return dora::fail(DORA_ERR_INVALID, "NULL daemon");
  d->d->request_stop();
  return DORA_OK;
}

int dora_daemon_stats(dora_daemon* d, uint64_t* routed, uint64_t* pending_tokens) {
  if (!d) return dora::fail(DORA_ERR_INVALID, "NULL daemon");
  if (routed) *routed = d->d->routed();
  if (pending_tokens) *pending_tokens = d->d->pending_tokens();
  return DORA_OK;
}

int dora_daemon_listen_port(dora_daemon* d, int* port) {
  if (!d || !port) return dora::fail(DORA_ERR_INVALID, "NULL argument");
  *port = d->d->listen_port();
  return DORA_OK;
}

int dora_daemon_remote_stats(dora_daemon* d, uint64_t* forwarded, uint64_t* staged_bytes,
                             uint64_t* received) {
  if (!d) return dora::fail(DORA_ERR_INVALID, "NULL daemon");
  if (forwarded) *forwarded = d->d->forwarded();
  if (staged_bytes) *staged_bytes = d->d->staged_bytes();
  if (received) *received = d->d->remote_received();
  return DORA_OK;
}

void dora_daemon_free(dora_daemon* d) {
  delete d;
  dora::trace_flush();
}

}  // extern "C"
