// TEST INFRASTRUCTURE ONLY — CPU baseline: a faithful C++ restatement of the reference's
// shared-memory data path, timed on the host cores beside the MI355X numbers.
// Never linked into the product; `bench.py`'s cpu_baseline leg runs it.
//
// Restated behaviour (reference v0.3.6):
//  sender  DoraNode::send_output_raw (apis/rust/node/src/node/mod.rs:180-196):
//          allocate_data_sample: >= 4096 B -> best-fit from a 20-entry cache of recycled shm
//          regions else shm_open+ftruncate+mmap (mod.rs:303-346, 364-371); < 4096 B -> zeroed
//          Vec; memcpy the payload; HLC timestamp after the fill (mod.rs:258); SendMessage over
//          TCP 127.0.0.1 with a u64 LE length prefix, two writes, no reply
//          (daemon_connection/tcp.rs:15-29, 82-88); region kept until its drop token returns;
//          a DropStream thread long-polls NextFinishedDropTokens (node/drop_stream.rs:93-141).
//  daemon  send_output_to_local_receivers (binaries/daemon/src/lib.rs:1314-1390): queue the
//          Input for the sink, register the pending drop token, and open + copy every shm
//          output into a fresh Vec (F8, lib.rs:1361-1376); drop_oldest_inputs with queue_size 10
//          (node_communication/mod.rs:320-359); NextEvent replies with all queued events
//          (:445-473); ReportDrop -> check_drop_token -> OutputDropped (lib.rs:890-917,1642-1672).
//  sink    examples/benchmark/sink: NextEvent{drop_tokens} request/reply, MappedInputData::map
//          per shm message (event_stream/event.rs:105-115), latency = now - metadata timestamp;
//          the token of a dropped input rides on the next NextEvent (event_stream/thread.rs:96-101).
// Each of the three processes is pinned to its own core (`--cores a,b,c`).
//
// Usage: shm_baseline --sizes 4096,40960000 --lat-n 50 --lat-gap-us 2000 --tp-n 50 --cores 0,1,2
// Prints one JSON document to stdout.
#include <arpa/inet.h>
#include <fcntl.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <poll.h>
#include <sched.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <mutex>
#include <random>
#include <set>
#include <string>
#include <thread>
#include <vector>

namespace {

uint64_t now_ns() {
  timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  return uint64_t(ts.tv_sec) * 1000000000ull + uint64_t(ts.tv_nsec);
}

void pin(int core) {
  if (core < 0) return;
  cpu_set_t s;
  CPU_ZERO(&s);
  CPU_SET(core, &s);
  sched_setaffinity(0, sizeof(s), &s);
}

// ---- framing (u64 LE length + payload, two writes like tcp_send) ----------------------------
bool write_all(int fd, const void* p, size_t n) {
  const char* c = static_cast<const char*>(p);
  while (n) {
    ssize_t k = write(fd, c, n);
    if (k <= 0) return false;
    c += k;
    n -= size_t(k);
  }
  return true;
}
bool read_all(int fd, void* p, size_t n) {
  char* c = static_cast<char*>(p);
  while (n) {
    ssize_t k = read(fd, c, n);
    if (k <= 0) return false;
    c += k;
    n -= size_t(k);
  }
  return true;
}
bool send_msg(int fd, const std::vector<uint8_t>& m) {
  uint64_t n = m.size();
  return write_all(fd, &n, 8) && write_all(fd, m.data(), m.size());
}
bool recv_msg(int fd, std::vector<uint8_t>& m) {
  uint64_t n;
  if (!read_all(fd, &n, 8)) return false;
  m.resize(n);
  return read_all(fd, m.data(), n);
}

struct W {
  std::vector<uint8_t> b;
  void u8(uint8_t v) { b.push_back(v); }
  void u64(uint64_t v) { b.insert(b.end(), (uint8_t*)&v, (uint8_t*)&v + 8); }
  void raw(const void* p, size_t n) { b.insert(b.end(), (const uint8_t*)p, (const uint8_t*)p + n); }
  void str(const std::string& s) {
    u64(s.size());
    raw(s.data(), s.size());
  }
};
struct R {
  const uint8_t* p;
  size_t n, i = 0;
  uint8_t u8() { return p[i++]; }
  uint64_t u64() {
    uint64_t v;
    std::memcpy(&v, p + i, 8);
    i += 8;
    return v;
  }
  std::string str() {
    uint64_t k = u64();
    std::string s((const char*)p + i, k);
    i += k;
    return s;
  }
};

enum : uint8_t {
  REG_CONTROL = 1, REG_DROP = 2, REG_EVENTS = 3,
  SEND_MESSAGE = 10, NEXT_EVENT = 11, NEXT_FINISHED_DROP_TOKENS = 12, OUTPUTS_DONE = 13,
  DATA_VEC = 0, DATA_SHM = 1,
};

struct Token {
  uint64_t a, b;
  bool operator<(const Token& o) const { return a < o.a || (a == o.a && b < o.b); }
};

// An Input event as queued by the daemon: the SendMessage body forwarded as-is.
struct Input {
  uint8_t output;  // 0 latency, 1 throughput
  std::vector<uint8_t> body;
  bool has_token;
  Token token;
};

int connect_to(int port) {
  int fd = socket(AF_INET, SOCK_STREAM, 0);
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons(uint16_t(port));
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  for (int k = 0; k < 1000; ++k) {
    if (connect(fd, (sockaddr*)&a, sizeof(a)) == 0) break;
    usleep(1000);
  }
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  return fd;
}

// ---------------------------------------------------------------------------------------------
// daemon
// ---------------------------------------------------------------------------------------------
int run_daemon(int lfd) {
  std::vector<pollfd> fds;
  std::map<int, uint8_t> role;
  fds.push_back({lfd, POLLIN, 0});
  std::deque<Input> queue;
  std::map<Token, int> pending;  // token -> number of pending receivers (only the sink here)
  std::vector<Token> finished;
  int events_fd = -1, drop_fd = -1;
  bool sink_waiting = false, drop_waiting = false, done = false, closed_sent = false;
  const size_t queue_size = 10;  // spawn.rs:56 default
  std::vector<uint8_t> m;
  uint64_t f8_bytes = 0;

  auto check_token = [&](const Token& t) {
    auto it = pending.find(t);
    if (it != pending.end() && it->second == 0) {
      pending.erase(it);
      finished.push_back(t);
    }
  };
  auto reply_drop = [&]() {
    if (!drop_waiting || finished.empty()) return;
    W w;
    w.u64(finished.size());
    for (auto& t : finished) {
      w.u64(t.a);
      w.u64(t.b);
    }
    finished.clear();
    drop_waiting = false;
    send_msg(drop_fd, w.b);
  };
  auto reply_events = [&]() {
    if (!sink_waiting) return;
    if (queue.empty() && !(done && !closed_sent)) return;
    W w;
    w.u64(queue.size());
    for (auto& in : queue) {
      w.u8(in.output);
      w.u64(in.body.size());
      w.raw(in.body.data(), in.body.size());
    }
    queue.clear();
    w.u8(done ? 1 : 0);  // AllInputsClosed
    if (done) closed_sent = true;
    sink_waiting = false;
    send_msg(events_fd, w.b);
  };
  for (;;) {
    if (poll(fds.data(), fds.size(), 1000) < 0) return 1;
    for (size_t i = 0; i < fds.size(); ++i) {
      if (!(fds[i].revents & (POLLIN | POLLHUP))) continue;
      int fd = fds[i].fd;
      if (fd == lfd) {
        int c = accept(lfd, nullptr, nullptr);
        int one = 1;
        setsockopt(c, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
        fds.push_back({c, POLLIN, 0});
        role[c] = 0;
        continue;
      }
      if (!recv_msg(fd, m)) {
        fds[i].fd = -fd - 1;  // ignore from now on
        continue;
      }
      R r{m.data(), m.size()};
      const uint8_t kind = r.u8();
      if (kind == REG_CONTROL || kind == REG_DROP || kind == REG_EVENTS) {
        role[fd] = kind;
        if (kind == REG_DROP) drop_fd = fd;
        if (kind == REG_EVENTS) events_fd = fd;
      } else if (kind == SEND_MESSAGE) {
        Input in;
        in.output = r.u8();
        in.body.assign(m.begin() + 2, m.end());
        // body: ts, t_start, data kind, ...
        R b{in.body.data(), in.body.size()};
        b.u64();
        b.u64();
        const uint8_t dk = b.u8();
        in.has_token = dk == DATA_SHM;
        if (in.has_token) {
          const std::string name = b.str();
          const uint64_t len = b.u64();
          in.token.a = b.u64();
          in.token.b = b.u64();
          // F8: open the sender's region and copy `len` bytes into a fresh Vec
          int sfd = shm_open(name.c_str(), O_RDONLY, 0);
          if (sfd >= 0) {
            void* p = mmap(nullptr, len, PROT_READ, MAP_SHARED, sfd, 0);
            close(sfd);
            if (p != MAP_FAILED) {
              std::vector<uint8_t> copy((const uint8_t*)p, (const uint8_t*)p + len);
              f8_bytes += copy.size();
              munmap(p, len);
            }
          }
          pending[in.token] = 1;
        }
        queue.push_back(std::move(in));
        // drop_oldest_inputs: newest first, keep queue_size per output
        std::map<uint8_t, size_t> seen;
        std::deque<Input> kept;
        for (auto it = queue.rbegin(); it != queue.rend(); ++it) {
          if (seen[it->output]++ < queue_size) {
            kept.push_front(std::move(*it));
          } else if (it->has_token) {
            pending[it->token] = 0;
            check_token(it->token);
          }
        }
        queue.swap(kept);
        reply_events();
        reply_drop();
      } else if (kind == NEXT_EVENT) {
        const uint64_t nt = r.u64();
        for (uint64_t k = 0; k < nt; ++k) {
          Token t{r.u64(), r.u64()};
          auto it = pending.find(t);
          if (it != pending.end()) {
            it->second = 0;
            check_token(t);
          }
        }
        sink_waiting = true;
        reply_events();
        reply_drop();
      } else if (kind == NEXT_FINISHED_DROP_TOKENS) {
        drop_waiting = true;
        reply_drop();
      } else if (kind == OUTPUTS_DONE) {
        done = true;
        reply_events();
      }
    }
    if (closed_sent && pending.empty()) {
      // tell the drop stream we're done
      if (drop_fd >= 0 && drop_waiting) {
        W w;
        w.u64(UINT64_MAX);
        send_msg(drop_fd, w.b);
      }
      break;
    }
  }
  return 0;
}

// ---------------------------------------------------------------------------------------------
// sender
// ---------------------------------------------------------------------------------------------
struct Region {
  std::string name;
  void* p;
  size_t len;
};

int run_sender(int port, const std::vector<uint64_t>& sizes, int lat_n, int lat_gap_us, int tp_n) {
  int ctl = connect_to(port), dfd = connect_to(port);
  W reg;
  reg.u8(REG_CONTROL);
  send_msg(ctl, reg.b);
  W reg2;
  reg2.u8(REG_DROP);
  send_msg(dfd, reg2.b);

  std::mutex mu;
  std::deque<Token> returned;
  std::atomic<bool> drop_done{false};
  std::thread drop_thread([&] {  // DropStream::drop_stream_loop
    std::vector<uint8_t> m;
    for (;;) {
      W q;
      q.u8(NEXT_FINISHED_DROP_TOKENS);
      if (!send_msg(dfd, q.b) || !recv_msg(dfd, m)) break;
      R r{m.data(), m.size()};
      uint64_t n = r.u64();
      if (n == UINT64_MAX) break;
      std::lock_guard<std::mutex> g(mu);
      for (uint64_t k = 0; k < n; ++k) returned.push_back({r.u64(), r.u64()});
    }
    drop_done = true;
  });

  std::deque<Region> cache;
  std::map<Token, Region> sent_out;
  std::mt19937_64 rng(0xD05A);
  uint64_t region_counter = 0;
  auto handle_finished = [&] {
    std::lock_guard<std::mutex> g(mu);
    while (!returned.empty()) {
      Token t = returned.front();
      returned.pop_front();
      auto it = sent_out.find(t);
      if (it == sent_out.end()) continue;
      cache.push_back(it->second);
      sent_out.erase(it);
      while (cache.size() > 20) {
        Region& old = cache.front();
        munmap(old.p, old.len);
        shm_unlink(old.name.c_str());
        cache.pop_front();
      }
    }
  };
  auto allocate = [&](size_t len) -> Region {
    int best = -1;
    for (int i = int(cache.size()) - 1; i >= 0; --i)
      if (cache[size_t(i)].len >= len && (best < 0 || cache[size_t(i)].len < cache[size_t(best)].len))
        best = i;
    if (best >= 0) {
      Region r = cache[size_t(best)];
      cache.erase(cache.begin() + best);
      return r;
    }
    Region r;
    char nm[96];
    std::snprintf(nm, sizeof(nm), "/dora-base-%d-%llu", getpid(),
                  (unsigned long long)region_counter++);
    r.name = nm;
    r.len = len;
    int fd = shm_open(nm, O_CREAT | O_EXCL | O_RDWR, 0600);
    if (ftruncate(fd, off_t(len)) != 0) std::abort();
    r.p = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    return r;
  };

  std::map<uint64_t, std::vector<uint8_t>> payload;
  for (uint64_t s : sizes) {  // splitmix64(seed = 0xD05A + size)
    std::vector<uint8_t> v(s);
    uint64_t seed = 0xD05A + s;
    for (uint64_t i = 0; 8 * i < s; ++i) {
      uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
      z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
      z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
      z ^= z >> 31;
      std::memcpy(v.data() + 8 * i, &z, std::min<uint64_t>(8, s - 8 * i));
    }
    payload[s] = std::move(v);
  }

  auto send_one = [&](uint8_t output, uint64_t size) {
    const uint64_t t_start = now_ns();
    handle_finished();
    const std::vector<uint8_t>& data = payload[size];
    W w;
    w.u8(SEND_MESSAGE);
    w.u8(output);
    if (size >= 4096) {
      Region r = allocate(size);
      std::memcpy(r.p, data.data(), size);  // `out.copy_from_slice(data)`
      const uint64_t ts = now_ns();          // metadata timestamp after the fill
      Token t{rng(), rng()};
      w.u64(ts);
      w.u64(t_start);
      w.u8(DATA_SHM);
      w.str(r.name);
      w.u64(size);
      w.u64(t.a);
      w.u64(t.b);
      send_msg(ctl, w.b);
      sent_out[t] = r;
    } else {
      std::vector<uint8_t> v(size, 0);
      std::memcpy(v.data(), data.data(), size);
      const uint64_t ts = now_ns();
      w.u64(ts);
      w.u64(t_start);
      w.u8(DATA_VEC);
      w.u64(size);
      w.raw(v.data(), size);
      send_msg(ctl, w.b);
    }
  };
  for (uint64_t s : sizes)
    for (int k = 0; k < lat_n; ++k) {
      send_one(0, s);
      usleep(useconds_t(lat_gap_us));
    }
  usleep(2000000);  // "wait a bit to ensure that all throughput messages reached their target"
  for (uint64_t s : sizes)
    for (int k = 0; k < tp_n; ++k) send_one(1, s);
  W done;
  done.u8(OUTPUTS_DONE);
  send_msg(ctl, done.b);
  // Drop for DoraNode: wait for outstanding tokens
  for (int k = 0; k < 10000 && !sent_out.empty() && !drop_done; ++k) {
    handle_finished();
    usleep(1000);
  }
  handle_finished();
  drop_thread.join();
  for (auto& r : cache) {
    munmap(r.p, r.len);
    shm_unlink(r.name.c_str());
  }
  for (auto& kv : sent_out) {
    munmap(kv.second.p, kv.second.len);
    shm_unlink(kv.second.name.c_str());
  }
  return 0;
}

// ---------------------------------------------------------------------------------------------
// sink
// ---------------------------------------------------------------------------------------------
struct Series {
  std::vector<double> lat, full;
  uint64_t n = 0, first_start = 0, last_recv = 0;
};

double pct(std::vector<double> v, double p) {
  if (v.empty()) return 0;
  std::sort(v.begin(), v.end());
  return v[std::min(v.size() - 1, size_t(p * double(v.size() - 1) + 0.5))];
}

int run_sink(int port, int out_fd) {
  int fd = connect_to(port);
  W reg;
  reg.u8(REG_EVENTS);
  send_msg(fd, reg.b);
  std::vector<Token> to_report;
  std::map<std::pair<int, uint64_t>, Series> st;
  std::vector<uint8_t> m;
  for (;;) {
    W q;
    q.u8(NEXT_EVENT);
    q.u64(to_report.size());
    for (auto& t : to_report) {
      q.u64(t.a);
      q.u64(t.b);
    }
    to_report.clear();
    if (!send_msg(fd, q.b) || !recv_msg(fd, m)) break;
    R r{m.data(), m.size()};
    uint64_t n = r.u64();
    for (uint64_t k = 0; k < n; ++k) {
      const uint8_t output = r.u8();
      const uint64_t blen = r.u64();
      R b{r.p + r.i, blen};
      r.i += blen;
      const uint64_t ts = b.u64(), t_start = b.u64();
      const uint8_t dk = b.u8();
      uint64_t len = 0;
      if (dk == DATA_SHM) {
        const std::string name = b.str();
        len = b.u64();
        Token tok{b.u64(), b.u64()};
        // MappedInputData::map: shm open + mmap per message, zero-copy view
        int sfd = shm_open(name.c_str(), O_RDONLY, 0);
        void* p = sfd >= 0 ? mmap(nullptr, len, PROT_READ, MAP_SHARED, sfd, 0) : MAP_FAILED;
        if (sfd >= 0) close(sfd);
        const uint64_t t = now_ns();
        Series& s = st[{output, len}];
        s.lat.push_back(double(t - ts) / 1000.0);
        s.full.push_back(double(t - t_start) / 1000.0);
        if (!s.n) s.first_start = t_start;
        s.last_recv = t;
        ++s.n;
        if (p != MAP_FAILED) munmap(p, len);  // ArrowData dropped -> token released
        to_report.push_back(tok);
      } else {
        len = b.u64();
        const uint64_t t = now_ns();
        Series& s = st[{output, len}];
        s.lat.push_back(double(t - ts) / 1000.0);
        s.full.push_back(double(t - t_start) / 1000.0);
        if (!s.n) s.first_start = t_start;
        s.last_recv = t;
        ++s.n;
      }
    }
    const uint8_t closed = r.u8();
    if (closed) {
      // report the last tokens
      W q2;
      q2.u8(NEXT_EVENT);
      q2.u64(to_report.size());
      for (auto& t : to_report) {
        q2.u64(t.a);
        q2.u64(t.b);
      }
      send_msg(fd, q2.b);
      break;
    }
  }
  std::string js = "[";
  bool first = true;
  for (auto& kv : st) {
    Series& s = kv.second;
    const double dur = double(s.last_recv - s.first_start) / 1e9;
    char buf[512];
    std::snprintf(buf, sizeof(buf),
                  "%s{\"mode\": \"%s\", \"size\": %llu, \"n\": %llu, \"p50_us\": %.3f, "
                  "\"p99_us\": %.3f, \"full_p50_us\": %.3f, \"full_p99_us\": %.3f, "
                  "\"msgs_per_s\": %.1f, \"GBps\": %.4f}",
                  first ? "" : ",", kv.first.first ? "throughput" : "latency",
                  (unsigned long long)kv.first.second, (unsigned long long)s.n, pct(s.lat, 0.5),
                  pct(s.lat, 0.99), pct(s.full, 0.5), pct(s.full, 0.99),
                  dur > 0 ? double(s.n) / dur : 0.0,
                  dur > 0 ? double(s.n) * double(kv.first.second) / dur / 1e9 : 0.0);
    js += buf;
    first = false;
  }
  js += "]";
  write_all(out_fd, js.data(), js.size());
  close(out_fd);
  return 0;
}

std::vector<long long> parse_list(const char* s) {
  std::vector<long long> v;
  while (*s) {
    v.push_back(std::atoll(s));
    while (*s && *s != ',') ++s;
    if (*s == ',') ++s;
  }
  return v;
}

}  // namespace

int main(int argc, char** argv) {
  std::vector<uint64_t> sizes = {4096, 40960, 409600, 4096000, 40960000};
  int lat_n = 50, lat_gap_us = 10000, tp_n = 50;
  std::vector<long long> cores = {0, 1, 2};
  for (int i = 1; i + 1 < argc; i += 2) {
    std::string a = argv[i];
    if (a == "--sizes") {
      sizes.clear();
      for (long long x : parse_list(argv[i + 1])) sizes.push_back(uint64_t(x));
    } else if (a == "--lat-n") lat_n = std::atoi(argv[i + 1]);
    else if (a == "--lat-gap-us") lat_gap_us = std::atoi(argv[i + 1]);
    else if (a == "--tp-n") tp_n = std::atoi(argv[i + 1]);
    else if (a == "--cores") cores = parse_list(argv[i + 1]);
  }
  while (cores.size() < 3) cores.push_back(-1);
  int lfd = socket(AF_INET, SOCK_STREAM, 0);
  int one = 1;
  setsockopt(lfd, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  a.sin_port = 0;
  if (bind(lfd, (sockaddr*)&a, sizeof(a)) != 0 || listen(lfd, 16) != 0) return 1;
  socklen_t al = sizeof(a);
  getsockname(lfd, (sockaddr*)&a, &al);
  const int port = ntohs(a.sin_port);
  int pfd[2];
  if (pipe(pfd) != 0) return 1;
  const uint64_t t0 = now_ns();
  pid_t d = fork();
  if (d == 0) {
    pin(int(cores[0]));
    _exit(run_daemon(lfd));
  }
  pid_t s = fork();
  if (s == 0) {
    close(pfd[0]);
    pin(int(cores[2]));
    _exit(run_sink(port, pfd[1]));
  }
  close(pfd[1]);
  pid_t p = fork();
  if (p == 0) {
    pin(int(cores[1]));
    _exit(run_sender(port, sizes, lat_n, lat_gap_us, tp_n));
  }
  std::string out;
  char buf[4096];
  ssize_t k;
  while ((k = read(pfd[0], buf, sizeof(buf))) > 0) out.append(buf, size_t(k));
  int st;
  waitpid(p, &st, 0);
  waitpid(s, &st, 0);
  waitpid(d, &st, 0);
  std::printf("{\"baseline\": \"reference shm path restated (C++)\", \"processes\": 3, "
              "\"cores\": [%lld, %lld, %lld], \"nproc\": %ld, \"wall_s\": %.3f, \"series\": %s}\n",
              cores[0], cores[1], cores[2], sysconf(_SC_NPROCESSORS_ONLN),
              double(now_ns() - t0) / 1e9, out.empty() ? "[]" : out.c_str());
  return 0;
}
