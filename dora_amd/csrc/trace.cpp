#include "trace.h"

#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <vector>

#include "shm.h"

namespace dora {
namespace {

struct Rec {
  uint64_t t;
  DropToken tok;
  uint8_t p;
};

struct Tracer {
  const char* dir = std::getenv("DORA_GPU_TRACE");
  std::vector<Rec> buf;
  std::atomic<size_t> n{0};
  std::string who = "proc";
  std::mutex mu;
  bool flushed = false;
  Tracer() {
    if (dir) buf.resize(1u << 20);
  }
  ~Tracer() { flush(); }
  void flush() {
    std::lock_guard<std::mutex> g(mu);
    if (!dir || flushed) return;
    flushed = true;
    const std::string path = std::string(dir) + "/" + who + "-" + std::to_string(getpid()) +
                             ".trace.csv";
    FILE* f = std::fopen(path.c_str(), "w");
    if (!f) return;
    std::fprintf(f, "who,point,token,t_ns\n");
    const size_t m = std::min(n.load(), buf.size());
    for (size_t i = 0; i < m; ++i) {
      std::fprintf(f, "%s,%u,", who.c_str(), unsigned(buf[i].p));
      for (int k = 0; k < 16; ++k) std::fprintf(f, "%02x", buf[i].tok.b[k]);
      std::fprintf(f, ",%llu\n", (unsigned long long)buf[i].t);
    }
    std::fclose(f);
  }
};

Tracer& tracer() {
  static Tracer t;
  return t;
}

}  // namespace

bool trace_enabled() { return tracer().dir != nullptr; }

void trace(TracePoint p, const DropToken& t) {
  Tracer& tr = tracer();
  if (!tr.dir) return;
  const size_t i = tr.n.fetch_add(1, std::memory_order_relaxed);
  if (i < tr.buf.size()) tr.buf[i] = {now_ns(), t, p};
}

void trace_at(TracePoint p, const DropToken& t, uint64_t t_ns) {
  Tracer& tr = tracer();
  if (!tr.dir) return;
  const size_t i = tr.n.fetch_add(1, std::memory_order_relaxed);
  if (i < tr.buf.size()) tr.buf[i] = {t_ns, t, p};
}

void trace_set_name(const std::string& who) { tracer().who = who; }

void trace_flush() { tracer().flush(); }

}  // namespace dora
