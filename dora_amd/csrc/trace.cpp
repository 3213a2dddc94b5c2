#include "trace.h"

#include <sched.h>
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <mutex>
#include <vector>

#include "shm.h"
#include "subprof.h"

namespace dora {
namespace {

struct Rec {
  uint64_t t;
  DropToken tok;
  uint8_t p;
  int16_t cpu;  // the CPU the stamp was taken on (whose interrupts / sibling load it saw)
};

// DORA_GPU_TRACE=<dir>: per-message trace files in <dir> (and the sub-phase profile below);
// "subphases": the sub-phase profile alone
const char* trace_dir() {
  const char* e = std::getenv("DORA_GPU_TRACE");
  if (!e || !*e || std::strcmp(e, "0") == 0 || std::strcmp(e, "subphases") == 0) return nullptr;
  return e;
}

struct Tracer {
  const char* dir = trace_dir();
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
    std::fprintf(f, "who,point,token,t_ns,cpu\n");
    const size_t m = std::min(n.load(), buf.size());
    for (size_t i = 0; i < m; ++i) {
      std::fprintf(f, "%s,%u,", who.c_str(), unsigned(buf[i].p));
      for (int k = 0; k < 16; ++k) std::fprintf(f, "%02x", buf[i].tok.b[k]);
      std::fprintf(f, ",%llu,%d\n", (unsigned long long)buf[i].t, int(buf[i].cpu));
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
  if (i < tr.buf.size()) tr.buf[i] = {now_ns(), t, p, int16_t(sched_getcpu())};
}

void trace_at(TracePoint p, const DropToken& t, uint64_t t_ns) {
  Tracer& tr = tracer();
  if (!tr.dir) return;
  const size_t i = tr.n.fetch_add(1, std::memory_order_relaxed);
  if (i < tr.buf.size()) tr.buf[i] = {t_ns, t, p, int16_t(sched_getcpu())};
}

void trace_set_name(const std::string& who) { tracer().who = who; }

DropToken ts_key(uint64_t ts) {
  DropToken k;
  std::memcpy(k.b, &ts, 8);
  std::memset(k.b + 8, 0xff, 8);
  return k;
}

void trace_flush() { tracer().flush(); }

namespace {

const char* const kSubNames[SP_COUNT] = {
    "send_plan",    "alloc_tokens", "alloc_wait",   "alloc_slot",    "stream_query",
    "aql_pack",     "aql_args",     "aql_dispatch", "send_ti",       "send_tokens",
    "send_lookup",  "send_request", "send_track",   "recv_drain",    "recv_encode",
    "recv_dropold", "recv_finish",  "recv_release", "daemon_route",  "slot_flag",
    "sample_new",   "send_source_wait"};

struct SubProf {
  const bool on = g_subprof_on;
  std::atomic<uint64_t> ticks[SP_COUNT] = {};
  std::atomic<uint64_t> calls[SP_COUNT] = {};
  uint64_t tsc0 = __rdtsc(), ns0 = mono_ns();
  ~SubProf() {
    if (!on) return;
    const double ns_per_tick = double(mono_ns() - ns0) / double(__rdtsc() - tsc0);
    std::fprintf(stderr, "{\"subphases\": {");
    bool first = true;
    for (int k = 0; k < SP_COUNT; ++k) {
      const uint64_t c = calls[k].load();
      if (!c) continue;
      std::fprintf(stderr, "%s\"%s\": [%.1f, %llu]", first ? "" : ", ", kSubNames[k],
                   double(ticks[k].load()) * ns_per_tick / double(c), (unsigned long long)c);
      first = false;
    }
    std::fprintf(stderr, "}, \"pid\": %d}\n", int(getpid()));
  }
};

SubProf& subprof() {
  static SubProf p;
  return p;
}

}  // namespace

// DORA_GPU_TRACE set (a directory, or "subphases" for the sub-phase profile alone)
const bool g_subprof_on = [] {
  const char* e = std::getenv("DORA_GPU_TRACE");
  return e && *e && std::strcmp(e, "0") != 0;
}();

void subprof_add(int phase, uint64_t ticks) {
  SubProf& p = subprof();
  p.ticks[phase].fetch_add(ticks, std::memory_order_relaxed);
  p.calls[phase].fetch_add(1, std::memory_order_relaxed);
}

}  // namespace dora
