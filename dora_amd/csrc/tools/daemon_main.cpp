// dora-gpu-daemon: runs the data-plane daemon of one local dataflow (the `dora daemon
// --run-dataflow` role of binaries/cli/src/main.rs:468-499, data plane only).
//   dora-gpu-daemon --shm /name --spec FILE [--ring-bytes N] [--timeout-ms T]
#include <time.h>

#include <csignal>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>

#include "dora_gpu.h"
#include "params.h"

static volatile sig_atomic_t g_stop = 0;
static uint64_t mono_ns_main() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return uint64_t(ts.tv_sec) * 1000000000ull + uint64_t(ts.tv_nsec);
}
static void on_signal(int) { g_stop = 1; }

int main(int argc, char** argv) {
  std::string shm, spec_file;
  size_t ring = 4u << 20;
  long long timeout_ms = -1;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto next = [&]() -> const char* { return i + 1 < argc ? argv[++i] : ""; };
    if (a == "--shm") shm = next();
    else if (a == "--spec") spec_file = next();
    else if (a == "--ring-bytes") ring = std::strtoull(next(), nullptr, 10);
    else if (a == "--timeout-ms") timeout_ms = std::atoll(next());
  }
  if (shm.empty() || spec_file.empty()) {
    std::fprintf(stderr, "usage: dora-gpu-daemon --shm /name --spec FILE\n");
    return 2;
  }
  std::ifstream f(spec_file);
  std::stringstream ss;
  ss << f.rdbuf();
  dora_daemon* d = nullptr;
  if (dora_daemon_create(shm.c_str(), ss.str().c_str(), ring, &d) != 0) {
    std::fprintf(stderr, "daemon: %s\n", dora_gpu_last_error());
    return 1;
  }
  std::signal(SIGTERM, on_signal);
  std::signal(SIGINT, on_signal);
  int port = -1;
  dora_daemon_listen_port(d, &port);
  std::printf("{\"daemon\": \"ready\", \"shm\": \"%s\", \"listen_port\": %d}\n", shm.c_str(),
              port);
  std::fflush(stdout);
  const uint64_t t_start = mono_ns_main();
  int rc;
  long long waited = 0;
  bool stop_sent = false;
  for (;;) {
    rc = dora_daemon_run(d, 200);
    if (rc != DORA_ERR_TIMEOUT) break;
    waited += 200;
    if (g_stop && !stop_sent) {  // ctrl-c: Event::Stop to every node, then keep routing
      dora_daemon_request_stop(d);
      stop_sent = true;
    }
    if (timeout_ms >= 0 && waited >= timeout_ms) break;
  }
  uint64_t routed = 0, pending = 0;
  dora_daemon_stats(d, &routed, &pending);
  uint64_t idle = 0;
  dora_gpu_busy_stats(&idle, nullptr);
  const double busy_us = (double(mono_ns_main() - t_start) - double(idle)) / 1e3;
  uint64_t fwd = 0, staged = 0, received = 0;
  dora_daemon_remote_stats(d, &fwd, &staged, &received);
  std::printf("{\"daemon\": \"done\", \"rc\": %d, \"routed\": %llu, \"pending_tokens\": %llu, "
              "\"busy_us\": %.1f, \"busy_us_per_routed\": %.3f, \"forwarded\": %llu, "
              "\"staged_bytes\": %llu, \"remote_received\": %llu, \"sched\": %s}\n",
              rc, (unsigned long long)routed, (unsigned long long)pending, busy_us,
              routed ? busy_us / double(routed) : 0.0, (unsigned long long)fwd,
              (unsigned long long)staged, (unsigned long long)received, sched_json().c_str());
  dora_daemon_free(d);
  return rc == 0 ? 0 : 1;
}
