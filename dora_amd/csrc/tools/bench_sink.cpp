// dora-gpu-bench-sink: the benchmark sink (examples/benchmark/sink/src/main.rs:6-87) on the
// device data plane.  For every input it records the latency from the sender's metadata
// timestamp (taken after the sample is filled, node/mod.rs:258) and, when the sender passes a
// `t_start` parameter, the latency including allocation + pack.  With `verify` it checksums the
// received device sample (csum64 kernel) against the sender's `csum` parameter.  Inputs with an
// `ack` parameter are acknowledged on the `ack` output (used by the bench to close a timed burst).
// With `verify_late` the input is held (its token not returned) and checksummed right after the
// next ack has gone out: the bench marks the last messages of its timed region so, and their
// bytes are verified without putting a checksum kernel inside the timed region.
// At the end of the stream it writes one JSON document with per-(input, size) statistics.
//   env: DORA_GPU_DATAFLOW, DORA_NODE_ID, DORA_GPU_DEVICE, DORA_BENCH_RESULT (path)
#include <algorithm>
#include <array>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "dora_gpu.h"
#include "params.h"

namespace {

struct Series {
  std::vector<double> lat_us, full_us;
  uint64_t first_ns = 0, last_ns = 0, n = 0, bytes = 0, verified = 0, mismatches = 0;
  // bursts: receipts between two acks (the source's barriers delimit its warmup, latency and
  // throughput phases); the longest one is the throughput phase, whose rate the bench reports
  uint64_t b_first = 0, b_last = 0, b_n = 0, tp_first = 0, tp_last = 0, tp_n = 0;
  void close_burst() {
    if (b_n > tp_n) {
      tp_n = b_n;
      tp_first = b_first;
      tp_last = b_last;
    }
    b_n = b_first = b_last = 0;
  }
};

double pct(std::vector<double> v, double p) {
  if (v.empty()) return 0;
  std::sort(v.begin(), v.end());
  size_t k = static_cast<size_t>(p * (v.size() - 1) + 0.5);
  return v[std::min(k, v.size() - 1)];
}

double mean(const std::vector<double>& v) {
  double s = 0;
  for (double x : v) s += x;
  return v.empty() ? 0 : s / v.size();
}

uint64_t mono() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return uint64_t(ts.tv_sec) * 1000000000ull + uint64_t(ts.tv_nsec);
}

// csum64 of host bytes (the csum_kernel's sum, include/dora_gpu.h dora_gpu_csum64), for inputs a
// receiver without a GPU got staged in host memory
uint64_t fmix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

uint64_t csum64_host(const uint8_t* p, size_t n) {
  constexpr uint64_t kGolden = 0x9E3779B97F4A7C15ull, kSeed = 0xD0A5D0A5D0A5D0A5ull;
  uint64_t s = 0;
  for (size_t i = 0; 8 * i < n; ++i) {
    uint64_t w = 0;
    std::memcpy(&w, p + 8 * i, std::min<size_t>(8, n - 8 * i));
    s += fmix64(w ^ (i * kGolden + kSeed));
  }
  return fmix64(s + n);
}

uint64_t now_ns() {
  timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  return uint64_t(ts.tv_sec) * 1000000000ull + uint64_t(ts.tv_nsec);
}

}  // namespace

int main() {
  dora_node* node = nullptr;
  if (dora_node_init_from_env(&node) != 0) {
    std::fprintf(stderr, "sink: init failed: %s\n", dora_gpu_last_error());
    return 1;
  }
  const char* out_path = std::getenv("DORA_BENCH_RESULT");
  std::map<std::pair<std::string, uint64_t>, Series> stats;
  uint64_t csum_buf_dummy = 0;
  (void)csum_buf_dummy;
  uint64_t* csum_dev = nullptr;
  dora_gpu_malloc(reinterpret_cast<void**>(&csum_dev), 8);
  // a stream of its own: every checksum below is synchronised before its input is released, so
  // the node stream stays unused and no release has to query it (node.cpp stream_used)
  dora_stream_t st = nullptr;
  const bool own_stream = dora_gpu_stream_create(&st) == 0;
  if (!own_stream) st = dora_node_stream(node);
  // the first checksum loads the kernel's code object (milliseconds): do it now, not while a
  // burst waits on this sink
  {
    uint64_t c = 0;
    if (csum_dev && dora_gpu_csum64(csum_dev, 8, csum_dev, st) == 0)
      (void)dora_gpu_memcpy_async(&c, csum_dev, 8, st);
    (void)dora_gpu_stream_sync(st);
  }
  int errors = 0;
  uint64_t t_next = 0, t_free = 0, n_inputs = 0;
  Series* last = nullptr;
  size_t last_len = 0;
  std::string last_id;
  struct Held {
    dora_event* ev;
    const void* p;
    size_t len;
    uint64_t csum;
    Series* s;
  };
  std::vector<Held> held;  // verify_late inputs, checksummed after the next ack
  // (seq, receipt ns, ack sent ns) of inputs that asked for an ack: the bench splits its
  // closing time into delivery and the ack's way back
  std::vector<std::array<uint64_t, 3>> acks;
  auto verify = [&](const void* p, size_t len, uint64_t want, Series& s) {
    uint64_t c = 0;
    if (dora_gpu_csum64(p, len, csum_dev, st) == 0 &&
        dora_gpu_memcpy_async(&c, csum_dev, 8, st) == 0 && dora_gpu_stream_sync(st) == 0) {
      ++s.verified;
      if (c != want) ++s.mismatches;
    } else {
      ++errors;
    }
  };
  // busy = wall - idle between the first and the last input (diagnostics)
  uint64_t w_first = 0, w_last = 0, idle_first = 0, idle_last = 0, fill_first = 0, fill_last = 0;
  for (;;) {
    dora_event* ev = nullptr;
    const uint64_t tn0 = mono();
    int rc = dora_node_next_event(node, -1, &ev);
    t_next += mono() - tn0;
    if (rc != 0) break;
    const int type = dora_event_type(ev);
    if (type == DORA_EVENT_INPUT) {
      // data access first: a cross-GPU input is pulled into local HBM there, and the latency
      // counts until the sample is readable on this GPU
      const void* p = nullptr;
      size_t len = 0;
      if (dora_event_data(ev, &p, &len) != 0) {
        std::fprintf(stderr, "sink: input data: %s\n", dora_gpu_last_error());
        ++errors;
      }
      const uint64_t t = now_ns();
      {
        uint64_t idle = 0, fw = 0;
        dora_gpu_busy_stats(&idle, &fw);
        if (!n_inputs) {
          w_first = mono();
          idle_first = idle;
          fill_first = fw;
        }
        w_last = mono();
        idle_last = idle;
        fill_last = fw;
      }
      const uint8_t* pp = nullptr;
      size_t pl = 0;
      dora_event_parameters(ev, &pp, &pl);
      std::map<std::string, Param> params;
      if (pl) params = decode_params(pp, pl);
      if (params.count("ack")) {
        // acknowledge first: the sender's clock waits on this (the data is complete and
        // readable here; the bookkeeping below does not delay the ack)
        std::map<std::string, Param> ap;
        ap["seq"].i = params.count("seq") ? params["seq"].i : -1;
        auto enc = encode_params(ap);
        if (dora_node_send_output_bytes(node, "ack", nullptr, 0, ARROW_DEVICE_ROCM, enc.data(),
                                        enc.size()) != 0) {
          std::fprintf(stderr, "sink: ack failed: %s\n", dora_gpu_last_error());
          ++errors;
        }
        if (acks.size() < 4096)
          acks.push_back({uint64_t(ap["seq"].i), t, now_ns()});
      } else if (params.count("mark") && acks.size() < 4096) {
        acks.push_back({uint64_t(params.count("seq") ? params["seq"].i : -1), t, 0});
      }
      // consecutive inputs mostly share (input, size): skip the keyed lookup then
      const char* id = dora_event_id(ev);
      if (!last || len != last_len || last_id != id) {
        last = &stats[{id, len}];
        last_len = len;
        last_id = id;
      }
      Series& s = *last;
      const uint64_t ts = dora_event_timestamp_ns(ev);
      s.lat_us.push_back((double(t) - double(ts)) / 1000.0);
      if (params.count("t_start"))
        s.full_us.push_back((double(t) - double(params["t_start"].i)) / 1000.0);
      if (!s.first_ns) s.first_ns = t;
      s.last_ns = t;
      ++s.n;
      if (!s.b_first) s.b_first = t;
      s.b_last = t;
      ++s.b_n;
      s.bytes += len;
      const bool dev = dora_event_is_device(ev);
      if (params.count("csum") && params.count("verify") && dev)
        verify(p, len, static_cast<uint64_t>(params["csum"].i), s);
      if (params.count("csum") && params.count("verify") && !dev && p) {
        ++s.verified;  // a host input (inline, shared memory, or a device sample staged here)
        if (csum64_host(static_cast<const uint8_t*>(p), len) !=
            static_cast<uint64_t>(params["csum"].i))
          ++s.mismatches;
      }
      const bool ack = params.count("ack") != 0;
      if (params.count("csum") && params.count("verify_late") && dev) {
        held.push_back({ev, p, len, static_cast<uint64_t>(params["csum"].i), &s});
      } else {
        const uint64_t tf0 = mono();
        dora_event_free(ev);  // zero-copy consumer done: token goes back to the sender
        t_free += mono() - tf0;
      }
      ++n_inputs;
      if (ack)
        for (auto& kv : stats) kv.second.close_burst();
      if (ack) {
        for (Held& h : held) {
          verify(h.p, h.len, h.csum, *h.s);
          dora_event_free(h.ev);
        }
        held.clear();
      }
      continue;
    }
    const bool end = type == DORA_EVENT_ALL_INPUTS_CLOSED || type == DORA_EVENT_STOP;
    if (type == DORA_EVENT_ERROR) {
      std::fprintf(stderr, "sink: error event: %s\n", dora_event_error(ev));
      ++errors;
    }
    dora_event_free(ev);
    if (end) break;
  }
  for (Held& h : held) {  // no ack followed them
    verify(h.p, h.len, h.csum, *h.s);
    dora_event_free(h.ev);
  }
  held.clear();
  uint64_t slots = 0, hits = 0, inflight = 0, dropped = 0;
  dora_node_stats(node, &slots, &hits, &inflight, &dropped);
  uint64_t pulls = 0, pull_bytes = 0, bgroups = 0, brecv = 0, brecv_bytes = 0;
  const char* berr = "";
  dora_node_peer_stats(node, &pulls, &pull_bytes);
  dora_node_bcast_stats(node, nullptr, &bgroups, nullptr, &brecv, &brecv_bytes, &berr);
  FILE* f = out_path ? std::fopen(out_path, "w") : stdout;
  std::fprintf(f,
               "{\"errors\": %d, \"dropped_inputs\": %llu, \"next_event_us\": %.3f, "
               "\"free_us\": %.3f, \"busy_us_per_input\": %.3f, "
               "\"fill_wait_us_per_input\": %.3f, \"pulls\": %llu, \"pull_bytes\": %llu, "
               "\"bcast_groups\": %llu, "
               "\"bcast_received\": %llu, \"bcast_error\": \"%s\", \"sched\": %s, "
               "\"series\": [",
               errors, (unsigned long long)dropped,
               n_inputs ? double(t_next) / n_inputs / 1000.0 : 0.0,
               n_inputs ? double(t_free) / n_inputs / 1000.0 : 0.0,
               n_inputs > 1 ? (double(w_last - w_first) - double(idle_last - idle_first)) / 1e3 /
                                  double(n_inputs - 1)
                            : 0.0,
               n_inputs > 1 ? double(fill_last - fill_first) / 1e3 / double(n_inputs - 1) : 0.0,
               (unsigned long long)pulls, (unsigned long long)pull_bytes,
               (unsigned long long)bgroups, (unsigned long long)brecv, json_safe(berr).c_str(),
               sched_json().c_str());
  bool first = true;
  for (auto& kv : stats) kv.second.close_burst();
  for (auto& kv : stats) {
    Series& s = kv.second;
    std::fprintf(f,
                 "%s\n {\"input\": \"%s\", \"size\": %llu, \"n\": %llu, \"p50_us\": %.3f, "
                 "\"p99_us\": %.3f, \"mean_us\": %.3f, \"min_us\": %.3f, \"full_p50_us\": %.3f, "
                 "\"full_p99_us\": %.3f, \"first_ns\": %llu, \"last_ns\": %llu, \"verified\": "
                 "%llu, \"mismatches\": %llu, \"burst_n\": %llu, \"burst_first_ns\": %llu, "
                 "\"burst_last_ns\": %llu}",
                 first ? "" : ",", kv.first.first.c_str(), (unsigned long long)kv.first.second,
                 (unsigned long long)s.n, pct(s.lat_us, 0.5), pct(s.lat_us, 0.99), mean(s.lat_us),
                 pct(s.lat_us, 0.0), pct(s.full_us, 0.5), pct(s.full_us, 0.99),
                 (unsigned long long)s.first_ns, (unsigned long long)s.last_ns,
                 (unsigned long long)s.verified, (unsigned long long)s.mismatches,
                 (unsigned long long)s.tp_n, (unsigned long long)s.tp_first,
                 (unsigned long long)s.tp_last);
    first = false;
  }
  std::fprintf(f, "\n], \"acks\": [");
  for (size_t k = 0; k < acks.size(); ++k)
    std::fprintf(f, "%s[%llu, %llu, %llu]", k ? ", " : "", (unsigned long long)acks[k][0],
                 (unsigned long long)acks[k][1], (unsigned long long)acks[k][2]);
  std::fprintf(f, "]}\n");
  if (f != stdout) std::fclose(f);
  dora_gpu_free(csum_dev);
  dora_node_free(node);
  if (own_stream) (void)dora_gpu_stream_destroy(st);
  return errors ? 1 : 0;
}
