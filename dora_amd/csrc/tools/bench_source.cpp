// dora-gpu-bench-source: the benchmark node (examples/benchmark/node/src/main.rs:1-73) as a
// native process for the multi-GPU configurations (BASELINE.json configs C4 fan-out and C5
// chain), where the producer sits on one GPU and its receivers on others.  Payloads are
// device-resident splitmix64 bytes (seed 0xD05A + size, like bench.py); the first messages of
// every size carry their csum64 so receivers verify them bit-exact after the xGMI pulls.
//
// Modes (reference: latency mode = spaced messages, throughput mode = back-to-back):
//   latency:    DORA_BENCH_LAT_SIZES (comma list) x DORA_BENCH_LAT_N messages,
//               DORA_BENCH_LAT_GAP_US apart (33333 = 30 Hz, C5);
//   throughput: DORA_BENCH_TP_N messages of DORA_BENCH_TP_SIZE bytes back-to-back, closed by an
//               ack request that every one of the DORA_BENCH_ACKS receivers acknowledges.
// DORA_BENCH_SAMPLE_PATH=1: every message takes the reference benchmark's own path
// (examples/benchmark/node/src/main.rs via allocate_data_sample + send_output_sample,
// apis/rust/node/src/node/mod.rs:246-346): a slot is allocated, a kernel on the node stream
// writes the payload into it in place, and the sample is sent — no pack, no source buffer.
// Outputs `latency` and `throughput` (warmup and ack requests go on `throughput`, like the
// reference node's two outputs); every input is an ack channel from a receiver.
//   env: DORA_GPU_DATAFLOW, DORA_NODE_ID, DORA_GPU_DEVICE, DORA_BENCH_RESULT (path)
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <set>
#include <string>
#include <vector>

#include "dora_gpu.h"
#include "params.h"

namespace {

uint64_t mono() {
  timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return uint64_t(ts.tv_sec) * 1000000000ull + uint64_t(ts.tv_nsec);
}

uint64_t realtime() {
  timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  return uint64_t(ts.tv_sec) * 1000000000ull + uint64_t(ts.tv_nsec);
}

long env_long(const char* k, long d) {
  const char* v = std::getenv(k);
  return v && *v ? std::atol(v) : d;
}

std::vector<uint64_t> env_sizes(const char* k) {
  std::vector<uint64_t> out;
  const char* v = std::getenv(k);
  if (!v) return out;
  std::string cur;
  for (const char* p = v;; ++p) {
    if (*p == ',' || !*p) {
      if (!cur.empty()) out.push_back(std::strtoull(cur.c_str(), nullptr, 10));
      cur.clear();
      if (!*p) break;
    } else {
      cur += *p;
    }
  }
  return out;
}

struct Source {
  void* ptr = nullptr;
  uint64_t csum = 0;
  std::vector<void*> extra;  // DORA_BENCH_TP_SOURCES - 1 more copies the throughput mode rotates over
};

}  // namespace

int main() {
  dora_node* node = nullptr;
  if (dora_node_init_from_env(&node) != 0) {
    std::fprintf(stderr, "source: init failed: %s\n", dora_gpu_last_error());
    return 1;
  }
  // the benchmark node never rewrites its sources: sends return as soon as their pack is queued
  // (DORA_SEND_ASYNC; DORA_BENCH_SYNC_SENDS=1 measures the default synchronous sends instead)
  if (env_long("DORA_BENCH_SYNC_SENDS", 0) == 0) dora_node_set_async_sends(node, 1);
  // bench.py --keep-awake-us: the warm thread's period (dora_gpu_set_keep_awake; 0: off)
  if (const char* v = std::getenv("DORA_BENCH_KEEP_AWAKE_US")) dora_gpu_set_keep_awake(std::atof(v));
  const char* out_path = std::getenv("DORA_BENCH_RESULT");
  const auto lat_sizes = env_sizes("DORA_BENCH_LAT_SIZES");
  const long lat_n = env_long("DORA_BENCH_LAT_N", 30);
  const long gap_us = env_long("DORA_BENCH_LAT_GAP_US", 33333);
  const uint64_t tp_size = static_cast<uint64_t>(env_long("DORA_BENCH_TP_SIZE", 0));
  const long tp_n = env_long("DORA_BENCH_TP_N", 100);
  const long acks = env_long("DORA_BENCH_ACKS", 1);
  const long verify_n = env_long("DORA_BENCH_VERIFY", 2);
  // the payloads are made (and synchronised) on a stream of its own before any send: the node
  // stream stays unused, so sends need not query it (node.cpp stream_used)
  dora_stream_t st = nullptr;
  const bool own_stream = dora_gpu_stream_create(&st) == 0;
  if (!own_stream) st = dora_node_stream(node);
  int errors = 0;

  // throughput mode: rotating source copies, so the sources of a burst are not all served from the
  // Infinity Cache (one resident source per size by default, as the reference node sends one Vec)
  const long tp_sources = std::max(1L, env_long("DORA_BENCH_TP_SOURCES", 1));
  std::map<uint64_t, Source> src;
  std::vector<uint64_t> all = lat_sizes;
  if (tp_size) all.push_back(tp_size);
  for (uint64_t s : all) {
    if (src.count(s) || s == 0) continue;
    Source& x = src[s];
    if (dora_gpu_malloc(&x.ptr, s) != 0 || dora_gpu_fill_splitmix(x.ptr, s, 0xD05A + s, st) != 0 ||
        dora_gpu_csum64_sync(x.ptr, s, st, &x.csum) != 0) {
      std::fprintf(stderr, "source: payload of %llu B: %s\n", (unsigned long long)s,
                   dora_gpu_last_error());
      return 1;
    }
    for (long k = 1; s == tp_size && k < tp_sources; ++k) {
      void* p = nullptr;
      if (dora_gpu_malloc(&p, s) != 0 || dora_gpu_fill_splitmix(p, s, 0xD05A + s, st) != 0) {
        std::fprintf(stderr, "source: payload copy: %s\n", dora_gpu_last_error());
        return 1;
      }
      x.extra.push_back(p);
    }
  }
  dora_gpu_stream_sync(st);

  // sample path: the node stream the payload kernels run on, and byte_array type infos by size
  const bool sample_path = env_long("DORA_BENCH_SAMPLE_PATH", 0) != 0;
  dora_stream_t nst = sample_path ? dora_node_stream(node) : nullptr;
  std::map<uint64_t, std::vector<uint8_t>> tis;
  auto type_info = [&](const void* data, uint64_t size) -> const std::vector<uint8_t>& {
    auto it = tis.find(size);
    if (it != tis.end()) return it->second;
    std::vector<uint8_t>& ti = tis[size];
    dora_plan* plan = nullptr;
    size_t n = 0;
    if (dora_gpu_plan_bytes(data, size, ARROW_DEVICE_ROCM, &plan) == 0) {
      ti.resize(4096);
      if (dora_gpu_plan_type_info(plan, ti.data(), ti.size(), &n) != 0) n = 0;
      dora_gpu_plan_free(plan);
    }
    ti.resize(n);
    return ti;
  };
  // one message of `size` bytes written in place by a kernel (sample path)
  auto send_in_place = [&](const char* output, uint64_t size, const uint8_t* params,
                           size_t params_len) -> int {
    dora_sample* smp = nullptr;
    if (dora_node_allocate_data_sample(node, size, &smp) != 0) return -1;
    if (size && dora_gpu_fill_splitmix(dora_sample_data(smp), size, 0xD05A + size, nst) != 0) {
      dora_sample_discard(node, smp);
      return -1;
    }
    const std::vector<uint8_t>& ti = type_info(dora_sample_data(smp), size);
    return dora_node_send_output_sample(node, output, ti.data(), ti.size(), params, params_len,
                                        smp);
  };

  int64_t seq = 0;
  // throughput-mode messages carry default parameters, like the reference node's
  // send_output_raw(.., Default::default(), ..): latency comes from the metadata timestamp
  auto send_plain = [&](const char* output, uint64_t size) {
    const Source& x = src[size];
    const size_t k = static_cast<size_t>(seq++ % tp_sources);
    const void* p = k == 0 ? x.ptr : x.extra[k - 1];
    if ((sample_path ? send_in_place(output, size, nullptr, 0)
                     : dora_node_send_output_bytes(node, output, p, size, ARROW_DEVICE_ROCM,
                                                   nullptr, 0)) != 0) {
      std::fprintf(stderr, "source: send failed: %s\n", dora_gpu_last_error());
      ++errors;
    }
  };
  auto send = [&](const char* output, uint64_t size, bool verify) {
    std::map<std::string, Param> p;
    p["seq"].i = seq++;
    p["t_start"].i = static_cast<int64_t>(realtime());
    if (verify) {
      p["csum"].i = static_cast<int64_t>(src[size].csum);
      p["verify"].tag = 0;
      p["verify"].i = 1;
    }
    auto enc = encode_params(p);
    if ((sample_path ? send_in_place(output, size, enc.data(), enc.size())
                     : dora_node_send_output_bytes(node, output, src[size].ptr, size,
                                                   ARROW_DEVICE_ROCM, enc.data(), enc.size())) != 0) {
      std::fprintf(stderr, "source: send failed: %s\n", dora_gpu_last_error());
      ++errors;
    }
  };
  // ack barrier: every receiver acknowledges `seq` (sink `ack` output, any input of ours)
  auto barrier = [&]() -> bool {
    std::map<std::string, Param> p;
    const int64_t want = seq++;
    p["seq"].i = want;
    p["ack"].tag = 0;
    p["ack"].i = 1;
    auto enc = encode_params(p);
    if (dora_node_send_output_bytes(node, "throughput", nullptr, 0, ARROW_DEVICE_ROCM, enc.data(),
                                    enc.size()) != 0) {
      ++errors;
      return false;
    }
    std::set<std::string> got;
    const uint64_t t0 = mono();
    while (static_cast<long>(got.size()) < acks) {
      if (mono() - t0 > 120000000000ull) {
        std::fprintf(stderr, "source: %zu/%ld acks for seq %lld\n", got.size(), acks,
                     (long long)want);
        ++errors;
        return false;
      }
      dora_event* ev = nullptr;
      if (dora_node_next_event(node, 1000000, &ev) != 0) continue;
      if (dora_event_type(ev) == DORA_EVENT_INPUT) {
        const uint8_t* pp = nullptr;
        size_t pl = 0;
        dora_event_parameters(ev, &pp, &pl);
        auto ap = decode_params(pp, pl);
        if (ap.count("seq") && ap["seq"].i == want) got.insert(dora_event_id(ev));
      }
      dora_event_free(ev);
    }
    return true;
  };

  // warmup: every size once per receiver path, first ones verified
  for (auto& kv : src)
    for (long k = 0; k < 3; ++k) send("throughput", kv.first, k < verify_n);
  bool ok = barrier();

  // latency mode
  for (uint64_t s : lat_sizes) {
    if (!ok) break;
    for (long k = 0; k < lat_n; ++k) {
      if (s) send("latency", s, k < verify_n);
      usleep(static_cast<useconds_t>(gap_us));
    }
  }
  if (ok && !lat_sizes.empty()) ok = barrier();

  // throughput mode
  double tp_s = 0;
  uint64_t idle0 = 0, idle1 = 0;
  if (ok && tp_size) {
    dora_node_set_profiling(node, 0);  // resets the send-phase counters, no kernel stamps
    dora_gpu_busy_stats(&idle0, nullptr);
    const uint64_t t0 = mono();
    for (long k = 0; k < tp_n; ++k) send_plain("throughput", tp_size);
    ok = barrier();
    tp_s = double(mono() - t0) / 1e9;
    dora_gpu_busy_stats(&idle1, nullptr);
  }
  double phase[4] = {0, 0, 0, 0};
  uint64_t cnt = 0;
  dora_node_send_profile(node, phase, 4, &cnt);
  uint64_t slots = 0, hits = 0, inflight = 0, dropped = 0;
  dora_node_stats(node, &slots, &hits, &inflight, &dropped);

  uint64_t batches = 0, batched = 0, backlogged = 0;
  {
    int dev = 0;
    dora_gpu_get_device(&dev);
    dora_gpu_aql_batch_stats(dev, &batches, &batched, &backlogged);
  }
  uint64_t bgroups = 0, bsent = 0;
  const char* berr = "";
  dora_node_bcast_stats(node, &bgroups, nullptr, &bsent, nullptr, nullptr, &berr);
  uint64_t branks = 0;
  dora_node_bcast_ranks(node, &branks);
  FILE* f = out_path ? std::fopen(out_path, "w") : stdout;
  const double delivered = double(tp_size) * double(tp_n) * double(acks);
  std::fprintf(f,
               "{\"errors\": %d, \"ok\": %s, \"receivers\": %ld, \"tp_size\": %llu, \"tp_n\": %ld, "
               "\"tp_seconds\": %.6f, \"tp_delivered_GBps\": %.3f, \"tp_per_receiver_GBps\": %.3f, "
               "\"send_phase_us\": {\"alloc_us\": %.2f, \"launch_us\": %.2f, \"fill_us\": %.2f, "
               "\"send_us\": %.2f}, \"slots_created\": %llu, \"cache_hits\": %llu, "
               "\"bcast_groups\": %llu, \"bcast_ranks\": %llu, \"bcast_sent\": %llu, "
               "\"bcast_error\": \"%s\", "
               "\"tp_busy_us_per_msg\": %.3f, \"aql_batches\": %llu, \"aql_batched_msgs\": %llu}\n",
               errors, ok ? "true" : "false", acks, (unsigned long long)tp_size, tp_n, tp_s,
               tp_s > 0 ? delivered / tp_s / 1e9 : 0.0,
               tp_s > 0 ? double(tp_size) * double(tp_n) / tp_s / 1e9 : 0.0, phase[0], phase[1],
               phase[2], phase[3], (unsigned long long)slots, (unsigned long long)hits,
               (unsigned long long)bgroups, (unsigned long long)branks, (unsigned long long)bsent,
               json_safe(berr).c_str(),
               tp_n > 0 ? (tp_s * 1e9 - double(idle1 - idle0)) / 1e3 / double(tp_n) : 0.0,
               (unsigned long long)batches, (unsigned long long)batched);
  if (f != stdout) std::fclose(f);
  for (auto& kv : src) {
    dora_gpu_free(kv.second.ptr);
    for (void* p : kv.second.extra) dora_gpu_free(p);
  }
  dora_node_free(node);
  if (own_stream) (void)dora_gpu_stream_destroy(st);
  return errors || !ok ? 1 : 0;
}
