// MetadataParameters encoding shared by the native tools (see include/dora_gpu.h).
#pragma once

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

struct Param {
  uint8_t tag = 1;  // 0 bool, 1 int, 2 string
  int64_t i = 0;
  std::string s;
};

inline std::vector<uint8_t> encode_params(const std::map<std::string, Param>& m) {
  std::vector<uint8_t> o;
  auto put = [&](const void* p, size_t n) {
    const auto* c = static_cast<const uint8_t*>(p);
    o.insert(o.end(), c, c + n);
  };
  uint32_t n = static_cast<uint32_t>(m.size());
  put(&n, 4);
  for (auto& kv : m) {
    uint64_t kl = kv.first.size();
    put(&kl, 8);
    put(kv.first.data(), kl);
    put(&kv.second.tag, 1);
    if (kv.second.tag == 0) {
      uint8_t b = kv.second.i ? 1 : 0;
      put(&b, 1);
    } else if (kv.second.tag == 1) {
      put(&kv.second.i, 8);
    } else {
      uint64_t sl = kv.second.s.size();
      put(&sl, 8);
      put(kv.second.s.data(), sl);
    }
  }
  return o;
}

inline std::map<std::string, Param> decode_params(const uint8_t* p, size_t n) {
  std::map<std::string, Param> m;
  size_t i = 0;
  auto get = [&](void* d, size_t k) {
    if (i + k > n) throw 1;
    std::memcpy(d, p + i, k);
    i += k;
  };
  try {
    if (n < 4) return m;
    uint32_t cnt;
    get(&cnt, 4);
    for (uint32_t c = 0; c < cnt; ++c) {
      uint64_t kl;
      get(&kl, 8);
      std::string key(kl, '\0');
      get(&key[0], kl);
      Param v;
      get(&v.tag, 1);
      if (v.tag == 0) {
        uint8_t b;
        get(&b, 1);
        v.i = b;
      } else if (v.tag == 1) {
        get(&v.i, 8);
      } else {
        uint64_t sl;
        get(&sl, 8);
        v.s.assign(sl, '\0');
        get(&v.s[0], sl);
      }
      m[key] = v;
    }
  } catch (int) {
  }
  return m;
}

// A C string as the body of a JSON string literal (quotes, backslashes and control bytes
// replaced).
inline std::string json_safe(const char* s) {
  std::string o;
  for (; s && *s; ++s) o += (*s == '"' || *s == '\\' || static_cast<unsigned char>(*s) < 0x20) ? ' ' : *s;
  return o;
}

// The calling process's main thread as the scheduler saw it (/proc/self/schedstat: time on the
// CPU, time runnable but waiting for one; /proc/self/status: context switches), as a JSON object.
// A spinning receiver that waited on the run queue or was switched out involuntarily lost the CPU
// to other load: the tail of its latencies is that, not its own work.
inline std::string sched_json() {
  unsigned long long run = 0, wait = 0, slices = 0, vol = 0, invol = 0;
  if (FILE* f = std::fopen("/proc/self/schedstat", "r")) {
    if (std::fscanf(f, "%llu %llu %llu", &run, &wait, &slices) != 3) run = wait = slices = 0;
    std::fclose(f);
  }
  if (FILE* f = std::fopen("/proc/self/status", "r")) {
    char line[256];
    while (std::fgets(line, sizeof(line), f)) {
      if (std::strncmp(line, "voluntary_ctxt_switches:", 24) == 0) vol = std::strtoull(line + 24, nullptr, 10);
      if (std::strncmp(line, "nonvoluntary_ctxt_switches:", 27) == 0)
        invol = std::strtoull(line + 27, nullptr, 10);
    }
    std::fclose(f);
  }
  char b[256];
  std::snprintf(b, sizeof(b),
                "{\"run_ms\": %.3f, \"runq_wait_ms\": %.3f, \"timeslices\": %llu, "
                "\"voluntary_switches\": %llu, \"involuntary_switches\": %llu}",
                run / 1e6, wait / 1e6, slices, vol, invol);
  return b;
}

