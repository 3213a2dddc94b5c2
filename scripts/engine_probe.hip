// Persistent pack-engine probe (experiment, not product code).  One resident kernel takes
// copy descriptors from a host-memory ring and signals a per-message flag in host memory, so a
// send costs a 64-byte descriptor write instead of an AQL dispatch.  Measures back-to-back
// throughput (in-flight cap like the node) and single-message latency, and checks every copy.
//   hipcc --offload-arch=gfx950 -O3 -o build/engine_probe scripts/engine_probe.hip
//   build/engine_probe [size_bytes] [n_msgs] [in_flight] [groups] [wgs_per_group]
//
// Roles (all in one launch, 256-thread workgroups):
//   copy WGs  G = groups x per_group: message m belongs to group m % groups; within the group
//             WG i copies chunks i, i + per_group, ... of it; then publishes done[w] = m + 1.
//   finisher  the last WG: for messages in order, waits for the done words of the message's
//             group, then stores the message's flag (system scope) and the host `completed`.
// Every WG polls the host ring's tail itself (system-scope loads, s_sleep between polls) and
// reads its descriptor from host memory.  Every loop is bounded by s_memrealtime: the kernel
// exits on the host's stop word or after `max_ms` without work.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      std::printf("%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                               \
    }                                                                             \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

constexpr int kThreads = 256;
constexpr uint32_t kRing = 1024;  // descriptors

struct Desc {  // 64 B, written by the host before it bumps `tail`
  const uint8_t* src;
  uint8_t* dst;
  uint64_t len;
  uint64_t* flag;
  uint64_t epoch;
  uint64_t pad[3];
};

struct Ctl {  // host memory
  alignas(64) uint64_t tail;       // descriptors posted (host)
  alignas(64) uint64_t stop;       // host asks the engine to exit
  alignas(64) uint64_t completed;  // messages signalled (finisher)
  alignas(64) uint64_t exited;     // WGs that left
};

__device__ __forceinline__ uint64_t ld_sys(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ void st_sys(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint32_t ld_dev(const uint32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_dev(uint32_t* p, uint32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st16_wt(uint8_t* p, u32x4 v) {
  asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" ::"v"(p), "v"(v) : "memory");
}
__device__ __forceinline__ uint64_t now_ticks() { return __builtin_amdgcn_s_memrealtime(); }  // 100 MHz

// gtail replicas: one word per (group, XCD), each on its own 128-B line, so a group's
// pollers spread over 8 lines (workgroups land on XCD blockIdx % 8) instead of one hot line.
constexpr uint32_t kXcds = 8, kLineWords = 32, kStopMark = 0xFFFFFFFFu;
__device__ __forceinline__ uint32_t* replica(uint32_t* gtail, uint32_t g, uint32_t x) {
  return gtail + (g * kXcds + x) * kLineWords;
}

__global__ __launch_bounds__(kThreads) void engine(Ctl* ctl, const Desc* ring, Desc* dring,
                                                   uint32_t* gtail, uint32_t* done,
                                                   uint32_t groups, uint32_t per_group,
                                                   uint32_t chunk, uint32_t max_ms) {
  // Only each group's leader (its WG 0) reads host memory: it polls the host tail and stop word
  // over PCIe, copies the descriptor into the device ring and publishes the group's replicas;
  // the other WGs poll their XCD's replica.
  const uint32_t G = groups * per_group;
  const uint32_t w = blockIdx.x;
  __shared__ uint64_t s_d[8];
  __shared__ int s_go;
  const uint64_t limit = uint64_t(max_ms) * 100000;  // ticks
  uint64_t last_work = now_ticks();
  if (w < G) {
    const uint32_t g = w / per_group, i = w % per_group;
    uint32_t* my_rep = replica(gtail, g, w % kXcds);
    for (uint64_t m = g;; m += groups) {
      if (threadIdx.x == 0) {
        int go = 0;
        for (uint32_t spin = 0;; ++spin) {
          if (i == 0) {
            if (ld_sys(&ctl->tail) > m) {
              const uint64_t* hd = reinterpret_cast<const uint64_t*>(&ring[m % kRing]);
              uint32_t* dd = reinterpret_cast<uint32_t*>(&dring[m % kRing]);
              uint64_t v[5];
              for (int k = 0; k < 5; ++k) v[k] = ld_sys(hd + k);
              for (int k = 0; k < 5; ++k) {
                st_dev(dd + 2 * k, uint32_t(v[k]));
                st_dev(dd + 2 * k + 1, uint32_t(v[k] >> 32));
              }
              asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
              for (uint32_t x = 0; x < kXcds; ++x) st_dev(replica(gtail, g, x), uint32_t(m + 1));
              go = 1;
              break;
            }
            if ((spin & 63) == 63 && (ld_sys(&ctl->stop) || now_ticks() - last_work > limit)) {
              for (uint32_t x = 0; x < kXcds; ++x) st_dev(replica(gtail, g, x), kStopMark);
              break;
            }
          } else {
            const uint32_t t = ld_dev(my_rep);
            if (t == kStopMark) break;
            if (int32_t(t - uint32_t(m + 1)) >= 0) {
              go = 1;
              break;
            }
            if (now_ticks() - last_work > 2 * limit) break;  // the leader is gone
          }
          __builtin_amdgcn_s_sleep(4);
        }
        s_go = go;
      }
      __syncthreads();
      if (!s_go) break;
      if (threadIdx.x < 10)
        reinterpret_cast<uint32_t*>(s_d)[threadIdx.x] =
            ld_dev(reinterpret_cast<const uint32_t*>(&dring[m % kRing]) + threadIdx.x);
      __syncthreads();
      const uint8_t* src = reinterpret_cast<const uint8_t*>(s_d[0]);
      uint8_t* dst = reinterpret_cast<uint8_t*>(s_d[1]);
      const uint64_t len = s_d[2];
      __syncthreads();
      const uint64_t nch = (len + chunk - 1) / chunk;
      for (uint64_t c = i; c < nch; c += per_group) {
        const uint64_t b0 = c * chunk, b1 = b0 + chunk < len ? b0 + chunk : len;
        const uint64_t nu = (b1 - b0) / 16;
        for (uint64_t u = threadIdx.x; u < nu; u += kThreads * 4) {
          u32x4 v[4];
#pragma unroll
          for (int k = 0; k < 4; ++k)
            if (u + k * kThreads < nu)
              v[k] = __builtin_nontemporal_load(
                  reinterpret_cast<const u32x4*>(src + b0) + u + k * kThreads);
#pragma unroll
          for (int k = 0; k < 4; ++k)
            if (u + k * kThreads < nu)
              st16_wt(dst + b0 + 16 * (u + k * kThreads), v[k]);
        }
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (threadIdx.x == 0) st_dev(done + w * kLineWords, uint32_t(m + 1));
      last_work = now_ticks();
    }
  } else {
    // finisher: messages in order; done words one per line
    for (uint64_t m = 0;; ++m) {
      const uint32_t g = uint32_t(m % groups);
      const uint32_t want = uint32_t(m + 1);
      bool alive = true;
      for (uint32_t round = 0;; ++round) {
        if (threadIdx.x == 0) s_go = 1;
        __syncthreads();
        for (uint32_t k = threadIdx.x; k < per_group; k += kThreads)
          if (int32_t(ld_dev(done + (g * per_group + k) * kLineWords) - want) < 0) s_go = 0;
        __syncthreads();
        const int ok = s_go;
        __syncthreads();
        if (ok) break;
        if ((round & 63) == 63) {
          if (threadIdx.x == 0)
            s_go = (ld_sys(&ctl->stop) || now_ticks() - last_work > 2 * limit) ? 0 : 1;
          __syncthreads();
          alive = s_go;
          __syncthreads();
          if (!alive) break;
        }
        __builtin_amdgcn_s_sleep(2);
      }
      if (!alive) break;
      if (threadIdx.x == 0) {
        const uint32_t* dd = reinterpret_cast<const uint32_t*>(&dring[m % kRing]);
        const uint64_t f = uint64_t(ld_dev(dd + 6)) | (uint64_t(ld_dev(dd + 7)) << 32);
        const uint64_t ep = uint64_t(ld_dev(dd + 8)) | (uint64_t(ld_dev(dd + 9)) << 32);
        st_sys(reinterpret_cast<uint64_t*>(f), ep);
        st_sys(&ctl->completed, m + 1);
      }
      last_work = now_ticks();
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) __hip_atomic_fetch_add(&ctl->exited, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void fill(uint8_t* p, uint64_t n, uint64_t seed) {
  for (uint64_t i = blockIdx.x * uint64_t(blockDim.x) + threadIdx.x; i < n / 8;
       i += uint64_t(gridDim.x) * blockDim.x)
    reinterpret_cast<uint64_t*>(p)[i] = (i + 1) * 0x9E3779B97F4A7C15ull ^ seed;
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(
             std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const uint64_t size = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : (4ull << 20);
  const int n = argc > 2 ? std::atoi(argv[2]) : 5000;
  const int cap = argc > 3 ? std::atoi(argv[3]) : 24;
  const uint32_t groups = argc > 4 ? std::atoi(argv[4]) : 4;
  const uint32_t per_group = argc > 5 ? std::atoi(argv[5]) : 256;
  const uint32_t chunk = argc > 6 ? std::atoi(argv[6]) : 16384;
  const int nsrc = int(std::max<uint64_t>(2, std::min<uint64_t>(160, (640ull << 20) / size)));
  const int nslot = 32;
  std::vector<uint8_t*> src(nsrc), dst(nslot);
  for (auto& p : src) CHECK(hipMalloc(&p, size));
  for (auto& p : dst) CHECK(hipMalloc(&p, size));
  for (int k = 0; k < nsrc; ++k) hipLaunchKernelGGL(fill, dim3(1024), dim3(256), 0, 0, src[k], size, uint64_t(k) * 7919);
  CHECK(hipDeviceSynchronize());
  Ctl* ctl = nullptr;
  Desc* ring = nullptr;
  uint64_t* flags = nullptr;
  CHECK(hipHostMalloc(&ctl, sizeof(Ctl), hipHostMallocCoherent | hipHostMallocMapped));
  CHECK(hipHostMalloc(&ring, sizeof(Desc) * kRing, hipHostMallocCoherent | hipHostMallocMapped));
  CHECK(hipHostMalloc(&flags, 64 * nslot, hipHostMallocCoherent | hipHostMallocMapped));
  std::memset(ctl, 0, sizeof(Ctl));
  std::memset(ring, 0, sizeof(Desc) * kRing);
  std::memset(flags, 0, 64 * nslot);
  uint32_t* done = nullptr;
  uint32_t* gtail = nullptr;
  Desc* dring = nullptr;
  const uint32_t G = groups * per_group;
  CHECK(hipMalloc(&done, 128 * G));
  CHECK(hipMemset(done, 0, 128 * G));
  CHECK(hipMalloc(&gtail, 128 * 8 * groups));
  CHECK(hipMemset(gtail, 0, 128 * 8 * groups));
  CHECK(hipMalloc(&dring, sizeof(Desc) * kRing));
  CHECK(hipDeviceSynchronize());
  hipStream_t st;
  CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipLaunchKernelGGL(engine, dim3(G + 1), dim3(kThreads), 0, st, ctl, ring, dring, gtail, done,
                     groups, per_group, chunk, 3000u);
  CHECK(hipGetLastError());
  volatile uint64_t* vtail = &ctl->tail;
  volatile uint64_t* vcomp = &ctl->completed;
  uint64_t posted = 0;
  auto post = [&](int k, uint64_t len) {
    Desc& d = ring[posted % kRing];
    d.src = src[k % nsrc];
    d.dst = dst[posted % nslot];
    d.len = len;
    d.flag = reinterpret_cast<uint64_t*>(reinterpret_cast<uint8_t*>(flags) + 64 * (posted % nslot));
    d.epoch = posted + 1;
    __atomic_store_n(vtail, posted + 1, __ATOMIC_RELEASE);
    ++posted;
  };
  auto wait_completed = [&](uint64_t upto) {
    const double t0 = now_us();
    while (__atomic_load_n(vcomp, __ATOMIC_ACQUIRE) < upto) {
      __builtin_ia32_pause();
      if (now_us() - t0 > 2e6) {
        std::printf("{\"error\": \"timeout waiting for %llu (completed %llu)\"}\n",
                    (unsigned long long)upto, (unsigned long long)*vcomp);
        ctl->stop = 1;
        return false;
      }
    }
    return true;
  };
  bool ok = true;
  // warm
  for (int k = 0; k < 64 && ok; ++k) {
    if (posted >= uint64_t(cap)) ok = wait_completed(posted - cap + 1);
    post(k, size);
  }
  ok = ok && wait_completed(posted);
  // throughput
  const double t0 = now_us();
  for (int k = 0; k < n && ok; ++k) {
    const uint64_t need = posted + 1 > uint64_t(cap) ? posted + 1 - cap : 0;
    if (need && *vcomp < need) ok = wait_completed(need);
    post(k, size);
  }
  ok = ok && wait_completed(posted);
  const double tp_us = now_us() - t0;
  // check the last nslot copies
  int bad = 0;
  if (ok) {
    std::vector<uint8_t> a(size), b(size);
    for (int j = 0; j < 4; ++j) {
      const uint64_t msg = posted - 1 - j;  // message index
      const int k = int((msg - 64) % nsrc);  // throughput message k = msg - 64
      CHECK(hipMemcpy(a.data(), dst[msg % nslot], size, hipMemcpyDeviceToHost));
      CHECK(hipMemcpy(b.data(), src[k], size, hipMemcpyDeviceToHost));
      bad += std::memcmp(a.data(), b.data(), size) != 0;
    }
  }
  // latency: one 4 KB message at a time
  std::vector<double> lat;
  for (int k = 0; k < 2000 && ok; ++k) {
    const double a = now_us();
    post(k, 4096);
    ok = wait_completed(posted);
    lat.push_back(now_us() - a);
  }
  std::sort(lat.begin(), lat.end());
  ctl->stop = 1;
  const double ts = now_us();
  while (hipStreamQuery(st) == hipErrorNotReady) {
    if (now_us() - ts > 5e6) {
      std::printf("{\"error\": \"engine did not exit\"}\n");
      return 2;
    }
  }
  const double per = tp_us / n;
  std::printf("{\"size\": %llu, \"n\": %d, \"cap\": %d, \"groups\": %u, \"per_group\": %u, "
              "\"chunk\": %u, \"us_per_msg\": %.3f, \"hbm_frac_2S\": %.4f, \"lat_p50_us\": %.2f, "
              "\"lat_p99_us\": %.2f, \"bad\": %d, \"ok\": %s}\n",
              (unsigned long long)size, n, cap, groups, per_group, chunk, per,
              2.0 * size / (per * 1e-6) / 8e12, lat.empty() ? 0 : lat[lat.size() / 2],
              lat.empty() ? 0 : lat[lat.size() * 99 / 100], bad, ok ? "true" : "false");
  return ok && !bad ? 0 : 1;
}
