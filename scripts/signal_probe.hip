// Fill-signal probe (tuning experiment, not product code): how a pack kernel should tell the
// receiver that a sample is complete.  HBM->HBM copy of S bytes (8 KiB chunks, one 256-thread
// workgroup each, 16-B loads/stores, 4 in flight per lane) with these completion forms:
//   nt        non-temporal stores, no signal                     (copy speed reference)
//   wt        write-through (sc1 nt) stores, no signal           (cost of write-through alone)
//   wt+ctr8   wt + 8 shard counters (blockIdx % 8) -> top counter; the last arriver stores the
//             host flag (system scope).  No polling workgroup, full grid.
//   wt+ctr8 16K  same, 16 KiB chunks (half the arrivals)
//   nt+wv     nt + hipStreamWriteValue64 of the host flag (stream packet)
//   nt+k1     nt + a 1-workgroup kernel that stores the host flag
// Throughput: HIP events around 30 back-to-back launches on rotating buffers (> 512 MiB).
// Latency: one isolated launch, host spins on the flag; launch call -> flag seen (host clock).
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/signal_probe scripts/signal_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                         \
  do {                                                                   \
    hipError_t e = (x);                                                  \
    if (e != hipSuccess) {                                               \
      std::printf("%s: %s\n", #x, hipGetErrorString(e));                 \
      std::exit(1);                                                      \
    }                                                                    \
  } while (0)

struct Args {
  const u32x4* s;
  u32x4* d;
  size_t n;      // 16-B units
  size_t per;    // units per workgroup
  unsigned long long* flag;  // host flag (mapped)
  unsigned int* ctr;         // shard counters + top counter (device), `pad` words apart
  unsigned long long epoch;
  unsigned pad;              // words between counters
  unsigned nsh;              // shards (power of two <= 64)
  unsigned* done;            // per-workgroup done words (MODE 3)
};

template <int MODE>  // 0 nt, 1 wt, 2 wt + sharded counters, 3 wt + done words polled by the last block
__global__ __launch_bounds__(256) void copyk(Args a) {
  const size_t b0 = size_t(blockIdx.x) * a.per;
  const size_t b1 = b0 + a.per < a.n ? b0 + a.per : a.n;
  for (size_t base = b0 + threadIdx.x; base < b1; base += 256 * 4) {
    u32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const size_t i = base + size_t(u) * 256;
      if (i < b1) v[u] = __builtin_nontemporal_load(a.s + i);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const size_t i = base + size_t(u) * 256;
      if (i < b1) {
        if constexpr (MODE == 0) __builtin_nontemporal_store(v[u], a.d + i);
        else asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" ::"v"(a.d + i), "v"(v[u]) : "memory");
      }
    }
  }
  if constexpr (MODE == 2) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned k = blockIdx.x & (a.nsh - 1);
      const unsigned cnt = (gridDim.x - k + a.nsh - 1) / a.nsh;
      const unsigned shards = gridDim.x < a.nsh ? gridDim.x : a.nsh;
      unsigned* top = a.ctr + a.nsh * a.pad;
      if (__hip_atomic_fetch_add(a.ctr + k * a.pad, 1u, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT) == cnt - 1) {
        if (__hip_atomic_fetch_add(top, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) ==
            shards - 1) {
          for (unsigned j = 0; j < a.nsh; ++j)
            __hip_atomic_store(a.ctr + j * a.pad, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(top, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(a.flag, a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
      }
    }
  }
  if constexpr (MODE == 3) {
    const unsigned e = unsigned(a.epoch);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0)
      __hip_atomic_store(a.done + blockIdx.x, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (blockIdx.x != gridDim.x - 1) return;
    bool ok = false;
    for (unsigned round = 0; round < (1u << 22); ++round) {
      bool mine = true;
      for (unsigned i = threadIdx.x; i < gridDim.x; i += 256)
        mine &= __hip_atomic_load(a.done + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == e;
      if (__syncthreads_and(mine)) { ok = true; break; }
      __builtin_amdgcn_s_sleep(1);
    }
    if (threadIdx.x == 0 && ok)
      __hip_atomic_store(a.flag, a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

__global__ void flagk(unsigned long long* flag, unsigned long long epoch) {
  if (threadIdx.x == 0) __hip_atomic_store(flag, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

struct Var {
  const char* name;
  int mode;      // kernel MODE
  int extra;     // 0 none, 1 write-value, 2 flag kernel
  size_t chunk;  // bytes per workgroup
  unsigned pad = 1, nsh = 8;
};

int main(int argc, char** argv) {
  std::vector<size_t> sizes = {4096000, 16777216, 40960000};
  if (argc > 1) sizes = {std::strtoull(argv[1], nullptr, 10)};
  const int iters = 30, rounds = 5, lat_n = 40;
  std::vector<Var> vars = {
      {"nt", 0, 0, 8192},
      {"wt", 1, 0, 8192},
      {"wt+ctr8 pad256B", 2, 0, 8192, 64, 8},
      {"wt+ctr8 pad4K", 2, 0, 8192, 1024, 8},
      {"wt+ctr64 pad256B", 2, 0, 8192, 64, 64},
      {"wt+ctr64 pad256B 16K", 2, 0, 16384, 64, 64},
      {"wt+done last-block poll", 3, 0, 8192},
      {"wt+done last-block poll 16K", 3, 0, 16384},
      {"nt+k1", 0, 2, 8192},
  };
  unsigned long long* hflag;
  CHECK(hipHostMalloc(reinterpret_cast<void**>(&hflag), 64, hipHostMallocMapped));
  unsigned long long* dflag;
  CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&dflag), hflag, 0));
  *reinterpret_cast<volatile unsigned long long*>(hflag) = 0;
  unsigned int* ctr;
  CHECK(hipMalloc(&ctr, 1 << 20));
  CHECK(hipMemset(ctr, 0, 1 << 20));
  unsigned* done;
  CHECK(hipMalloc(&done, 1 << 20));
  CHECK(hipMemset(done, 0, 1 << 20));
  hipStream_t st;
  CHECK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  unsigned long long epoch = 0;
  for (size_t S : sizes) {
    const size_t n = S / 16;
    const int nbuf = int(std::max<size_t>(2, std::min<size_t>(64, (640u << 20) / (2 * S))));
    std::vector<u32x4*> src(nbuf), dst(nbuf);
    for (int i = 0; i < nbuf; ++i) {
      CHECK(hipMalloc(&src[i], S));
      CHECK(hipMalloc(&dst[i], S));
      CHECK(hipMemset(src[i], i, S));
    }
    CHECK(hipDeviceSynchronize());
    std::vector<std::vector<float>> thr(vars.size());
    std::vector<std::vector<double>> lat(vars.size());
    for (int r = 0; r < rounds; ++r) {
      for (size_t v = 0; v < vars.size(); ++v) {
        const Var& x = vars[v];
        auto launch = [&](int k) {
          Args a;
          a.s = src[k];
          a.d = dst[k];
          a.n = n;
          a.per = x.chunk / 16;
          a.flag = dflag;
          a.ctr = ctr;
          a.epoch = ++epoch;
          a.pad = x.pad;
          a.nsh = x.nsh;
          a.done = done;
          const unsigned grid = unsigned((n + a.per - 1) / a.per);
          if (x.mode == 0) hipLaunchKernelGGL(copyk<0>, dim3(grid), dim3(256), 0, st, a);
          else if (x.mode == 1) hipLaunchKernelGGL(copyk<1>, dim3(grid), dim3(256), 0, st, a);
          else if (x.mode == 2) hipLaunchKernelGGL(copyk<2>, dim3(grid), dim3(256), 0, st, a);
          else hipLaunchKernelGGL(copyk<3>, dim3(grid), dim3(256), 0, st, a);
          if (x.extra == 1) CHECK(hipStreamWriteValue64(st, dflag, a.epoch, 0));
          if (x.extra == 2) hipLaunchKernelGGL(flagk, dim3(1), dim3(64), 0, st, dflag, a.epoch);
          return a.epoch;
        };
        for (int w = 0; w < 3; ++w) launch(w % nbuf);
        CHECK(hipEventRecord(e0, st));
        for (int i = 0; i < iters; ++i) launch(i % nbuf);
        CHECK(hipEventRecord(e1, st));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        thr[v].push_back(ms / iters);
        if (x.mode >= 2 || x.extra) {
          for (int i = 0; i < lat_n / rounds; ++i) {
            CHECK(hipStreamSynchronize(st));
            const auto t0 = std::chrono::steady_clock::now();
            const unsigned long long e = launch(i % nbuf);
            const volatile unsigned long long* f = hflag;
            while (*f < e) {
              if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
                std::printf("flag timeout in %s\n", x.name);
                std::exit(2);
              }
            }
            lat[v].push_back(
                std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0)
                    .count());
          }
        }
      }
    }
    CHECK(hipStreamSynchronize(st));
    for (size_t v = 0; v < vars.size(); ++v) {
      auto t = thr[v];
      std::sort(t.begin(), t.end());
      const float med = t[t.size() / 2];
      double lmed = 0;
      if (!lat[v].empty()) {
        auto l = lat[v];
        std::sort(l.begin(), l.end());
        lmed = l[l.size() / 2];
      }
      std::printf("{\"variant\": \"%s\", \"size\": %zu, \"us_per_launch\": %.2f, \"TBps_2S\": %.3f, "
                  "\"signal_latency_p50_us\": %.2f}\n",
                  vars[v].name, S, med * 1e3, 2.0 * S / (med * 1e-3) / 1e12, lmed);
      std::fflush(stdout);
    }
    for (int i = 0; i < nbuf; ++i) {
      CHECK(hipFree(src[i]));
      CHECK(hipFree(dst[i]));
    }
  }
  return 0;
}
