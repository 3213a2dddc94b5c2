// Multi-stream pack probe (tuning experiment, not product code): does spreading consecutive
// sends over P HIP streams (P hardware queues) hide the per-launch ramp/drain and the fill-signal
// tail?  Each message = one HBM->HBM copy of S bytes (8 KiB chunks, nt) + a 1-workgroup kernel
// that stores the message's epoch into its host fill flag (system scope).  At most D messages
// in flight (the node's backpressure): message i launches after the host saw the flag of i-D.
// Throughput = host wall clock over N messages, from the first launch to the last flag.
// `dep`: each send also records an event on its pack stream and makes a "node stream" wait on
// it (keeps later node-stream work ordered after the pack).
//   hipcc --offload-arch=gfx950 -O3 -o build/stream_probe scripts/stream_probe.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                         \
  do {                                                                   \
    hipError_t err_ = (x);                                                  \
    if (err_ != hipSuccess) {                                             \
      std::printf("%s: %s\n", #x, hipGetErrorString(err_));               \
      std::exit(1);                                                      \
    }                                                                    \
  } while (0)

__global__ __launch_bounds__(256) void copyk(const u32x4* __restrict__ s, u32x4* __restrict__ d,
                                             size_t n, size_t per) {
  const size_t b0 = size_t(blockIdx.x) * per;
  const size_t b1 = b0 + per < n ? b0 + per : n;
  for (size_t base = b0 + threadIdx.x; base < b1; base += 256 * 4) {
    u32x4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const size_t i = base + size_t(u) * 256;
      if (i < b1) v[u] = __builtin_nontemporal_load(s + i);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const size_t i = base + size_t(u) * 256;
      if (i < b1) __builtin_nontemporal_store(v[u], d + i);
    }
  }
}

// In-kernel fill signal: write-through (sc1 nt) stores; every workgroup drains and publishes
// the epoch in its done word; one workgroup polls all done words, then stores the host flag.
// POLLER 0: the last block polls (full grid, one chunk per workgroup);
// POLLER 1: block 0 polls, grid capped at `cap` workgroups striding over the chunks.
template <int POLLER>
__global__ __launch_bounds__(256) void copysig(const u32x4* __restrict__ s, u32x4* __restrict__ d,
                                               size_t n, size_t per, unsigned* done,
                                               unsigned long long* flag, unsigned long long epoch) {
  const size_t nch = (n + per - 1) / per;
  for (size_t c = blockIdx.x; c < nch; c += gridDim.x) {
    const size_t b0 = c * per;
    const size_t b1 = b0 + per < n ? b0 + per : n;
    for (size_t base = b0 + threadIdx.x; base < b1; base += 256 * 4) {
      u32x4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const size_t i = base + size_t(u) * 256;
        if (i < b1) v[u] = __builtin_nontemporal_load(s + i);
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const size_t i = base + size_t(u) * 256;
        if (i < b1)
          asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" ::"v"(d + i), "v"(v[u]) : "memory");
      }
    }
  }
  const unsigned e = unsigned(epoch);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    __hip_atomic_store(done + blockIdx.x, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  const unsigned poller = POLLER == 0 ? gridDim.x - 1 : 0;
  if (blockIdx.x != poller) return;
  bool ok = false;
  for (unsigned round = 0; round < (1u << 22); ++round) {
    bool mine = true;
    for (unsigned i = threadIdx.x; i < gridDim.x; i += 256)
      mine &= __hip_atomic_load(done + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == e;
    if (__syncthreads_and(mine)) { ok = true; break; }
    __builtin_amdgcn_s_sleep(1);
  }
  if (threadIdx.x == 0 && ok)
    __hip_atomic_store(flag, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__global__ void flagk(unsigned long long* flag, unsigned long long epoch) {
  if (threadIdx.x == 0) __hip_atomic_store(flag, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

int main(int argc, char** argv) {
  std::vector<size_t> sizes = {1 << 20, 4096000, 16777216, 40960000};
  const int N = 200, D = 8, rounds = 3;
  // sig: 0 = copy + flag kernel, 1 = in-kernel (last block polls), 2 = in-kernel (block 0
  // polls, grid capped at 1024)
  struct Var { int P; bool dep; int sig; size_t chunk; };
  std::vector<Var> vars = {{1, false, 0, 8192},  {2, false, 0, 8192},  {3, false, 0, 8192},
                           {1, false, 1, 8192},  {2, false, 1, 8192},  {3, false, 1, 8192},
                           {1, false, 1, 16384}, {2, false, 1, 16384}, {3, false, 1, 16384},
                           {1, false, 2, 8192},  {2, false, 2, 8192},  {3, false, 2, 8192}};
  unsigned* done;
  CHECK(hipMalloc(&done, D * 8192 * sizeof(unsigned)));
  CHECK(hipMemset(done, 0, D * 8192 * sizeof(unsigned)));
  unsigned long long* hflag;
  CHECK(hipHostMalloc(reinterpret_cast<void**>(&hflag), 64 * D, hipHostMallocMapped));
  unsigned long long* dflag;
  CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&dflag), hflag, 0));
  for (int i = 0; i < 8 * D; ++i) reinterpret_cast<volatile unsigned long long*>(hflag)[i] = 0;
  std::vector<hipStream_t> st(4);
  for (auto& s : st) CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipStream_t node;
  CHECK(hipStreamCreateWithFlags(&node, hipStreamNonBlocking));
  std::vector<hipEvent_t> ev(D);
  for (auto& e : ev) CHECK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  unsigned long long epoch = 0;
  for (size_t S : sizes) {
    const size_t n = S / 16;
    const int nbuf = int(std::max<size_t>(D + 1, std::min<size_t>(64, (640u << 20) / (2 * S))));
    std::vector<u32x4*> src(nbuf), dst(nbuf);
    for (int i = 0; i < nbuf; ++i) {
      CHECK(hipMalloc(&src[i], S));
      CHECK(hipMalloc(&dst[i], S));
      CHECK(hipMemset(src[i], i, S));
    }
    CHECK(hipDeviceSynchronize());
    std::vector<std::vector<double>> res(vars.size()), host(vars.size());
    for (int r = 0; r < rounds; ++r) {
      for (size_t v = 0; v < vars.size(); ++v) {
        const Var x = vars[v];
        std::vector<unsigned long long> want(D, 0);
        double launch_us = 0;
        const auto t0 = std::chrono::steady_clock::now();
        for (int i = 0; i < N; ++i) {
          const int slot = i % D;
          const volatile unsigned long long* f = hflag + 8 * slot;
          while (*f < want[slot]) {
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(5)) {
              std::printf("flag timeout\n");
              return 2;
            }
          }
          const auto l0 = std::chrono::steady_clock::now();
          hipStream_t s = st[i % x.P];
          const int b = i % nbuf;
          const size_t per = x.chunk / 16;
          unsigned grid = unsigned((n + per - 1) / per);
          want[slot] = ++epoch;
          if (x.sig == 0) {
            hipLaunchKernelGGL(copyk, dim3(grid), dim3(256), 0, s, src[b], dst[b], n, per);
            hipLaunchKernelGGL(flagk, dim3(1), dim3(64), 0, s, dflag + 8 * slot, want[slot]);
          } else if (x.sig == 1) {
            hipLaunchKernelGGL(copysig<0>, dim3(grid), dim3(256), 0, s, src[b], dst[b], n, per,
                               done + 8192 * slot, dflag + 8 * slot, want[slot]);
          } else {
            grid = std::min(grid, 1024u);
            hipLaunchKernelGGL(copysig<1>, dim3(grid), dim3(256), 0, s, src[b], dst[b], n, per,
                               done + 8192 * slot, dflag + 8 * slot, want[slot]);
          }
          if (x.dep) {
            CHECK(hipEventRecord(ev[slot], s));
            CHECK(hipStreamWaitEvent(node, ev[slot], 0));
          }
          launch_us += std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - l0).count();
        }
        for (int slot = 0; slot < D; ++slot) {
          const volatile unsigned long long* f = hflag + 8 * slot;
          while (*f < want[slot]) {
          }
        }
        const double us =
            std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
        res[v].push_back(us / N);
        host[v].push_back(launch_us / N);
        CHECK(hipDeviceSynchronize());
      }
    }
    for (size_t v = 0; v < vars.size(); ++v) {
      auto t = res[v];
      std::sort(t.begin(), t.end());
      auto h = host[v];
      std::sort(h.begin(), h.end());
      const double med = t[t.size() / 2];
      std::printf("{\"streams\": %d, \"sig\": \"%s\", \"chunk\": %zu, \"node_dep\": %s, \"size\": %zu, \"us_per_msg\": %.2f, "
                  "\"host_launch_us\": %.2f, \"TBps_2S\": %.3f, \"payload_GBps\": %.1f}\n",
                  vars[v].P, vars[v].sig == 0 ? "flag-kernel" : vars[v].sig == 1 ? "inkernel-last" : "inkernel-wg0-cap1024",
                  vars[v].chunk, vars[v].dep ? "true" : "false", S, med, h[h.size() / 2],
                  2.0 * S / (med * 1e-6) / 1e12, S / (med * 1e-6) / 1e9);
      std::fflush(stdout);
    }
    for (int i = 0; i < nbuf; ++i) {
      CHECK(hipFree(src[i]));
      CHECK(hipFree(dst[i]));
    }
  }
  return 0;
}
