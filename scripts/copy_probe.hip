// Copy-kernel structure probe (tuning experiment, not product code): HBM->HBM copy of S bytes
// with several workgroup shapes / grid policies / cache policies, each timed with hipEvents
// over back-to-back launches on rotating buffers (> 512 MiB so the Infinity Cache cannot hold
// them).  Variants are interleaved over rounds in one process.
//   hipcc --offload-arch=gfx950 -O3 -o copy_probe scripts/copy_probe.hip && ./copy_probe
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e = (x);                                                           \
    if (e != hipSuccess) {                                                        \
      std::printf("%s: %s\n", #x, hipGetErrorString(e));                          \
      std::exit(1);                                                               \
    }                                                                             \
  } while (0)

template <bool NT>
__device__ __forceinline__ u32x4 ld(const u32x4* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  return *p;
}
template <bool NT>
__device__ __forceinline__ void st(u32x4* p, u32x4 v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// chunked: block b copies units [b*per, (b+1)*per), U loads in flight per lane
template <int T, int U, bool NT>
__global__ __launch_bounds__(T) void chunked(const u32x4* __restrict__ s, u32x4* __restrict__ d,
                                             size_t n, size_t per) {
  size_t b0 = size_t(blockIdx.x) * per, b1 = b0 + per < n ? b0 + per : n;
  for (size_t base = b0 + threadIdx.x; base < b1; base += size_t(T) * U) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      size_t i = base + size_t(u) * T;
      if (i < b1) v[u] = ld<NT>(s + i);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      size_t i = base + size_t(u) * T;
      if (i < b1) st<NT>(d + i, v[u]);
    }
  }
}

// grid-stride: all blocks sweep the whole buffer, U units per lane per sweep
template <int T, int U, bool NT>
__global__ __launch_bounds__(T) void strided(const u32x4* __restrict__ s, u32x4* __restrict__ d,
                                             size_t n, size_t) {
  const size_t stride = size_t(gridDim.x) * T * U;
  for (size_t base = size_t(blockIdx.x) * T * U + threadIdx.x; base < n; base += stride) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      size_t i = base + size_t(u) * T;
      if (i < n) v[u] = ld<NT>(s + i);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      size_t i = base + size_t(u) * T;
      if (i < n) st<NT>(d + i, v[u]);
    }
  }
}

using Kern = void (*)(const u32x4*, u32x4*, size_t, size_t);

struct Var {
  const char* name;
  Kern k;
  int threads, unroll;
  int grid_mode;  // 0: chunk = per bytes; 1: fixed grid
  size_t param;   // bytes per block (mode 0) or number of blocks (mode 1)
};

int main(int argc, char** argv) {
  size_t S = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 40960000;
  const int iters = 30, rounds = 5;
  const size_t n = S / 16;
  const int nbuf = int(std::max<size_t>(2, std::min<size_t>(16, (640u << 20) / (2 * S))));
  std::vector<u32x4*> src(nbuf), dst(nbuf);
  for (int i = 0; i < nbuf; ++i) {
    CHECK(hipMalloc(&src[i], S));
    CHECK(hipMalloc(&dst[i], S));
    CHECK(hipMemset(src[i], i, S));
  }
  std::vector<Var> vars = {
      {"chunk T256 U4 nt 8K", chunked<256, 4, true>, 256, 4, 0, 8192},
      {"chunk T256 U8 nt 20K", chunked<256, 8, true>, 256, 8, 0, 20480},
      {"chunk T256 U8 nt 32K", chunked<256, 8, true>, 256, 8, 0, 32768},
      {"chunk T512 U4 nt 32K", chunked<512, 4, true>, 512, 4, 0, 32768},
      {"chunk T512 U8 nt 64K", chunked<512, 8, true>, 512, 8, 0, 65536},
      {"chunk T1024 U4 nt 64K", chunked<1024, 4, true>, 1024, 4, 0, 65536},
      {"chunk T256 U8 plain 32K", chunked<256, 8, false>, 256, 8, 0, 32768},
      {"stride T256 U4 nt 2048blk", strided<256, 4, true>, 256, 4, 1, 2048},
      {"stride T256 U8 nt 1024blk", strided<256, 8, true>, 256, 8, 1, 1024},
      {"stride T256 U8 nt 2048blk", strided<256, 8, true>, 256, 8, 1, 2048},
      {"stride T512 U4 nt 1024blk", strided<512, 4, true>, 512, 4, 1, 1024},
      {"stride T512 U8 nt 512blk", strided<512, 8, true>, 512, 8, 1, 512},
      {"stride T1024 U4 nt 512blk", strided<1024, 4, true>, 1024, 4, 1, 512},
      {"stride T256 U16 nt 1024blk", strided<256, 16, true>, 256, 16, 1, 1024},
  };
  hipStream_t st;
  CHECK(hipStreamCreate(&st));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  std::vector<std::vector<float>> res(vars.size() + 1);
  for (int r = 0; r < rounds; ++r) {
    for (size_t v = 0; v <= vars.size(); ++v) {
      auto launch = [&](int k) {
        if (v == vars.size()) {
          CHECK(hipMemcpyAsync(dst[k], src[k], S, hipMemcpyDeviceToDevice, st));
          return;
        }
        const Var& x = vars[v];
        size_t per = x.param / 16, grid;
        if (x.grid_mode == 0) grid = (n + per - 1) / per;
        else grid = x.param, per = 0;
        hipLaunchKernelGGL(x.k, dim3(unsigned(grid)), dim3(x.threads), 0, st, src[k], dst[k], n,
                           per);
      };
      for (int w = 0; w < 3; ++w) launch(w % nbuf);
      CHECK(hipEventRecord(e0, st));
      for (int i = 0; i < iters; ++i) launch(i % nbuf);
      CHECK(hipEventRecord(e1, st));
      CHECK(hipEventSynchronize(e1));
      float ms;
      CHECK(hipEventElapsedTime(&ms, e0, e1));
      res[v].push_back(ms / iters);
    }
  }
  for (size_t v = 0; v <= vars.size(); ++v) {
    auto x = res[v];
    std::sort(x.begin(), x.end());
    const float med = x[x.size() / 2];
    std::printf("{\"variant\": \"%s\", \"size\": %zu, \"us\": %.2f, \"TBps_2S\": %.3f}\n",
                v == vars.size() ? "hipMemcpyAsync" : vars[v].name, S, med * 1e3,
                2.0 * S / (med * 1e-3) / 1e12);
  }
  return 0;
}
