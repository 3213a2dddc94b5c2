// Misaligned-source copy probe (tuning experiment, not product code).  A pack segment whose
// source and sample offsets disagree mod 16 (C3: x/y/z/intensity land at 4 mod 16) is copied
// today by funnel-shifting two aligned 16-B loads per 16-B store (pack_device.h copy_shifted).
// Variants, each a 256-thread workgroup per 8 KiB chunk, 4 units in flight per lane, nt hints:
//   funnel   two aligned loads per unit + v_alignbyte_b32 (current)
//   direct   one 16-B load straight from the misaligned source (unaligned access mode)
//   dpp      one aligned load per unit; the upper half comes from the next lane (ds_bpermute),
//            the wave's last lane loads its own
//   aligned  reference: source and sample both 16-aligned
// Kernel time from HIP events around 20 back-to-back launches over buffers rotating across
// > 512 MiB (no Infinity Cache hits); every variant's output is checked against the source.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 scripts/shift_probe.hip -o build/shift_probe
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      std::printf("%s: %s\n", #x, hipGetErrorString(e_));                         \
      std::exit(1);                                                               \
    }                                                                             \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
constexpr int kThreads = 256;
constexpr int U = 4;
constexpr uint64_t kChunk = 8192;

__device__ __forceinline__ u32x4 ld(const uint8_t* p) {
  return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
}
__device__ __forceinline__ void st(uint8_t* p, u32x4 v) {
  __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
}

template <int Q>
__device__ __forceinline__ u32x4 funnel(u32x4 lo, u32x4 hi, uint32_t b) {
  const uint32_t w[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
  u32x4 o;
  o.x = __builtin_amdgcn_alignbyte(w[Q + 1], w[Q + 0], b);
  o.y = __builtin_amdgcn_alignbyte(w[Q + 2], w[Q + 1], b);
  o.z = __builtin_amdgcn_alignbyte(w[Q + 3], w[Q + 2], b);
  o.w = __builtin_amdgcn_alignbyte(w[Q + 4], w[Q + 3], b);
  return o;
}

__device__ __forceinline__ u32x4 from_next_lane(u32x4 v) {
  const int addr = ((__lane_id() + 1) & 63) << 2;
  u32x4 o;
  o.x = __builtin_amdgcn_ds_bpermute(addr, v.x);
  o.y = __builtin_amdgcn_ds_bpermute(addr, v.y);
  o.z = __builtin_amdgcn_ds_bpermute(addr, v.z);
  o.w = __builtin_amdgcn_ds_bpermute(addr, v.w);
  return o;
}

// dst 16-aligned; src = dst-relative misaligned by r (src & 15 == r) when r > 0.
template <int MODE, int Q>
__global__ __launch_bounds__(kThreads) void copy_kernel(uint8_t* dst, const uint8_t* src,
                                                        uint64_t nunits, uint32_t b) {
  const uint64_t per = kChunk / 16;
  const uint64_t u0 = uint64_t(blockIdx.x) * per;
  const uint64_t u1 = u0 + per < nunits ? u0 + per : nunits;
  const uint8_t* sbase = reinterpret_cast<const uint8_t*>(reinterpret_cast<uintptr_t>(src) & ~uintptr_t(15));
  for (uint64_t base = u0 + threadIdx.x; base < u1; base += kThreads * U) {
    u32x4 v[U];
    if constexpr (MODE == 0) {  // funnel
      u32x4 lo[U], hi[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint64_t i = base + uint64_t(u) * kThreads;
        if (i < u1) {
          lo[u] = ld(sbase + 16 * i);
          hi[u] = ld(sbase + 16 * i + 16);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = funnel<Q>(lo[u], hi[u], b);
    } else if constexpr (MODE == 1) {  // direct unaligned
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint64_t i = base + uint64_t(u) * kThreads;
        if (i < u1) v[u] = ld(src + 16 * i);
      }
    } else if constexpr (MODE == 2) {  // dpp: neighbour's lo
      u32x4 lo[U], hi[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint64_t i = base + uint64_t(u) * kThreads;
        if (i < u1) lo[u] = ld(sbase + 16 * i);
      }
      const bool last = __lane_id() == 63;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint64_t i = base + uint64_t(u) * kThreads;
        hi[u] = from_next_lane(lo[u]);
        if (last || i + 1 >= u1) {
          if (i < u1) hi[u] = ld(sbase + 16 * i + 16);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) v[u] = funnel<Q>(lo[u], hi[u], b);
    } else {  // aligned reference
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint64_t i = base + uint64_t(u) * kThreads;
        if (i < u1) v[u] = ld(src + 16 * i);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = base + uint64_t(u) * kThreads;
      if (i < u1) st(dst + 16 * i, v[u]);
    }
  }
}

template <int MODE>
void launch(uint8_t* dst, const uint8_t* src, uint64_t nunits, hipStream_t s) {
  const uint32_t r = uint32_t(reinterpret_cast<uintptr_t>(src) & 15);
  const uint32_t grid = uint32_t((nunits * 16 + kChunk - 1) / kChunk);
  const uint32_t b = r & 3;
  switch (r >> 2) {
    case 0: copy_kernel<MODE, 0><<<grid, kThreads, 0, s>>>(dst, src, nunits, b); break;
    case 1: copy_kernel<MODE, 1><<<grid, kThreads, 0, s>>>(dst, src, nunits, b); break;
    case 2: copy_kernel<MODE, 2><<<grid, kThreads, 0, s>>>(dst, src, nunits, b); break;
    default: copy_kernel<MODE, 3><<<grid, kThreads, 0, s>>>(dst, src, nunits, b); break;
  }
}

int main() {
  const uint64_t sizes[] = {4096000, 13000000, 40960000};
  const int offs[] = {4, 12, 7};
  const char* names[] = {"funnel", "direct", "dpp", "aligned"};
  const int nbuf = 14;  // 14 x 2 x 40.96 MB > 1 GiB
  std::vector<uint8_t*> src(nbuf), dst(nbuf);
  for (int i = 0; i < nbuf; ++i) {
    CHECK(hipMalloc(&src[i], 41000000 + 64));
    CHECK(hipMalloc(&dst[i], 41000000 + 64));
  }
  std::vector<uint8_t> h(41000000 + 64);
  for (size_t i = 0; i < h.size(); ++i) h[i] = uint8_t((i * 2654435761u) >> 13);
  for (int i = 0; i < nbuf; ++i) CHECK(hipMemcpy(src[i], h.data(), h.size(), hipMemcpyHostToDevice));
  hipStream_t s;
  CHECK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  std::vector<uint8_t> back(41000000);
  for (uint64_t size : sizes) {
    const uint64_t nunits = size / 16;
    for (int off : offs) {
      for (int mode = 0; mode < 4; ++mode) {
        const int o = mode == 3 ? 0 : off;
        auto run = [&](int k) {
          uint8_t* d = dst[k % nbuf];
          const uint8_t* sp = src[k % nbuf] + o;
          switch (mode) {
            case 0: launch<0>(d, sp, nunits, s); break;
            case 1: launch<1>(d, sp, nunits, s); break;
            case 2: launch<2>(d, sp, nunits, s); break;
            default: launch<3>(d, sp, nunits, s); break;
          }
        };
        for (int k = 0; k < 4; ++k) run(k);
        CHECK(hipStreamSynchronize(s));
        float best = 1e9f;
        for (int rep = 0; rep < 3; ++rep) {
          CHECK(hipEventRecord(e0, s));
          for (int k = 0; k < 20; ++k) run(k);
          CHECK(hipEventRecord(e1, s));
          CHECK(hipEventSynchronize(e1));
          float ms = 0;
          CHECK(hipEventElapsedTime(&ms, e0, e1));
          best = ms < best ? ms : best;
        }
        run(0);
        CHECK(hipStreamSynchronize(s));
        CHECK(hipMemcpy(back.data(), dst[0], nunits * 16, hipMemcpyDeviceToHost));
        bool ok = true;
        for (uint64_t i = 0; i < nunits * 16; ++i)
          if (back[i] != h[i + o]) {
            ok = false;
            break;
          }
        const double us = best * 1000.0 / 20;
        std::printf("{\"variant\": \"%s\", \"size\": %llu, \"src_mod16\": %d, \"us_per_launch\": %.2f, "
                    "\"TBps_2S\": %.3f, \"ok\": %s}\n",
                    names[mode], (unsigned long long)size, o, us, 2.0 * size / us / 1e6,
                    ok ? "true" : "false");
        std::fflush(stdout);
      }
    }
  }
  return 0;
}
