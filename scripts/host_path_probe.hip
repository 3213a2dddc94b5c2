// Host <-> HBM sample paths probe (experiment, not product code; DESIGN §2 host sources, §2
// host-only receivers).  For each size it times, per message, with inputs warm in the host cache
// for small sizes:
//   h2d_pageable   hipMemcpyAsync(dev, pageable host) + stream sync   (the r05 host-source path)
//   h2d_pinned     memcpy into pinned staging + hipMemcpyAsync + sync
//   bar_memcpy     CPU stores straight into a hipMalloc slot mapped for the CPU (BAR):
//                  memcpy / AVX2 streaming stores, sfence, HDP flush, one read-back
//   h2d_kernel     memcpy into pinned staging + a copy kernel reading host memory + sync
//   d2h_pinned     hipMemcpyAsync(pinned, dev) + sync   (host-only receiver staging)
//   d2h_kernel     a copy kernel writing pinned host memory + sync
//   d2h_pageable   hipMemcpy(pageable, dev)
// and checks that every path delivered the bytes, and that a BAR-mapped slot still exports an
// IPC handle.
//   hipcc --offload-arch=gfx950 -O3 -mavx2 -o build/host_path_probe scripts/host_path_probe.hip \
//         -lhsa-runtime64
//   build/host_path_probe [reps_small] [reps_large]
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <immintrin.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CHECK(x)                                                                    \
  do {                                                                              \
    hipError_t e_ = (x);                                                            \
    if (e_ != hipSuccess) {                                                         \
      std::printf("%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                 \
    }                                                                               \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void copy16(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                              uint64_t n16) {
  for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n16; i += uint64_t(gridDim.x) * 256)
    __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
}

namespace {

double now_us() {
  return std::chrono::duration<double, std::micro>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

struct Agents {
  uint32_t bdf = 0;
  hsa_agent_t gpu{}, cpu{};
  bool gpu_ok = false, cpu_ok = false;
};

hsa_status_t on_agent(hsa_agent_t a, void* p) {
  auto* f = static_cast<Agents*>(p);
  hsa_device_type_t t;
  hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t == HSA_DEVICE_TYPE_GPU) {
    uint32_t bdf = 0;
    hsa_agent_get_info(a, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_BDFID), &bdf);
    if (bdf == f->bdf) {
      f->gpu = a;
      f->gpu_ok = true;
    }
  } else if (t == HSA_DEVICE_TYPE_CPU && !f->cpu_ok) {
    f->cpu = a;
    f->cpu_ok = true;
  }
  return HSA_STATUS_SUCCESS;
}

void stream_copy(void* dst, const void* src, size_t n) {
  // 32-B streaming stores to a 32-B aligned destination (slots are 2 MiB aligned), tail bytes
  // with plain stores
  auto* d = static_cast<uint8_t*>(dst);
  auto* s = static_cast<const uint8_t*>(src);
  size_t i = 0;
  for (; i + 128 <= n; i += 128) {
    __m256i a = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i));
    __m256i b = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i + 32));
    __m256i c = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i + 64));
    __m256i e = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i + 96));
    _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i), a);
    _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i + 32), b);
    _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i + 64), c);
    _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i + 96), e);
  }
  if (i < n) std::memcpy(d + i, s + i, n - i);
}

struct Stat {
  double p50, p10, mn;
};

Stat stat(std::vector<double> v) {
  std::sort(v.begin(), v.end());
  return {v[v.size() / 2], v[v.size() / 10], v[0]};
}

}  // namespace

int main(int argc, char** argv) {
  const int reps_small = argc > 1 ? std::atoi(argv[1]) : 300;
  const int reps_large = argc > 2 ? std::atoi(argv[2]) : 30;
  CHECK(hipSetDevice(0));
  int bus = 0, devn = 0;
  CHECK(hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, 0));
  CHECK(hipDeviceGetAttribute(&devn, hipDeviceAttributePciDeviceId, 0));
  if (hsa_init() != HSA_STATUS_SUCCESS) {
    std::printf("hsa_init failed\n");
    return 1;
  }
  Agents ag;
  ag.bdf = (uint32_t(bus) << 8) | (uint32_t(devn) << 3);
  hsa_iterate_agents(on_agent, &ag);
  if (!ag.gpu_ok || !ag.cpu_ok) {
    std::printf("agents not found\n");
    return 1;
  }
  hsa_amd_hdp_flush_t hdp{};
  hsa_agent_get_info(ag.gpu, static_cast<hsa_agent_info_t>(HSA_AMD_AGENT_INFO_HDP_FLUSH), &hdp);
  volatile uint32_t* hdp_reg = hdp.HDP_MEM_FLUSH_CNTL;
  std::printf("{\"probe\": \"host_path\", \"hdp\": %s}\n", hdp_reg ? "true" : "false");

  hipStream_t st;
  CHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  const size_t sizes[] = {4096, 16384, 65536, 1 << 20, 4 << 20, 6220800, 40960000};
  const size_t maxz = 40960000;
  uint8_t* host = static_cast<uint8_t*>(std::aligned_alloc(4096, maxz));
  uint8_t* back = static_cast<uint8_t*>(std::aligned_alloc(4096, maxz));
  for (size_t i = 0; i < maxz; ++i) host[i] = uint8_t(i * 2654435761u >> 13);
  uint8_t* pinned = nullptr;
  uint8_t* pinned2 = nullptr;
  CHECK(hipHostMalloc(reinterpret_cast<void**>(&pinned), maxz, hipHostMallocDefault));
  CHECK(hipHostMalloc(reinterpret_cast<void**>(&pinned2), maxz, hipHostMallocDefault));
  uint8_t* dev = nullptr;
  CHECK(hipMalloc(&dev, (maxz + (2 << 20)) & ~size_t((2 << 20) - 1)));
  hsa_status_t aa = hsa_amd_agents_allow_access(1, &ag.cpu, nullptr, dev);
  hipIpcMemHandle_t ih;
  hipError_t ipc = hipIpcGetMemHandle(&ih, dev);
  std::printf("{\"allow_access_cpu\": %d, \"ipc_after_allow\": \"%s\"}\n", int(aa),
              hipGetErrorString(ipc));
  (void)hipGetLastError();
  const bool bar = aa == HSA_STATUS_SUCCESS;

  auto verify = [&](size_t z, const char* what) {
    std::memset(back, 0, z);
    CHECK(hipMemcpy(back, dev, z, hipMemcpyDeviceToHost));
    if (std::memcmp(back, host, z) != 0) std::printf("{\"MISMATCH\": \"%s\", \"size\": %zu}\n", what, z);
  };
  auto report = [&](const char* what, size_t z, std::vector<double>& v) {
    Stat s = stat(v);
    std::printf("{\"path\": \"%s\", \"size\": %zu, \"p50_us\": %.2f, \"p10_us\": %.2f, "
                "\"min_us\": %.2f, \"GBps_p50\": %.2f}\n",
                what, z, s.p50, s.p10, s.mn, z / s.p50 / 1e3);
    std::fflush(stdout);
  };

  for (size_t z : sizes) {
    const int reps = z >= (4u << 20) ? reps_large : reps_small;
    std::vector<double> v;
    auto run = [&](const char* what, auto&& fn) {
      v.clear();
      for (int r = 0; r < reps + 5; ++r) {
        const double t0 = now_us();
        fn();
        const double t1 = now_us();
        if (r >= 5) v.push_back(t1 - t0);
      }
      report(what, z, v);
    };
    const unsigned grid = unsigned(std::min<uint64_t>(1024, (z / 16 + 255) / 256));
    // ---- H2D ----
    CHECK(hipMemset(dev, 0, z));
    CHECK(hipDeviceSynchronize());
    run("h2d_pageable", [&] {
      CHECK(hipMemcpyAsync(dev, host, z, hipMemcpyHostToDevice, st));
      CHECK(hipStreamSynchronize(st));
    });
    verify(z, "h2d_pageable");
    CHECK(hipMemset(dev, 0, z));
    CHECK(hipDeviceSynchronize());
    run("h2d_pinned", [&] {
      std::memcpy(pinned, host, z);
      CHECK(hipMemcpyAsync(dev, pinned, z, hipMemcpyHostToDevice, st));
      CHECK(hipStreamSynchronize(st));
    });
    verify(z, "h2d_pinned");
    run("memcpy_to_pinned_only", [&] { std::memcpy(pinned2, host, z); });
    CHECK(hipMemset(dev, 0, z));
    CHECK(hipDeviceSynchronize());
    run("h2d_kernel", [&] {
      std::memcpy(pinned, host, z);
      hipLaunchKernelGGL(copy16, dim3(grid), dim3(256), 0, st,
                         reinterpret_cast<const u32x4*>(pinned), reinterpret_cast<u32x4*>(dev),
                         uint64_t(z / 16));
      CHECK(hipStreamSynchronize(st));
    });
    verify(z, "h2d_kernel");
    if (bar) {
      CHECK(hipMemset(dev, 0, z));
      CHECK(hipDeviceSynchronize());
      run("bar_memcpy", [&] {
        std::memcpy(dev, host, z);
        _mm_sfence();
        if (hdp_reg) *hdp_reg = 1;
        (void)*reinterpret_cast<volatile uint32_t*>(dev + ((z - 4) & ~size_t(3)));
      });
      verify(z, "bar_memcpy");
      CHECK(hipMemset(dev, 0, z));
      CHECK(hipDeviceSynchronize());
      run("bar_stream", [&] {
        stream_copy(dev, host, z);
        _mm_sfence();
        if (hdp_reg) *hdp_reg = 1;
        (void)*reinterpret_cast<volatile uint32_t*>(dev + ((z - 4) & ~size_t(3)));
      });
      verify(z, "bar_stream");
      run("bar_stream_noreadback", [&] {
        stream_copy(dev, host, z);
        _mm_sfence();
        if (hdp_reg) *hdp_reg = 1;
      });
      run("bar_readback_only", [&] {
        if (hdp_reg) *hdp_reg = 1;
        (void)*reinterpret_cast<volatile uint32_t*>(dev + ((z - 4) & ~size_t(3)));
      });
    }
    // ---- D2H ----
    CHECK(hipMemcpy(dev, host, z, hipMemcpyHostToDevice));
    run("d2h_pinned", [&] {
      CHECK(hipMemcpyAsync(pinned, dev, z, hipMemcpyDeviceToHost, st));
      CHECK(hipStreamSynchronize(st));
    });
    if (std::memcmp(pinned, host, z)) std::printf("{\"MISMATCH\": \"d2h_pinned\"}\n");
    std::memset(pinned, 0, z);
    run("d2h_kernel", [&] {
      hipLaunchKernelGGL(copy16, dim3(grid), dim3(256), 0, st, reinterpret_cast<const u32x4*>(dev),
                         reinterpret_cast<u32x4*>(pinned), uint64_t(z / 16));
      CHECK(hipStreamSynchronize(st));
    });
    if (std::memcmp(pinned, host, z & ~size_t(15))) std::printf("{\"MISMATCH\": \"d2h_kernel\"}\n");
    run("d2h_pageable", [&] { CHECK(hipMemcpy(back, dev, z, hipMemcpyDeviceToHost)); });
    run("d2h_pinned_plus_memcpy_out", [&] {
      CHECK(hipMemcpyAsync(pinned, dev, z, hipMemcpyDeviceToHost, st));
      CHECK(hipStreamSynchronize(st));
      std::memcpy(back, pinned, z);
    });
    if (z >= (1u << 20)) {
      run("host_register_unregister", [&] {
        CHECK(hipHostRegister(back, z, hipHostRegisterDefault));
        CHECK(hipHostUnregister(back));
      });
    }
  }
  std::printf("{\"done\": true}\n");
  return 0;
}
