// Host cost of the calls a send makes (tuning experiment, not product code): hipLaunchKernelGGL
// with a small (64 B) vs the pack's ~1 KB kernarg block, on one stream vs three round-robin, and
// hipStreamQuery.  Tiny kernels (1 workgroup) so the GPU never backs up; host clock per call.
//   hipcc --offload-arch=gfx950 -O3 -o build/launch_probe scripts/launch_probe.hip
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHECK(x)                                                          \
  do {                                                                    \
    hipError_t err_ = (x);                                                \
    if (err_ != hipSuccess) {                                             \
      std::printf("%s: %s\n", #x, hipGetErrorString(err_));               \
      std::exit(1);                                                       \
    }                                                                     \
  } while (0)

struct Small {
  void* p[8];
};
struct Big {
  void* p[8];
  unsigned long long seg[112];  // ~960 B like PackArgs with 32 segments
};

__global__ void ksmall(Small a) {
  if (threadIdx.x == 0 && a.p[0]) *static_cast<int*>(a.p[0]) = 1;
}
__global__ void kbig(Big a) {
  if (threadIdx.x == 0 && a.p[0]) *static_cast<int*>(a.p[0]) = int(a.seg[5]);
}

int main() {
  std::vector<hipStream_t> st(3);
  for (auto& s : st) CHECK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  Small sa{};
  Big ba{};
  const int N = 3000;
  auto bench = [&](const char* name, auto fn) {
    for (int w = 0; w < 200; ++w) fn(w);
    CHECK(hipDeviceSynchronize());
    std::vector<double> per;
    for (int r = 0; r < 5; ++r) {
      const auto t0 = std::chrono::steady_clock::now();
      for (int i = 0; i < N; ++i) fn(i);
      const double us =
          std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
      per.push_back(us / N);
      CHECK(hipDeviceSynchronize());
    }
    std::sort(per.begin(), per.end());
    std::printf("{\"call\": \"%s\", \"host_us\": %.3f}\n", name, per[per.size() / 2]);
    std::fflush(stdout);
  };
  bench("launch small 1 stream", [&](int) { hipLaunchKernelGGL(ksmall, dim3(1), dim3(64), 0, st[0], sa); });
  bench("launch big 1 stream", [&](int) { hipLaunchKernelGGL(kbig, dim3(1), dim3(64), 0, st[0], ba); });
  bench("launch small 3 streams", [&](int i) { hipLaunchKernelGGL(ksmall, dim3(1), dim3(64), 0, st[i % 3], sa); });
  bench("launch big 3 streams", [&](int i) { hipLaunchKernelGGL(kbig, dim3(1), dim3(64), 0, st[i % 3], ba); });
  bench("launch big 5000 wg 3 streams", [&](int i) { hipLaunchKernelGGL(kbig, dim3(5000), dim3(256), 0, st[i % 3], ba); });
  bench("hipStreamQuery idle", [&](int) { (void)hipStreamQuery(st[0]); });
  bench("hipExtLaunchKernelGGL big", [&](int i) {
    hipExtLaunchKernelGGL(kbig, dim3(1), dim3(64), 0, st[i % 3], nullptr, nullptr, 0, ba);
  });
  return 0;
}
