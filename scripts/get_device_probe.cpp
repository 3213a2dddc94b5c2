// Host cost of hipGetDevice / hipSetDevice (same device) per call: what node.cpp's DeviceScope
// adds to every entry point.   hipcc -O2 scripts/get_device_probe.cpp -o build/get_device_probe
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>

int main() {
  if (hipSetDevice(0) != hipSuccess) return 1;
  int d = -1;
  const int n = 1000000;
  for (int i = 0; i < 1000; ++i) (void)hipGetDevice(&d);
  auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < n; ++i) (void)hipGetDevice(&d);
  auto t1 = std::chrono::steady_clock::now();
  for (int i = 0; i < n; ++i) (void)hipSetDevice(0);
  auto t2 = std::chrono::steady_clock::now();
  std::printf("{\"hipGetDevice_ns\": %.1f, \"hipSetDevice_same_ns\": %.1f}\n",
              std::chrono::duration<double, std::nano>(t1 - t0).count() / n,
              std::chrono::duration<double, std::nano>(t2 - t1).count() / n);
  return 0;
}
