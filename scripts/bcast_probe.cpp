// Exercises the RCCL loader and group calls of dora_amd/csrc/bcast.cpp on one GPU: a one-rank
// group (the only group a one-GPU box can form: RCCL refuses two ranks on one device) is
// formed through the same non-blocking init / settle path, broadcasts a buffer in place and is
// closed.  Multi-rank groups run only on the driver's multi-GPU node (bench.py c4_fanout_rccl).
//   hipcc -O2 -std=c++17 -Iinclude -Idora_amd/csrc scripts/bcast_probe.cpp -Ldora_amd/lib -ldora_gpu
//         -Wl,-rpath,'$ORIGIN/../dora_amd/lib' -o build/bcast_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

#include "bcast.h"
#include "dora_gpu.h"

int main() {
  std::string why;
  if (!dora::bcast_available(&why)) {
    std::printf("{\"ok\": false, \"error\": \"%s\"}\n", why.c_str());
    return 1;
  }
  uint8_t uid[dora::kBcastIdBytes];
  if (dora::bcast_unique_id(uid) != DORA_OK) {
    std::printf("{\"ok\": false, \"error\": \"unique id: %s\"}\n", dora_gpu_last_error());
    return 1;
  }
  dora::BcastComm* c = nullptr;
  if (dora::bcast_join(uid, 1, 0, 30000, &c) != DORA_OK) {
    std::printf("{\"ok\": false, \"error\": \"join: %s\"}\n", dora_gpu_last_error());
    return 1;
  }
  const size_t n = 6220800;
  std::vector<uint8_t> h(n), back(n);
  for (size_t i = 0; i < n; ++i) h[i] = static_cast<uint8_t>(i * 131 + 7);
  void* d = nullptr;
  hipStream_t st;
  (void)hipStreamCreate(&st);
  (void)hipMalloc(&d, n);
  (void)hipMemcpy(d, h.data(), n, hipMemcpyHostToDevice);
  int rc = dora::bcast_enqueue(c, d, n, st);
  (void)hipStreamSynchronize(st);
  (void)hipMemcpy(back.data(), d, n, hipMemcpyDeviceToHost);
  dora::bcast_close(c, st, 10000);
  const bool same = back == h;
  std::printf("{\"ok\": %s, \"enqueue_rc\": %d, \"bytes\": %zu, \"intact\": %s}\n",
              rc == DORA_OK && same ? "true" : "false", rc, n, same ? "true" : "false");
  (void)hipFree(d);
  (void)hipStreamDestroy(st);
  return rc == DORA_OK && same ? 0 : 1;
}
