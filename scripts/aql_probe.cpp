// Direct AQL dispatch probe (tuning experiment, not product code): a node-owned HSA queue with
// raw kernel-dispatch packets vs hipLaunchKernelGGL, for the signalling copy of
// scripts/aql_kernel.hip.  Measures host cost per dispatch, dispatch -> fill flag seen on the
// host (isolated), back-to-back throughput with <= 8 messages in flight, and checks every
// copy's bytes.
//   hipcc --genco --offload-arch=gfx950 -O3 --offload-device-only --no-gpu-bundle-output \
//       scripts/aql_kernel.hip -o build/aql_kernel.co
//   hipcc -O3 -o build/aql_probe scripts/aql_probe.cpp -lhsa-runtime64 && build/aql_probe
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <iterator>
#include <string>
#include <vector>

#define CHECK(x)                                                         \
  do {                                                                   \
    hipError_t err_ = (x);                                               \
    if (err_ != hipSuccess) {                                            \
      std::printf("%s: %s\n", #x, hipGetErrorString(err_));              \
      std::exit(1);                                                      \
    }                                                                    \
  } while (0)
#define HSA(x)                                                           \
  do {                                                                   \
    hsa_status_t st_ = (x);                                              \
    if (st_ != HSA_STATUS_SUCCESS) {                                     \
      const char* m_ = nullptr;                                          \
      hsa_status_string(st_, &m_);                                       \
      std::printf("%s: %s\n", #x, m_ ? m_ : "?");                        \
      std::exit(1);                                                      \
    }                                                                    \
  } while (0)

struct AqlArgs {
  const void* s;
  void* d;
  unsigned long long n;
  unsigned long long* flag;
  unsigned* done;
  unsigned long long epoch;
  unsigned grid;
  unsigned per;
};
static_assert(sizeof(AqlArgs) == 56, "kernarg layout");

double now_us() {
  return std::chrono::duration<double, std::micro>(
             std::chrono::steady_clock::now().time_since_epoch())
      .count();
}

struct Found {
  hsa_agent_t gpu{}, cpu{};
  uint32_t want_bdf = 0;
  bool gpu_ok = false, cpu_ok = false;
  hsa_amd_memory_pool_t kernarg{};
  bool ka_ok = false;
  hsa_amd_memory_pool_t devpool{};  // GPU global pool (fine-grained preferred)
  bool dev_ok = false, dev_fine = false;
};

hsa_status_t find_dev_pool(hsa_amd_memory_pool_t pool, void* p) {
  Found* f = static_cast<Found*>(p);
  hsa_amd_segment_t seg;
  hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
  if (seg != HSA_AMD_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
  bool alloc_ok = false;
  hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_RUNTIME_ALLOC_ALLOWED, &alloc_ok);
  if (!alloc_ok) return HSA_STATUS_SUCCESS;
  uint32_t flags = 0;
  hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
  const bool fine = flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_FINE_GRAINED;
  if (!f->dev_ok || (fine && !f->dev_fine)) {
    f->devpool = pool;
    f->dev_ok = true;
    f->dev_fine = fine;
  }
  return HSA_STATUS_SUCCESS;
}

hsa_status_t find_agents(hsa_agent_t a, void* p) {
  Found* f = static_cast<Found*>(p);
  hsa_device_type_t t;
  hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t == HSA_DEVICE_TYPE_GPU && !f->gpu_ok) {
    uint32_t bdf = 0;
    hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf);
    if (bdf == f->want_bdf) {
      f->gpu = a;
      f->gpu_ok = true;
    }
  }
  if (t == HSA_DEVICE_TYPE_CPU && !f->cpu_ok) {
    f->cpu = a;
    f->cpu_ok = true;
  }
  return HSA_STATUS_SUCCESS;
}

hsa_status_t find_kernarg_pool(hsa_amd_memory_pool_t pool, void* p) {
  Found* f = static_cast<Found*>(p);
  hsa_amd_segment_t seg;
  hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
  if (seg != HSA_AMD_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
  uint32_t flags = 0;
  hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
  if ((flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_KERNARG_INIT) && !f->ka_ok) {
    f->kernarg = pool;
    f->ka_ok = true;
  }
  return HSA_STATUS_SUCCESS;
}

void queue_error(hsa_status_t st, hsa_queue_t*, void*) {
  const char* m = nullptr;
  hsa_status_string(st, &m);
  std::printf("queue error: %s\n", m ? m : "?");
  std::exit(3);
}

__global__ void hip_copy_sig_stub() {}

int main() {
  CHECK(hipSetDevice(0));
  CHECK(hipFree(nullptr));
  int bus = 0, devn = 0, dom = 0;
  CHECK(hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, 0));
  CHECK(hipDeviceGetAttribute(&devn, hipDeviceAttributePciDeviceId, 0));
  CHECK(hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, 0));
  HSA(hsa_init());
  Found f;
  f.want_bdf = (uint32_t(bus) << 8) | (uint32_t(devn) << 3);  // function 0
  HSA(hsa_iterate_agents(find_agents, &f));
  if (!f.gpu_ok || !f.cpu_ok) {
    std::printf("agent not found (bdf %x)\n", f.want_bdf);
    return 2;
  }
  HSA(hsa_amd_agent_iterate_memory_pools(f.cpu, find_kernarg_pool, &f));
  if (!f.ka_ok) {
    std::printf("no kernarg pool\n");
    return 2;
  }
  // code object
  const char* co_path = std::getenv("CO") ? std::getenv("CO") : "build/aql_kernel.co";
  std::ifstream in(co_path, std::ios::binary);
  std::vector<char> co((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
  if (co.empty()) {
    std::printf("build/aql_kernel.co missing\n");
    return 2;
  }
  hsa_code_object_reader_t reader;
  HSA(hsa_code_object_reader_create_from_memory(co.data(), co.size(), &reader));
  hsa_executable_t exe;
  HSA(hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, nullptr,
                                &exe));
  HSA(hsa_executable_load_agent_code_object(exe, f.gpu, reader, nullptr, nullptr));
  HSA(hsa_executable_freeze(exe, nullptr));
  hsa_executable_symbol_t sym;
  HSA(hsa_executable_get_symbol_by_name(exe, "aql_copy_sig.kd", &f.gpu, &sym));
  uint64_t kobj = 0;
  uint32_t ka_size = 0, grp = 0, priv = 0;
  HSA(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &kobj));
  HSA(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE,
                                     &ka_size));
  HSA(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE,
                                     &grp));
  HSA(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE,
                                     &priv));
  std::printf("{\"kernarg_size\": %u, \"group\": %u, \"private\": %u}\n", ka_size, grp, priv);
  if (ka_size != sizeof(AqlArgs)) {
    std::printf("unexpected kernarg size\n");
    return 2;
  }
  // queue and kernarg ring
  const int nq = std::getenv("Q") ? std::atoi(std::getenv("Q")) : 1;
  std::vector<hsa_queue_t*> qs(nq);
  for (int i = 1; i < nq; ++i)
    HSA(hsa_queue_create(f.gpu, 1024, HSA_QUEUE_TYPE_SINGLE, queue_error, nullptr, UINT32_MAX,
                         UINT32_MAX, &qs[i]));
  hsa_queue_t* q = nullptr;
  HSA(hsa_queue_create(f.gpu, 1024, HSA_QUEUE_TYPE_SINGLE, queue_error, nullptr, UINT32_MAX,
                       UINT32_MAX, &q));
  const int kRing = 256;
  void* ka = nullptr;
  const char* kae = std::getenv("KA");
  const bool dev_ka = kae && (std::string(kae) == "dev" || std::string(kae) == "devhdp");
  const bool hdp = kae && std::string(kae) == "devhdp";
  hsa_amd_hdp_flush_t hdpf{};
  if (hdp) HSA(hsa_agent_get_info(f.gpu, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_HDP_FLUSH, &hdpf));
  if (dev_ka) {
    HSA(hsa_amd_agent_iterate_memory_pools(f.gpu, find_dev_pool, &f));
    if (!f.dev_ok) {
      std::printf("no device pool\n");
      return 2;
    }
    HSA(hsa_amd_memory_pool_allocate(f.devpool, kRing * 64, 0, &ka));
    HSA(hsa_amd_agents_allow_access(1, &f.cpu, nullptr, ka));
  } else {
    HSA(hsa_amd_memory_pool_allocate(f.kernarg, kRing * 64, 0, &ka));
    HSA(hsa_amd_agents_allow_access(1, &f.gpu, nullptr, ka));
  }
  const char* fe = std::getenv("FENCE");
  const int acq = fe && std::string(fe) == "agent" ? HSA_FENCE_SCOPE_AGENT
                  : fe && std::string(fe) == "none" ? HSA_FENCE_SCOPE_NONE : HSA_FENCE_SCOPE_SYSTEM;
  int rel = acq;
  int acq2 = acq;
  if (fe && std::string(fe) == "sysacq") {  // system-scope acquire, agent-scope release
    acq2 = HSA_FENCE_SCOPE_SYSTEM;
    rel = HSA_FENCE_SCOPE_AGENT;
  }
  std::printf("{\"kernarg\": \"%s\", \"dev_fine\": %d, \"fence\": %d}\n",
              dev_ka ? "device" : "host", int(f.dev_fine), acq);
  // flags (mapped pinned host), done words (device)
  unsigned long long* hflag;
  CHECK(hipHostMalloc(reinterpret_cast<void**>(&hflag), 64 * 16, hipHostMallocMapped));
  unsigned long long* dflag;
  CHECK(hipHostGetDevicePointer(reinterpret_cast<void**>(&dflag), hflag, 0));
  std::memset(hflag, 0, 64 * 16);
  unsigned* done;
  CHECK(hipMalloc(&done, 16 * 4096 * 4));
  CHECK(hipMemset(done, 0, 16 * 4096 * 4));
  CHECK(hipDeviceSynchronize());
  // every ring slot starts with harmless arguments (no bytes, dummy flag 15): a dispatch that
  // read a stale slot could only re-run an earlier, valid copy
  for (int r = 0; r < kRing; ++r) {
    AqlArgs z{};
    z.flag = dflag + 8 * 15;
    z.done = done + 4096 * 15;
    z.grid = 1;
    z.per = 512;
    std::memcpy(static_cast<char*>(ka) + 64 * r, &z, sizeof(z));
  }
  __builtin_ia32_sfence();
  (void)*reinterpret_cast<volatile unsigned*>(static_cast<char*>(ka) + 64 * (kRing - 1));

  uint64_t epoch = 0;
  int ring_next = 0;
  std::vector<uint64_t> ring_epoch(kRing, 0);
  std::vector<int> ring_flag(kRing, 0);
  auto dispatch = [&](const void* s, void* d, size_t bytes, int slot) -> uint64_t {
    const int r = ring_next++ % kRing;
    const volatile unsigned long long* rf = hflag + 8 * ring_flag[r];
    while (*rf < ring_epoch[r]) {
    }  // kernarg slot still in use
    AqlArgs* a = reinterpret_cast<AqlArgs*>(static_cast<char*>(ka) + 64 * r);
    a->s = s;
    a->d = d;
    a->n = bytes / 16;
    a->flag = dflag + 8 * slot;
    a->done = done + 4096 * slot;
    a->epoch = ++epoch;
    a->per = 8192 / 16;
    const unsigned long long nch = (a->n + a->per - 1) / a->per;
    a->grid = unsigned(std::min<unsigned long long>(std::max<unsigned long long>(nch, 1), 1024));
    ring_epoch[r] = epoch;
    ring_flag[r] = slot;
    qs[0] = q;
    hsa_queue_t* const qq = qs[epoch % nq];
    const uint64_t idx = hsa_queue_add_write_index_relaxed(qq, 1);
    while (idx - hsa_queue_load_read_index_relaxed(qq) >= qq->size) {
    }
    hsa_kernel_dispatch_packet_t* p =
        static_cast<hsa_kernel_dispatch_packet_t*>(qq->base_address) + (idx & (qq->size - 1));
    p->workgroup_size_x = 256;
    p->workgroup_size_y = 1;
    p->workgroup_size_z = 1;
    p->reserved0 = 0;
    p->grid_size_x = a->grid * 256;
    p->grid_size_y = 1;
    p->grid_size_z = 1;
    p->private_segment_size = priv;
    p->group_segment_size = grp;
    p->kernel_object = kobj;
    p->kernarg_address = a;
    p->reserved2 = 0;
    p->completion_signal.handle = 0;
    if (hdp) {
      // write-combined kernargs leave the CPU, then the HDP flush makes them visible to the
      // GPU (posted writes, ordered before the doorbell); no PCIe read round trip
      __builtin_ia32_sfence();
      *reinterpret_cast<volatile uint32_t*>(hdpf.HDP_MEM_FLUSH_CNTL) = 1;
      __builtin_ia32_sfence();
    } else if (dev_ka) {
      __builtin_ia32_sfence();  // write-combined kernargs reach the device before the packet
      (void)*reinterpret_cast<volatile unsigned*>(a);
    }
    const uint16_t header = (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                            (acq2 << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                            (rel << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
    const uint16_t setup = 1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;
    __atomic_store_n(reinterpret_cast<uint32_t*>(p), header | (uint32_t(setup) << 16),
                     __ATOMIC_RELEASE);
    hsa_signal_store_relaxed(qq->doorbell_signal, idx);
    return epoch;
  };
  auto wait_flag = [&](int slot, uint64_t e) {
    const volatile unsigned long long* fl = hflag + 8 * slot;
    const double t0 = now_us();
    while (*fl < e) {
      if (now_us() - t0 > 2e6) {
        std::printf("flag timeout slot %d epoch %llu\n", slot, (unsigned long long)e);
        std::exit(4);
      }
    }
  };

  std::vector<size_t> sizes = {4096, 65536, 1 << 20, 4096000, 16777216, 40960000};
  const size_t maxs = 40960000;
  std::vector<void*> src(4), dst(8);
  for (auto& p : src) {
    CHECK(hipMalloc(&p, maxs));
  }
  for (auto& p : dst) CHECK(hipMalloc(&p, maxs));
  for (int i = 0; i < 4; ++i) CHECK(hipMemset(src[i], 0x11 * (i + 1), maxs));
  CHECK(hipDeviceSynchronize());
  std::vector<unsigned char> host(maxs);

  for (size_t S : sizes) {
    // correctness: one copy per destination, compare bytes
    for (int k = 0; k < 8; ++k) {
      CHECK(hipMemset(dst[k], 0, S));
      CHECK(hipDeviceSynchronize());
      const uint64_t e = dispatch(src[k % 4], dst[k], S, k);
      wait_flag(k, e);
      CHECK(hipMemcpy(host.data(), dst[k], S, hipMemcpyDeviceToHost));
      for (size_t i = 0; i < S; ++i)
        if (host[i] != (unsigned char)(0x11 * (k % 4 + 1))) {
          std::printf("mismatch size %zu dst %d at %zu\n", S, k, i);
          return 5;
        }
    }
    // isolated latency: dispatch -> flag seen
    std::vector<double> lat, host_cost;
    for (int i = 0; i < 50; ++i) {
      const double t0 = now_us();
      const uint64_t e = dispatch(src[i % 4], dst[i % 8], S, i % 8);
      const double t1 = now_us();
      wait_flag(i % 8, e);
      lat.push_back(now_us() - t0);
      host_cost.push_back(t1 - t0);
    }
    std::sort(lat.begin(), lat.end());
    std::sort(host_cost.begin(), host_cost.end());
    // back-to-back, <= 8 in flight
    const int N = 400;
    std::vector<uint64_t> want(8, 0);
    const double t0 = now_us();
    double hc = 0;
    for (int i = 0; i < N; ++i) {
      const int slot = i % 8;
      wait_flag(slot, want[slot]);
      const double a = now_us();
      want[slot] = dispatch(src[i % 4], dst[slot], S, slot);
      hc += now_us() - a;
    }
    for (int slot = 0; slot < 8; ++slot) wait_flag(slot, want[slot]);
    const double us = (now_us() - t0) / N;
    std::printf("{\"path\": \"aql-%s-f%d\", \"size\": %zu, \"dispatch_host_us_p50\": %.3f, "
                "\"isolated_flag_latency_us_p50\": %.2f, \"b2b_us_per_msg\": %.3f, "
                "\"b2b_host_us\": %.3f, \"TBps_2S\": %.3f, \"queues\": %d, \"code_object\": \"%s\"}\n",
                hdp ? (nq == 1 ? "devka-hdp" : nq == 2 ? "devka-hdp-q2" : "devka-hdp-q3") : dev_ka ? "devka" : "hostka", acq2 * 10 + rel, S, host_cost[host_cost.size() / 2], lat[lat.size() / 2], us, hc / N,
                2.0 * S / (us * 1e-6) / 1e12, nq, co_path);
    std::fflush(stdout);
  }
  HSA(hsa_queue_destroy(q));
  return 0;
}
