// HIP kernels of the data plane (gfx950): launches of the batched segmented pack (device code in
// pack_device.h) that replaces `copy_array_into_sample` (apis/rust/node/src/node/
// arrow_utils.rs:23-71), the compacting transforms, the csum64 parity reduction and the
// splitmix64 payload generator.
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <mutex>
#include <cstring>
#include <string>
#include <vector>

#include "aql.h"
#include "common.h"
#include "pack_device.h"
#include "plan.h"

namespace dora {
namespace {

using namespace pack;

template <int U, int NT>
__global__ __launch_bounds__(kThreads) void pack_kernel(PackArgs args) {
  // grid = chunks (one chunk per workgroup), or fewer workgroups striding over the chunks when
  // the launch signals its fill (fewer workgroups to count in)
  pack_body<U, NT>(args, blockIdx.x, gridDim.x);
}

// Workgroups at most of a pack the command processor signals: a synchronous 40.96 MB send
// (5,000 chunks) takes 21.7-22.0 us with 3584 workgroups against 22.0-22.7 with 4096, 22.9 with
// one per chunk, 22.7-23.3 with 3072 and 24.6-25.3 with fewer, larger chunks, in four interleaved
// rounds of 200 sends (profiles/r04_sync_ab.jsonl batches sy4-sy6; packs below 28 MiB have fewer
// chunks than that).
constexpr uint32_t kCpGrid = 3584;
// Workgroups at most of a multi-segment pack the command processor signals.  Such packs (C3's
// 13 MB clouds) run up to four at once, one per queue: 640 workgroups each (2.5 per CU) against
// the single-segment cap of 3584, C3's 20-cloud burst 0.67-0.72 -> 0.72-0.75 and its 200-cloud
// steady state 0.71-0.72 -> 0.77-0.79 of HBM (caps 512-1536 interleaved over four boxes,
// profiles/r05_c3_cp_grid_b.jsonl, r05_c3_multi_grid_*.jsonl).
constexpr uint32_t kCpGridMulti = 640;

// The HIP-launched pack: 4 x 16-B loads in flight per lane, non-temporal loads and stores (the
// r01 sweep, profiles/r01_pack_sweep*.jsonl: 10-12 % at 16-40 MB, the sample is consumed by
// another process; neutral below); its signalling launch stores write-through (NT = 2).  The
// sweep's other variants (2 / 8 loads, cached stores) and their tuning hooks were removed in r06
// (verdict r05 item 6): the product library carries no variant only a microbenchmark selects.
constexpr int kUnroll = 4;

// ------------------------------------------------------------------------------------------
// Transform segments of compacting plans: bitmap slices shifted to bit 0 and offsets rebased to
// 0.  Elementwise and tiny next to the value buffers (a bitmap is len/8 bytes, offsets
// 4-8 B per list), so one simple grid over all transform segments.
// ------------------------------------------------------------------------------------------
struct XSeg {
  const uint8_t* src;
  uint64_t dst_off;
  uint64_t len;      // output bytes
  uint64_t src_len;  // readable source bytes (bitshift)
  uint32_t op;
  uint32_t aux;      // bit offset (bitshift)
};

struct XArgs {
  uint8_t* dst;
  uint32_t nseg;
  uint32_t block_end[kMaxSegs];
  XSeg seg[kMaxSegs];
};

constexpr uint64_t kXElems = 4096;  // output elements per workgroup

template <typename T>
__device__ __forceinline__ void rebase(const uint8_t* src, uint8_t* dst, uint64_t count,
                                       uint64_t e0, uint64_t e1) {
  T base;
  __builtin_memcpy(&base, src, sizeof(T));
  const bool aligned = ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) &
                        (sizeof(T) - 1)) == 0;
  for (uint64_t i = e0 + threadIdx.x; i < e1 && i < count; i += kThreads) {
    if (aligned) {
      reinterpret_cast<T*>(dst)[i] = reinterpret_cast<const T*>(src)[i] - base;
    } else {
      T v;
      __builtin_memcpy(&v, src + i * sizeof(T), sizeof(T));
      v -= base;
      __builtin_memcpy(dst + i * sizeof(T), &v, sizeof(T));
    }
  }
}

__global__ __launch_bounds__(kThreads) void transform_kernel(XArgs a) {
  const uint32_t blk = blockIdx.x;
  uint32_t s = 0;
  while (s + 1 < a.nseg && blk >= a.block_end[s]) ++s;
  const XSeg g = a.seg[s];
  const uint64_t c = blk - (s ? a.block_end[s - 1] : 0u);
  const uint64_t e0 = c * kXElems, e1 = e0 + kXElems;
  uint8_t* dst = a.dst + g.dst_off;
  if (g.op == SEG_BITSHIFT) {
    for (uint64_t j = e0 + threadIdx.x; j < e1 && j < g.len; j += kThreads) {
      const uint32_t lo = g.src[j];
      const uint32_t hi = j + 1 < g.src_len ? g.src[j + 1] : 0u;
      dst[j] = static_cast<uint8_t>(g.aux ? ((lo >> g.aux) | (hi << (8 - g.aux))) : lo);
    }
  } else if (g.op == SEG_REBASE32) {
    rebase<int32_t>(g.src, dst, g.len / 4, e0, e1);
  } else if (g.op == SEG_REBASE64) {
    rebase<int64_t>(g.src, dst, g.len / 8, e0, e1);
  }
}

uint64_t xseg_elems(const Segment& s) {
  return s.op == SEG_REBASE32 ? s.len / 4 : s.op == SEG_REBASE64 ? s.len / 8 : s.len;
}

// Loads in flight per lane: 4 at every size.  r01's isolated-pack probes preferred 8 loads over
// 32 KiB chunks for 8-32 MB bodies; under the node's overlapping AQL packs (line-aligned chunks,
// no release fence) 4 loads over 8 KiB chunks are faster there: C3 4.70-4.91 -> 4.56 us per
// cloud, a flat 13 MB pack 4.81-4.91 -> 4.33-4.37 us, 16 MB unchanged
// (profiles/r02_u4_mid_ab.jsonl, r02_c3_final_knobs_ab.jsonl).
uint32_t choose_chunk_bytes(uint64_t body_bytes) {
  // r01 probes (profiles/r01_copy_probe.jsonl): at >= 32 MB the best shape is many small
  // workgroups (8 KiB each, 4 loads in flight per lane: 40.96 MB in 14.6 us launch-to-launch);
  // below that ~2k workgroups of >= 8 KiB.
  constexpr uint64_t kGrain = 8192;
  if (body_bytes >= (32u << 20)) return kGrain;
  uint64_t cb = (body_bytes / 2048 + kGrain - 1) / kGrain * kGrain;
  cb = std::max<uint64_t>(cb, kGrain);
  cb = std::min<uint64_t>(cb, uint64_t(1) << 22);
  return static_cast<uint32_t>(cb);
}

// ------------------------------------------------------------------------------------------
// csum64 (oracle/checksum_ref.py): S = sum_i fmix64(word_i ^ (i * GOLDEN + SEED)); fmix64(S+n)
// ------------------------------------------------------------------------------------------
constexpr uint64_t kGolden = 0x9E3779B97F4A7C15ull;
constexpr uint64_t kSeed = 0xD0A5D0A5D0A5D0A5ull;

__host__ __device__ __forceinline__ uint64_t fmix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ __launch_bounds__(kThreads) void csum_kernel(const uint8_t* __restrict__ p, uint64_t n,
                                                        unsigned long long* __restrict__ acc) {
  const uint64_t nw = (n + 7) / 8;
  const uint64_t full = n / 8;
  const bool aligned8 = (reinterpret_cast<uintptr_t>(p) & 7) == 0;
  uint64_t s = 0;
  for (uint64_t i = blockIdx.x * uint64_t(kThreads) + threadIdx.x; i < nw;
       i += uint64_t(gridDim.x) * kThreads) {
    uint64_t w = 0;
    if (aligned8 && i < full) {
      w = reinterpret_cast<const uint64_t*>(p)[i];
    } else {
      const uint64_t lim = (i < full) ? 8 : (n - 8 * i);
      for (uint64_t k = 0; k < lim; ++k) w |= uint64_t(p[8 * i + k]) << (8 * k);
    }
    s += fmix64(w ^ (i * kGolden + kSeed));
  }
  for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
  if ((threadIdx.x & 63) == 0 && s) atomicAdd(acc, static_cast<unsigned long long>(s));
}

__global__ void csum_finalize(unsigned long long* acc, uint64_t n) {
  *acc = fmix64(static_cast<uint64_t>(*acc) + n);
}

// splitmix64 payload: word k = fmix64(seed + (k + 1) * GOLDEN), little-endian bytes.
__global__ __launch_bounds__(kThreads) void fill_kernel(uint8_t* __restrict__ p, uint64_t n,
                                                        uint64_t seed) {
  const uint64_t nw = (n + 7) / 8;
  const bool aligned8 = (reinterpret_cast<uintptr_t>(p) & 7) == 0;
  for (uint64_t i = blockIdx.x * uint64_t(kThreads) + threadIdx.x; i < nw;
       i += uint64_t(gridDim.x) * kThreads) {
    const uint64_t w = fmix64(seed + (i + 1) * kGolden);
    if (aligned8 && 8 * i + 8 <= n) {
      reinterpret_cast<uint64_t*>(p)[i] = w;
    } else {
      for (uint64_t k = 0; k < 8 && 8 * i + k < n; ++k) p[8 * i + k] = uint8_t(w >> (8 * k));
    }
  }
}

// Test tool (the acquire-fence negative control, tests/test_gpu_fence.py): every workgroup reads
// all of [p, p + n) with plain cached loads, so that each XCD's L2 ends up holding the lines
// (one workgroup per CU: 32 per XCD, dispatched round robin over the XCDs).  The reduction is
// stored only under a condition the data never meets, so the loads cannot be elided.
__global__ __launch_bounds__(kThreads) void l2_touch_kernel(const uint8_t* __restrict__ p,
                                                            uint64_t n, uint32_t* __restrict__ sink) {
  const uint64_t nu = n / 16;
  uint32_t x = 0;
  for (uint64_t i = threadIdx.x; i < nu; i += kThreads) {
    const uint32_t* w = reinterpret_cast<const uint32_t*>(p + 16 * i);
    x ^= w[0] ^ w[1] ^ w[2] ^ w[3];
  }
  if (x == 0x5EEDF00Du && n == 1) sink[blockIdx.x] = x;
}

// Test tool (the fence probe's failing control, tests/test_gpu_fence.py): can a CU's cache hand
// a wave stale source bytes inside ONE dispatch?  One 64-lane workgroup per CU reads 64 words of
// `src` (coarse-grained device memory the host then rewrites through the BAR) into `first`,
// reports its arrival on a host counter, waits (bounded) for the host's `go` — given after the
// rewrite — and reads the same words again into `second`.  `mode` picks the loads: 0 plain
// (L1-cached), 1 non-temporal (the pack's default loads), 2 agent-coherent sc1 (the coherent
// pack's).  A plain load served by the CU's L1 returns the old words; a load that bypasses L1
// cannot.  The arrival counter is a vector atomic, the poll a system-scope load; every wave
// leaves after at most ~2^22 sleeps, so a host that never answers cannot hang the device.
template <int MODE>
__device__ __forceinline__ uint32_t probe_load(const uint32_t* p) {
  if constexpr (MODE == 0) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
  if constexpr (MODE == 1) return __builtin_nontemporal_load(p);
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int MODE>
__global__ __launch_bounds__(64) void l1_stale_kernel(const uint32_t* src, uint32_t* first,
                                                      uint32_t* second, uint32_t* arrived,
                                                      const uint32_t* go) {
  const uint32_t t = threadIdx.x, b = blockIdx.x;
  asm volatile("" ::: "memory");
  first[b * 64 + t] = probe_load<MODE>(src + t);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (t == 0) {
    __hip_atomic_fetch_add(arrived, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    for (uint32_t i = 0; i < (1u << 22); ++i) {
      if (__hip_atomic_load(go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) break;
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  asm volatile("" ::: "memory");
  second[b * 64 + t] = probe_load<MODE>(src + t);
}

unsigned grid_for(uint64_t items) {
  uint64_t g = (items + kThreads - 1) / kThreads;
  return static_cast<unsigned>(std::max<uint64_t>(1, std::min<uint64_t>(g, 4096)));
}

}  // namespace

// Boundary units written whole (PackArgsT::edge_mask) for one launch holding every segment of
// its plan: a segment's unaligned head / tail unit is stitched when it lies inside the writable
// destination [dst, dst + cap).  Segments must be sorted by destination offset and disjoint, as
// plans are (else nothing is stitched), so every byte of such a unit belongs to a segment of
// this launch or is padding.  cap 0 (unknown extent, host destinations): nothing is stitched.
uint64_t edge_mask(const Segment* segs, size_t n, const uint8_t* dst, uint64_t cap) {
  if (!cap || n > 32) return 0;
  for (size_t k = 1; k < n; ++k)
    if (segs[k].dst_off < segs[k - 1].dst_off + segs[k - 1].len) return 0;
  const uint64_t base = reinterpret_cast<uintptr_t>(dst);
  auto inside = [&](uint64_t unit) { return unit >= base && unit + 16 <= base + cap; };
  uint64_t mask = 0;
  for (size_t k = 0; k < n; ++k) {
    const uint64_t d0 = base + segs[k].dst_off, d1 = d0 + segs[k].len;
    if (d1 == d0) continue;
    const uint64_t A0 = (d0 + 15) & ~uint64_t(15);
    if (A0 > d0 && inside(A0 - 16)) mask |= uint64_t(1) << (2 * k);
    if (A0 < d1 && (d1 & 15) && inside(d1 & ~uint64_t(15))) mask |= uint64_t(2) << (2 * k);
  }
  return mask;
}

// Launch the pack of `n` segments into `dst` (device).  Copy segments with device sources go
// to pack_kernel in batches of kMaxSegs, transform segments (compacting plans) to
// transform_kernel; host sources are DMA'd with hipMemcpyAsync.  With timing events the
// launches go through hipExtLaunchKernelGGL, whose dispatch packet stamps the first kernel's
// begin into `ev_start` and the last kernel's end into `ev_stop`.
int launch_pack(const Segment* segs_in, size_t n_in, ArrowDeviceType dev, uint8_t* dst,
                hipStream_t stream, hipEvent_t ev_start, hipEvent_t ev_stop,
                const FillSignal* signal, bool* signalled, uint64_t dst_cap) {
  if (signalled) *signalled = false;
  bool any_x = false;
  for (size_t i = 0; i < n_in; ++i) any_x |= segs_in[i].op != SEG_COPY;
  if (dev == ARROW_DEVICE_CPU) {
    if (any_x) return fail(DORA_ERR_UNSUPPORTED, "compacting plans need device-resident arrays");
    for (size_t i = 0; i < n_in; ++i)
      DORA_HIP(hipMemcpyAsync(dst + segs_in[i].dst_off, segs_in[i].src, segs_in[i].len,
                              hipMemcpyHostToDevice, stream));
    return DORA_OK;
  }
  std::vector<Segment> copies, xforms;
  const Segment* segs = segs_in;
  size_t n = n_in;
  if (any_x) {
    for (size_t i = 0; i < n_in; ++i) (segs_in[i].op == SEG_COPY ? copies : xforms).push_back(segs_in[i]);
    segs = copies.data();
    n = copies.size();
  }
  const size_t n_launch_x = (xforms.size() + kMaxSegs - 1) / kMaxSegs;
  size_t launch = 0;
  const size_t n_launch = (n + kMaxSegs - 1) / kMaxSegs + n_launch_x;
  size_t i = 0;
  while (i < n) {
    PackArgs a;
    std::memset(&a, 0, sizeof(a));
    a.dst = dst;
    uint64_t body = 0;
    const size_t m = std::min<size_t>(kMaxSegs, n - i);
    for (size_t k = 0; k < m; ++k) body += segs[i + k].len;
    a.chunk_bytes = choose_chunk_bytes(body);
    uint64_t chunks = 0;
    for (size_t k = 0; k < m; ++k) {
      const Segment& s = segs[i + k];
      a.seg[k] = {static_cast<const uint8_t*>(s.src), s.dst_off, s.len};
      chunks += segment_chunks(reinterpret_cast<uintptr_t>(dst), s.dst_off, s.len, a.chunk_bytes);
      if (chunks > 0x7fffffffull) return fail(DORA_ERR_INVALID, "pack: too many chunks");
      a.chunk_end[k] = static_cast<uint32_t>(chunks);
    }
    a.nseg = static_cast<uint32_t>(m);
    // one launch holding the whole plan: its boundary units may be written whole
    if (!any_x && m == n) a.edge_mask = edge_mask(segs, n, dst, dst_cap);
    const bool first = launch == 0, last = launch + 1 == n_launch;
    a.n_chunks = static_cast<uint32_t>(chunks);
    uint64_t grid = chunks;
    void (*kern)(PackArgs) = pack_kernel<kUnroll, 1>;
    if (last && signal) {
      // signalling launch: write-through stores, at most kSignalGrid workgroups
      a.flag = signal->flag;
      a.done = signal->done;
      a.epoch = signal->epoch;
      if (grid > kSignalGrid) grid = kSignalGrid;
      kern = pack_kernel<kUnroll, 2>;
    }
    a.grid = static_cast<uint32_t>(grid);
    if (ev_start || ev_stop) {
      hipExtLaunchKernelGGL(kern, dim3(static_cast<unsigned>(grid)), dim3(kThreads), 0, stream,
                            first ? ev_start : nullptr, last ? ev_stop : nullptr, 0, a);
    } else {
      hipLaunchKernelGGL(kern, dim3(static_cast<unsigned>(grid)), dim3(kThreads), 0, stream, a);
    }
    DORA_HIP(hipGetLastError());
    if (a.flag && signalled) *signalled = true;
    i += m;
    ++launch;
  }
  for (size_t j = 0; j < xforms.size(); j += kMaxSegs) {
    XArgs x;
    std::memset(&x, 0, sizeof(x));
    x.dst = dst;
    const size_t m = std::min<size_t>(kMaxSegs, xforms.size() - j);
    uint64_t blocks = 0;
    for (size_t k = 0; k < m; ++k) {
      const Segment& s = xforms[j + k];
      x.seg[k] = {static_cast<const uint8_t*>(s.src), s.dst_off, s.len, s.src_len, s.op, s.aux};
      blocks += std::max<uint64_t>(1, (xseg_elems(s) + kXElems - 1) / kXElems);
      if (blocks > 0x7fffffffull) return fail(DORA_ERR_INVALID, "pack: too many blocks");
      x.block_end[k] = static_cast<uint32_t>(blocks);
    }
    x.nseg = static_cast<uint32_t>(m);
    const bool first = launch == 0, last = launch + 1 == n_launch;
    if (ev_start || ev_stop) {
      hipExtLaunchKernelGGL(transform_kernel, dim3(static_cast<unsigned>(blocks)), dim3(kThreads),
                            0, stream, first ? ev_start : nullptr, last ? ev_stop : nullptr, 0, x);
    } else {
      hipLaunchKernelGGL(transform_kernel, dim3(static_cast<unsigned>(blocks)), dim3(kThreads), 0,
                         stream, x);
    }
    DORA_HIP(hipGetLastError());
    ++launch;
  }
  return DORA_OK;
}

// Launch a pack and wait for it by spinning on a host flag the launch writes itself (a
// blocking stream synchronise sleeps and wakes tens of microseconds late).  Per thread and
// device: the pinned flag, its device view and the done words.  Falls back to a stream
// synchronise when the launch cannot signal (transform segments) or the flag does not come.
int launch_pack_wait(const Segment* segs, size_t n, uint8_t* dst, hipStream_t stream) {
  struct WaitCtx {
    int device = -1;
    uint64_t* host = nullptr;
    uint64_t* dev = nullptr;
    uint32_t* done = nullptr;
    uint64_t epoch = 0;
  };
  thread_local std::vector<WaitCtx> ctxs;
  int device = 0;
  DORA_HIP(hipGetDevice(&device));
  WaitCtx* c = nullptr;
  for (auto& x : ctxs)
    if (x.device == device) c = &x;
  if (!c) {
    WaitCtx x;
    x.device = device;
    void* dv = nullptr;
    DORA_HIP(hipHostMalloc(reinterpret_cast<void**>(&x.host), 64, hipHostMallocMapped));
    DORA_HIP(hipHostGetDevicePointer(&dv, x.host, 0));
    x.dev = static_cast<uint64_t*>(dv);
    *reinterpret_cast<volatile uint64_t*>(x.host) = 0;
    DORA_HIP(hipMalloc(&x.done, kMaxSignalWgs * sizeof(uint32_t)));
    DORA_HIP(hipMemset(x.done, 0, kMaxSignalWgs * sizeof(uint32_t)));
    DORA_HIP(hipDeviceSynchronize());
    ctxs.push_back(x);
    c = &ctxs.back();
  }
  FillSignal sig{c->dev, ++c->epoch, c->done};
  bool signalled = false;
  int rc = launch_pack(segs, n, ARROW_DEVICE_ROCM, dst, stream, nullptr, nullptr, &sig,
                       &signalled);
  if (rc != DORA_OK) return rc;
  if (signalled) {
    const volatile uint64_t* f = c->host;
    const auto t0 = std::chrono::steady_clock::now();
    unsigned spins = 0;
    while (*f < sig.epoch) {
      __builtin_ia32_pause();
      if (++spins % 4096 == 0 &&
          std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(200))
        break;  // slow or failed signal: the stream synchronise below decides
    }
    if (*f >= sig.epoch) return DORA_OK;
  }
  DORA_HIP(hipStreamSynchronize(stream));
  return DORA_OK;
}

size_t aql_args_size() { return sizeof(AqlPackArgs); }
size_t aql_batch_args_size() { return sizeof(dora::pack::AqlBatchArgs); }

// The chunk size a message's pack would use on its own (a batch holds messages of one size).
uint32_t aql_chunk_bytes(const Segment* segs, size_t n) {
  uint64_t body = 0;
  for (size_t k = 0; k < n; ++k) body += segs[k].len;
  return choose_chunk_bytes(body);  // the AQL kernels keep 4 loads in flight per lane
}

// Arguments of dora_aql_packb_u4: the segments of `n` messages with absolute destinations,
// sorted by address, each message's stitched-edge bits carried over from its own edge_mask.
int build_aql_batch_args(const BatchItem* items, size_t n, uint8_t* out, size_t cap,
                         uint32_t* grid_out) {
  using dora::pack::AqlBatchArgs;
  using dora::pack::kMaxBatchMsgs;
  using dora::pack::kMaxBatchSegs;
  if (n == 0 || n > size_t(kMaxBatchMsgs)) return fail(DORA_ERR_INVALID, "batch of %zu", n);
  if (cap < sizeof(AqlBatchArgs)) return fail(DORA_ERR_INVALID, "AQL batch: argument buffer");
  struct S {
    uint64_t dst;
    const uint8_t* src;
    uint64_t len;
    uint32_t edge;
  };
  S all[kMaxBatchSegs];
  size_t ns = 0;
  const uint32_t chunk = aql_chunk_bytes(items[0].segs, items[0].n);
  for (size_t m = 0; m < n; ++m) {
    const BatchItem& it = items[m];
    if (ns + it.n > size_t(kMaxBatchSegs)) return fail(DORA_ERR_INVALID, "AQL batch: segments");
    if (aql_chunk_bytes(it.segs, it.n) != chunk)
      return fail(DORA_ERR_INVALID, "AQL batch: messages of different chunk sizes");
    const uint64_t em = edge_mask(it.segs, it.n, it.dst, it.dst_cap);
    for (size_t k = 0; k < it.n; ++k) {
      if (it.segs[k].op != SEG_COPY) return fail(DORA_ERR_INVALID, "AQL batch: transform");
      all[ns++] = {reinterpret_cast<uintptr_t>(it.dst) + it.segs[k].dst_off,
                   static_cast<const uint8_t*>(it.segs[k].src), it.segs[k].len,
                   static_cast<uint32_t>(em >> (2 * k)) & 3u};
    }
  }
  std::sort(all, all + ns, [](const S& a, const S& b) { return a.dst < b.dst; });
  AqlBatchArgs a;
  std::memset(&a, 0, sizeof(a));
  a.chunk_bytes = chunk;
  uint64_t chunks = 0;
  for (size_t k = 0; k < ns; ++k) {
    a.seg[k] = {all[k].src, all[k].dst, all[k].len};
    chunks += segment_chunks(0, all[k].dst, all[k].len, chunk);
    if (chunks > 0x7fffffffull) return fail(DORA_ERR_INVALID, "pack: too many chunks");
    a.chunk_end[k] = static_cast<uint32_t>(chunks);
    a.edge_mask |= uint64_t(all[k].edge) << (2 * k);
  }
  a.nseg = static_cast<uint32_t>(ns);
  a.n_chunks = static_cast<uint32_t>(chunks);
  a.grid = static_cast<uint32_t>(std::min<uint64_t>(chunks, kSignalGrid));
  a.flag = items[0].sig.flag;
  a.done = items[0].sig.done;
  a.epoch = items[0].sig.epoch;
  a.nmsg = static_cast<uint32_t>(n);
  for (size_t m = 0; m < n; ++m) a.msg[m] = {items[m].sig.flag, items[m].sig.epoch};
  std::memcpy(out, &a, sizeof(a));
  *grid_out = a.grid;
  return DORA_OK;
}

// Workgroups of an AQL pack signalled as `sig` says.  In-kernel signals (a flag): the signalling
// grid (kSignalGrid).  Signalled by the command processor (no flag): nothing to poll, so up to
// kCpGrid workgroups — a lone 40.96 MB pack capped at 1024 keeps 8 MiB in flight, half of what
// HBM needs.
uint64_t signal_grid_cap(const FillSignal& sig) { return sig.flag ? kSignalGrid : kCpGrid; }

// Arguments of one AQL-dispatched signalling pack (aql.cpp): the same chunking and signalling
// grid as launch_pack's last launch.
int build_aql_args(const Segment* segs, size_t n, uint8_t* dst, const FillSignal& sig,
                   uint8_t* out, size_t cap, uint32_t* grid_out, uint64_t dst_cap) {
  if (n == 0 || n > size_t(kMaxAqlSegs)) return fail(DORA_ERR_INVALID, "AQL pack: %zu segments", n);
  if (cap < sizeof(AqlPackArgs)) return fail(DORA_ERR_INVALID, "AQL pack: argument buffer");
  AqlPackArgs a;
  std::memset(&a, 0, sizeof(a));
  a.dst = dst;
  uint64_t body = 0;
  for (size_t k = 0; k < n; ++k) {
    if (segs[k].op != SEG_COPY) return fail(DORA_ERR_INVALID, "AQL pack: transform segment");
    body += segs[k].len;
  }
  a.chunk_bytes = choose_chunk_bytes(body);
  const uint64_t base = reinterpret_cast<uintptr_t>(dst);
  uint64_t chunks = 0;
  for (size_t k = 0; k < n; ++k) {
    const Segment& s = segs[k];
    a.seg[k] = {static_cast<const uint8_t*>(s.src), s.dst_off, s.len};
    chunks += segment_chunks(base, s.dst_off, s.len, a.chunk_bytes);
    if (chunks > 0x7fffffffull) return fail(DORA_ERR_INVALID, "pack: too many chunks");
    a.chunk_end[k] = static_cast<uint32_t>(chunks);
  }
  a.nseg = static_cast<uint32_t>(n);
  a.edge_mask = edge_mask(segs, n, dst, dst_cap);
  a.n_chunks = static_cast<uint32_t>(chunks);
  const uint64_t grid_cap = sig.flag ? kSignalGrid : kCpGridMulti;
  a.grid = static_cast<uint32_t>(std::min<uint64_t>(chunks, grid_cap));
  a.flag = sig.flag;
  a.done = sig.done;
  a.epoch = sig.epoch;
  std::memcpy(out, &a, sizeof(a));
  *grid_out = a.grid;
  return DORA_OK;
}

// Arguments of the preloaded single-segment AQL kernels (aql_kernels.hip dora_aql_pack1_*):
// dst, src, len, flag, done, epoch, chunk_bytes, grid — 56 bytes, the same chunk shape and grid
// build_aql_args chooses for one segment at sample offset 0.
int build_aql_args1(const Segment& sg, uint8_t* dst, const FillSignal& sig, uint8_t* out,
                    uint32_t* grid_out) {
  if (sg.op != SEG_COPY || sg.dst_off != 0)
    return fail(DORA_ERR_INVALID, "AQL single-segment pack: segment at offset %llu",
                (unsigned long long)sg.dst_off);
  const uint64_t base = reinterpret_cast<uintptr_t>(dst);
  const uint64_t cap = signal_grid_cap(sig);
  const uint32_t chunk_bytes = choose_chunk_bytes(sg.len);
  const uint64_t chunks = segment_chunks(base, 0, sg.len, chunk_bytes);
  if (chunks > 0x7fffffffull) return fail(DORA_ERR_INVALID, "pack: too many chunks");
  const uint32_t grid = static_cast<uint32_t>(std::min<uint64_t>(chunks, cap));
  const uint64_t words[6] = {reinterpret_cast<uintptr_t>(dst), reinterpret_cast<uintptr_t>(sg.src),
                             sg.len, reinterpret_cast<uintptr_t>(sig.flag),
                             reinterpret_cast<uintptr_t>(sig.done), sig.epoch};
  std::memcpy(out, words, sizeof(words));
  std::memcpy(out + 48, &chunk_bytes, 4);
  std::memcpy(out + 52, &grid, 4);
  *grid_out = grid;
  return DORA_OK;
}

int launch_csum(const void* data, size_t len, uint64_t* out_dev, hipStream_t stream) {
  DORA_HIP(hipMemsetAsync(out_dev, 0, sizeof(uint64_t), stream));
  if (len) {
    hipLaunchKernelGGL(csum_kernel, dim3(grid_for((len + 7) / 8)), dim3(kThreads), 0, stream,
                       static_cast<const uint8_t*>(data), uint64_t(len),
                       reinterpret_cast<unsigned long long*>(out_dev));
    DORA_HIP(hipGetLastError());
  }
  hipLaunchKernelGGL(csum_finalize, dim3(1), dim3(1), 0, stream,
                     reinterpret_cast<unsigned long long*>(out_dev), uint64_t(len));
  DORA_HIP(hipGetLastError());
  return DORA_OK;
}

int launch_l2_touch(const void* p, size_t len, hipStream_t stream) {
  if (len < 16) return DORA_OK;
  int cus = 0, dev = 0;
  DORA_HIP(hipGetDevice(&dev));
  DORA_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  hipLaunchKernelGGL(l2_touch_kernel, dim3(std::max(cus, 1)), dim3(kThreads), 0, stream,
                     static_cast<const uint8_t*>(p), uint64_t(len), nullptr);
  DORA_HIP(hipGetLastError());
  return DORA_OK;
}

// One run of l1_stale_kernel (see there): `src` holds 64 words of pattern A, the host rewrites
// them to pattern B once every workgroup has read them.  Out: workgroups whose first read was
// not A (setup failures), whose second read still held A words (stale), and the workgroups.
int l1_stale_probe(int device, int mode, uint32_t* bad_first, uint32_t* stale, uint32_t* blocks) {
  *bad_first = *stale = *blocks = 0;
  DORA_HIP(hipSetDevice(device));
  int cus = 0;
  DORA_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, device));
  const uint32_t nb = uint32_t(std::max(cus, 1));
  void* bar = nullptr;
  int rc = bar_alloc(device, 4096, &bar);
  if (rc != DORA_OK) return rc;
  uint32_t A[64], B[64];
  for (uint32_t i = 0; i < 64; ++i) {
    A[i] = 0xA0000000u | i;
    B[i] = 0xB0000000u | i;
  }
  uint32_t *first = nullptr, *second = nullptr, *ctl = nullptr;
  auto cleanup = [&] {
    if (first) (void)hipFree(first);
    if (second) (void)hipFree(second);
    if (ctl) (void)hipHostFree(ctl);
    bar_free(bar);
  };
  if (bar_write(device, bar, A, sizeof(A)) != DORA_OK ||
      hipMalloc(&first, size_t(nb) * 256) != hipSuccess ||
      hipMalloc(&second, size_t(nb) * 256) != hipSuccess ||
      hipHostMalloc(&ctl, 128, hipHostMallocMapped | hipHostMallocCoherent) != hipSuccess) {
    cleanup();
    return fail(DORA_ERR_HIP, "l1 stale probe: setup");
  }
  volatile uint32_t* arrived = ctl;
  volatile uint32_t* go = ctl + 16;  // its own cache line
  *arrived = 0;
  *go = 0;
  uint32_t *d_arr = nullptr, *d_go = nullptr;
  (void)hipHostGetDevicePointer(reinterpret_cast<void**>(&d_arr), ctl, 0);
  d_go = d_arr + 16;
  hipStream_t st = nullptr;
  DORA_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  auto kern = mode == 0 ? l1_stale_kernel<0> : mode == 1 ? l1_stale_kernel<1> : l1_stale_kernel<2>;
  hipLaunchKernelGGL(kern, dim3(nb), dim3(64), 0, st, static_cast<const uint32_t*>(bar), first,
                     second, d_arr, d_go);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) {
    // every workgroup has read A (bounded: a workgroup that never got a CU is just not counted)
    const auto t0 = std::chrono::steady_clock::now();
    while (*arrived < nb && std::chrono::steady_clock::now() - t0 < std::chrono::seconds(2)) {
    }
    (void)bar_write(device, bar, B, sizeof(B));
    __atomic_store_n(const_cast<uint32_t*>(go), 1u, __ATOMIC_SEQ_CST);
    e = hipStreamSynchronize(st);
  }
  (void)hipStreamDestroy(st);
  if (e != hipSuccess) {
    cleanup();
    return fail(DORA_ERR_HIP, "l1 stale probe: %s", hipGetErrorString(e));
  }
  std::vector<uint32_t> f(size_t(nb) * 64), g(size_t(nb) * 64);
  DORA_HIP(hipMemcpy(f.data(), first, f.size() * 4, hipMemcpyDeviceToHost));
  DORA_HIP(hipMemcpy(g.data(), second, g.size() * 4, hipMemcpyDeviceToHost));
  for (uint32_t b = 0; b < nb; ++b) {
    bool bf = false, bs = false;
    for (uint32_t i = 0; i < 64; ++i) {
      bf |= f[b * 64 + i] != A[i];
      bs |= g[b * 64 + i] == A[i];
    }
    *bad_first += bf;
    *stale += bs;
  }
  *blocks = nb;
  cleanup();
  return DORA_OK;
}

int launch_fill(void* dst, size_t len, uint64_t seed, hipStream_t stream) {
  if (!len) return DORA_OK;
  hipLaunchKernelGGL(fill_kernel, dim3(grid_for((len + 7) / 8)), dim3(kThreads), 0, stream,
                     static_cast<uint8_t*>(dst), uint64_t(len), seed);
  DORA_HIP(hipGetLastError());
  return DORA_OK;
}

}  // namespace dora

extern "C" {

int dora_gpu_pack(const dora_plan* plan, void* dst, size_t dst_len, dora_stream_t stream) {
  if (!plan) return dora::fail(DORA_ERR_INVALID, "plan is NULL");
  if (dst_len < plan->size)
    // arrow_utils.rs:37-42 asserts; the C ABI reports instead
    return dora::fail(DORA_ERR_TOO_SMALL,
                      "target buffer too small (total_len: %zu, required_len: %llu)", dst_len,
                      static_cast<unsigned long long>(plan->size));
  if (plan->segs.empty()) return DORA_OK;
  if (!dst) return dora::fail(DORA_ERR_INVALID, "dst is NULL");
  return dora::launch_pack(plan->segs.data(), plan->segs.size(), plan->dev,
                           static_cast<uint8_t*>(dst), static_cast<hipStream_t>(stream), nullptr,
                           nullptr, nullptr, nullptr, dst_len);
}

int dora_gpu_csum64(const void* data, size_t len, uint64_t* out_dev, dora_stream_t stream) {
  if (!out_dev || (!data && len)) return dora::fail(DORA_ERR_INVALID, "NULL argument");
  return dora::launch_csum(data, len, out_dev, static_cast<hipStream_t>(stream));
}

int dora_gpu_csum64_sync(const void* data, size_t len, dora_stream_t stream, uint64_t* out) {
  if (!out || (!data && len)) return dora::fail(DORA_ERR_INVALID, "NULL argument");
  uint64_t* d = nullptr;
  DORA_HIP(hipMalloc(&d, sizeof(uint64_t)));
  int rc = dora::launch_csum(data, len, d, static_cast<hipStream_t>(stream));
  if (rc == DORA_OK) {
    hipError_t e = hipMemcpyAsync(out, d, sizeof(uint64_t), hipMemcpyDeviceToHost,
                                  static_cast<hipStream_t>(stream));
    if (e == hipSuccess) e = hipStreamSynchronize(static_cast<hipStream_t>(stream));
    if (e != hipSuccess) rc = dora::fail(DORA_ERR_HIP, "csum64 readback: %s", hipGetErrorString(e));
  }
  (void)hipFree(d);
  return rc;
}

int dora_gpu_fill_splitmix(void* dst, size_t len, uint64_t seed, dora_stream_t stream) {
  if (!dst && len) return dora::fail(DORA_ERR_INVALID, "dst is NULL");
  return dora::launch_fill(dst, len, seed, static_cast<hipStream_t>(stream));
}

}  // extern "C"
