// The pack kernels of the AQL path (aql.cpp): the same device code as the HIP-launched
// signalling packs (pack_device.h), as plain extern "C" entry points that take no hidden kernel
// arguments (grid size in the arguments, workgroup id from its SGPR), so that a node can
// dispatch them with raw AQL packets on its own HSA queue.  Built as a standalone gfx950 code
// object (dora_amd/build.py) and embedded in libdora_gpu.so.
#include "pack_device.h"

using dora::pack::AqlPackArgs;
using dora::pack::kThreads;

extern "C" __global__ __launch_bounds__(kThreads) void dora_aql_pack_u4(AqlPackArgs a) {
  dora::pack::pack_body<4, 2>(a, __builtin_amdgcn_workgroup_id_x(), a.grid);
}

// Batch packs (aql.cpp): up to kMaxBatchMsgs queued sends in one dispatch, each signalled
// on its own flag when the batch completes.
extern "C" __global__ __launch_bounds__(kThreads) void dora_aql_packb_u4(
    dora::pack::AqlBatchArgs a) {
  dora::pack::pack_body<4, 2>(a, __builtin_amdgcn_workgroup_id_x(), a.grid);
}

// Single-segment packs (a UInt8 payload at sample offset 0: send_output_raw / _bytes, the C2
// benchmark) with every argument in SGPRs: the 56 bytes below are preloaded by the command
// processor once per dispatch (gfx950 kernarg preload, built with
// -mllvm -amdgpu-kernarg-preload-count=14), so they can sit in host memory — no BAR writes and
// no HDP flush per send (aql.cpp; profiles/r01_aql_preload_probe.jsonl: 0.15 vs 1.6 us host
// time per dispatch at the same device time).  The chunk count is derived here as
// build_aql_args derives it for one segment.
template <int U, int NT = 2>
__device__ __forceinline__ void pack1(uint8_t* dst, const uint8_t* src, uint64_t len,
                                      uint64_t* flag, uint32_t* done, uint64_t epoch,
                                      uint32_t chunk_bytes, uint32_t grid) {
  const uint64_t nc =
      dora::pack::segment_chunks(reinterpret_cast<uintptr_t>(dst), 0, len, chunk_bytes);
  dora::pack::PackArgsT<1> a;
  a.dst = dst;
  a.flag = flag;
  a.done = done;
  a.epoch = epoch;
  a.n_chunks = static_cast<uint32_t>(nc);
  a.nseg = 1;
  a.chunk_bytes = chunk_bytes;
  a.grid = grid;
  a.edge_mask = 0;  // a tail unit past `len` may lie outside the destination: bytes one by one
  a.chunk_end[0] = static_cast<uint32_t>(nc);
  a.seg[0] = {src, 0, len};
  dora::pack::pack_body<U, NT>(a, __builtin_amdgcn_workgroup_id_x(), grid);
}

extern "C" __global__ __launch_bounds__(kThreads) void dora_aql_pack1_u4(
    uint8_t* dst, const uint8_t* src, uint64_t len, uint64_t* flag, uint32_t* done,
    uint64_t epoch, uint32_t chunk_bytes, uint32_t grid) {
  pack1<4>(dst, src, len, flag, done, epoch, chunk_bytes, grid);
}

// As dora_aql_pack1_u4, reading the source with agent-coherent loads (pack_device.h kCoherent):
// dispatched without the packet's acquire fence (aql.cpp dispatch_locked: lone packs and packs
// the command processor signals inside its window).
extern "C" __global__ __launch_bounds__(kThreads) void dora_aql_pack1c_u4(
    uint8_t* dst, const uint8_t* src, uint64_t len, uint64_t* flag, uint32_t* done,
    uint64_t epoch, uint32_t chunk_bytes, uint32_t grid) {
  pack1<4, dora::pack::kCoherent>(dst, src, len, flag, done, epoch, chunk_bytes, grid);
}

// Region-end reduction of CP-signalled packs' stamp areas (aql.cpp aql_stamp_reduce, node.cpp
// dora_node_region_end): workgroup i reads area `areas[i]` of `base` (area_words words: [0] the
// first workgroup's start, then the end stamps of pack_body's CP branch) and writes (start,
// latest end) to out[2i], out[2i + 1] in host memory.  The words were written by system-scope
// atomics (performed in memory); system-scope loads read them there.
extern "C" __global__ __launch_bounds__(kThreads) void dora_aql_stamp_reduce(
    const uint64_t* base, const uint32_t* areas, uint64_t* out, uint32_t n, uint32_t area_words) {
  const uint32_t i = __builtin_amdgcn_workgroup_id_x(), t = threadIdx.x;
  if (i >= n) return;
  const uint64_t* a = base + uint64_t(areas[i]) * area_words;
  uint64_t m = 0;
  for (uint32_t w = 1 + t; w < area_words; w += kThreads) {
    const uint64_t v = __hip_atomic_load(a + w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    m = v > m ? v : m;
  }
  __shared__ uint64_t red[kThreads];
  red[t] = m;
  __syncthreads();
  for (uint32_t k = kThreads / 2; k > 0; k >>= 1) {
    if (t < k && red[t + k] > red[t]) red[t] = red[t + k];
    __syncthreads();
  }
  if (t == 0) {
    __hip_atomic_store(out + 2 * i, __hip_atomic_load(a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(out + 2 * i + 1, red[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}
