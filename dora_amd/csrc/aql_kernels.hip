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

// Read-signalled single-segment pack (aql.cpp: a synchronous send of 1-192 MiB, source and slot
// 16-byte aligned).  The reference's send_output returns once its source has been copied; a pack
// that loads and stores chunk by chunk has read its last source byte only about when it has
// written its last sample byte, so a synchronous send waited for the whole pack plus the host
// round trip (0.47 of HBM per 40.96 MB message).  Here every workgroup first loads
// its whole share of the source into VGPRs (<= kReadLaneUnits 16-B units per lane, plan.h),
// publishes that in its done word once all its loads have returned, and only then stores;
// workgroup 0 waits for every done word and raises the flag line's read word — the send returns
// there, and the next send's loads overlap this pack's stores.  The other workgroups hold their
// stores until workgroup 0 raises a go word with it (≤ 20 us): early stores slowed the loads
// the read word waits for (40.96 MB synchronous sends 18.3-18.9 -> 16.8-17.3 us per message,
// profiles/r06_gate_ab.jsonl).  The fill itself is the
// dispatch's completion signal (every wave waits for its own stores), as for the other lone
// packs; stamps as pack_body's CP branch.
extern "C" __global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(8)))
void dora_aql_pack1r_u4(
    uint8_t* dst, const uint8_t* src, uint64_t len, uint64_t* rflag, uint32_t* done,
    uint64_t epoch, uint64_t* stamps, uint32_t grid, uint32_t per) {
  using namespace dora;
  using namespace dora::pack;
  const uint32_t blk = __builtin_amdgcn_workgroup_id_x(), t = threadIdx.x;
  const uint64_t t_start = blk == 0 ? __builtin_amdgcn_s_memrealtime() : 0;
  // lane t holds units u0 + t + 256 k, k < nk: one VGPR offset, the stride in SGPR offsets
  // (few VGPRs, so every workgroup of the grid is resident at once)
  const uint32_t units = static_cast<uint32_t>(len >> 4);
  const uint32_t u0 = blk * per;
  const uint32_t u1 = u0 + per < units ? u0 + per : units;
  const uint32_t mine = u0 + t < u1 ? (u1 - u0 - t + kThreads - 1) / kThreads : 0;
  const uint32_t off = 16 * (u0 + t);
  const __amdgpu_buffer_rsrc_t rs = src_rsrc(src), rd = src_rsrc(dst);
  u32x4 v[kReadLaneUnits];
#pragma unroll
  for (int k = 0; k < int(kReadLaneUnits); ++k)
    if (uint32_t(k) < mine)
      v[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 16 * kThreads * k, kCoherentPolicy);
  const uint32_t tail = static_cast<uint32_t>(len & 15);
  const bool tail_lane = blk == grid - 1 && t < tail;
  uint8_t tb = 0;
  if (tail_lane) tb = ld1<kCoherent>(src + 16 * uint64_t(units) + t);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every load of this workgroup has returned
  __syncthreads();
  const uint32_t e = static_cast<uint32_t>(epoch);
  if (t == 0) __hip_atomic_store(done + blk, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  // workgroup 0's go for the stores: the flag's last done word, free below kMaxSignalWgs.  Only
  // for grids an idle GPU holds at once (<= 1024 of these 63-VGPR workgroups, a 50 MB pack): a
  // larger one would hold its resident workgroups for the whole bound while the rest wait
  uint32_t* const go = grid <= 1024 ? done + (kMaxSignalWgs - 1) : nullptr;
  if (blk == 0) {
    // as signal_fill: every done word at once per round, bounded (a lost workgroup leaves the
    // read word unset; the send then waits for the fill instead)
    constexpr int kPer = kMaxSignalWgs / kThreads;
    __shared__ uint32_t missing;
    for (uint32_t round = 0; round < (1u << 22); ++round) {
      if (t == 0) missing = 0;
      __syncthreads();
      // four loads in flight per lane at a time: this workgroup's source bytes stay in VGPRs
      // meanwhile, and few registers keep every workgroup of the grid resident
      bool all_mine = true;
#pragma unroll 1
      for (int k0 = 0; k0 < kPer; k0 += 4) {
        uint32_t w[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint32_t i = t + (k0 + j) * kThreads;
          w[j] = i < grid ? __hip_atomic_load(done + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : e;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) all_mine &= w[j] == e;
      }
      if (!all_mine) missing = 1;
      __syncthreads();
      const bool all = missing == 0;
      __syncthreads();
      if (all) {
        if (t == 0) {
          __hip_atomic_store(rflag, epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          if (go) __hip_atomic_store(go, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  } else if (go) {
    // the stores wait for every workgroup's loads (the go word, raised with the read word), so
    // the loads run alone at the read rate and the send returns sooner; bounded (a workgroup
    // that is not resident yet cannot hold the others past kGoWaitTicks)
    constexpr uint64_t kGoWaitTicks = 2000;  // 20 us at 100 MHz
    if (t == 0) {
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      while (__hip_atomic_load(go, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != e &&
             __builtin_amdgcn_s_memrealtime() - t0 < kGoWaitTicks)
        __builtin_amdgcn_s_sleep(1);
    }
    __syncthreads();
  }
  // write-through to device scope, as st16<kCoherent> (sc1 nt)
#pragma unroll
  for (int k = 0; k < int(kReadLaneUnits); ++k)
    if (uint32_t(k) < mine)
      __builtin_amdgcn_raw_buffer_store_b128(v[k], rd, off, 16 * kThreads * k, kCoherentPolicy);
  if (tail_lane) st1<kCoherent>(dst + 16 * uint64_t(units) + t, tb);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the fill: complete before the waves end
  if (stamps) {
    __syncthreads();
    if (t == 0) {
      __hip_atomic_fetch_max(stamps + 1 + (blk % kCpStampWgs), __builtin_amdgcn_s_memrealtime(),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      if (blk == 0) __hip_atomic_store(stamps, t_start, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
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
