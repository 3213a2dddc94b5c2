// Device code of the pack (replaces `copy_array_into_sample`, apis/rust/node/src/node/
// arrow_utils.rs:23-71), shared by the HIP-launched kernels (kernels.hip) and the AQL code
// object dispatched on a node's own HSA queue (aql_kernels.hip, aql.cpp).
//
// Pack = pure HBM streaming: read S bytes + write S bytes, no MFMA, no LDS.  Every chunk of a
// segment is one 256-thread workgroup.  The destination is written with 16-byte aligned
// `global_store_dwordx4`; the source is read with `global_load_dwordx4` too.  When source and
// destination disagree mod 16 by whole dwords (C3's x/y/z/intensity at sample offsets 4 mod 16)
// the load is simply issued at the dword-aligned source address: gfx950 runs in unaligned
// access mode and the wave's 64 consecutive 16-B loads still coalesce into whole cache lines
// (profiles/r01_shift_probe.jsonl: 13 MB at src 4 mod 16, 6.02 us vs 5.91 aligned and 6.87 for
// the two-load funnel).  Byte-granular disagreements funnel-shift two aligned loads with
// v_alignbyte_b32.  The shift is uniform per segment, so the per-segment loop is specialised
// on it and no lane diverges.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "plan.h"

namespace dora {
namespace pack {

constexpr int kThreads = 256;
constexpr int kMaxSegs = 32;       // segments of a HIP-launched pack
constexpr int kMaxAqlSegs = 8;     // segments of an AQL-dispatched pack (smaller kernargs)
// Workgroups of a signalling pack (r01 sweep, profiles/r01_signal_sweep.jsonl: 1024 beats 512
// and 2048-4096 at 16-40 MB, flat at 4 MB).  Packs signalled by the command processor have no
// done words to poll and take up to cp_grid() workgroups instead (aql.cpp).
constexpr uint32_t kSignalGrid = 1024;
// Chunk windows start on a cache line: a segment's body is cut into chunks from the 128-byte
// line holding its first aligned unit, so every wave's 1 KiB store covers whole lines (64-byte
// HBM write sectors) and no two waves write parts of one sector.  A body at 16 mod 64 — C3's
// x/y/z/intensity after 68 bytes of list offsets — otherwise gave every wave store two partial
// sectors, each a read-modify-write in the memory controller: ~10 % of the pack's device time
// (profiles/r02_c3_edges_ab.jsonl, the same cloud with every buffer at 0 mod 64).
constexpr uint64_t kLine = 128;

// Chunks of one segment [d0, d0 + len) of a destination at `base` (host and device agree).
__host__ __device__ inline uint64_t segment_chunks(uint64_t base, uint64_t d0, uint64_t len,
                                                   uint64_t chunk_bytes) {
  const uint64_t A0 = (base + d0 + 15) & ~uint64_t(15);
  const uint64_t A1 = (base + d0 + len) & ~uint64_t(15);
  if (A1 <= A0) return 1;
  const uint64_t O = A0 & ~(kLine - 1);
  return (A1 - O + chunk_bytes - 1) / chunk_bytes;
}

struct PackSeg {
  const uint8_t* src;
  uint64_t dst_off;
  uint64_t len;
};

template <int MAXSEG>
struct PackArgsT {
  uint8_t* dst;
  uint64_t* flag;        // fill flag to signal at the end (null: none)
  uint32_t* done;        // per workgroup: epoch (low 32 bits) once its stores are complete
  uint64_t epoch;
  uint32_t n_chunks;     // chunks of this launch (>= grid size)
  uint32_t nseg;
  uint32_t chunk_bytes;  // multiple of 16
  uint32_t grid;         // workgroups launched (AQL kernels cannot read gridDim)
  // Bits 2k / 2k+1: the 16-byte unit holding segment k's unaligned head / tail bytes is written
  // whole (edge_mask(), kernels.hip); clear: those bytes are stored one by one.
  uint64_t edge_mask;
  uint32_t chunk_end[MAXSEG];
  PackSeg seg[MAXSEG];
};
using PackArgs = PackArgsT<kMaxSegs>;
using AqlPackArgs = PackArgsT<kMaxAqlSegs>;

// A batch pack (aql.cpp: sends queued behind busy AQL queues go out together in one dispatch):
// the segments of up to kMaxBatchMsgs messages, each into its own slot.  `dst` is null and every
// segment's `dst_off` is its absolute destination address, so pack_chunk's alignment arithmetic
// and stitched edges work unchanged; the segments are sorted by address (slots never overlap), so
// a segment's predecessor never shares a 16-byte unit with it unless it is of the same message.
// Every message keeps its own fill flag and epoch; the done words and their epoch are the first
// message's.
constexpr int kMaxBatchSegs = 16;
constexpr int kMaxBatchMsgs = 8;
struct BatchMsg {
  uint64_t* flag;
  uint64_t epoch;
};
struct AqlBatchArgs {
  uint8_t* dst;          // null: segment dst_off are absolute addresses
  uint64_t* flag;        // message 0's flag (non-null: the launch signals)
  uint32_t* done;        // message 0's done words
  uint64_t epoch;        // message 0's epoch
  uint32_t n_chunks;
  uint32_t nseg;
  uint32_t chunk_bytes;
  uint32_t grid;
  uint64_t edge_mask;
  uint32_t nmsg;
  uint32_t pad;
  uint32_t chunk_end[kMaxBatchSegs];
  PackSeg seg[kMaxBatchSegs];
  BatchMsg msg[kMaxBatchMsgs];
};

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x4_a4 __attribute__((ext_vector_type(4), aligned(4)));

// Memory policy NT: 0 plain, 1 non-temporal loads and stores, 2/3 non-temporal loads and stores
// written through to device (sc1) / system (sc0 sc1) scope — no L2 write-back needed before a
// fill signal.  4: as 2, and the source is read with agent-coherent loads (buffer_load sc1 nt),
// which never return a line another XCD's writer has since replaced, so the dispatch needs no
// acquire fence (its L2 invalidation) to see a source rewritten since an earlier pack read it.
constexpr int kCoherent = 4;
// raw buffer loads: cache policy bits sc1 (16) | nt (2); resource word 3 as for gfx9 raw buffers
constexpr int kCoherentPolicy = 16 | 2;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t src_rsrc(const uint8_t* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(p), 0, 0x7fffffff, 0x00020000);
}
__device__ __forceinline__ u32x4 ldc16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, kCoherentPolicy);
}
// one source byte (heads, tails, stitched units)
template <int NT>
__device__ __forceinline__ uint8_t ld1(const uint8_t* p) {
  if constexpr (NT == kCoherent) return __builtin_amdgcn_raw_buffer_load_b8(src_rsrc(p), 0, 0, kCoherentPolicy);
  return *p;
}

template <int NT, bool DW = false>
__device__ __forceinline__ u32x4 ld16(const uint8_t* p) {
  constexpr bool nt = NT != 0;
  if constexpr (DW) {  // p only 4-byte aligned
    if constexpr (nt) return __builtin_nontemporal_load(reinterpret_cast<const u32x4_a4*>(p));
    return *reinterpret_cast<const u32x4_a4*>(p);
  }
  if constexpr (nt) return __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p));
  return *reinterpret_cast<const u32x4*>(p);
}
template <int NT>
__device__ __forceinline__ void st16(uint8_t* p, u32x4 v) {
  if constexpr (NT == 2 || NT == kCoherent) {
    asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" ::"v"(p), "v"(v) : "memory");
  } else if constexpr (NT == 3) {
    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt" ::"v"(p), "v"(v) : "memory");
  } else if constexpr (NT == 1) {
    __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
  } else {
    *reinterpret_cast<u32x4*>(p) = v;
  }
}

template <int NT>
__device__ __forceinline__ void st1(uint8_t* p, uint8_t v) {
  if constexpr (NT >= 2) {
    const uint32_t w = v;
    asm volatile("global_store_byte %0, %1, off sc1" ::"v"(p), "v"(w) : "memory");
  } else {
    *p = v;
  }
}

// Bytes [4Q + b, 4Q + b + 16) of the 32-byte little-endian concatenation lo|hi.
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

// Body copy of `nunits` 16-byte units: dst 16-aligned, source `sp` 16-aligned (DW: 4-aligned).
// U loads of 16 B per lane in flight before the stores.
// Units [skip, nunits) are copied; the first `skip` (< 8, a chunk starting mid-line) only keep
// the lanes' windows on whole lines, their addresses are never dereferenced.
template <int U, int NT, bool DW = false>
__device__ __forceinline__ void copy_aligned(uint8_t* dp, const uint8_t* sp, uint64_t skip,
                                             uint64_t nunits) {
  [[maybe_unused]] __amdgpu_buffer_rsrc_t r;
  if constexpr (NT == kCoherent) r = src_rsrc(sp);
  for (uint64_t base = threadIdx.x; base < nunits; base += kThreads * U) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = base + uint64_t(u) * kThreads;
      if (i >= skip && i < nunits) {
        if constexpr (NT == kCoherent) v[u] = ldc16(r, static_cast<uint32_t>(16 * i));
        else v[u] = ld16<NT, DW>(sp + 16 * i);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = base + uint64_t(u) * kThreads;
      if (i >= skip && i < nunits) st16<NT>(dp + 16 * i, v[u]);
    }
  }
}

template <int U, int NT, int Q>
__device__ __forceinline__ void copy_shifted(uint8_t* dp, const uint8_t* sbase, uint32_t b,
                                             uint64_t skip, uint64_t nunits) {
  // sbase = 16-aligned address holding the first source byte at byte 4Q+b.
  [[maybe_unused]] __amdgpu_buffer_rsrc_t r;
  if constexpr (NT == kCoherent) r = src_rsrc(sbase);
  for (uint64_t base = threadIdx.x; base < nunits; base += kThreads * U) {
    u32x4 lo[U], hi[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = base + uint64_t(u) * kThreads;
      if (i >= skip && i < nunits) {
        if constexpr (NT == kCoherent) {
          lo[u] = ldc16(r, static_cast<uint32_t>(16 * i));
          hi[u] = ldc16(r, static_cast<uint32_t>(16 * i + 16));
        } else {
          lo[u] = ld16<NT>(sbase + 16 * i);
          hi[u] = ld16<NT>(sbase + 16 * i + 16);
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = base + uint64_t(u) * kThreads;
      if (i >= skip && i < nunits) st16<NT>(dp + 16 * i, funnel<Q>(lo[u], hi[u], b));
    }
  }
}

// Byte `o` (sample offset) of a stitched boundary unit: from the segment that holds it, else
// the byte the destination already has (padding stays as it was, arrow_utils.rs:48).
template <int NT, class A>
__device__ __forceinline__ uint8_t unit_byte(const A& a, uint64_t o) {
  for (uint32_t k = 0; k < a.nseg; ++k) {
    const PackSeg g = a.seg[k];
    if (o - g.dst_off < g.len) return ld1<NT>(g.src + (o - g.dst_off));  // o in [dst_off, +len)
  }
  return a.dst[o];
}

template <int U, int NT, class A>
__device__ __forceinline__ void pack_chunk(const A& args, uint32_t chunk) {
  const uint32_t nseg = args.nseg;
  uint32_t s = 0;
  while (s + 1 < nseg && chunk >= args.chunk_end[s]) ++s;  // uniform, <= 32 steps
  const PackSeg sg = args.seg[s];
  const uint32_t c = chunk - (s ? args.chunk_end[s - 1] : 0u);

  // 16-byte alignment is taken on absolute addresses (the sample base may be unaligned).
  const uint64_t base = reinterpret_cast<uintptr_t>(args.dst);
  const uint64_t d0 = sg.dst_off, d1 = sg.dst_off + sg.len;
  const uint64_t A0 = (base + d0 + 15) & ~uint64_t(15);
  const uint64_t A1 = (base + d1) & ~uint64_t(15);
  const uint64_t a0 = A0 - base;
  const uint64_t a1 = A1 > A0 ? A1 - base : a0;  // body [a0, a1) empty unless A1 > A0
  uint8_t* const dst = args.dst;
  const uint8_t* const src = sg.src;  // source byte of sample offset d is src[d - d0]

  if (c == 0) {
    // Unaligned head [d0, min(a0, d1)) and tail [max(a1, a0), d1) (< 16 bytes each).  Their
    // 16-byte units (shared with the neighbouring segment or padding) are either written whole —
    // "stitched": one lane-group gathers the unit's 16 bytes from every segment that holds one
    // and one lane stores it with the body's full-width store — or byte by byte.  Sub-dword
    // write-through stores made a C3 pack ~10 % slower than the same sample with every buffer at
    // 0 mod 16 (profiles/r02_c3_edges_ab.jsonl).
    const uint32_t em = static_cast<uint32_t>(args.edge_mask >> (2 * s)) & 3u;
    const bool has_head = d1 > d0 && a0 > d0;
    const bool has_tail = a0 < d1 && ((base + d1) & 15u) != 0;
    const bool st_head = has_head && (em & 1u), st_tail = has_tail && (em & 2u);
    const uint32_t t = threadIdx.x;
    if (has_head && !st_head) {
      const uint64_t hend = a0 < d1 ? a0 : d1;
      if (t < hend - d0) st1<NT>(dst + d0 + t, ld1<NT>(src + t));
    }
    if (has_tail && !st_tail) {
      const uint64_t t0 = a1 > a0 ? a1 : a0;
      if (t >= 64 && t - 64 < d1 - t0) {
        const uint64_t d = t0 + (t - 64);
        st1<NT>(dst + d, ld1<NT>(src + (d - d0)));
      }
    }
    if (st_head || st_tail) {  // uniform over the workgroup
      __shared__ u32x4 unit[2];
      uint8_t* const ub = reinterpret_cast<uint8_t*>(unit);
      const uint64_t H = a0 - 16;                            // head unit (sample offset)
      const uint64_t T = ((base + d1) & ~uint64_t(15)) - base;  // tail unit
      // a unit shared with the previous segment is written by that segment (the lowest one
      // holding a byte of it); a tail unit always belongs to its segment
      const bool own_head = st_head && (s == 0 || args.seg[s - 1].dst_off + args.seg[s - 1].len <= H);
      if (own_head && t < 16) ub[t] = unit_byte<NT>(args, H + t);
      if (st_tail && t >= 64 && t < 80) ub[16 + (t - 64)] = unit_byte<NT>(args, T + (t - 64));
      __syncthreads();
      if (own_head && t == 0) st16<NT>(dst + H, unit[0]);
      if (st_tail && t == 64) st16<NT>(dst + T, unit[1]);
      __syncthreads();  // unit[] is reused by this workgroup's next segment
    }
  }
  if (a0 >= a1) return;
  // chunk c covers [O + c * chunk_bytes, +chunk_bytes) of the body, O = the line of its first
  // aligned unit (kLine; segment_chunks counts them the same way).  Absolute addresses: O may
  // lie before the destination's base.
  const uint64_t E0 = base + a0, E1 = base + a1;  // the body, absolute (A0, A1 when non-empty)
  const uint64_t O = E0 & ~(kLine - 1);
  const uint64_t B0 = O + uint64_t(c) * args.chunk_bytes;
  if (B0 >= E1) return;
  const uint64_t B1 = (E1 - B0) > args.chunk_bytes ? B0 + args.chunk_bytes : E1;
  const uint64_t skip = B0 < E0 ? (E0 - B0) >> 4 : 0;
  const uint64_t nunits = (B1 - B0) >> 4;
  uint8_t* dp = reinterpret_cast<uint8_t*>(B0);
  // the source byte of B0 (before src for skipped units: never dereferenced)
  const uint8_t* sp = src + (static_cast<int64_t>(B0 - base) - static_cast<int64_t>(d0));
  const uint32_t r = static_cast<uint32_t>(reinterpret_cast<uintptr_t>(sp) & 15);
  if (r == 0) {
    copy_aligned<U, NT>(dp, sp, skip, nunits);
    return;
  }
  if ((r & 3) == 0) {  // whole-dword disagreement: one 16-B load at the source address
    copy_aligned<U, NT, true>(dp, sp, skip, nunits);
    return;
  }
  const uint8_t* sbase = sp - r;
  const uint32_t b = r & 3;
  switch (r >> 2) {
    case 0: copy_shifted<U, NT, 0>(dp, sbase, b, skip, nunits); break;
    case 1: copy_shifted<U, NT, 1>(dp, sbase, b, skip, nunits); break;
    case 2: copy_shifted<U, NT, 2>(dp, sbase, b, skip, nunits); break;
    default: copy_shifted<U, NT, 3>(dp, sbase, b, skip, nunits); break;
  }
}

// In-kernel fill signal.  A signalling launch writes the sample through to device scope (sc1:
// no dirty lines left in the per-XCD L2s, so no cache write-back is needed), every workgroup
// waits for its stores to complete and publishes the epoch in its own done word, and
// workgroup 0 — dispatched first — polls all done words and then stores the epoch into the
// host fill flag with a system-scope release.  No same-address atomics (those serialise at
// ~0.1 us each across XCDs) and no L2 write-back per workgroup (~0.1 us each, serial per
// XCD): this replaces the stream write-value packet, a ~4 us blit kernel plus a kernel
// boundary per message on ROCm 7.
// `blk`/`nblk`: this workgroup and the launch's workgroup count, passed in so that the AQL
// kernels need no hidden kernel arguments.
// Workgroup 0 also stamps the launch (s_memrealtime, 100 MHz) into the flag's line: its own
// start, taken on entry, and the time it signals — the fill's device time without a profiled
// queue or timing events.
__device__ __forceinline__ void stamp_fill(uint64_t* flag, uint64_t t_start) {
  __hip_atomic_store(flag + 1, t_start, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store(flag + 2, __builtin_amdgcn_s_memrealtime(), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_SYSTEM);
}

template <class A>
__device__ __forceinline__ void signal_fill(const A& a, uint32_t blk, uint32_t nblk,
                                            uint64_t t_start) {
  const uint32_t e = static_cast<uint32_t>(a.epoch);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's sample stores are complete
  __syncthreads();
  if (nblk == 1) {  // nothing to wait for but this workgroup's own stores
    if (threadIdx.x == 0) {
      stamp_fill(a.flag, t_start);
      __hip_atomic_store(a.flag, a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    return;
  }
  if (threadIdx.x == 0) __hip_atomic_store(a.done + blk, e, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
  if (blk != 0) return;
  // Poll every done word at once per round (up to kMaxSignalWgs / kThreads = 16 independent
  // loads in flight per lane), so completion is seen one load round trip after the last
  // workgroup.  Bounded (~seconds): a lost workgroup must not hang the device; the flag then
  // stays unset and the receiver reports the fill as failed.  The workgroup vote goes through
  // one LDS word (__syncthreads_and would read the workgroup size from hidden arguments).
  constexpr int kPer = kMaxSignalWgs / kThreads;
  __shared__ uint32_t missing;
  bool ok = false;
  for (uint32_t round = 0; round < (1u << 22); ++round) {
    if (threadIdx.x == 0) missing = 0;
    __syncthreads();
    uint32_t v[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
      const uint32_t i = threadIdx.x + k * kThreads;
      v[k] = i < nblk ? __hip_atomic_load(a.done + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                      : e;
    }
    bool mine = true;
#pragma unroll
    for (int k = 0; k < kPer; ++k) mine &= v[k] == e;
    if (!mine) missing = 1;
    __syncthreads();
    const bool all = missing == 0;
    __syncthreads();
    if (all) {
      ok = true;
      break;
    }
    __builtin_amdgcn_s_sleep(1);
  }
  // Relaxed: everything this store publishes is already written through (sample stores and done
  // words are device-scope write-through and complete), and it issues only after every done
  // word was observed; a release would write back this XCD's whole L2 for nothing.
  if (threadIdx.x == 0 && ok) {
    stamp_fill(a.flag, t_start);
    __hip_atomic_store(a.flag, a.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// A batch's signal: as signal_fill, and workgroup 0's lanes k < nmsg then stamp and signal
// message k's flag (every message completes with the whole batch).
__device__ __forceinline__ void signal_batch(const AqlBatchArgs& a, uint32_t blk, uint32_t nblk,
                                             uint64_t t_start) {
  const uint32_t e = static_cast<uint32_t>(a.epoch);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (nblk > 1) {
    if (threadIdx.x == 0)
      __hip_atomic_store(a.done + blk, e, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (blk != 0) return;
    constexpr int kPer = kMaxSignalWgs / kThreads;
    __shared__ uint32_t missing;
    bool ok = false;
    for (uint32_t round = 0; round < (1u << 22); ++round) {
      if (threadIdx.x == 0) missing = 0;
      __syncthreads();
      uint32_t v[kPer];
#pragma unroll
      for (int k = 0; k < kPer; ++k) {
        const uint32_t i = threadIdx.x + k * kThreads;
        v[k] = i < nblk ? __hip_atomic_load(a.done + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                        : e;
      }
      bool mine = true;
#pragma unroll
      for (int k = 0; k < kPer; ++k) mine &= v[k] == e;
      if (!mine) missing = 1;
      __syncthreads();
      const bool all = missing == 0;
      __syncthreads();
      if (all) {
        ok = true;
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (!ok) return;  // a lost workgroup: the flags stay unset, receivers report the failure
  }
  if (threadIdx.x < a.nmsg) {
    const BatchMsg m = a.msg[threadIdx.x];
    stamp_fill(m.flag, t_start);
    __hip_atomic_store(m.flag, m.epoch, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

// A pack launch: its workgroups stride over the chunks; a signalling launch (NT >= 2) then
// signals the fill flag.
template <int U, int NT, class A>
__device__ __forceinline__ void pack_body(const A& args, uint32_t blk, uint32_t nblk) {
  uint64_t t_start = 0;
  if constexpr (NT >= 2) {
    if (blk == 0) t_start = __builtin_amdgcn_s_memrealtime();
  }
  for (uint32_t c = blk; c < args.n_chunks; c += nblk) pack_chunk<U, NT>(args, c);
  if constexpr (NT >= 2) {
    if (args.flag) {  // all-zero arguments are a no-op
      if constexpr (__is_same(A, AqlBatchArgs)) {
        signal_batch(args, blk, nblk, t_start);
      } else {
        signal_fill(args, blk, nblk, t_start);
      }
    } else if (args.done) {
      // done words but no flag: the dispatch's completion signal reports the fill (the command
      // processor's, aql.cpp aql_cp_candidate); every wave's stores are complete before it ends
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (args.epoch) {
        // a pack inside a timed region: `epoch` is its stamp area (device memory, zeroed by the
        // host, read once the region's packs have all completed) — [0] the first workgroup's
        // start, [1 + blk mod kCpStampWgs] the latest time a workgroup mapping there had all its
        // stores complete (system-scope atomic max: performed past the L2s, where the host's BAR
        // read finds it; a grid of any size fits the area)
        uint64_t* st = reinterpret_cast<uint64_t*>(static_cast<uintptr_t>(args.epoch));
        __syncthreads();
        if (threadIdx.x == 0) {
          __hip_atomic_fetch_max(st + 1 + (blk % kCpStampWgs), __builtin_amdgcn_s_memrealtime(),
                                 __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          if (blk == 0)
            __hip_atomic_store(st, t_start, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        }
      }
    }
  }
}

}  // namespace pack
}  // namespace dora
