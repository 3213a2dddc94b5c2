// Internal plan structures shared by plan.cpp and the pack launcher.
#pragma once

#include <cstdint>
#include <string>
#include <utility>
#include <vector>

#include <hip/hip_runtime_api.h>

#include "dora_gpu.h"

namespace dora {

struct BufSpec {
  enum Kind { Fixed, Bitmap, Var } kind;
  uint32_t width;  // bytes per element for Fixed
  uint32_t align;  // FixedWidth alignment (arrow-data layout())
};

// At most three buffer specs per Arrow layout: a fixed-capacity list (no heap allocation per
// planned node).
struct SpecList {
  BufSpec v[3];
  size_t n = 0;
  void push_back(const BufSpec& b) { v[n++] = b; }
  size_t size() const { return n; }
  bool empty() const { return n == 0; }
  const BufSpec& operator[](size_t i) const { return v[i]; }
  const BufSpec* begin() const { return v; }
  const BufSpec* end() const { return v + n; }
};

struct Layout {
  SpecList specs;
  bool can_null = true;
  bool offsets_first = false;  // first non-null buffer is an offsets buffer of len+1 entries
};

// ArrowTypeInfo (libraries/message/src/metadata.rs:51-59) with the data type as a signature.
struct TypeInfoNode {
  std::vector<uint8_t> schema;      // serialized DataType (see serialize_schema)
  uint64_t len = 0;
  uint64_t null_count = 0;
  bool has_validity = false;
  std::vector<uint8_t> validity;
  // Node sends of device arrays: the bitmap travels in the sample itself, in the slot's tail
  // past the reference layout's `size` bytes ([validity_off, +validity_len)), instead of inline
  // in the metadata; receivers import it zero-copy and dora_event_type_info restores the
  // inline form on demand.
  bool validity_in_sample = false;
  uint64_t validity_off = 0, validity_len = 0;
  uint64_t offset = 0;
  std::vector<std::pair<uint64_t, uint64_t>> bufs;  // BufferOffset {offset, len}
  std::vector<TypeInfoNode> children;
};

// One copy of `copy_array_into_sample_inner` (arrow_utils.rs:48): src -> sample[dst_off..+len].
// Compacting plans (dora_gpu_plan_compact) also carry transforms: a bit-shifted bitmap slice
// and rebased offsets.
enum SegOp : uint32_t {
  SEG_COPY = 0,      // len bytes verbatim
  SEG_BITSHIFT = 1,  // len bytes of bitmap starting `aux` bits into src (src_len readable bytes)
  SEG_REBASE32 = 2,  // len/4 int32 offsets minus src[0]
  SEG_REBASE64 = 3,  // len/8 int64 offsets minus src[0]
};

struct Segment {
  const void* src;
  uint64_t dst_off;
  uint64_t len;
  uint32_t op = SEG_COPY;
  uint32_t aux = 0;
  uint64_t src_len = 0;
};

// Fill signal written by a pack launch itself (kernels.hip): once every workgroup's stores are
// complete, a system-scope store of `epoch` into `flag` (device view of a host-registered fill
// flag), preceded by the launch's start / signal times into flag[1], flag[2] (the flag must own
// 24 bytes).  `done` = kMaxSignalWgs device words owned by this flag (zeroed once).
struct FillSignal {
  uint64_t* flag;
  uint64_t epoch;
  uint32_t* done;
};
constexpr uint32_t kMaxSignalWgs = 4096;
// Completion-stamp words of a CP-signalled pack inside a timed region (aql.h): workgroup k
// raises word 1 + (k mod kCpStampWgs) to its end time (atomic max), so a grid of any size fits.
// 1024 words: a few arrivals per word.  (16 words made every 40.96 MB pack of 5,000 workgroups
// take 33 instead of 15 us: ~300 system-scope atomics per address serialise at ~60 ns each.)
// The host does not read the words through the BAR (8 KiB of uncached reads per pack, ~57 ms
// for a 200-send region, r04 trace): one AQL dispatch reduces them (aql_stamp_reduce).
constexpr uint32_t kCpStampWgs = 1024;
// Read-signalled packs (aql_kernels.hip dora_aql_pack1r_u4): 16-byte units of the source each
// lane holds in VGPRs at most (62 VGPRs at 12: every workgroup of two 40.96 MB packs resident).
constexpr uint32_t kReadLaneUnits = 12;

// One message of a batch pack (aql.cpp): its copy segments, slot, fill signal, writable bytes.
struct BatchItem {
  const Segment* segs;
  size_t n;
  uint8_t* dst;
  FillSignal sig;
  uint64_t dst_cap;
};

// Launch the pack of `segs` into `dst` on `stream` (kernels.hip).  With `signal`, the last
// launch writes the fill flag itself when it can (`*signalled` says whether it did; compacting
// transforms and host sources leave it to the caller).  `dst_cap`: bytes writable from `dst`
// (0: unknown), which lets the boundary units of the segments be written whole.
int launch_pack(const Segment* segs, size_t n, ArrowDeviceType dev, uint8_t* dst,
                hipStream_t stream, hipEvent_t ev_start, hipEvent_t ev_stop,
                const FillSignal* signal = nullptr, bool* signalled = nullptr,
                uint64_t dst_cap = 0);

// Pack device segments into `dst` (device or mapped host memory) and return once complete,
// waiting on the launch's own fill signal instead of a blocking stream synchronise.
int launch_pack_wait(const Segment* segs, size_t n, uint8_t* dst, hipStream_t stream);

void serialize_type_info(const TypeInfoNode& t, std::vector<uint8_t>& out);
// DataType as a schema tree: str format, str name, i64 flags, u8 has_meta [str meta],
// u32 n_children × Schema, u8 has_dict [Schema].  The top level carries no name and only the
// type-relevant flags (dictionary ordered / map keys sorted).
void serialize_schema(const ArrowSchema* s, bool top, std::vector<uint8_t>& out);
std::string schema_sig(const ArrowSchema* s);
uint64_t metadata_len(const char* meta);
// Everything a plan of (array, schema) depends on when it reads no array bytes, as words: per
// node in walk order the schema's identity and strings (hashed), flags, and the array's length,
// offset, null count, buffer addresses and child counts.  Equal keys give equal plans (a node's
// plan cache, node.cpp).  False when the tree is too large to key.
bool plan_key(const ArrowArray* array, const ArrowSchema* schema, std::vector<uint64_t>& out);

Layout layout_of(const char* format);
inline Layout layout_of(const std::string& format) { return layout_of(format.c_str()); }
int build_plan(const ArrowArray* array, const ArrowSchema* schema, ArrowDeviceType dev,
               dora_plan** out, bool validity_in_sample = false);
int build_plan_compact(const ArrowArray* array, const ArrowSchema* schema, ArrowDeviceType dev,
                       dora_plan** out);

}  // namespace dora

struct dora_plan {
  ArrowDeviceType dev = ARROW_DEVICE_ROCM;
  bool compact = false;  // built by dora_gpu_plan_compact (carries transform segments)
  uint64_t size = 0;      // required_data_size: the reference sample
  uint64_t ext_size = 0;  // bytes to allocate and fill incl. a validity tail (0: == size)
  bool read_device = false;  // planning read bytes of the array (last offsets, bitmaps)
  std::vector<dora::Segment> segs;
  dora::TypeInfoNode root;
  uint64_t fill_size() const { return ext_size > size ? ext_size : size; }
};
