// Host-side planning of a pack: the a1 walk (`required_data_size_inner`,
// apis/rust/node/src/node/arrow_utils.rs:9-21) and the ArrowTypeInfo half of
// `copy_array_into_sample_inner` (arrow_utils.rs:28-71), over the Arrow C Data Interface.
//
// Restated third-party rules (arrow-rs 53.2.0, pinned by Cargo.lock, not vendored):
//   * layout(): arrow-data `layout()` buffer specs and alignments (Rust 1.76: i128 align 8);
//   * buffer lengths: arrow-rs FFI import `buffer_len` (offsets (len+offset+1)*w, Utf8/Binary
//     data = last offset, everything else ceil((len+offset)*bits/8));
//   * nulls: kept only when the null count is non-zero (ArrayDataBuilder::build filter).
#include <hip/hip_runtime_api.h>

#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "common.h"
#include "plan.h"

namespace dora {

namespace {

bool starts_with(const char* s, const char* p) { return std::strncmp(s, p, std::strlen(p)) == 0; }
bool eq(const char* a, const char* b) { return std::strcmp(a, b) == 0; }

}  // namespace

// arrow-data 53.2.0 `layout()`; throws std::domain_error for types outside the parity set.
// Matched on the C format string without building a std::string (a plan walks it per node).
Layout layout_of(const char* f) {
  Layout l;
  auto fixed = [&](uint32_t w, uint32_t a) { l.specs.push_back({BufSpec::Fixed, w, a}); };
  const bool one = f[0] && !f[1];  // single-character primitive formats
  if (one && f[0] == 'n') {
    l.can_null = false;
  } else if (one && f[0] == 'b') {
    l.specs.push_back({BufSpec::Bitmap, 0, 1});
  } else if (one && (f[0] == 'c' || f[0] == 'C')) {
    fixed(1, 1);
  } else if (one && (f[0] == 's' || f[0] == 'S' || f[0] == 'e')) {
    fixed(2, 2);
  } else if ((one && (f[0] == 'i' || f[0] == 'I' || f[0] == 'f')) || eq(f, "tdD") ||
             eq(f, "tts") || eq(f, "ttm") || eq(f, "tiM")) {
    fixed(4, 4);
  } else if ((one && (f[0] == 'l' || f[0] == 'L' || f[0] == 'g')) || eq(f, "tdm") ||
             eq(f, "ttu") || eq(f, "ttn") || starts_with(f, "ts") || starts_with(f, "tD")) {
    fixed(8, 8);
  } else if (eq(f, "tiD")) {
    fixed(8, 4);  // IntervalDayTime {i32, i32}
  } else if (eq(f, "tin")) {
    fixed(16, 8);  // IntervalMonthDayNano {i32, i32, i64}
  } else if (starts_with(f, "d:")) {
    // "d:precision,scale[,bitwidth]"; i128 / i256 have align 8 on the pinned Rust 1.76
    int commas = 0;
    const char* last = nullptr;
    for (const char* p = f; *p; ++p)
      if (*p == ',') ++commas, last = p;
    const int bw = commas >= 2 ? std::atoi(last + 1) : 128;
    if (bw != 128 && bw != 256) throw std::invalid_argument(std::string("decimal bit width ") + f);
    fixed(static_cast<uint32_t>(bw / 8), 8);
  } else if (starts_with(f, "w:")) {
    fixed(static_cast<uint32_t>(std::strtoul(f + 2, nullptr, 10)), 1);
  } else if (one && (f[0] == 'z' || f[0] == 'u')) {
    fixed(4, 4);
    l.specs.push_back({BufSpec::Var, 0, 1});
    l.offsets_first = true;
  } else if (one && (f[0] == 'Z' || f[0] == 'U')) {
    fixed(8, 8);
    l.specs.push_back({BufSpec::Var, 0, 1});
    l.offsets_first = true;
  } else if (eq(f, "+l") || eq(f, "+m")) {
    fixed(4, 4);
    l.offsets_first = true;
  } else if (eq(f, "+L")) {
    fixed(8, 8);
    l.offsets_first = true;
  } else if (starts_with(f, "+w:") || eq(f, "+s")) {
    // children only
  } else if (eq(f, "+r")) {
    l.can_null = false;
  } else {
    // views (vz/vu: the reference's zip drops variadic buffers), unions, list views
    throw std::domain_error(std::string("arrow format '") + f +
                            "' is outside the supported parity set");
  }
  return l;
}

uint64_t metadata_len(const char* meta) {
  // Arrow C metadata: i32 n, then n × (i32 klen, key, i32 vlen, value)
  if (!meta) return 0;
  int32_t n;
  std::memcpy(&n, meta, 4);
  uint64_t off = 4;
  for (int32_t i = 0; i < n; ++i)
    for (int kv = 0; kv < 2; ++kv) {
      int32_t l;
      std::memcpy(&l, meta + off, 4);
      off += 4 + static_cast<uint64_t>(l);
    }
  return off;
}

std::string schema_sig(const ArrowSchema* s) {
  std::string fmt = s->format ? s->format : "";
  if (s->dictionary) {
    std::string out = "dict<" + fmt + "," + schema_sig(s->dictionary);
    if (s->flags & ARROW_FLAG_DICTIONARY_ORDERED) out += ",ordered";
    return out + ">";
  }
  std::string out = fmt;
  if (fmt == "+m" && (s->flags & ARROW_FLAG_MAP_KEYS_SORTED)) out += "s";
  if (s->n_children > 0) {
    out += "[";
    for (int64_t i = 0; i < s->n_children; ++i) {
      const ArrowSchema* c = s->children[i];
      if (i) out += ",";
      out += c->name ? c->name : "";
      out += ":";
      out += (c->flags & ARROW_FLAG_NULLABLE) ? "?" : "!";
      out += schema_sig(c);
    }
    out += "]";
  }
  return out;
}

namespace {

void put_str(std::vector<uint8_t>& o, const char* p, uint64_t n) {
  for (int i = 0; i < 4; ++i) o.push_back(static_cast<uint8_t>(n >> (8 * i)));
  o.insert(o.end(), p, p + n);
}

}  // namespace

void serialize_schema(const ArrowSchema* s, bool top, std::vector<uint8_t>& o) {
  const char* f = s->format ? s->format : "";
  put_str(o, f, std::strlen(f));
  const char* nm = (!top && s->name) ? s->name : "";
  put_str(o, nm, std::strlen(nm));
  int64_t flags = s->flags;
  if (top) flags &= (ARROW_FLAG_DICTIONARY_ORDERED | ARROW_FLAG_MAP_KEYS_SORTED);
  for (int i = 0; i < 8; ++i) o.push_back(static_cast<uint8_t>(uint64_t(flags) >> (8 * i)));
  const uint64_t ml = top ? 0 : metadata_len(s->metadata);
  o.push_back(ml ? 1 : 0);
  if (ml) put_str(o, s->metadata, ml);
  const uint32_t nc = static_cast<uint32_t>(s->n_children);
  for (int i = 0; i < 4; ++i) o.push_back(static_cast<uint8_t>(nc >> (8 * i)));
  for (uint32_t i = 0; i < nc; ++i) serialize_schema(s->children[i], false, o);
  o.push_back(s->dictionary ? 1 : 0);
  if (s->dictionary) serialize_schema(s->dictionary, false, o);
}

namespace {

// Host reads a plan needs from the array (last offsets of Utf8/Binary data, validity bitmaps).
// Device arrays: DIRECT does one blocking hipMemcpy per read; the reference walk (build_plan)
// instead runs twice — COLLECT records every read (no address depends on a value read, so the
// second walk asks for the same ranges in the same order), one gather launch of the pack kernel
// copies them all into pinned host memory, REPLAY serves them from there.  One launch + one
// sync per plan instead of one blocking copy per buffer.
struct Reader {
  ArrowDeviceType dev = ARROW_DEVICE_CPU;
  enum Mode { DIRECT, COLLECT, REPLAY } mode = DIRECT;
  mutable std::vector<Segment> reqs;  // src, offset in the staging buffer, len
  mutable uint64_t total = 0;
  mutable size_t cursor = 0;
  const uint8_t* staged = nullptr;
  // validity bitmaps of device arrays with a known null count go to the sample's tail
  bool defer_validity = false;
  mutable std::vector<const void*> deferred;  // their sources, in walk (DFS pre-order) order

  void read(void* dst, const void* src, size_t n) const {
    if (n == 0) return;
    if (dev != ARROW_DEVICE_ROCM) {
      std::memcpy(dst, src, n);
      return;
    }
    if (mode == COLLECT) {
      reqs.push_back({src, total, n});
      total += (n + 15) / 16 * 16;
      std::memset(dst, 0, n);
    } else if (mode == REPLAY) {
      if (cursor >= reqs.size() || reqs[cursor].src != src || reqs[cursor].len != n)
        throw std::logic_error("plan: replayed read differs from the collected one");
      std::memcpy(dst, staged + reqs[cursor++].dst_off, n);
    } else {
      hipError_t e = hipMemcpy(dst, src, n, hipMemcpyDeviceToHost);
      if (e != hipSuccess)
        throw std::runtime_error(std::string("hipMemcpy D2H during plan: ") +
                                 hipGetErrorString(e));
    }
  }
};

// Pinned staging buffer + stream of this thread for the current device (plans are built on the
// caller's thread; the stream is a blocking one, ordered after legacy-stream work like the
// hipMemcpy it replaces).
struct GatherCtx {
  int device = -1;
  hipStream_t stream = nullptr;
  uint8_t* host = nullptr;
  void* host_dev = nullptr;
  uint64_t cap = 0;
};

const uint8_t* gather_to_host(const std::vector<Segment>& reqs, uint64_t total) {
  thread_local std::vector<GatherCtx> ctxs;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) throw std::runtime_error("plan: no current device");
  GatherCtx* c = nullptr;
  for (auto& x : ctxs)
    if (x.device == dev) c = &x;
  if (!c) {
    ctxs.push_back(GatherCtx{});
    c = &ctxs.back();
    c->device = dev;
    if (hipStreamCreate(&c->stream) != hipSuccess)
      throw std::runtime_error("plan: gather stream");
  }
  if (c->cap < total) {
    if (c->host) (void)hipHostFree(c->host);
    c->host = nullptr;
    c->cap = 0;
    const uint64_t cap = std::max<uint64_t>(total, 1 << 20);
    if (hipHostMalloc(reinterpret_cast<void**>(&c->host), cap, hipHostMallocMapped) !=
            hipSuccess ||
        hipHostGetDevicePointer(&c->host_dev, c->host, 0) != hipSuccess)
      throw std::runtime_error("plan: pinned staging buffer");
    c->cap = cap;
  }
  int rc = launch_pack_wait(reqs.data(), reqs.size(), static_cast<uint8_t*>(c->host_dev),
                            c->stream);
  if (rc != DORA_OK) throw std::runtime_error(std::string("plan: gather: ") + dora_gpu_last_error());
  return c->host;
}

uint64_t count_nulls(const std::vector<uint8_t>& v, uint64_t off, uint64_t len) {
  uint64_t n = 0;
  for (uint64_t i = off; i < off + len; ++i) n += ((v[i >> 3] >> (i & 7)) & 1) ? 0 : 1;
  return n;
}

uint64_t pad_to(uint64_t x, const BufSpec& sp) {
  if (sp.kind != BufSpec::Fixed) return x;
  return (x + sp.align - 1) / sp.align * sp.align;
}

// One ArrayData node: buffers in layout order, then children (DFS pre-order), exactly as
// copy_array_into_sample_inner walks it.
void walk(const ArrowArray* a, const ArrowSchema* s, const Reader& rd, uint64_t& next,
          std::vector<Segment>& segs, TypeInfoNode& ti) {
  if (!a || !s || !s->format) throw std::invalid_argument("null ArrowArray/ArrowSchema node");
  const char* fmt = s->format;
  const bool is_dict = s->dictionary != nullptr;
  Layout l = layout_of(fmt);  // dictionary: layout(key type) == layout(index format)
  if (is_dict) l.offsets_first = false;
  if (a->length < 0 || a->offset < 0) throw std::invalid_argument("negative length/offset");
  const uint64_t len = static_cast<uint64_t>(a->length);
  const uint64_t off = static_cast<uint64_t>(a->offset);
  const uint64_t total = len + off;
  const int64_t begin = l.can_null ? 1 : 0;
  if (a->n_buffers < begin + static_cast<int64_t>(l.specs.size()))
    throw std::invalid_argument(std::string("ArrowArray for '") + fmt + "' has too few buffers");

  serialize_schema(s, true, ti.schema);
  ti.len = len;
  ti.offset = off;
  ti.null_count = 0;
  ti.has_validity = false;

  uint64_t lens[3] = {0, 0, 0};
  for (size_t k = 0; k < l.specs.size(); ++k) {
    const BufSpec& sp = l.specs[k];
    const void* p = a->buffers[begin + static_cast<int64_t>(k)];
    uint64_t blen;
    if (sp.kind == BufSpec::Var) {
      if (len == 0) {
        blen = 0;
      } else {
        const uint32_t ow = l.specs[0].width;
        const uint64_t last = lens[0] / ow - 1;
        const uint8_t* op = static_cast<const uint8_t*>(a->buffers[begin]) + last * ow;
        if (ow == 4) {
          int32_t v;
          rd.read(&v, op, 4);
          if (v < 0) throw std::invalid_argument("negative last offset");
          blen = static_cast<uint64_t>(v);
        } else {
          int64_t v;
          rd.read(&v, op, 8);
          if (v < 0) throw std::invalid_argument("negative last offset");
          blen = static_cast<uint64_t>(v);
        }
      }
    } else if (k == 0 && l.offsets_first) {
      blen = (total + 1) * sp.width;
    } else {
      const uint64_t bits = sp.kind == BufSpec::Bitmap ? 1 : uint64_t(sp.width) * 8;
      blen = (total * bits + 7) / 8;
    }
    lens[k] = blen;
    if (!p && blen != 0)
      throw std::invalid_argument("buffer " + std::to_string(begin + k) + " of '" + fmt +
                                  "' is null but has length " + std::to_string(blen));
    next = pad_to(next, sp);
    ti.bufs.push_back({next, blen});
    if (blen) segs.push_back({p, next, blen});
    next += blen;
  }

  if (l.can_null && a->n_buffers > 0 && a->buffers[0]) {
    if (rd.defer_validity && rd.dev == ARROW_DEVICE_ROCM && a->null_count >= 0) {
      // the same bytes the inline form would carry, copied on the device (no read-back)
      if (a->null_count != 0) {
        ti.has_validity = true;
        ti.validity_in_sample = true;
        ti.validity_len = (total + 7) / 8;
        ti.null_count = static_cast<uint64_t>(a->null_count);
        rd.deferred.push_back(a->buffers[0]);
      }
    } else {
      std::vector<uint8_t> v((total + 7) / 8);
      rd.read(v.data(), a->buffers[0], v.size());
      uint64_t nc = a->null_count >= 0 ? static_cast<uint64_t>(a->null_count)
                                       : count_nulls(v, off, len);
      if (nc != 0) {
        ti.has_validity = true;
        ti.validity = std::move(v);
        ti.null_count = nc;
      }
    }
  }

  if (is_dict) {
    if (!a->dictionary) throw std::invalid_argument("dictionary schema without dictionary data");
    ti.children.emplace_back();
    walk(a->dictionary, s->dictionary, rd, next, segs, ti.children.back());
  } else {
    if (a->n_children != s->n_children)
      throw std::invalid_argument(std::string("array/schema child count mismatch for '") + fmt +
                                  "'");
    ti.children.resize(static_cast<size_t>(a->n_children));
    for (int64_t i = 0; i < a->n_children; ++i)
      walk(a->children[i], s->children[i], rd, next, segs, ti.children[static_cast<size_t>(i)]);
  }
}

// ---------------------------------------------------------------------------------------------
// Compacting walk (new capability; the reference copies sliced buffers whole and passes the
// offset through, F3): every node is reduced to exactly its logical range [phys, phys + len) of
// its buffers — fixed-width values sliced, Boolean bitmaps bit-shifted to bit 0, offsets rebased
// to start at 0 with the child / value ranges they address sliced recursively, validity
// bit-shifted on the host for the type info — so a slice moves only its own bytes and the
// receiver gets offset 0 everywhere.  `phys` is the element index into this node's buffers.
// ---------------------------------------------------------------------------------------------
std::vector<uint8_t> shift_bits_host(const std::vector<uint8_t>& src, uint64_t bit0,
                                     uint64_t nbits) {
  std::vector<uint8_t> out((nbits + 7) / 8, 0);
  for (uint64_t i = 0; i < nbits; ++i)
    if ((src[(bit0 + i) >> 3] >> ((bit0 + i) & 7)) & 1) out[i >> 3] |= uint8_t(1u << (i & 7));
  return out;
}

void walk_compact(const ArrowArray* a, const ArrowSchema* s, const Reader& rd, uint64_t phys,
                  uint64_t len, uint64_t& next, std::vector<Segment>& segs, TypeInfoNode& ti) {
  if (!a || !s || !s->format) throw std::invalid_argument("null ArrowArray/ArrowSchema node");
  const std::string fmt = s->format;
  const bool is_dict = s->dictionary != nullptr;
  if (fmt == "+r") throw std::domain_error("run-end encoded arrays cannot be compacted");
  Layout l = layout_of(fmt);
  if (is_dict) l.offsets_first = false;
  const int64_t begin = l.can_null ? 1 : 0;
  if (a->n_buffers < begin + static_cast<int64_t>(l.specs.size()))
    throw std::invalid_argument("ArrowArray for '" + fmt + "' has too few buffers");
  serialize_schema(s, true, ti.schema);
  ti.len = len;
  ti.offset = 0;
  ti.null_count = 0;
  ti.has_validity = false;

  uint64_t o_start = 0, o_end = 0;  // child / value range addressed by an offsets buffer
  for (size_t k = 0; k < l.specs.size(); ++k) {
    const BufSpec& sp = l.specs[k];
    const uint8_t* p = static_cast<const uint8_t*>(a->buffers[begin + static_cast<int64_t>(k)]);
    Segment seg{nullptr, 0, 0};
    if (sp.kind == BufSpec::Bitmap) {
      seg.len = (len + 7) / 8;
      seg.src = p + phys / 8;
      seg.op = SEG_BITSHIFT;
      seg.aux = static_cast<uint32_t>(phys % 8);
      seg.src_len = (phys + len + 7) / 8 - phys / 8;
    } else if (k == 0 && l.offsets_first) {
      const uint32_t w = sp.width;
      seg.len = (len + 1) * w;
      seg.src = p + phys * w;
      seg.op = w == 4 ? SEG_REBASE32 : SEG_REBASE64;
      if (w == 4) {
        int32_t v[2];
        rd.read(&v[0], p + phys * 4, 4);
        rd.read(&v[1], p + (phys + len) * 4, 4);
        if (v[0] < 0 || v[1] < v[0]) throw std::invalid_argument("bad offsets");
        o_start = uint64_t(v[0]);
        o_end = uint64_t(v[1]);
      } else {
        int64_t v[2];
        rd.read(&v[0], p + phys * 8, 8);
        rd.read(&v[1], p + (phys + len) * 8, 8);
        if (v[0] < 0 || v[1] < v[0]) throw std::invalid_argument("bad offsets");
        o_start = uint64_t(v[0]);
        o_end = uint64_t(v[1]);
      }
    } else if (sp.kind == BufSpec::Var) {
      seg.len = o_end - o_start;
      seg.src = p + o_start;
    } else {
      seg.len = len * sp.width;
      seg.src = p + phys * sp.width;
    }
    if (!p && seg.len) throw std::invalid_argument("null buffer with data in '" + fmt + "'");
    next = pad_to(next, sp);
    seg.dst_off = next;
    ti.bufs.push_back({next, seg.len});
    if (seg.len) segs.push_back(seg);
    next += seg.len;
  }

  if (l.can_null && a->n_buffers > 0 && a->buffers[0] && len) {
    std::vector<uint8_t> v((phys + len + 7) / 8);
    rd.read(v.data(), a->buffers[0], v.size());
    std::vector<uint8_t> sv = shift_bits_host(v, phys, len);
    const uint64_t nc = count_nulls(sv, 0, len);
    if (nc != 0) {
      ti.has_validity = true;
      ti.validity = std::move(sv);
      ti.null_count = nc;
    }
  }

  if (is_dict) {
    if (!a->dictionary) throw std::invalid_argument("dictionary schema without dictionary data");
    ti.children.emplace_back();
    const ArrowArray* d = a->dictionary;
    walk_compact(d, s->dictionary, rd, uint64_t(d->offset), uint64_t(d->length), next, segs,
                 ti.children.back());
    return;
  }
  if (a->n_children != s->n_children)
    throw std::invalid_argument("array/schema child count mismatch for '" + fmt + "'");
  for (int64_t i = 0; i < a->n_children; ++i) {
    const ArrowArray* c = a->children[i];
    uint64_t cphys, clen;
    if (l.offsets_first) {  // list / large list / map: the offsets address the child range
      cphys = uint64_t(c->offset) + o_start;
      clen = o_end - o_start;
    } else if (fmt.rfind("+w:", 0) == 0) {  // fixed-size list of k
      const uint64_t kk = std::stoull(fmt.substr(3));
      cphys = uint64_t(c->offset) + phys * kk;
      clen = len * kk;
    } else {  // struct: children are indexed by the parent's physical index
      cphys = uint64_t(c->offset) + phys;
      clen = len;
    }
    ti.children.emplace_back();
    walk_compact(c, s->children[i], rd, cphys, clen, next, segs, ti.children.back());
  }
}

void put_u8(std::vector<uint8_t>& o, uint8_t v) { o.push_back(v); }
void put_u32(std::vector<uint8_t>& o, uint32_t v) {
  for (int i = 0; i < 4; ++i) o.push_back(static_cast<uint8_t>(v >> (8 * i)));
}
void put_u64(std::vector<uint8_t>& o, uint64_t v) {
  for (int i = 0; i < 8; ++i) o.push_back(static_cast<uint8_t>(v >> (8 * i)));
}

}  // namespace

void serialize_type_info(const TypeInfoNode& t, std::vector<uint8_t>& o) {
  put_u32(o, static_cast<uint32_t>(t.schema.size()));
  o.insert(o.end(), t.schema.begin(), t.schema.end());
  put_u64(o, t.len);
  put_u64(o, t.null_count);
  // validity tag: 0 none, 1 inline bytes (the reference's Option<Vec<u8>>), 2 in the sample
  put_u8(o, !t.has_validity ? 0 : t.validity_in_sample ? 2 : 1);
  if (t.has_validity && t.validity_in_sample) {
    put_u64(o, t.validity_off);
    put_u64(o, t.validity_len);
  } else if (t.has_validity) {
    put_u64(o, t.validity.size());
    o.insert(o.end(), t.validity.begin(), t.validity.end());
  }
  put_u64(o, t.offset);
  put_u32(o, static_cast<uint32_t>(t.bufs.size()));
  for (auto& b : t.bufs) {
    put_u64(o, b.first);
    put_u64(o, b.second);
  }
  put_u32(o, static_cast<uint32_t>(t.children.size()));
  for (auto& c : t.children) serialize_type_info(c, o);
}

int build_plan_compact(const ArrowArray* array, const ArrowSchema* schema, ArrowDeviceType dev,
                       dora_plan** out) {
  if (!out) return fail(DORA_ERR_INVALID, "out is NULL");
  *out = nullptr;
  // host arrays can be planned (sizes, type info) but only device arrays packed
  if (dev != ARROW_DEVICE_CPU && dev != ARROW_DEVICE_ROCM && dev != ARROW_DEVICE_ROCM_HOST)
    return fail(DORA_ERR_INVALID, "unsupported device_type %d", dev);
  if (!array || !schema) return fail(DORA_ERR_INVALID, "null ArrowArray/ArrowSchema");
  auto* p = new dora_plan();
  p->dev = dev;
  p->compact = true;
  try {
    Reader rd;
    rd.dev = dev;
    uint64_t next = 0;
    walk_compact(array, schema, rd, uint64_t(array->offset), uint64_t(array->length), next,
                 p->segs, p->root);
    p->size = next;
  } catch (const std::domain_error& e) {
    delete p;
    return fail(DORA_ERR_UNSUPPORTED, "%s", e.what());
  } catch (const std::exception& e) {
    delete p;
    return fail(DORA_ERR_INVALID, "plan: %s", e.what());
  }
  *out = p;
  return DORA_OK;
}

namespace {

uint64_t hash_bytes(const char* p, size_t n) {
  uint64_t h = 0xcbf29ce484222325ull;
  for (size_t i = 0; i < n; ++i) h = (h ^ uint8_t(p[i])) * 0x100000001b3ull;
  return h ^ n;
}

bool key_node(const ArrowArray* a, const ArrowSchema* s, std::vector<uint64_t>& o) {
  if (!a || !s || !s->format || o.size() > 4096) return false;
  const size_t fl = std::strlen(s->format);
  o.push_back(reinterpret_cast<uintptr_t>(s));
  o.push_back(hash_bytes(s->format, fl));
  o.push_back(s->name ? hash_bytes(s->name, std::strlen(s->name)) : 0);
  o.push_back(static_cast<uint64_t>(s->flags));
  o.push_back(s->metadata ? hash_bytes(s->metadata, metadata_len(s->metadata)) : 0);
  o.push_back(static_cast<uint64_t>(a->length));
  o.push_back(static_cast<uint64_t>(a->offset));
  o.push_back(static_cast<uint64_t>(a->null_count));
  o.push_back(static_cast<uint64_t>(a->n_buffers) | (uint64_t(a->n_children) << 32));
  o.push_back(static_cast<uint64_t>(s->n_children) | (uint64_t(s->dictionary != nullptr) << 32) |
              (uint64_t(a->dictionary != nullptr) << 33));
  for (int64_t k = 0; k < a->n_buffers; ++k) o.push_back(reinterpret_cast<uintptr_t>(a->buffers[k]));
  if (s->dictionary) return a->dictionary && key_node(a->dictionary, s->dictionary, o);
  if (a->n_children != s->n_children) return false;
  for (int64_t i = 0; i < a->n_children; ++i)
    if (!key_node(a->children[i], s->children[i], o)) return false;
  return true;
}

}  // namespace

bool plan_key(const ArrowArray* array, const ArrowSchema* schema, std::vector<uint64_t>& out) {
  out.clear();
  return key_node(array, schema, out);
}

namespace {

// Validity tail of a plan with deferred bitmaps: 64-B aligned after the sample, in walk order.
void place_validity(TypeInfoNode& t, const std::vector<const void*>& src, size_t& k,
                    uint64_t& next, std::vector<Segment>& segs) {
  if (t.validity_in_sample) {
    next = (next + 63) / 64 * 64;
    t.validity_off = next;
    segs.push_back({src.at(k++), next, t.validity_len});
    next += t.validity_len;
  }
  for (auto& c : t.children) place_validity(c, src, k, next, segs);
}

}  // namespace

int build_plan(const ArrowArray* array, const ArrowSchema* schema, ArrowDeviceType dev,
               dora_plan** out, bool validity_in_sample) {
  if (!out) return fail(DORA_ERR_INVALID, "out is NULL");
  *out = nullptr;
  if (dev != ARROW_DEVICE_CPU && dev != ARROW_DEVICE_ROCM && dev != ARROW_DEVICE_ROCM_HOST)
    return fail(DORA_ERR_INVALID, "unsupported device_type %d", dev);
  auto* p = new dora_plan();
  p->dev = dev;
  try {
    Reader rd;
    rd.dev = dev;
    rd.defer_validity = validity_in_sample;
    uint64_t next = 0;
    bool done = false;
    if (dev == ARROW_DEVICE_ROCM) {
      rd.mode = Reader::COLLECT;
      walk(array, schema, rd, next, p->segs, p->root);
      // no device bytes read (e.g. fixed-width / nested arrays with in-sample validity): the
      // collecting walk is the plan; otherwise replay it with the gathered bytes
      done = rd.reqs.empty();
      p->read_device = !done;
      if (!done) {
        rd.staged = gather_to_host(rd.reqs, rd.total);
        rd.mode = Reader::REPLAY;
        next = 0;
        rd.deferred.clear();
        p->segs.clear();
        p->root = TypeInfoNode();
      }
    }
    if (!done) walk(array, schema, rd, next, p->segs, p->root);
    p->size = next;
    if (!rd.deferred.empty()) {
      size_t k = 0;
      place_validity(p->root, rd.deferred, k, next, p->segs);
      p->ext_size = next;
    }
  } catch (const std::domain_error& e) {
    delete p;
    return fail(DORA_ERR_UNSUPPORTED, "%s", e.what());
  } catch (const std::exception& e) {
    delete p;
    return fail(DORA_ERR_INVALID, "plan: %s", e.what());
  }
  *out = p;
  return DORA_OK;
}

}  // namespace dora

extern "C" {

int dora_gpu_plan(const struct ArrowArray* array, const struct ArrowSchema* schema,
                  ArrowDeviceType device_type, dora_plan** out) {
  return dora::build_plan(array, schema, device_type, out);
}

int dora_gpu_plan_compact(const struct ArrowArray* array, const struct ArrowSchema* schema,
                          ArrowDeviceType device_type, dora_plan** out) {
  return dora::build_plan_compact(array, schema, device_type, out);
}

int dora_gpu_plan_bytes(const void* src, size_t len, ArrowDeviceType device_type,
                        dora_plan** out) {
  if (!out) return dora::fail(DORA_ERR_INVALID, "out is NULL");
  if (!src && len) return dora::fail(DORA_ERR_INVALID, "src is NULL");
  DORA_GUARD_BEGIN
  auto* p = new dora_plan();
  p->dev = device_type;
  p->size = len;
  // ArrowTypeInfo::byte_array(len), libraries/message/src/metadata.rs:74-87
  {
    ArrowSchema u8{};
    u8.format = "C";
    dora::serialize_schema(&u8, true, p->root.schema);
  }
  p->root.len = len;
  p->root.bufs.push_back({0, len});
  if (len) p->segs.push_back({src, 0, len});
  *out = p;
  return DORA_OK;
  DORA_GUARD_END
}

void dora_gpu_plan_free(dora_plan* plan) { delete plan; }

size_t dora_gpu_plan_size(const dora_plan* plan) { return plan ? plan->size : 0; }

size_t dora_gpu_plan_num_segments(const dora_plan* plan) { return plan ? plan->segs.size() : 0; }

int dora_gpu_plan_segment(const dora_plan* plan, size_t i, const void** src, uint64_t* dst_off,
                          uint64_t* len) {
  if (!plan || i >= plan->segs.size())
    return dora::fail(DORA_ERR_INVALID, "segment index %zu out of range", i);
  if (src) *src = plan->segs[i].src;
  if (dst_off) *dst_off = plan->segs[i].dst_off;
  if (len) *len = plan->segs[i].len;
  return DORA_OK;
}

int dora_gpu_plan_type_info(const dora_plan* plan, uint8_t* buf, size_t cap, size_t* len) {
  if (!plan || !len) return dora::fail(DORA_ERR_INVALID, "plan/len is NULL");
  DORA_GUARD_BEGIN
  std::vector<uint8_t> o;
  dora::serialize_type_info(plan->root, o);
  *len = o.size();
  if (!buf) return DORA_OK;
  if (cap < o.size())
    return dora::fail(DORA_ERR_TOO_SMALL, "type info needs %zu bytes, buffer has %zu", o.size(),
                      cap);
  std::memcpy(buf, o.data(), o.size());
  return DORA_OK;
  DORA_GUARD_END
}

}  // extern "C"
