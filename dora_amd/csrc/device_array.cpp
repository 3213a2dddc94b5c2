// Device-resident Arrow arrays over the Arrow C Data Interface.
//
//  * dora_gpu_array_upload   : host ArrowArray -> HBM copy with the same structure (how a Python
//                              node's pyarrow array reaches a device sample, F12 workaround).
//  * dora_gpu_sample_import  : receiver side of a sample, `RawData::into_arrow_array` +
//                              `buffer_into_arrow_array` (apis/rust/node/src/event_stream/
//                              event.rs:35-91): zero-copy slices of the device sample per
//                              BufferOffset, validity from the type info, children recursively;
//                              an empty sample yields `ArrayData::new_empty(data_type)`.
//  * dora_gpu_array_download : device ArrowArray -> host ArrowArray (host staging for consumers
//                              that need CPU memory, e.g. pyarrow, which cannot import ROCm).
#include <hip/hip_runtime_api.h>

#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "aql.h"
#include "common.h"
#include "device_array.h"
#include "plan.h"

namespace dora {
namespace {

struct HipError : std::runtime_error {
  using std::runtime_error::runtime_error;
};

void hip_ok(hipError_t e, const char* what) {
  if (e != hipSuccess) throw HipError(std::string(what) + ": " + hipGetErrorString(e));
}

// ---------------------------------------------------------------------------------------------
// Owned ArrowArray: buffers either owned (device or host allocations) or borrowed from a shared
// keep-alive (the received sample).
// ---------------------------------------------------------------------------------------------
struct ArrayPrivate {
  std::vector<const void*> buffers;
  std::vector<void*> dev_owned;
  std::vector<void*> host_owned;
  std::vector<ArrowArray*> children;
  ArrowArray* dictionary = nullptr;
  std::shared_ptr<void> keepalive;
};

void release_array(ArrowArray* a) {
  if (!a || !a->release) return;
  auto* p = static_cast<ArrayPrivate*>(a->private_data);
  for (ArrowArray* c : p->children) {
    if (c->release) c->release(c);
    delete c;
  }
  if (p->dictionary) {
    if (p->dictionary->release) p->dictionary->release(p->dictionary);
    delete p->dictionary;
  }
  if (!p->dev_owned.empty()) aql_fence_all();  // AQL packs may still read these buffers
  for (void* d : p->dev_owned) (void)hipFree(d);
  for (void* h : p->host_owned) std::free(h);
  delete p;
  a->release = nullptr;
  a->private_data = nullptr;
}

ArrayPrivate* init_array(ArrowArray* out, int64_t length, int64_t null_count, int64_t offset,
                         size_t n_buffers) {
  auto* p = new ArrayPrivate();
  p->buffers.assign(n_buffers, nullptr);
  std::memset(out, 0, sizeof(*out));
  out->length = length;
  out->null_count = null_count;
  out->offset = offset;
  out->n_buffers = static_cast<int64_t>(n_buffers);
  out->buffers = p->buffers.data();
  out->release = release_array;
  out->private_data = p;
  return p;
}

void finish_children(ArrowArray* out, ArrayPrivate* p) {
  out->n_children = static_cast<int64_t>(p->children.size());
  out->children = p->children.empty() ? nullptr : p->children.data();
  out->dictionary = p->dictionary;
  out->buffers = p->buffers.data();
}

// Per C-struct buffer index: byte length under the arrow-rs FFI import rules.  `last_offset`
// reads the last offset value (host pointer) for variable-width data buffers.
std::vector<uint64_t> buffer_lengths(const ArrowArray* a, const ArrowSchema* s, bool host_reads) {
  const std::string fmt = s->format;
  Layout l = layout_of(fmt);
  if (s->dictionary) l.offsets_first = false;
  const uint64_t total = uint64_t(a->length) + uint64_t(a->offset);
  std::vector<uint64_t> lens;
  if (l.can_null) lens.push_back((total + 7) / 8);
  for (size_t k = 0; k < l.specs.size(); ++k) {
    const BufSpec& sp = l.specs[k];
    if (sp.kind == BufSpec::Var) {
      uint64_t blen = 0;
      if (a->length != 0) {
        const uint32_t ow = l.specs[0].width;
        const size_t oi = l.can_null ? 1 : 0;
        const uint8_t* op = static_cast<const uint8_t*>(a->buffers[oi]) + (total)*ow;
        if (host_reads) {
          if (ow == 4) {
            int32_t v;
            std::memcpy(&v, op, 4);
            blen = uint64_t(v);
          } else {
            int64_t v;
            std::memcpy(&v, op, 8);
            blen = uint64_t(v);
          }
        } else {
          if (ow == 4) {
            int32_t v;
            hip_ok(hipMemcpy(&v, op, 4, hipMemcpyDeviceToHost), "read last offset");
            blen = uint64_t(v);
          } else {
            int64_t v;
            hip_ok(hipMemcpy(&v, op, 8, hipMemcpyDeviceToHost), "read last offset");
            blen = uint64_t(v);
          }
        }
      }
      lens.push_back(blen);
    } else if (k == 0 && l.offsets_first) {
      lens.push_back((total + 1) * sp.width);
    } else {
      const uint64_t bits = sp.kind == BufSpec::Bitmap ? 1 : uint64_t(sp.width) * 8;
      lens.push_back((total * bits + 7) / 8);
    }
  }
  if (a->n_buffers != static_cast<int64_t>(lens.size()))
    throw std::domain_error("'" + fmt + "' exported with " + std::to_string(a->n_buffers) +
                            " buffers, expected " + std::to_string(lens.size()));
  return lens;
}

enum class Dir { ToDevice, ToHost };

void deep_copy(const ArrowArray* a, const ArrowSchema* s, Dir dir, ArrowArray* out) {
  const bool host_src = dir == Dir::ToDevice;
  const std::vector<uint64_t> lens = buffer_lengths(a, s, host_src);
  ArrayPrivate* p = init_array(out, a->length, a->null_count, a->offset, lens.size());
  try {
    for (size_t i = 0; i < lens.size(); ++i) {
      const void* src = a->buffers[i];
      if (!src) continue;  // absent validity / empty buffer stays NULL
      const uint64_t n = lens[i];
      if (dir == Dir::ToDevice) {
        void* d = nullptr;
        hip_ok(hipMalloc(&d, n ? n : 1), "hipMalloc");
        p->dev_owned.push_back(d);
        if (n) hip_ok(hipMemcpy(d, src, n, hipMemcpyHostToDevice), "upload");
        p->buffers[i] = d;
      } else {
        void* h = std::malloc(n ? n : 1);
        if (!h) throw std::bad_alloc();
        p->host_owned.push_back(h);
        if (n) hip_ok(hipMemcpy(h, src, n, hipMemcpyDeviceToHost), "download");
        p->buffers[i] = h;
      }
    }
    for (int64_t i = 0; i < a->n_children; ++i) {
      auto* c = new ArrowArray();
      p->children.push_back(c);
      deep_copy(a->children[i], s->children[i], dir, c);
    }
    if (s->dictionary) {
      p->dictionary = new ArrowArray();
      deep_copy(a->dictionary, s->dictionary, dir, p->dictionary);
    }
  } catch (...) {
    finish_children(out, p);
    release_array(out);
    throw;
  }
  finish_children(out, p);
}

// ---------------------------------------------------------------------------------------------
// Schema tree decoded from the type-info blob.
// ---------------------------------------------------------------------------------------------
struct SchemaPrivate {
  std::string format, name, metadata;
  std::vector<ArrowSchema*> children;
  ArrowSchema* dictionary = nullptr;
};

void release_schema(ArrowSchema* s) {
  if (!s || !s->release) return;
  auto* p = static_cast<SchemaPrivate*>(s->private_data);
  for (ArrowSchema* c : p->children) {
    if (c->release) c->release(c);
    delete c;
  }
  if (p->dictionary) {
    if (p->dictionary->release) p->dictionary->release(p->dictionary);
    delete p->dictionary;
  }
  delete p;
  s->release = nullptr;
  s->private_data = nullptr;
}

struct Cursor {
  const uint8_t* p;
  size_t n, i = 0;
  void need(size_t k) {
    if (i + k > n) throw std::invalid_argument("truncated type info");
  }
  uint8_t u8() {
    need(1);
    return p[i++];
  }
  uint32_t u32() {
    need(4);
    uint32_t v;
    std::memcpy(&v, p + i, 4);
    i += 4;
    return v;
  }
  uint64_t u64() {
    need(8);
    uint64_t v;
    std::memcpy(&v, p + i, 8);
    i += 8;
    return v;
  }
  std::string str() {
    uint32_t k = u32();
    need(k);
    std::string s(reinterpret_cast<const char*>(p + i), k);
    i += k;
    return s;
  }
};

void decode_schema(Cursor& c, ArrowSchema* out) {
  auto* p = new SchemaPrivate();
  std::memset(out, 0, sizeof(*out));
  out->release = release_schema;
  out->private_data = p;
  p->format = c.str();
  p->name = c.str();
  out->flags = static_cast<int64_t>(c.u64());
  if (c.u8()) p->metadata = c.str();
  const uint32_t nc = c.u32();
  for (uint32_t k = 0; k < nc; ++k) {
    auto* ch = new ArrowSchema();
    p->children.push_back(ch);
    decode_schema(c, ch);
  }
  if (c.u8()) {
    p->dictionary = new ArrowSchema();
    decode_schema(c, p->dictionary);
  }
  out->format = p->format.c_str();
  out->name = p->name.c_str();
  out->metadata = p->metadata.empty() ? nullptr : p->metadata.c_str();
  out->n_children = static_cast<int64_t>(p->children.size());
  out->children = p->children.empty() ? nullptr : p->children.data();
  out->dictionary = p->dictionary;
}

struct TiNode {
  std::vector<uint8_t> schema;
  uint64_t len = 0, null_count = 0, offset = 0;
  bool has_validity = false;
  std::vector<uint8_t> validity;
  bool in_sample = false;  // tag 2: bitmap at sample[voff, voff + vlen)
  uint64_t voff = 0, vlen = 0;
  std::vector<std::pair<uint64_t, uint64_t>> bufs;
  std::vector<TiNode> children;
};

void decode_ti(Cursor& c, TiNode& t) {
  const uint32_t sl = c.u32();
  c.need(sl);
  t.schema.assign(c.p + c.i, c.p + c.i + sl);
  c.i += sl;
  t.len = c.u64();
  t.null_count = c.u64();
  const uint8_t tag = c.u8();
  if (tag > 2) throw std::invalid_argument("unknown validity tag in type info");
  t.has_validity = tag != 0;
  t.in_sample = tag == 2;
  if (tag == 1) {
    const uint64_t vl = c.u64();
    c.need(vl);
    t.validity.assign(c.p + c.i, c.p + c.i + vl);
    c.i += vl;
  } else if (tag == 2) {
    t.voff = c.u64();
    t.vlen = c.u64();
  }
  t.offset = c.u64();
  const uint32_t nb = c.u32();
  for (uint32_t k = 0; k < nb; ++k) {
    uint64_t o = c.u64(), l = c.u64();
    t.bufs.push_back({o, l});
  }
  const uint32_t nch = c.u32();
  t.children.resize(nch);
  for (uint32_t k = 0; k < nch; ++k) decode_ti(c, t.children[k]);
}

// buffer_into_arrow_array (event.rs:61-91) on a device sample.
// `host`: the sample is in host memory (an inline Vec sample): bitmaps from the type info stay
// on the host.
void build_from_sample(const TiNode& t, const ArrowSchema* s, const uint8_t* sample,
                       uint64_t sample_len, uint64_t ext_len, const std::shared_ptr<void>& keep,
                       ArrowArray* out, bool host) {
  Layout l = layout_of(s->format);
  const size_t nbuf = (l.can_null ? 1 : 0) + t.bufs.size();
  if (t.bufs.size() != l.specs.size())
    throw std::invalid_argument("type info buffer count does not match the layout");
  ArrayPrivate* p = init_array(out, int64_t(t.len), int64_t(t.null_count), int64_t(t.offset), nbuf);
  p->keepalive = keep;
  try {
    size_t bi = 0;
    if (l.can_null) {
      if (t.in_sample) {
        // the bitmap travelled in the slot's tail: zero-copy like the buffers
        if (t.voff < sample_len || t.voff + t.vlen > ext_len)
          throw std::invalid_argument("in-sample validity outside the slot's tail");
        p->buffers[0] = sample + t.voff;
      } else if (t.has_validity && host) {
        void* h = std::malloc(t.validity.size() ? t.validity.size() : 1);
        if (!h) throw std::bad_alloc();
        p->host_owned.push_back(h);
        if (!t.validity.empty()) std::memcpy(h, t.validity.data(), t.validity.size());
        p->buffers[0] = h;
      } else if (t.has_validity) {
        void* d = nullptr;
        hip_ok(hipMalloc(&d, t.validity.size() ? t.validity.size() : 1), "hipMalloc validity");
        p->dev_owned.push_back(d);
        if (!t.validity.empty())
          hip_ok(hipMemcpy(d, t.validity.data(), t.validity.size(), hipMemcpyHostToDevice),
                 "validity upload");
        p->buffers[0] = d;
      } else {
        out->null_count = 0;
      }
      bi = 1;
    }
    for (auto& b : t.bufs) {
      // Buffer::slice_with_length asserts offset + len <= buffer len
      if (b.first + b.second > sample_len)
        throw std::invalid_argument("buffer offset " + std::to_string(b.first) + "+" +
                                    std::to_string(b.second) + " exceeds sample length " +
                                    std::to_string(sample_len));
      p->buffers[bi++] = sample + b.first;
    }
    const ArrowSchema* const* kids = s->children;
    if (s->dictionary) {
      if (t.children.size() != 1) throw std::invalid_argument("dictionary needs one child");
      p->dictionary = new ArrowArray();
      build_from_sample(t.children[0], s->dictionary, sample, sample_len, ext_len, keep,
                        p->dictionary, host);
    } else {
      if (t.children.size() != size_t(s->n_children))
        throw std::invalid_argument("type info child count does not match the data type");
      for (size_t k = 0; k < t.children.size(); ++k) {
        auto* ch = new ArrowArray();
        p->children.push_back(ch);
        build_from_sample(t.children[k], kids[k], sample, sample_len, ext_len, keep, ch, host);
      }
    }
  } catch (...) {
    finish_children(out, p);
    release_array(out);
    throw;
  }
  finish_children(out, p);
}

// ArrayData::new_empty(data_type) on the device: zero-length buffers, one zero offset for
// offsets buffers, children empty too.
void build_empty(const ArrowSchema* s, ArrowArray* out, bool host) {
  Layout l = layout_of(s->format);
  if (s->dictionary) l.offsets_first = false;
  const size_t nbuf = (l.can_null ? 1 : 0) + l.specs.size();
  ArrayPrivate* p = init_array(out, 0, 0, 0, nbuf);
  try {
    size_t bi = l.can_null ? 1 : 0;
    for (size_t k = 0; k < l.specs.size(); ++k, ++bi) {
      const uint64_t n = (k == 0 && l.offsets_first) ? l.specs[0].width : 0;
      void* d = nullptr;
      if (host) {
        d = std::calloc(1, n ? n : 16);
        if (!d) throw std::bad_alloc();
        p->host_owned.push_back(d);
      } else {
        hip_ok(hipMalloc(&d, n ? n : 16), "hipMalloc empty");
        p->dev_owned.push_back(d);
        if (n) hip_ok(hipMemset(d, 0, n), "memset empty offsets");
      }
      p->buffers[bi] = d;
    }
    if (s->dictionary) {
      p->dictionary = new ArrowArray();
      build_empty(s->dictionary, p->dictionary, host);
    } else {
      for (int64_t k = 0; k < s->n_children; ++k) {
        auto* ch = new ArrowArray();
        p->children.push_back(ch);
        build_empty(s->children[k], ch, host);
      }
    }
  } catch (...) {
    finish_children(out, p);
    release_array(out);
    throw;
  }
  finish_children(out, p);
}

int guarded(const std::function<void()>& fn) {
  try {
    fn();
    return DORA_OK;
  } catch (const HipError& e) {
    return fail(DORA_ERR_HIP, "%s", e.what());
  } catch (const std::domain_error& e) {
    return fail(DORA_ERR_UNSUPPORTED, "%s", e.what());
  } catch (const std::exception& e) {
    return fail(DORA_ERR_INVALID, "%s", e.what());
  }
}

}  // namespace

int import_sample(const void* sample, uint64_t sample_len, const uint8_t* ti, size_t ti_len,
                  std::shared_ptr<void> keep, ArrowArray* out_array, ArrowSchema* out_schema,
                  uint64_t ext_len, bool host) {
  if (ext_len < sample_len) ext_len = sample_len;
  return guarded([&] {
    Cursor c{ti, ti_len};
    TiNode root;
    decode_ti(c, root);
    if (c.i != ti_len) throw std::invalid_argument("trailing bytes after type info");
    Cursor sc{root.schema.data(), root.schema.size()};
    decode_schema(sc, out_schema);
    try {
      if (sample_len == 0) {
        build_empty(out_schema, out_array, host);  // event.rs:65-67
      } else {
        build_from_sample(root, out_schema, static_cast<const uint8_t*>(sample), sample_len,
                          ext_len, keep, out_array, host);
      }
    } catch (...) {
      release_schema(out_schema);
      throw;
    }
  });
}

namespace {

void copy_bytes(Cursor& c, std::vector<uint8_t>& o, size_t k) {
  c.need(k);
  o.insert(o.end(), c.p + c.i, c.p + c.i + k);
  c.i += k;
}

void put64(std::vector<uint8_t>& o, uint64_t v) {
  for (int i = 0; i < 8; ++i) o.push_back(static_cast<uint8_t>(v >> (8 * i)));
}

// One type-info node (serialize_type_info's layout) copied to `o` with tag-2 bitmaps inlined.
void inline_ti(Cursor& c, std::vector<uint8_t>& o, const uint8_t* sample, uint64_t ext_len,
               bool host) {
  Cursor sc = c;
  const uint32_t sl = sc.u32();
  copy_bytes(c, o, 4 + size_t(sl) + 16);  // schema, len, null_count
  const uint8_t tag = c.u8();
  if (tag == 2) {
    const uint64_t off = c.u64(), vl = c.u64();
    if (off + vl > ext_len) throw std::invalid_argument("in-sample validity outside the slot");
    o.push_back(1);
    put64(o, vl);
    const size_t at = o.size();
    o.resize(at + vl);
    if (vl && host) std::memcpy(o.data() + at, sample + off, vl);
    else if (vl) hip_ok(hipMemcpy(o.data() + at, sample + off, vl, hipMemcpyDeviceToHost),
                        "validity read-back");
  } else {
    o.push_back(tag);
    if (tag == 1) {
      Cursor vc = c;
      copy_bytes(c, o, 8 + size_t(vc.u64()));
    } else if (tag != 0) {
      throw std::invalid_argument("unknown validity tag in type info");
    }
  }
  Cursor bc = c;
  bc.u64();
  const uint32_t nb = bc.u32();
  copy_bytes(c, o, 8 + 4 + 16 * size_t(nb));  // offset, buffer offsets
  const uint32_t nch = c.u32();
  for (int i = 0; i < 4; ++i) o.push_back(static_cast<uint8_t>(nch >> (8 * i)));
  for (uint32_t k = 0; k < nch; ++k) inline_ti(c, o, sample, ext_len, host);
}

bool has_in_sample(const TiNode& t) {
  if (t.in_sample) return true;
  for (auto& ch : t.children)
    if (has_in_sample(ch)) return true;
  return false;
}

}  // namespace

int inline_type_info(const uint8_t* ti, size_t ti_len, const void* sample, uint64_t ext_len,
                     std::vector<uint8_t>* out, bool* changed, bool host) {
  return guarded([&] {
    *changed = false;
    Cursor c{ti, ti_len};
    TiNode root;
    decode_ti(c, root);
    if (!has_in_sample(root)) return;
    if (!sample) throw std::invalid_argument("in-sample validity without sample data");
    Cursor w{ti, ti_len};
    std::vector<uint8_t> o;
    o.reserve(ti_len + 4096);
    inline_ti(w, o, static_cast<const uint8_t*>(sample), ext_len, host);
    out->swap(o);
    *changed = true;
  });
}

}  // namespace dora

extern "C" {

int dora_gpu_array_upload(const struct ArrowArray* array, const struct ArrowSchema* schema,
                          struct ArrowArray* out) {
  if (!array || !schema || !out) return dora::fail(DORA_ERR_INVALID, "NULL argument");
  return dora::guarded([&] { dora::deep_copy(array, schema, dora::Dir::ToDevice, out); });
}

int dora_gpu_array_download(const struct ArrowArray* array, const struct ArrowSchema* schema,
                            struct ArrowArray* out) {
  if (!array || !schema || !out) return dora::fail(DORA_ERR_INVALID, "NULL argument");
  return dora::guarded([&] { dora::deep_copy(array, schema, dora::Dir::ToHost, out); });
}

int dora_gpu_sample_import(const void* sample, size_t sample_len, const uint8_t* type_info,
                           size_t type_info_len, struct ArrowArray* out_array,
                           struct ArrowSchema* out_schema) {
  if (!type_info || !out_array || !out_schema || (!sample && sample_len))
    return dora::fail(DORA_ERR_INVALID, "NULL argument");
  return dora::import_sample(sample, sample_len, type_info, type_info_len, nullptr, out_array,
                             out_schema);
}

int dora_gpu_type_info_schema(const uint8_t* type_info, size_t type_info_len,
                              struct ArrowSchema* out_schema) {
  if (!type_info || !out_schema) return dora::fail(DORA_ERR_INVALID, "NULL argument");
  return dora::guarded([&] {
    dora::Cursor c{type_info, type_info_len};
    dora::TiNode root;
    dora::decode_ti(c, root);
    dora::Cursor sc{root.schema.data(), root.schema.size()};
    dora::decode_schema(sc, out_schema);
  });
}

void dora_gpu_array_release(struct ArrowArray* array) {
  if (array && array->release) array->release(array);
}

void dora_gpu_schema_release(struct ArrowSchema* schema) {
  if (schema && schema->release) schema->release(schema);
}

}  // extern "C"
