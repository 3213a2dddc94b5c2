// bincode of Timestamped<InterDaemonEvent> (see bincode.h for the layouts and their sources).
#include "bincode.h"

#include "common.h"
#include "dora_gpu.h"

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <map>
#include <stdexcept>

namespace dora {

namespace {

[[noreturn]] void bad(const std::string& what) { throw std::invalid_argument(what); }

// ---- this library's serialized schema tree (plan.cpp serialize_schema) ----
struct SNode {
  std::string format, name;
  int64_t flags = 0;
  bool has_meta = false;
  std::string meta;  // Arrow C metadata bytes
  std::vector<SNode> children;
  std::vector<SNode> dict;  // 0 or 1: the dictionary's value type
};

constexpr int64_t kDictOrdered = 1, kNullable = 2, kMapKeysSorted = 4;  // ARROW_FLAG_*

// plan.cpp's strings carry u32 lengths
struct R32 {
  const uint8_t* p;
  size_t n, i = 0;
  void need(size_t k) {
    if (i + k > n) bad("truncated type info");
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
  uint8_t u8() {
    need(1);
    return p[i++];
  }
  std::string str() {
    const uint32_t k = u32();
    need(k);
    std::string s(reinterpret_cast<const char*>(p + i), k);
    i += k;
    return s;
  }
};

SNode read_schema(R32& r, int depth = 0) {
  if (depth > 64) bad("type nested too deeply");
  SNode s;
  s.format = r.str();
  s.name = r.str();
  s.flags = static_cast<int64_t>(r.u64());
  s.has_meta = r.u8() != 0;
  if (s.has_meta) s.meta = r.str();
  const uint32_t nc = r.u32();
  for (uint32_t k = 0; k < nc; ++k) s.children.push_back(read_schema(r, depth + 1));
  if (r.u8()) s.dict.push_back(read_schema(r, depth + 1));
  return s;
}

void put32(std::vector<uint8_t>& o, uint32_t v) {
  for (int k = 0; k < 4; ++k) o.push_back(static_cast<uint8_t>(v >> (8 * k)));
}
void put64(std::vector<uint8_t>& o, uint64_t v) {
  for (int k = 0; k < 8; ++k) o.push_back(static_cast<uint8_t>(v >> (8 * k)));
}
void putstr32(std::vector<uint8_t>& o, const std::string& s) {
  put32(o, static_cast<uint32_t>(s.size()));
  o.insert(o.end(), s.begin(), s.end());
}

void write_schema(const SNode& s, std::vector<uint8_t>& o) {
  putstr32(o, s.format);
  putstr32(o, s.name);
  put64(o, static_cast<uint64_t>(s.flags));
  o.push_back(s.has_meta ? 1 : 0);
  if (s.has_meta) putstr32(o, s.meta);
  put32(o, static_cast<uint32_t>(s.children.size()));
  for (const SNode& c : s.children) write_schema(c, o);
  o.push_back(s.dict.empty() ? 0 : 1);
  if (!s.dict.empty()) write_schema(s.dict[0], o);
}

// ---- arrow-schema 53.2.0 DataType (datatype.rs declaration order) ----
enum : uint32_t {
  DT_NULL = 0, DT_BOOLEAN, DT_INT8, DT_INT16, DT_INT32, DT_INT64, DT_UINT8, DT_UINT16, DT_UINT32,
  DT_UINT64, DT_FLOAT16, DT_FLOAT32, DT_FLOAT64, DT_TIMESTAMP, DT_DATE32, DT_DATE64, DT_TIME32,
  DT_TIME64, DT_DURATION, DT_INTERVAL, DT_BINARY, DT_FIXED_SIZE_BINARY, DT_LARGE_BINARY,
  DT_BINARY_VIEW, DT_UTF8, DT_LARGE_UTF8, DT_UTF8_VIEW, DT_LIST, DT_LIST_VIEW,
  DT_FIXED_SIZE_LIST, DT_LARGE_LIST, DT_LARGE_LIST_VIEW, DT_STRUCT, DT_UNION, DT_DICTIONARY,
  DT_DECIMAL128, DT_DECIMAL256, DT_MAP, DT_RUN_END_ENCODED,
};
// single-character C formats of the variants without parameters
constexpr struct {
  char f;
  uint32_t v;
} kSimple[] = {{'n', DT_NULL},    {'b', DT_BOOLEAN}, {'c', DT_INT8},    {'s', DT_INT16},
               {'i', DT_INT32},   {'l', DT_INT64},   {'C', DT_UINT8},   {'S', DT_UINT16},
               {'I', DT_UINT32},  {'L', DT_UINT64},  {'e', DT_FLOAT16}, {'f', DT_FLOAT32},
               {'g', DT_FLOAT64}, {'z', DT_BINARY},  {'Z', DT_LARGE_BINARY}, {'u', DT_UTF8},
               {'U', DT_LARGE_UTF8}};
constexpr char kUnits[] = "smun";  // TimeUnit: Second, Millisecond, Microsecond, Nanosecond

uint32_t unit_of(char c, const std::string& f) {
  const char* u = std::strchr(kUnits, c);
  if (!c || !u) bad("arrow format '" + f + "': unknown time unit");
  return static_cast<uint32_t>(u - kUnits);
}

// Arrow C metadata (i32 n, n x (i32 klen, key, i32 vlen, value)) as HashMap<String, String>
void put_c_metadata(const SNode& s, WBuf& w) {
  if (!s.has_meta || s.meta.size() < 4) {
    w.u64(0);
    return;
  }
  R32 r{reinterpret_cast<const uint8_t*>(s.meta.data()), s.meta.size()};
  const uint32_t n = r.u32();
  w.u64(n);
  for (uint32_t k = 0; k < n; ++k) {
    w.str(r.str());
    w.str(r.str());
  }
}

void put_datatype(const SNode& s, WBuf& w, int depth = 0);

// Field (FieldRef = Arc<Field> serializes the field itself)
void put_field(const SNode& s, WBuf& w, int depth) {
  w.str(s.name);
  put_datatype(s, w, depth + 1);
  w.u8((s.flags & kNullable) ? 1 : 0);
  w.u64(0);  // dict_id
  w.u8(!s.dict.empty() && (s.flags & kDictOrdered) ? 1 : 0);
  put_c_metadata(s, w);
}

void put_datatype(const SNode& s, WBuf& w, int depth) {
  if (depth > 64) bad("type nested too deeply");
  const std::string& f = s.format;
  if (!s.dict.empty()) {  // Dictionary(Box<key type>, Box<value type>)
    w.u32(DT_DICTIONARY);
    SNode key;
    key.format = f;
    put_datatype(key, w, depth + 1);
    put_datatype(s.dict[0], w, depth + 1);
    return;
  }
  if (f.size() == 1) {
    for (const auto& k : kSimple)
      if (k.f == f[0]) {
        w.u32(k.v);
        return;
      }
  }
  auto need_children = [&](size_t k) {
    if (s.children.size() != k) bad("arrow format '" + f + "': wrong number of children");
  };
  if (f == "tdD") return w.u32(DT_DATE32);
  if (f == "tdm") return w.u32(DT_DATE64);
  if (f == "tts" || f == "ttm") {
    w.u32(DT_TIME32);
    return w.u32(unit_of(f[2], f));
  }
  if (f == "ttu" || f == "ttn") {
    w.u32(DT_TIME64);
    return w.u32(unit_of(f[2], f));
  }
  if (f.size() == 3 && f.compare(0, 2, "tD") == 0) {
    w.u32(DT_DURATION);
    return w.u32(unit_of(f[2], f));
  }
  if (f.size() >= 4 && f.compare(0, 2, "ts") == 0 && f[3] == ':') {  // tsu:UTC
    w.u32(DT_TIMESTAMP);
    w.u32(unit_of(f[2], f));
    const std::string tz = f.substr(4);
    w.u8(tz.empty() ? 0 : 1);
    if (!tz.empty()) w.str(tz);
    return;
  }
  if (f == "tiM" || f == "tiD" || f == "tin") {  // IntervalUnit: YearMonth, DayTime, MonthDayNano
    w.u32(DT_INTERVAL);
    return w.u32(f == "tiM" ? 0 : f == "tiD" ? 1 : 2);
  }
  if (f.compare(0, 2, "w:") == 0) {
    w.u32(DT_FIXED_SIZE_BINARY);
    return w.i32(std::stoi(f.substr(2)));
  }
  if (f.compare(0, 2, "d:") == 0) {  // d:precision,scale[,bitwidth]
    int p = 0, sc = 0, bw = 128;
    if (std::sscanf(f.c_str(), "d:%d,%d,%d", &p, &sc, &bw) < 2) bad("arrow format '" + f + "'");
    if (bw != 128 && bw != 256) bad("arrow format '" + f + "': decimal bit width");
    w.u32(bw == 128 ? DT_DECIMAL128 : DT_DECIMAL256);
    w.u8(static_cast<uint8_t>(p));
    return w.u8(static_cast<uint8_t>(static_cast<int8_t>(sc)));
  }
  if (f == "+l" || f == "+L") {
    need_children(1);
    w.u32(f == "+l" ? DT_LIST : DT_LARGE_LIST);
    return put_field(s.children[0], w, depth);
  }
  if (f.compare(0, 3, "+w:") == 0) {
    need_children(1);
    w.u32(DT_FIXED_SIZE_LIST);
    put_field(s.children[0], w, depth);
    return w.i32(std::stoi(f.substr(3)));
  }
  if (f == "+s") {
    w.u32(DT_STRUCT);
    w.u64(s.children.size());
    for (const SNode& c : s.children) put_field(c, w, depth);
    return;
  }
  if (f == "+m") {
    need_children(1);
    w.u32(DT_MAP);
    put_field(s.children[0], w, depth);
    return w.u8((s.flags & kMapKeysSorted) ? 1 : 0);
  }
  if (f == "+r") {
    need_children(2);
    w.u32(DT_RUN_END_ENCODED);
    put_field(s.children[0], w, depth);
    return put_field(s.children[1], w, depth);
  }
  bad("arrow format '" + f + "' is outside the data plane's parity set");
}

// HashMap<String, String> -> Arrow C metadata
void get_c_metadata(RBuf& r, SNode& s) {
  const uint64_t n = r.u64();
  if (n == 0) return;
  if (n > r.size()) bad("metadata count");
  std::vector<uint8_t> m;
  put32(m, static_cast<uint32_t>(n));
  for (uint64_t k = 0; k < n; ++k) {
    putstr32(m, r.str());
    putstr32(m, r.str());
  }
  s.has_meta = true;
  s.meta.assign(m.begin(), m.end());
}

SNode get_datatype(RBuf& r, int depth = 0);

SNode get_field(RBuf& r, int depth) {
  std::string name = r.str();
  SNode s = get_datatype(r, depth + 1);
  s.name = std::move(name);
  s.flags &= ~kNullable;  // the field's own nullability (below), not a dictionary default
  const uint8_t nullable = r.u8();
  (void)r.u64();  // dict_id
  const uint8_t ordered = r.u8();
  s.flags |= (nullable ? kNullable : 0) | (ordered && !s.dict.empty() ? kDictOrdered : 0);
  get_c_metadata(r, s);
  return s;
}

SNode get_datatype(RBuf& r, int depth) {
  if (depth > 64) bad("type nested too deeply");
  SNode s;
  const uint32_t v = r.u32();
  for (const auto& k : kSimple)
    if (k.v == v) {
      s.format = std::string(1, k.f);
      return s;
    }
  auto unit = [&] {
    const uint32_t u = r.u32();
    if (u > 3) bad("time unit");
    return kUnits[u];
  };
  switch (v) {
    case DT_TIMESTAMP: {
      s.format = std::string("ts") + unit() + ":";
      if (r.u8()) s.format += r.str();
      return s;
    }
    case DT_DATE32: s.format = "tdD"; return s;
    case DT_DATE64: s.format = "tdm"; return s;
    case DT_TIME32:
    case DT_TIME64: s.format = std::string("tt") + unit(); return s;
    case DT_DURATION: s.format = std::string("tD") + unit(); return s;
    case DT_INTERVAL: {
      const uint32_t u = r.u32();
      if (u > 2) bad("interval unit");
      s.format = u == 0 ? "tiM" : u == 1 ? "tiD" : "tin";
      return s;
    }
    case DT_FIXED_SIZE_BINARY: s.format = "w:" + std::to_string(r.i32()); return s;
    case DT_LIST:
    case DT_LARGE_LIST:
      s.format = v == DT_LIST ? "+l" : "+L";
      s.children.push_back(get_field(r, depth));
      return s;
    case DT_FIXED_SIZE_LIST:
      s.children.push_back(get_field(r, depth));
      s.format = "+w:" + std::to_string(r.i32());
      return s;
    case DT_STRUCT: {
      s.format = "+s";
      const uint64_t n = r.u64();
      if (n > r.size()) bad("struct field count");
      for (uint64_t k = 0; k < n; ++k) s.children.push_back(get_field(r, depth));
      return s;
    }
    case DT_DICTIONARY: {
      SNode key = get_datatype(r, depth + 1);
      if (!key.dict.empty() || !key.children.empty()) bad("dictionary key type");
      s.format = key.format;
      s.dict.push_back(get_datatype(r, depth + 1));
      // the wire's value type carries no nullability; C Data Interface exporters (pyarrow,
      // arrow-rs) mark a dictionary's values nullable
      s.dict[0].flags |= kNullable;
      return s;
    }
    case DT_DECIMAL128:
    case DT_DECIMAL256: {
      const int p = r.u8();
      const int sc = static_cast<int8_t>(r.u8());
      s.format = "d:" + std::to_string(p) + "," + std::to_string(sc) +
                 (v == DT_DECIMAL256 ? ",256" : "");
      return s;
    }
    case DT_MAP:
      s.format = "+m";
      s.children.push_back(get_field(r, depth));
      if (r.u8()) s.flags |= kMapKeysSorted;
      return s;
    case DT_RUN_END_ENCODED:
      s.format = "+r";
      s.children.push_back(get_field(r, depth));
      s.children.push_back(get_field(r, depth));
      return s;
    default:
      bad("arrow DataType variant " + std::to_string(v) + " is outside the data plane's parity set");
  }
}

// ---- ArrowTypeInfo ----
void put_type_info(R32& r, WBuf& w, int depth) {
  if (depth > 64) bad("type info nested too deeply");
  const uint32_t sl = r.u32();
  r.need(sl);
  R32 sr{r.p + r.i, sl};
  r.i += sl;
  const SNode s = read_schema(sr);
  put_datatype(s, w);
  w.u64(r.u64());  // len
  w.u64(r.u64());  // null_count
  const uint8_t vt = r.u8();
  if (vt == 2) bad("validity bitmap in the sample: stage it inline first");
  w.u8(vt ? 1 : 0);
  if (vt) {
    const uint64_t n = r.u64();
    r.need(n);
    w.bytes(r.p + r.i, n);
    r.i += n;
  }
  w.u64(r.u64());  // offset
  const uint32_t nb = r.u32();
  w.u64(nb);
  for (uint32_t k = 0; k < nb; ++k) {
    w.u64(r.u64());
    w.u64(r.u64());
  }
  const uint32_t nc = r.u32();
  w.u64(nc);
  for (uint32_t k = 0; k < nc; ++k) put_type_info(r, w, depth + 1);
}

void get_type_info(RBuf& r, std::vector<uint8_t>& o, int depth) {
  if (depth > 64) bad("type info nested too deeply");
  SNode s = get_datatype(r);
  // a node's own schema is written as plan.cpp writes a top-level one: no name, no metadata,
  // only the type's own flags
  s.flags &= kDictOrdered | kMapKeysSorted;
  std::vector<uint8_t> sch;
  write_schema(s, sch);
  put32(o, static_cast<uint32_t>(sch.size()));
  o.insert(o.end(), sch.begin(), sch.end());
  put64(o, r.u64());  // len
  put64(o, r.u64());  // null_count
  const uint8_t has_v = r.u8();
  if (has_v > 1) bad("Option tag");
  o.push_back(has_v);
  if (has_v) {
    const std::vector<uint8_t> v = r.bytes();
    put64(o, v.size());
    o.insert(o.end(), v.begin(), v.end());
  }
  put64(o, r.u64());  // offset
  const uint64_t nb = r.u64();
  if (nb > r.size()) bad("buffer count");
  put32(o, static_cast<uint32_t>(nb));
  for (uint64_t k = 0; k < nb; ++k) {
    put64(o, r.u64());
    put64(o, r.u64());
  }
  const uint64_t nc = r.u64();
  if (nc > r.size()) bad("child count");
  put32(o, static_cast<uint32_t>(nc));
  for (uint64_t k = 0; k < nc; ++k) get_type_info(r, o, depth + 1);
}

// ---- uhlc ----
void put_timestamp(WBuf& w, uint64_t ns, const std::array<uint8_t, 16>& id) {
  w.u64(ntp64_of_ns(ns));
  w.raw(id.data(), 16);  // ID(NonZeroU128): u128, little endian
}
uint64_t get_timestamp(RBuf& r) {
  const uint64_t t = r.u64();
  r.skip(16);
  return ns_of_ntp64(t);
}

void put_uuid(WBuf& w, const std::array<uint8_t, 16>& u) { w.bytes(u.data(), 16); }
std::array<uint8_t, 16> get_uuid(RBuf& r) {
  if (r.u64() != 16) bad("Uuid length");
  std::array<uint8_t, 16> u;
  r.raw(u.data(), 16);
  return u;
}

}  // namespace

uint64_t ntp64_of_ns(uint64_t ns) {
  const uint64_t s = ns / 1000000000ull, sub = ns % 1000000000ull;
  // fraction rounded up: floor(frac * 1e9 / 2^32) gives back `sub` exactly
  const uint64_t frac = ((sub << 32) + 999999999ull) / 1000000000ull;
  return (s << 32) + frac;
}

uint64_t ns_of_ntp64(uint64_t t) {
  const uint64_t s = t >> 32, frac = t & 0xFFFFFFFFull;
  return s * 1000000000ull + ((frac * 1000000000ull) >> 32);
}

std::array<uint8_t, 16> dataflow_uuid(const std::string& id) {
  std::array<uint8_t, 16> u{};
  auto hex = [](char c) -> int {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
  };
  if (id.size() == 36 && id[8] == '-' && id[13] == '-' && id[18] == '-' && id[23] == '-') {
    size_t k = 0;
    bool ok = true;
    for (size_t i = 0; i < id.size() && ok; ++i) {
      if (i == 8 || i == 13 || i == 18 || i == 23) continue;
      const int h = hex(id[i]), l = i + 1 < id.size() ? hex(id[i + 1]) : -1;
      ok = h >= 0 && l >= 0 && k < 16;
      if (ok) u[k++] = static_cast<uint8_t>(h << 4 | l);
      ++i;
    }
    if (ok && k == 16) return u;
  }
  // two FNV-1a-64 passes with different offsets, then the version-8 / RFC 4122 variant bits
  uint64_t h1 = 0xcbf29ce484222325ull, h2 = 0x84222325cbf29ce4ull;
  for (unsigned char c : id) {
    h1 = (h1 ^ c) * 0x100000001b3ull;
    h2 = (h2 ^ c) * 0x100000001b3ull;
  }
  std::memcpy(u.data(), &h1, 8);
  std::memcpy(u.data() + 8, &h2, 8);
  u[6] = static_cast<uint8_t>((u[6] & 0x0F) | 0x80);
  u[8] = static_cast<uint8_t>((u[8] & 0x3F) | 0x80);
  return u;
}

void bincode_type_info(const uint8_t* ti, size_t n, WBuf& w) {
  R32 r{ti, n};
  put_type_info(r, w, 0);
  if (r.i != n) bad("trailing bytes in type info");
}

std::vector<uint8_t> type_info_from_bincode(RBuf& r) {
  std::vector<uint8_t> o;
  get_type_info(r, o, 0);
  return o;
}

void bincode_parameters(const uint8_t* p, size_t n, WBuf& w) {
  if (n == 0) {
    w.u64(0);
    return;
  }
  RBuf r(p, n);
  const uint32_t k = r.u32();
  // BTreeMap order: keys sorted bytewise
  std::map<std::string, std::pair<uint8_t, std::vector<uint8_t>>> m;
  for (uint32_t i = 0; i < k; ++i) {
    std::string key = r.str();
    const uint8_t tag = r.u8();
    std::vector<uint8_t> v;
    if (tag == 0) {
      v.push_back(r.u8() ? 1 : 0);
    } else if (tag == 1) {
      const uint64_t x = r.u64();
      v.resize(8);
      std::memcpy(v.data(), &x, 8);
    } else if (tag == 2) {
      const std::string s = r.str();
      WBuf sw;
      sw.str(s);
      v.assign(sw.data(), sw.data() + sw.size());
    } else {
      bad("parameter tag");
    }
    m[std::move(key)] = {tag, std::move(v)};
  }
  if (r.pos() != r.size()) bad("trailing bytes in parameters");
  w.u64(m.size());
  for (const auto& kv : m) {
    w.str(kv.first);
    w.u32(kv.second.first);  // Parameter: Bool 0, Integer 1, String 2
    w.raw(kv.second.second.data(), kv.second.second.size());
  }
}

std::vector<uint8_t> parameters_from_bincode(RBuf& r) {
  const uint64_t n = r.u64();
  if (n == 0) return {};
  if (n > r.size()) bad("parameter count");
  WBuf w;
  w.u32(static_cast<uint32_t>(n));
  for (uint64_t i = 0; i < n; ++i) {
    w.str(r.str());
    const uint32_t tag = r.u32();
    w.u8(static_cast<uint8_t>(tag));
    if (tag == 0) {
      w.u8(r.u8() ? 1 : 0);
    } else if (tag == 1) {
      w.u64(r.u64());
    } else if (tag == 2) {
      w.str(r.str());
    } else {
      bad("Parameter variant " + std::to_string(tag));
    }
  }
  return w.take();
}

void encode_ide(const InterDaemonEvent& e, std::vector<uint8_t>& out) {
  WBuf w;
  const std::array<uint8_t, 16> df = dataflow_uuid(e.dataflow_id);
  if (e.kind == IDE_OUTPUT) {
    w.u32(0);
    put_uuid(w, df);
    w.str(e.node_id);
    w.str(e.output_id);
    w.u16(e.meta_version);
    put_timestamp(w, e.timestamp_ns, e.hlc_id);
    bincode_type_info(e.type_info.data(), e.type_info.size(), w);
    bincode_parameters(e.parameters.data(), e.parameters.size(), w);
    w.u8(e.has_data ? 1 : 0);
    if (e.has_data) w.bytes(e.data);
  } else if (e.kind == IDE_INPUTS_CLOSED) {
    w.u32(1);
    put_uuid(w, df);
    std::vector<std::pair<std::string, std::string>> in(e.inputs);  // BTreeSet order
    std::sort(in.begin(), in.end());
    in.erase(std::unique(in.begin(), in.end()), in.end());
    w.u64(in.size());
    for (const auto& p : in) {
      w.str(p.first);
      w.str(p.second);
    }
  } else {
    bad("event kind has no wire form");
  }
  put_timestamp(w, e.event_ns, e.hlc_id);
  out = w.take();
}

InterDaemonEvent decode_ide(const uint8_t* p, size_t n) {
  RBuf r(p, n);
  InterDaemonEvent e;
  const uint32_t v = r.u32();
  e.dataflow_uuid = get_uuid(r);
  if (v == 0) {
    e.kind = IDE_OUTPUT;
    e.node_id = r.str();
    e.output_id = r.str();
    e.meta_version = r.u16();
    e.timestamp_ns = get_timestamp(r);
    e.type_info = type_info_from_bincode(r);
    e.parameters = parameters_from_bincode(r);
    const uint8_t has = r.u8();
    if (has > 1) bad("Option tag");
    e.has_data = has != 0;
    if (e.has_data) e.data = r.bytes();
  } else if (v == 1) {
    e.kind = IDE_INPUTS_CLOSED;
    const uint64_t k = r.u64();
    if (k > r.size()) bad("input count");
    for (uint64_t i = 0; i < k; ++i) {
      std::string node = r.str();
      e.inputs.emplace_back(std::move(node), r.str());
    }
  } else {
    bad("InterDaemonEvent variant " + std::to_string(v));
  }
  e.event_ns = get_timestamp(r);
  if (r.pos() != r.size()) bad("trailing bytes in inter-daemon event");
  return e;
}

}  // namespace dora

// ---- test hooks (dora_gpu.h) ----
