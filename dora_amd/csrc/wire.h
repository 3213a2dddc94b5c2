// Wire types of the data plane (little-endian, length-prefixed) — the MI355X counterparts of
// libraries/message: DataMessage (common.rs:135-152) with a DeviceIpc variant, DropToken
// (common.rs:175-184), Metadata (metadata.rs:9-34), DaemonRequest / NodeEvent / NodeDropEvent
// (node_to_daemon.rs:9-69, daemon_to_node.rs:48-77).
#pragma once

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

namespace dora {

struct DropToken {
  uint8_t b[16];
  bool operator==(const DropToken& o) const { return std::memcmp(b, o.b, 16) == 0; }
  bool operator<(const DropToken& o) const { return std::memcmp(b, o.b, 16) < 0; }
};
struct DropTokenHash {
  size_t operator()(const DropToken& t) const {
    uint64_t a, c;
    std::memcpy(&a, t.b, 8);
    std::memcpy(&c, t.b + 8, 8);
    return static_cast<size_t>(a * 0x9E3779B97F4A7C15ull ^ c);
  }
};
DropToken generate_drop_token();  // UUIDv7 (common.rs:181-183)

// Request kinds (node -> daemon), event kinds (daemon -> node), drop kinds.
enum : uint32_t {
  REQ_SUBSCRIBE = 1,
  REQ_SEND_MESSAGE = 2,
  REQ_REPORT_DROP_TOKENS = 3,
  REQ_CLOSE_OUTPUTS = 4,
  REQ_OUTPUTS_DONE = 5,
  REQ_BCAST_GROUP = 6,  // {output, ncclUniqueId}: form an RCCL group of the output's receivers
  EV_READY = 101,
  EV_INPUT = 102,
  EV_INPUT_CLOSED = 103,
  EV_ALL_INPUTS_CLOSED = 104,
  EV_STOP = 105,
  EV_BCAST_JOIN = 106,  // {input, ncclUniqueId, nranks, rank}: join the producer's group
  DROP_OUTPUT_DROPPED = 201,
  DROP_BCAST_GROUP = 202,  // {output, nranks}: the daemon's answer to REQ_BCAST_GROUP (0: none)
};

enum : uint8_t { DATA_NONE = 0, DATA_VEC = 1, DATA_DEVICE_IPC = 2, DATA_SHMEM = 3 };

// DataMessage::SharedMemory {shared_memory_id, len, drop_token} (libraries/message/src/
// common.rs:135-152): a host-only node's sample >= 4096 B in a POSIX shared-memory region.
struct SharedMem {
  std::string name;  // shm_open name ("/dora-gpu-s-<pid>-<slot id>")
  uint64_t len = 0;
  DropToken token{};
};

// DataMessage::DeviceIpc — the sample lives in an exported hipMalloc slot of `owner_pid`.
struct DeviceIpc {
  uint8_t handle[64];  // hipIpcMemHandle_t of the slot allocation
  int32_t device;      // GPU ordinal of the slot
  int32_t owner_pid;
  uint64_t slot_id;    // unique per owner process
  uint64_t offset;     // sample offset inside the slot allocation
  uint64_t len;
  uint64_t ext_len;    // bytes filled from `offset`: len + the validity tail (>= len)
  DropToken token;
  // How the receiver learns that the fill is complete:
  //   FILL_DONE  the sender synchronised before sending;
  //   FILL_FLAG  poll region node `flag_node`'s FillFlag[flag_index] until >= epoch;
  //   FILL_EVENT wait on the interprocess event `event` (fallback when no flag is free);
  //   FILL_BCAST the producer broadcasts the sample over the output's RCCL group: the receiver
  //              posts the matching receive into local HBM (`epoch` = the group's sequence).
  uint8_t fill = 0;
  uint32_t flag_node = 0, flag_index = 0;
  uint64_t epoch = 0;
  uint8_t event[64];  // hipIpcEventHandle_t
};
enum : uint8_t { FILL_DONE = 0, FILL_FLAG = 1, FILL_EVENT = 2, FILL_BCAST = 3 };

struct DataMsg {
  uint8_t kind = DATA_NONE;
  std::vector<uint8_t> vec;  // DATA_VEC
  DeviceIpc ipc{};           // DATA_DEVICE_IPC
  SharedMem shm;             // DATA_SHMEM
  bool has_token() const { return kind == DATA_DEVICE_IPC || kind == DATA_SHMEM; }
  const DropToken& token() const { return kind == DATA_SHMEM ? shm.token : ipc.token; }
};

struct Metadata {
  uint16_t version = 0;
  uint64_t timestamp_ns = 0;
  std::vector<uint8_t> type_info;
  std::vector<uint8_t> parameters;  // BTreeMap<String, Parameter> encoding (node.cpp)
};

// Encoder.  Tracks its own length over storage that only grows: a send encodes ~25 fields, and
// std::vector bookkeeping per field cost ~190 ns per message against ~20 ns for plain copies.
class WBuf {
 public:
  void clear() { n_ = 0; }
  const uint8_t* data() const { return buf_.data(); }
  size_t size() const { return n_; }
  // The encoded bytes as a vector (the storage moves out; the buffer is empty afterwards).
  std::vector<uint8_t> take() {
    buf_.resize(n_);
    n_ = 0;
    return std::move(buf_);
  }
  void u8(uint8_t v) { raw(&v, 1); }
  void u16(uint16_t v) { raw(&v, 2); }
  void u32(uint32_t v) { raw(&v, 4); }
  void u64(uint64_t v) { raw(&v, 8); }
  void i32(int32_t v) { raw(&v, 4); }
  void raw(const void* p, size_t n) {
    if (buf_.size() - n_ < n) buf_.resize(std::max(2 * buf_.size(), n_ + n + 256));
    if (n) std::memcpy(buf_.data() + n_, p, n);
    n_ += n;
  }
  void bytes(const uint8_t* p, size_t n) {
    u64(n);
    raw(p, n);
  }
  void bytes(const std::vector<uint8_t>& v) { bytes(v.data(), v.size()); }
  void str(const std::string& s) { bytes(reinterpret_cast<const uint8_t*>(s.data()), s.size()); }
  void str(const char* s) { bytes(reinterpret_cast<const uint8_t*>(s), std::strlen(s)); }
  void token(const DropToken& t) { raw(t.b, 16); }
  void data(const DataMsg& d) {
    u8(d.kind);
    if (d.kind == DATA_VEC) bytes(d.vec);
    if (d.kind == DATA_DEVICE_IPC) {
      raw(d.ipc.handle, 64);
      i32(d.ipc.device);
      i32(d.ipc.owner_pid);
      u64(d.ipc.slot_id);
      u64(d.ipc.offset);
      u64(d.ipc.len);
      u64(d.ipc.ext_len);
      token(d.ipc.token);
      u8(d.ipc.fill);
      if (d.ipc.fill == FILL_FLAG) {
        u32(d.ipc.flag_node);
        u32(d.ipc.flag_index);
        u64(d.ipc.epoch);
      }
      if (d.ipc.fill == FILL_EVENT) raw(d.ipc.event, 64);
      if (d.ipc.fill == FILL_BCAST) u64(d.ipc.epoch);
    }
    if (d.kind == DATA_SHMEM) {
      str(d.shm.name);
      u64(d.shm.len);
      token(d.shm.token);
    }
  }
  void metadata(const Metadata& m) {
    u16(m.version);
    u64(m.timestamp_ns);
    bytes(m.type_info);
    bytes(m.parameters);
  }

 private:
  std::vector<uint8_t> buf_;
  size_t n_ = 0;
};

class RBuf {
 public:
  RBuf(const uint8_t* p, size_t n) : p_(p), n_(n) {}
  explicit RBuf(const std::vector<uint8_t>& v) : p_(v.data()), n_(v.size()) {}
  void need(size_t k) {
    if (i_ + k > n_) throw std::invalid_argument("truncated message");
  }
  void raw(void* out, size_t k) {
    need(k);
    std::memcpy(out, p_ + i_, k);
    i_ += k;
  }
  uint8_t u8() {
    uint8_t v;
    raw(&v, 1);
    return v;
  }
  uint16_t u16() {
    uint16_t v;
    raw(&v, 2);
    return v;
  }
  uint32_t u32() {
    uint32_t v;
    raw(&v, 4);
    return v;
  }
  uint64_t u64() {
    uint64_t v;
    raw(&v, 8);
    return v;
  }
  int32_t i32() {
    int32_t v;
    raw(&v, 4);
    return v;
  }
  std::vector<uint8_t> bytes() {
    const uint64_t k = u64();
    need(k);
    std::vector<uint8_t> v(p_ + i_, p_ + i_ + k);
    i_ += k;
    return v;
  }
  std::string str() {
    const uint64_t k = u64();
    need(k);
    std::string s(reinterpret_cast<const char*>(p_ + i_), k);
    i_ += k;
    return s;
  }
  DropToken token() {
    DropToken t;
    raw(t.b, 16);
    return t;
  }
  DataMsg data() {
    DataMsg d;
    d.kind = u8();
    if (d.kind == DATA_VEC) d.vec = bytes();
    if (d.kind == DATA_DEVICE_IPC) {
      raw(d.ipc.handle, 64);
      d.ipc.device = i32();
      d.ipc.owner_pid = i32();
      d.ipc.slot_id = u64();
      d.ipc.offset = u64();
      d.ipc.len = u64();
      d.ipc.ext_len = u64();
      if (d.ipc.ext_len < d.ipc.len) throw std::invalid_argument("sample ext_len < len");
      d.ipc.token = token();
      d.ipc.fill = u8();
      if (d.ipc.fill == FILL_FLAG) {
        d.ipc.flag_node = u32();
        d.ipc.flag_index = u32();
        d.ipc.epoch = u64();
      }
      if (d.ipc.fill == FILL_EVENT) raw(d.ipc.event, 64);
      if (d.ipc.fill == FILL_BCAST) d.ipc.epoch = u64();
      if (d.ipc.fill > FILL_BCAST) throw std::invalid_argument("unknown fill kind");
    }
    if (d.kind == DATA_SHMEM) {
      d.shm.name = str();
      d.shm.len = u64();
      d.shm.token = token();
    }
    if (d.kind > DATA_SHMEM) throw std::invalid_argument("unknown DataMessage kind");
    return d;
  }
  Metadata metadata() {
    Metadata m;
    m.version = u16();
    m.timestamp_ns = u64();
    m.type_info = bytes();
    m.parameters = bytes();
    return m;
  }
  size_t pos() const { return i_; }
  size_t size() const { return n_; }
  const uint8_t* ptr() const { return p_ + i_; }
  void skip(size_t k) {
    need(k);
    i_ += k;
  }

 private:
  const uint8_t* p_;
  size_t n_;
  size_t i_ = 0;
};

}  // namespace dora
