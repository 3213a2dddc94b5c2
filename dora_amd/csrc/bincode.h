// The reference's inter-daemon wire format: `bincode::serialize(&Timestamped<InterDaemonEvent>)`
// (binaries/daemon/src/inter_daemon.rs:66) in a u64 little-endian length frame
// (binaries/daemon/src/socket_stream_utils.rs:3-12).
//
// bincode 1.3.3 (Cargo.lock), whose `serialize` uses fixed-width little-endian integers, u64
// lengths for strings, byte strings, sequences and maps, u32 enum variant indices, one byte for
// bool and for an Option's tag, u128 as 16 bytes, structs and tuples as their fields in order,
// newtype structs as their content.  The serde layouts of the types inside, in declaration order:
//   Timestamped<T> { inner: T, timestamp: uhlc::Timestamp }           libraries/message/src/common.rs:128-131
//   InterDaemonEvent { Output { dataflow_id: Uuid, node_id: NodeId, output_id: DataId,
//                      metadata: Metadata, data: Option<AVec<u8>> } = 0,
//                      InputsClosed { dataflow_id: Uuid, inputs: BTreeSet<(NodeId, DataId)> } = 1 }
//                                                                    libraries/message/src/daemon_to_daemon.rs:9-21
//   Metadata { metadata_version: u16, timestamp: uhlc::Timestamp, type_info: ArrowTypeInfo,
//              parameters: BTreeMap<String, Parameter> }             libraries/message/src/metadata.rs:9-15
//   ArrowTypeInfo { data_type: DataType, len, null_count: usize, validity: Option<Vec<u8>>,
//                   offset: usize, buffer_offsets: Vec<BufferOffset>, child_data: Vec<Self> }
//                                                                    metadata.rs:51-59, 140-143
//   Parameter { Bool(bool) = 0, Integer(i64) = 1, String(String) = 2 } metadata.rs:133-137
//   NodeId(String), DataId(String)                                   libraries/core/src/config.rs:16,78
// and of third-party types absent from /root/reference (restated from their published sources;
// no fixture in the reference holds their bytes, so these are parity-unpinned):
//   uuid 1.11.0   Uuid: non-human-readable serializers get `serialize_bytes` of the 16 bytes;
//   uhlc 0.5.2    Timestamp { time: NTP64(u64), id: ID(NonZeroU128) }; NTP64 = seconds since
//                 the UNIX epoch in the high 32 bits, the fraction of a second in the low 32;
//   aligned-vec 0.5.0  AVec<u8> serializes as a sequence of its bytes (= Vec<u8>);
//   arrow-schema 53.2.0  DataType, variants in declaration order (bincode_datatype below), its
//                 Field { name, data_type, nullable, dict_id: i64, dict_is_ordered, metadata:
//                 HashMap<String, String> }, Fields / FieldRef as sequences / the field itself.
#pragma once

#include <array>
#include <cstdint>
#include <string>
#include <vector>

#include "interdaemon.h"
#include "wire.h"

namespace dora {

// Timestamped<InterDaemonEvent> <-> the daemon's event (throws std::invalid_argument on input
// it cannot represent: a validity bitmap left in the sample, an Arrow type outside the data
// plane's parity set, a malformed or truncated frame).
void encode_ide(const InterDaemonEvent& e, std::vector<uint8_t>& out);
InterDaemonEvent decode_ide(const uint8_t* p, size_t n);

// The pieces, for tests (runtime.cpp test hooks):
// this library's serialized ArrowTypeInfo (plan.cpp serialize_type_info, validity inline) as
// bincode of the reference's ArrowTypeInfo, and back
void bincode_type_info(const uint8_t* ti, size_t n, WBuf& w);
std::vector<uint8_t> type_info_from_bincode(RBuf& r);
// MetadataParameters: this library's encoding (u32 count, per entry u64-length key, u8 tag,
// value) <-> bincode of BTreeMap<String, Parameter>
void bincode_parameters(const uint8_t* p, size_t n, WBuf& w);
std::vector<uint8_t> parameters_from_bincode(RBuf& r);
// NTP64 of a UNIX-epoch nanosecond time, and back (exact for every ns value)
uint64_t ntp64_of_ns(uint64_t ns);
uint64_t ns_of_ntp64(uint64_t t);
// The dataflow id as the reference's Uuid: a UUID's text parsed, any other name hashed into a
// version-8 UUID (every daemon of a dataflow derives the same one)
std::array<uint8_t, 16> dataflow_uuid(const std::string& id);

}  // namespace dora
