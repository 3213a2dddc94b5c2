//! `DataMessage::DeviceIpc`: a sample that lives in an exported `hipMalloc` slot of its
//! producer, described by its IPC handle instead of a shared-memory id.  Mirrors
//! `dora_amd/csrc/wire.h` (`struct DeviceIpc`, `WBuf::data` / `RBuf::data`).
//!
//! In the dora tree the variant is added to `DataMessage` next to `Vec` and `SharedMemory`
//! (`libraries/message/src/common.rs:135-152`):
//!
//! ```ignore
//! pub enum DataMessage {
//!     Vec(AVec<u8, ConstAlign<128>>),
//!     SharedMemory { shared_memory_id: String, len: usize, drop_token: DropToken },
//!     /// device-resident sample (MI355X data plane): routed by handle, never copied by the daemon
//!     DeviceIpc(dora_node_api_gpu::device_ipc::DeviceIpc),
//! }
//! // and in DataMessage::drop_token:  DataMessage::DeviceIpc(d) => Some(d.drop_token),
//!
//! // DropToken (common.rs:175-184) keeps its Uuid private; the C side exchanges raw bytes:
//! impl DropToken {
//!     pub fn from_bytes(b: [u8; 16]) -> Self { Self(Uuid::from_bytes(b)) }
//!     pub fn as_bytes(&self) -> &[u8; 16] { self.0.as_bytes() }
//! }
//! ```
//!
//! The daemon treats it like `SharedMemory` minus the F8 copy: it forwards the descriptor to
//! every receiver and keeps the drop token pending until each has reported it
//! (`binaries/daemon/src/lib.rs:1314-1390`), and for a remote receiver it stages the bytes to
//! the host (`InterDaemonEvent::Output { data: Some(..) }`).
use dora_message::common::DropToken;
use eyre::{bail, eyre, Result};
use serde::{Deserialize, Serialize};

/// How the receiver learns that the producer's fill of the slot is complete.
#[derive(Debug, Clone, Copy, PartialEq, Eq, Serialize, Deserialize)]
pub enum Fill {
    /// The producer synchronised before sending.
    Done,
    /// Poll fill flag `index` of node `node` in the dataflow's control region until it is >= `epoch`
    /// (the pack kernel stores the epoch itself once every workgroup's stores are complete).
    Flag { node: u32, index: u32, epoch: u64 },
    /// Wait on the interprocess HIP event (fallback when no flag was free).
    Event { handle: [u8; 64] },
    /// The producer broadcasts the sample over the output's RCCL group; post the receive
    /// (`seq` = the group's sequence number).
    Bcast { seq: u64 },
}

#[derive(Debug, Clone, PartialEq, Eq, Serialize, Deserialize)]
pub struct DeviceIpc {
    /// `hipIpcMemHandle_t` of the slot allocation.
    #[serde(with = "serde_bytes_64")]
    pub handle: [u8; 64],
    /// GPU ordinal of the slot (a receiver on another GPU pulls the bytes over xGMI).
    pub device: i32,
    pub owner_pid: i32,
    /// Unique per owner process (receivers key their mapping cache on (pid, slot, handle)).
    pub slot_id: u64,
    /// Sample offset inside the slot allocation.
    pub offset: u64,
    pub len: u64,
    /// Bytes filled from `offset`: `len` plus the validity tail (>= len).
    pub ext_len: u64,
    pub drop_token: DropToken,
    pub fill: Fill,
}

mod serde_bytes_64 {
    use serde::{de::Error, Deserialize, Deserializer, Serializer};
    pub fn serialize<S: Serializer>(b: &[u8; 64], s: S) -> Result<S::Ok, S::Error> {
        s.serialize_bytes(b)
    }
    pub fn deserialize<'de, D: Deserializer<'de>>(d: D) -> Result<[u8; 64], D::Error> {
        let v: Vec<u8> = Deserialize::deserialize(d)?;
        v.try_into().map_err(|_| D::Error::custom("IPC handle must be 64 bytes"))
    }
}

const DATA_DEVICE_IPC: u8 = 2;

impl DeviceIpc {
    /// The C data plane's wire form (`WBuf::data` for kind DATA_DEVICE_IPC).
    pub fn encode(&self, o: &mut Vec<u8>) {
        o.push(DATA_DEVICE_IPC);
        o.extend_from_slice(&self.handle);
        o.extend_from_slice(&self.device.to_le_bytes());
        o.extend_from_slice(&self.owner_pid.to_le_bytes());
        for v in [self.slot_id, self.offset, self.len, self.ext_len] {
            o.extend_from_slice(&v.to_le_bytes());
        }
        o.extend_from_slice(self.drop_token.as_bytes());
        match self.fill {
            Fill::Done => o.push(0),
            Fill::Flag { node, index, epoch } => {
                o.push(1);
                o.extend_from_slice(&node.to_le_bytes());
                o.extend_from_slice(&index.to_le_bytes());
                o.extend_from_slice(&epoch.to_le_bytes());
            }
            Fill::Event { handle } => {
                o.push(2);
                o.extend_from_slice(&handle);
            }
            Fill::Bcast { seq } => {
                o.push(3);
                o.extend_from_slice(&seq.to_le_bytes());
            }
        }
    }

    /// Inverse of [`encode`](Self::encode); returns the descriptor and the bytes consumed.
    pub fn decode(b: &[u8]) -> Result<(Self, usize)> {
        let mut i = 0usize;
        let mut take = |n: usize| -> Result<&[u8]> {
            let s = b.get(i..i + n).ok_or_else(|| eyre!("DeviceIpc: truncated"))?;
            i += n;
            Ok(s)
        };
        if take(1)?[0] != DATA_DEVICE_IPC {
            bail!("not a DeviceIpc data message");
        }
        let handle: [u8; 64] = take(64)?.try_into().unwrap();
        let device = i32::from_le_bytes(take(4)?.try_into().unwrap());
        let owner_pid = i32::from_le_bytes(take(4)?.try_into().unwrap());
        let mut u = [0u64; 4];
        for x in &mut u {
            *x = u64::from_le_bytes(take(8)?.try_into().unwrap());
        }
        let [slot_id, offset, len, ext_len] = u;
        if ext_len < len {
            bail!("DeviceIpc: ext_len < len");
        }
        let drop_token = DropToken::from_bytes(take(16)?.try_into().unwrap());
        let fill = match take(1)?[0] {
            0 => Fill::Done,
            1 => Fill::Flag {
                node: u32::from_le_bytes(take(4)?.try_into().unwrap()),
                index: u32::from_le_bytes(take(4)?.try_into().unwrap()),
                epoch: u64::from_le_bytes(take(8)?.try_into().unwrap()),
            },
            2 => Fill::Event { handle: take(64)?.try_into().unwrap() },
            3 => Fill::Bcast { seq: u64::from_le_bytes(take(8)?.try_into().unwrap()) },
            k => bail!("DeviceIpc: unknown fill kind {k}"),
        };
        let d = DeviceIpc { handle, device, owner_pid, slot_id, offset, len, ext_len, drop_token, fill };
        Ok((d, i))
    }
}
