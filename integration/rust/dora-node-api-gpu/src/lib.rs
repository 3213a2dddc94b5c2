//! dora's Rust node API on the MI355X device data plane.
//!
//! * [`type_info`]: the C ABI's serialized ArrowTypeInfo <-> `dora_message::metadata::ArrowTypeInfo`
//!   (schema tree <-> `arrow_schema::DataType`, validity tags 0 / 1 / 2).
//! * [`device_ipc`]: the `DataMessage::DeviceIpc` variant (wire form of `dora_amd/csrc/wire.h`).
//! * [`arrow_utils`]: `required_data_size` / `copy_array_into_sample` with the reference
//!   signatures (`apis/rust/node/src/node/arrow_utils.rs:4-71`), packing on the GPU.
//! * [`node`]: `GpuNode`, the device-first node over `dora_node_*` (device samples and
//!   zero-copy device inputs).
//! * [`api`]: the reference's `DoraNode` / `EventStream` / `Event` surface (drop-in: an
//!   existing node changes only its `use` line), re-exported at the crate root with the
//!   reference's re-exports (`dora_node_api::{arrow, dora_core, Metadata, ...}`).
pub mod api;
pub mod arrow_utils;
pub mod device_ipc;
pub mod node;
pub mod type_info;

pub use api::{DataSample, DoraNode, Event, EventStream};
pub use arrow;
pub use dora_arrow_convert::*;
pub use dora_core::{self, uhlc};
pub use dora_message::{
    metadata::{Metadata, MetadataParameters, Parameter},
    DataflowId,
};
pub use node::{DeviceInput, GpuEvent, GpuNode};

use std::os::raw::c_int;

/// `Ok(())` for DORA_OK, else the library's thread-local error message.
pub(crate) fn check(rc: c_int) -> eyre::Result<()> {
    if rc == dora_gpu_sys::DORA_OK {
        Ok(())
    } else {
        Err(eyre::eyre!("dora-gpu error {rc}: {}", dora_gpu_sys::last_error()))
    }
}
