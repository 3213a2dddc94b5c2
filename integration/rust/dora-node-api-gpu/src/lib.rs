//! dora's Rust node API on the MI355X device data plane.
//!
//! * [`type_info`]: the C ABI's serialized ArrowTypeInfo <-> `dora_message::metadata::ArrowTypeInfo`
//!   (schema tree <-> `arrow_schema::DataType`, validity tags 0 / 1 / 2).
//! * [`device_ipc`]: the `DataMessage::DeviceIpc` variant (wire form of `dora_amd/csrc/wire.h`).
//! * [`arrow_utils`]: `required_data_size` / `copy_array_into_sample` with the reference
//!   signatures (`apis/rust/node/src/node/arrow_utils.rs:4-71`), packing on the GPU.
//! * [`node`]: `GpuNode`, the `DoraNode` + `EventStream` surface over `dora_node_*`.
pub mod arrow_utils;
pub mod device_ipc;
pub mod node;
pub mod type_info;

use std::os::raw::c_int;

/// `Ok(())` for DORA_OK, else the library's thread-local error message.
pub(crate) fn check(rc: c_int) -> eyre::Result<()> {
    if rc == dora_gpu_sys::DORA_OK {
        Ok(())
    } else {
        Err(eyre::eyre!("dora-gpu error {rc}: {}", dora_gpu_sys::last_error()))
    }
}
