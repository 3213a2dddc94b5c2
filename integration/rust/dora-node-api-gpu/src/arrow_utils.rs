//! `required_data_size` / `copy_array_into_sample` with the reference signatures
//! (`apis/rust/node/src/node/arrow_utils.rs:4-71`) on top of the C ABI's plan, plus the device
//! forms a GPU node uses.
//!
//! The plan (`dora_gpu_plan`) is the reference's DFS: buffers in layout order at offsets
//! padded to the arrow-data `layout()` alignment, children after their parent, lengths from the
//! arrow-rs FFI import rules.  Its segment table is what `copy_array_into_sample_inner` copies;
//! its type info is the `ArrowTypeInfo` that function returns.
use std::os::raw::c_void;
use std::ptr;

use arrow::array::ArrayData;
use arrow::ffi::{FFI_ArrowArray, FFI_ArrowSchema};
use dora_gpu_sys as sys;
use dora_message::metadata::ArrowTypeInfo;
use eyre::{Context, Result};

use crate::{check, type_info};

/// A planned pack; keeps the exported C structs of the array alive while the plan borrows them.
pub struct Plan {
    raw: *mut sys::dora_plan,
    _array: Option<FFI_ArrowArray>,
    _schema: Option<FFI_ArrowSchema>,
}

impl Plan {
    /// Plan a host-resident `ArrayData` (its buffers in host memory).
    pub fn of_host(array: &ArrayData) -> Result<Self> {
        let a = FFI_ArrowArray::new(array);
        let s = FFI_ArrowSchema::try_from(array.data_type()).context("export schema")?;
        let mut raw = ptr::null_mut();
        check(unsafe {
            sys::dora_gpu_plan(
                &a as *const FFI_ArrowArray as *const sys::ArrowArray,
                &s as *const FFI_ArrowSchema as *const sys::ArrowSchema,
                sys::ARROW_DEVICE_CPU,
                &mut raw,
            )
        })?;
        Ok(Plan { raw, _array: Some(a), _schema: Some(s) })
    }

    /// Plan a device-resident array given through the Arrow C Device Data Interface (buffers
    /// in HBM, e.g. from `DeviceInput::device_array` or a producer kernel).
    ///
    /// # Safety
    /// `array` / `schema` must be valid and stay so (buffers included) until the pack that uses
    /// this plan has completed on its stream.
    pub unsafe fn of_device(array: *const sys::ArrowArray, schema: *const sys::ArrowSchema) -> Result<Self> {
        let mut raw = ptr::null_mut();
        check(sys::dora_gpu_plan(array, schema, sys::ARROW_DEVICE_ROCM, &mut raw))?;
        Ok(Plan { raw, _array: None, _schema: None })
    }

    /// `required_data_size` (arrow_utils.rs:4-8).
    pub fn size(&self) -> usize {
        unsafe { sys::dora_gpu_plan_size(self.raw) }
    }

    /// The serialized type info of the C ABI (what a send puts on the wire).
    pub fn type_info_bytes(&self) -> Result<Vec<u8>> {
        let mut n = 0usize;
        check(unsafe { sys::dora_gpu_plan_type_info(self.raw, ptr::null_mut(), 0, &mut n) })?;
        let mut b = vec![0u8; n];
        check(unsafe { sys::dora_gpu_plan_type_info(self.raw, b.as_mut_ptr(), n, &mut n) })?;
        Ok(b)
    }

    /// The `ArrowTypeInfo` `copy_array_into_sample` returns (validity inline).
    pub fn type_info(&self) -> Result<ArrowTypeInfo> {
        type_info::decode_inline(&self.type_info_bytes()?)
    }

    /// Pack into a device sample on `stream` (async): one HIP pack kernel for device arrays, DMA
    /// for host arrays.
    ///
    /// # Safety
    /// `dst` must be device memory of at least `dst_len` bytes.
    pub unsafe fn pack_device(&self, dst: *mut c_void, dst_len: usize, stream: sys::dora_stream_t) -> Result<()> {
        check(sys::dora_gpu_pack(self.raw, dst, dst_len, stream))
    }

    /// Copy into a host buffer from the segment table (the reference's host path, byte for
    /// byte; padding is left as it was).
    pub fn pack_host(&self, target: &mut [u8]) -> Result<()> {
        let n = unsafe { sys::dora_gpu_plan_num_segments(self.raw) };
        for i in 0..n {
            let (mut src, mut off, mut len) = (ptr::null(), 0u64, 0u64);
            check(unsafe { sys::dora_gpu_plan_segment(self.raw, i, &mut src, &mut off, &mut len) })?;
            let (off, len) = (off as usize, len as usize);
            assert!(
                target.len() >= off + len,
                "target buffer too small (total_len: {}, offset: {off}, required_len: {len})",
                target.len()
            );
            let src = unsafe { std::slice::from_raw_parts(src as *const u8, len) };
            target[off..off + len].copy_from_slice(src);
        }
        Ok(())
    }
}

impl Drop for Plan {
    fn drop(&mut self) {
        unsafe { sys::dora_gpu_plan_free(self.raw) }
    }
}

/// arrow_utils.rs:4-8, same signature.
pub fn required_data_size(array: &ArrayData) -> usize {
    Plan::of_host(array).expect("plan").size()
}

/// arrow_utils.rs:23-26, same signature: the host sample (a reference shared-memory sample or a
/// `DataSample` in host memory) filled from the plan's segment table.
pub fn copy_array_into_sample(target_buffer: &mut [u8], arrow_array: &ArrayData) -> ArrowTypeInfo {
    let plan = Plan::of_host(arrow_array).expect("plan");
    plan.pack_host(target_buffer).expect("pack");
    plan.type_info().expect("type info")
}

/// The device form: pack `arrow_array` (host or device resident) into a device sample `dst`
/// on `stream` with the GPU pack kernel and return its `ArrowTypeInfo`.  What
/// `DoraNode::send_output` does for a device node (`GpuNode::send_output` does all of it,
/// slot allocation and send included).
///
/// # Safety
/// `dst` must be device memory of at least `dst_len` bytes; for a device array the buffers
/// must stay valid until the pack completed on `stream`.
pub unsafe fn copy_array_into_device_sample(
    dst: *mut c_void,
    dst_len: usize,
    plan: &Plan,
    stream: sys::dora_stream_t,
) -> Result<ArrowTypeInfo> {
    plan.pack_device(dst, dst_len, stream)?;
    plan.type_info()
}
