//! Raw bindings of `include/dora_gpu.h`, the C ABI of the MI355X device-resident message data
//! plane (hipcc-built `libdora_gpu`, see build.rs).  The declarations live in `ffi.rs`,
//! generated from the header (`integration/rust/gen_ffi.py`); this file holds the types they
//! name.  Safe wrappers are in the `dora-node-api-gpu` crate.
#![allow(non_camel_case_types)]

use std::os::raw::{c_char, c_void};

mod ffi;
pub use ffi::*;

/// Arrow C Data Interface (public Arrow ABI, spec v1).  Layout-identical to
/// `arrow::ffi::FFI_ArrowArray` / `FFI_ArrowSchema`, so pointers to those cast to these.
#[repr(C)]
pub struct ArrowSchema {
    pub format: *const c_char,
    pub name: *const c_char,
    pub metadata: *const c_char,
    pub flags: i64,
    pub n_children: i64,
    pub children: *mut *mut ArrowSchema,
    pub dictionary: *mut ArrowSchema,
    pub release: Option<unsafe extern "C" fn(*mut ArrowSchema)>,
    pub private_data: *mut c_void,
}

#[repr(C)]
pub struct ArrowArray {
    pub length: i64,
    pub null_count: i64,
    pub offset: i64,
    pub n_buffers: i64,
    pub n_children: i64,
    pub buffers: *mut *const c_void,
    pub children: *mut *mut ArrowArray,
    pub dictionary: *mut ArrowArray,
    pub release: Option<unsafe extern "C" fn(*mut ArrowArray)>,
    pub private_data: *mut c_void,
}

pub type ArrowDeviceType = i32;
pub const ARROW_DEVICE_CPU: ArrowDeviceType = 1;
pub const ARROW_DEVICE_ROCM: ArrowDeviceType = 10;
pub const ARROW_DEVICE_ROCM_HOST: ArrowDeviceType = 11;

pub const DORA_OK: i32 = 0;
pub const DORA_ERR_INVALID: i32 = -1;
pub const DORA_ERR_HIP: i32 = -2;
pub const DORA_ERR_TOO_SMALL: i32 = -3;
pub const DORA_ERR_UNSUPPORTED: i32 = -4;
pub const DORA_ERR_CLOSED: i32 = -5;
pub const DORA_ERR_TIMEOUT: i32 = -6;
pub const DORA_ERR_NOT_FOUND: i32 = -7;

/// Flags of dora_node_send_output_ex / _bytes_ex.
pub const DORA_SEND_ASYNC: u32 = 1;

pub const DORA_EVENT_STOP: i32 = 0;
pub const DORA_EVENT_INPUT: i32 = 1;
pub const DORA_EVENT_INPUT_CLOSED: i32 = 2;
pub const DORA_EVENT_ERROR: i32 = 3;
pub const DORA_EVENT_ALL_INPUTS_CLOSED: i32 = 4;

/// A `hipStream_t` / `hipEvent_t`; null = the device's null stream.
pub type dora_stream_t = *mut c_void;
pub type dora_event_t = *mut c_void;

/// Opaque handles of the library.
#[repr(C)]
pub struct dora_plan {
    _p: [u8; 0],
}
#[repr(C)]
pub struct dora_node {
    _p: [u8; 0],
}
#[repr(C)]
pub struct dora_sample {
    _p: [u8; 0],
}
#[repr(C)]
pub struct dora_event {
    _p: [u8; 0],
}
#[repr(C)]
pub struct dora_daemon {
    _p: [u8; 0],
}

/// `dora_gpu_last_error()` as an owned string.
pub fn last_error() -> String {
    unsafe {
        let p = dora_gpu_last_error();
        if p.is_null() {
            return String::new();
        }
        std::ffi::CStr::from_ptr(p).to_string_lossy().into_owned()
    }
}
