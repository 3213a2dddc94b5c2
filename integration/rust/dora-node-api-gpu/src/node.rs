//! `GpuNode`: `DoraNode` + `EventStream` (apis/rust/node/src/node/mod.rs:42-503,
//! event_stream/mod.rs) over the C node API (`dora_node_*`, `dora_event_*`).
//!
//! The device-first surface: samples live in HBM (`DataSample::as_mut_ptr` is a device
//! pointer; there is no `Deref<[u8]>` for them), and an input's data is a device array
//! (`DeviceInput::device_array`) — arrow-rs cannot import device buffers as `ArrayData`
//! (it reads offsets while importing), so `DeviceInput::to_host` stages a host copy when a
//! CPU consumer needs one.  The reference's own surface (`DoraNode`, `EventStream`, `Event`)
//! is in `api.rs`, built on this.
use std::ffi::{CStr, CString};
use std::os::raw::c_void;
use std::ptr;
use std::sync::{Arc, Mutex, MutexGuard};
use std::time::Duration;

use arrow::array::{Array, ArrayData};
use arrow::ffi::{from_ffi, FFI_ArrowArray, FFI_ArrowSchema};
use dora_gpu_sys as sys;
use dora_message::metadata::{ArrowTypeInfo, MetadataParameters, Parameter};
use eyre::{bail, Result};

use crate::{check, type_info};

/// MetadataParameters in the C ABI's encoding: u32 n, then per entry u64 klen, key, u8 tag
/// (0 bool, 1 int, 2 string), value (u8 | i64 | u64 len + bytes); BTreeMap order.
pub fn encode_parameters(p: &MetadataParameters) -> Vec<u8> {
    let mut o = (p.len() as u32).to_le_bytes().to_vec();
    for (k, v) in p {
        o.extend_from_slice(&(k.len() as u64).to_le_bytes());
        o.extend_from_slice(k.as_bytes());
        match v {
            Parameter::Bool(b) => o.extend_from_slice(&[0, u8::from(*b)]),
            Parameter::Integer(i) => {
                o.push(1);
                o.extend_from_slice(&i.to_le_bytes());
            }
            Parameter::String(s) => {
                o.push(2);
                o.extend_from_slice(&(s.len() as u64).to_le_bytes());
                o.extend_from_slice(s.as_bytes());
            }
        }
    }
    o
}

pub fn decode_parameters(b: &[u8]) -> Result<MetadataParameters> {
    let mut out = MetadataParameters::new();
    if b.len() < 4 {
        return Ok(out);
    }
    let mut i = 4usize;
    let n = u32::from_le_bytes(b[..4].try_into().unwrap());
    let mut take = |k: usize| -> Result<&[u8]> {
        let s = b.get(i..i + k).ok_or_else(|| eyre::eyre!("parameters: truncated"))?;
        i += k;
        Ok(s)
    };
    for _ in 0..n {
        let kl = u64::from_le_bytes(take(8)?.try_into().unwrap()) as usize;
        let key = String::from_utf8(take(kl)?.to_vec())?;
        let v = match take(1)?[0] {
            0 => Parameter::Bool(take(1)?[0] != 0),
            1 => Parameter::Integer(i64::from_le_bytes(take(8)?.try_into().unwrap())),
            2 => {
                let sl = u64::from_le_bytes(take(8)?.try_into().unwrap()) as usize;
                Parameter::String(String::from_utf8(take(sl)?.to_vec())?)
            }
            t => bail!("parameters: tag {t}"),
        };
        out.insert(key, v);
    }
    Ok(out)
}

/// The C node handle, shared by the `GpuNode` (or `DoraNode` + `EventStream`) and every sample
/// and input that calls back into it: freed (`dora_node_free`, the reference's Drop for
/// DoraNode) when the last of them goes, so no sample or input can outlive its node.  The
/// mutex serialises calls into the node from different threads.
pub(crate) struct NodeRef {
    pub(crate) raw: *mut sys::dora_node,
}

unsafe impl Send for NodeRef {}

impl Drop for NodeRef {
    /// Drop for DoraNode (mod.rs:384-431): close outputs, wait <= 10 s for drop tokens.
    fn drop(&mut self) {
        unsafe { sys::dora_node_free(self.raw) }
    }
}

pub(crate) type SharedNode = Arc<Mutex<NodeRef>>;

pub(crate) fn lock(n: &SharedNode) -> MutexGuard<'_, NodeRef> {
    n.lock().unwrap_or_else(|e| e.into_inner())
}

pub struct GpuNode {
    node: SharedNode,
}

/// A device sample (`DataSample`, mod.rs:434-503): an HBM slot from the node's recycled cache.
/// It keeps its node alive: dropping it unsent returns the slot to that node's cache.
pub struct DataSample {
    raw: *mut sys::dora_sample,
    node: SharedNode,
}

unsafe impl Send for DataSample {}

impl DataSample {
    /// Device pointer of the slot: fill it with kernels on `GpuNode::stream()` (or any stream,
    /// synchronised before `send_output_sample`).
    pub fn as_mut_ptr(&mut self) -> *mut u8 {
        unsafe { sys::dora_sample_data(self.raw) as *mut u8 }
    }
    pub fn len(&self) -> usize {
        unsafe { sys::dora_sample_len(self.raw) }
    }
    pub fn is_empty(&self) -> bool {
        self.len() == 0
    }
    /// Hand the raw sample to a send (which consumes it).
    pub(crate) fn take(mut self) -> *mut sys::dora_sample {
        std::mem::replace(&mut self.raw, ptr::null_mut())
    }
}

impl Drop for DataSample {
    fn drop(&mut self) {
        if !self.raw.is_null() {
            let g = lock(&self.node);
            unsafe { sys::dora_sample_discard(g.raw, self.raw) }
        }
    }
}

/// An event of `GpuNode::recv` / `EventStream::recv_device`: inputs stay device-resident.
pub enum GpuEvent {
    Input { id: String, metadata: InputMetadata, data: DeviceInput },
    InputClosed { id: String },
    Stop,
    Error(String),
}

pub struct InputMetadata {
    pub timestamp_ns: u64,
    pub parameters: MetadataParameters,
}

/// One received input; its drop token goes back when this (and every array imported from it)
/// is dropped.  It keeps its node alive.
pub struct DeviceInput {
    ev: *mut sys::dora_event,
    node: SharedNode,
}

unsafe impl Send for DeviceInput {}

impl DeviceInput {
    /// The reference `ArrowTypeInfo` (validity inline, restored from the sample's tail).
    pub fn type_info(&self) -> Result<ArrowTypeInfo> {
        let _g = lock(&self.node);
        let (mut p, mut n) = (ptr::null(), 0usize);
        check(unsafe { sys::dora_event_type_info(self.ev, &mut p, &mut n) })?;
        type_info::decode_inline(unsafe { std::slice::from_raw_parts(p, n) })
    }
    /// Raw sample: device pointer (or host pointer of an inline Vec sample) and length.
    pub fn raw(&self) -> Result<(*const c_void, usize)> {
        let _g = lock(&self.node);
        let (mut p, mut n) = (ptr::null(), 0usize);
        check(unsafe { sys::dora_event_data(self.ev, &mut p, &mut n) })?;
        Ok((p, n))
    }
    pub fn is_device(&self) -> bool {
        unsafe { sys::dora_event_is_device(self.ev) != 0 }
    }
    /// `RawData::into_arrow_array` (event.rs:35-91) as a zero-copy device array over the
    /// sample (C Device Data Interface structs; release them to let the token go).
    pub fn device_array(&self) -> Result<(FFI_ArrowArray, FFI_ArrowSchema)> {
        let _g = lock(&self.node);
        let mut a = FFI_ArrowArray::empty();
        let mut s = FFI_ArrowSchema::empty();
        check(unsafe {
            sys::dora_event_array(
                self.ev,
                &mut a as *mut FFI_ArrowArray as *mut sys::ArrowArray,
                &mut s as *mut FFI_ArrowSchema as *mut sys::ArrowSchema,
            )
        })?;
        Ok((a, s))
    }
    /// A host `ArrayData` copy of the input (device -> host staging for CPU consumers).
    pub fn to_host(&self) -> Result<ArrayData> {
        let (a, s) = self.device_array()?;
        if !self.is_device() {
            return Ok(unsafe { from_ffi(a, &s)? });
        }
        let mut host = FFI_ArrowArray::empty();
        check(unsafe {
            sys::dora_gpu_array_download(
                &a as *const FFI_ArrowArray as *const sys::ArrowArray,
                &s as *const FFI_ArrowSchema as *const sys::ArrowSchema,
                &mut host as *mut FFI_ArrowArray as *mut sys::ArrowArray,
            )
        })?;
        Ok(unsafe { from_ffi(host, &s)? })
    }
}

impl Drop for DeviceInput {
    fn drop(&mut self) {
        let _g = lock(&self.node);
        unsafe { sys::dora_event_free(self.ev) }
    }
}

fn cstr(s: &str) -> Result<CString> {
    Ok(CString::new(s)?)
}

/// `dora_node_next_event` once (timeout in us, -1: wait) -> the next event, Ok(None) at the end
/// of the stream, Err on a timeout.
pub(crate) fn next_event(node: &SharedNode, timeout_us: i64) -> Result<Option<GpuEvent>, i32> {
    let mut ev = ptr::null_mut();
    let g = lock(node);
    let rc = unsafe { sys::dora_node_next_event(g.raw, timeout_us, &mut ev) };
    drop(g);
    if rc == sys::DORA_ERR_TIMEOUT {
        return Err(rc);
    }
    if rc != sys::DORA_OK {
        return Ok(None);
    }
    let kind = unsafe { sys::dora_event_type(ev) };
    let id = unsafe { CStr::from_ptr(sys::dora_event_id(ev)) }.to_string_lossy().into_owned();
    match kind {
        sys::DORA_EVENT_INPUT => {
            let (mut p, mut n) = (ptr::null(), 0usize);
            let params = if unsafe { sys::dora_event_parameters(ev, &mut p, &mut n) } == sys::DORA_OK {
                decode_parameters(unsafe { std::slice::from_raw_parts(p, n) }).unwrap_or_default()
            } else {
                MetadataParameters::new()
            };
            let timestamp_ns = unsafe { sys::dora_event_timestamp_ns(ev) };
            Ok(Some(GpuEvent::Input {
                id,
                metadata: InputMetadata { timestamp_ns, parameters: params },
                data: DeviceInput { ev, node: node.clone() },
            }))
        }
        other => {
            let out = match other {
                sys::DORA_EVENT_INPUT_CLOSED => Some(GpuEvent::InputClosed { id }),
                sys::DORA_EVENT_STOP => Some(GpuEvent::Stop),
                sys::DORA_EVENT_ERROR => Some(GpuEvent::Error(
                    unsafe { CStr::from_ptr(sys::dora_event_error(ev)) }.to_string_lossy().into_owned(),
                )),
                _ => None, // ALL_INPUTS_CLOSED: the stream ends
            };
            let _g = lock(node);
            unsafe { sys::dora_event_free(ev) };
            Ok(out)
        }
    }
}

impl GpuNode {
    pub(crate) fn from_raw(raw: *mut sys::dora_node) -> Self {
        GpuNode { node: Arc::new(Mutex::new(NodeRef { raw })) }
    }

    pub(crate) fn shared(&self) -> SharedNode {
        self.node.clone()
    }

    /// DoraNode::init_from_env (mod.rs:65-76): DORA_GPU_DATAFLOW, DORA_NODE_ID, DORA_GPU_DEVICE.
    pub fn init_from_env() -> Result<Self> {
        let mut raw = ptr::null_mut();
        check(unsafe { sys::dora_node_init_from_env(&mut raw) })?;
        Ok(Self::from_raw(raw))
    }

    /// A node of the dataflow whose control region is `dataflow` (DORA_GPU_DATAFLOW) on HIP
    /// device `device`: a dynamic node (`path: dynamic`) started by hand.
    pub fn init(dataflow: &str, node_id: &str, device: i32) -> Result<Self> {
        let mut raw = ptr::null_mut();
        check(unsafe {
            sys::dora_node_init(cstr(dataflow)?.as_ptr(), cstr(node_id)?.as_ptr(), device, &mut raw)
        })?;
        Ok(Self::from_raw(raw))
    }

    /// The node's HIP stream: consumers run their kernels on it, so a token returns only after
    /// they have read the sample.
    pub fn stream(&self) -> sys::dora_stream_t {
        let g = lock(&self.node);
        unsafe { sys::dora_node_stream(g.raw) }
    }

    /// send_output (mod.rs:198-215) of a host-resident array: planned on the host, DMA'd into a
    /// device sample (the array may be reused when the call returns).
    pub fn send_output(&mut self, output_id: &str, parameters: MetadataParameters, data: impl Array) -> Result<()> {
        let d = data.to_data();
        let a = FFI_ArrowArray::new(&d);
        let s = FFI_ArrowSchema::try_from(d.data_type())?;
        let p = encode_parameters(&parameters);
        let g = lock(&self.node);
        check(unsafe {
            sys::dora_node_send_output(
                g.raw,
                cstr(output_id)?.as_ptr(),
                &a as *const FFI_ArrowArray as *const sys::ArrowArray,
                &s as *const FFI_ArrowSchema as *const sys::ArrowSchema,
                sys::ARROW_DEVICE_CPU,
                p.as_ptr(),
                p.len(),
            )
        })
    }

    /// send_output of a device-resident array: host plan + one pack kernel.  Returns once the
    /// pack has read the array (the reference copies inside send_output), so the buffers may be
    /// rewritten on any stream afterwards.
    ///
    /// # Safety
    /// `array` / `schema` must point to a valid Arrow C Device array with ROCm buffers.
    pub unsafe fn send_output_device(
        &mut self,
        output_id: &str,
        parameters: MetadataParameters,
        array: *const sys::ArrowArray,
        schema: *const sys::ArrowSchema,
    ) -> Result<()> {
        self.send_output_device_flags(output_id, parameters, array, schema, 0)
    }

    /// As `send_output_device`, returning as soon as the pack is queued (DORA_SEND_ASYNC).
    ///
    /// # Safety
    /// As `send_output_device`; in addition the array's buffers must not be written until
    /// `sync()` or only by work queued on `stream()` fetched after this call.
    pub unsafe fn send_output_device_async(
        &mut self,
        output_id: &str,
        parameters: MetadataParameters,
        array: *const sys::ArrowArray,
        schema: *const sys::ArrowSchema,
    ) -> Result<()> {
        self.send_output_device_flags(output_id, parameters, array, schema, sys::DORA_SEND_ASYNC)
    }

    unsafe fn send_output_device_flags(
        &mut self,
        output_id: &str,
        parameters: MetadataParameters,
        array: *const sys::ArrowArray,
        schema: *const sys::ArrowSchema,
        flags: u32,
    ) -> Result<()> {
        let p = encode_parameters(&parameters);
        let g = lock(&self.node);
        check(sys::dora_node_send_output_ex(
            g.raw,
            cstr(output_id)?.as_ptr(),
            array,
            schema,
            sys::ARROW_DEVICE_ROCM,
            p.as_ptr(),
            p.len(),
            flags,
        ))
    }

    /// Wait until every fill of this node has completed (dora_node_sync).
    pub fn sync(&mut self) -> Result<()> {
        let g = lock(&self.node);
        check(unsafe { sys::dora_node_sync(g.raw) })
    }

    /// send_output_raw (mod.rs:180-196): `data` fills a host staging buffer of `data_len`
    /// bytes, which is DMA'd into a device sample (ArrowTypeInfo::byte_array).
    pub fn send_output_raw<F: FnOnce(&mut [u8])>(
        &mut self,
        output_id: &str,
        parameters: MetadataParameters,
        data_len: usize,
        data: F,
    ) -> Result<()> {
        let mut buf = vec![0u8; data_len];
        data(&mut buf);
        self.send_output_bytes(output_id, parameters, &buf)
    }

    /// send_output_bytes (mod.rs:217-228) of host bytes.
    pub fn send_output_bytes(&mut self, output_id: &str, parameters: MetadataParameters, data: &[u8]) -> Result<()> {
        let p = encode_parameters(&parameters);
        let g = lock(&self.node);
        check(unsafe {
            sys::dora_node_send_output_bytes(
                g.raw,
                cstr(output_id)?.as_ptr(),
                data.as_ptr() as *const c_void,
                data.len(),
                sys::ARROW_DEVICE_CPU,
                p.as_ptr(),
                p.len(),
            )
        })
    }

    /// allocate_data_sample (mod.rs:303-346): a device slot.
    pub fn allocate_data_sample(&mut self, data_len: usize) -> Result<DataSample> {
        let mut raw = ptr::null_mut();
        let g = lock(&self.node);
        check(unsafe { sys::dora_node_allocate_data_sample(g.raw, data_len, &mut raw) })?;
        Ok(DataSample { raw, node: self.node.clone() })
    }

    /// send_output_sample (mod.rs:246-275).  The sample must be fully written (its stream
    /// synchronised) before the call.
    pub fn send_output_sample(
        &mut self,
        output_id: &str,
        parameters: MetadataParameters,
        data: Option<DataSample>,
        type_info: ArrowTypeInfo,
    ) -> Result<()> {
        let ti = type_info::encode(&type_info)?;
        let p = encode_parameters(&parameters);
        let raw = data.map(DataSample::take).unwrap_or(ptr::null_mut());
        let g = lock(&self.node);
        check(unsafe {
            sys::dora_node_send_output_sample(
                g.raw,
                cstr(output_id)?.as_ptr(),
                ti.as_ptr(),
                ti.len(),
                p.as_ptr(),
                p.len(),
                raw,
            )
        })
    }

    /// close_outputs (mod.rs:277-289).
    pub fn close_outputs(&mut self, outputs: &[&str]) -> Result<()> {
        let owned: Vec<CString> = outputs.iter().map(|o| cstr(o)).collect::<Result<_>>()?;
        let ptrs: Vec<*const std::os::raw::c_char> = owned.iter().map(|c| c.as_ptr()).collect();
        let g = lock(&self.node);
        check(unsafe { sys::dora_node_close_outputs(g.raw, ptrs.as_ptr(), ptrs.len()) })
    }

    /// EventStream::recv / recv_timeout (event_stream/mod.rs:121-140) with device-resident
    /// inputs; None once the stream ended or on a timeout.  Waits in 1 ms slices, releasing the
    /// node's lock between them: a `DeviceInput` dropped on another thread (its drop token)
    /// or a send there never waits for the next event to arrive.
    pub fn recv(&mut self, timeout: Option<Duration>) -> Option<GpuEvent> {
        let t0 = std::time::Instant::now();
        let slice = Duration::from_millis(1);
        loop {
            let wait = match timeout {
                None => slice,
                Some(d) => d.saturating_sub(t0.elapsed()).min(slice),
            };
            match next_event(&self.node, wait.as_micros() as i64) {
                Ok(e) => return e,
                Err(_) if timeout.map_or(false, |d| t0.elapsed() >= d) => return None,
                Err(_) => {}
            }
        }
    }
}
