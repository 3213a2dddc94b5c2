//! The reference's node API surface on the device data plane: `DoraNode`
//! (apis/rust/node/src/node/mod.rs:42-431), `EventStream` (event_stream/mod.rs:27-214) and
//! `Event` (event_stream/event.rs:10-26) with the reference's signatures, so an existing Rust
//! node compiles against this crate with only its `use` line changed.
//!
//! What moves where: outputs are packed into device samples in HBM and routed as handles
//! (`DataMessage::DeviceIpc`); `Event::Input::data` is host `ArrowData`, as the reference's
//! CPU consumers expect — a device input is staged to the host (one D2H copy) and its drop
//! token returned at once.  A consumer that can use HBM directly takes
//! `EventStream::recv_device` (zero-copy `DeviceInput`).  `send_output*` return once the sample
//! no longer needs the caller's data, as the reference's.
use std::future::Future;
use std::pin::Pin;
use std::task::{Context, Poll};
use std::time::{Duration, Instant};

use arrow::array::{make_array, new_empty_array, Array};
use dora_arrow_convert::ArrowData;
use dora_core::config::{DataId, NodeId, OperatorId};
use dora_core::uhlc;
use dora_message::metadata::{ArrowTypeInfo, Metadata, MetadataParameters};
use dora_gpu_sys as sys;
use eyre::{bail, Result, WrapErr};

use crate::check;
use crate::node::{self, DeviceInput, GpuEvent, GpuNode, SharedNode};

/// `DoraNode` (mod.rs:42): sends outputs of this node.
pub struct DoraNode {
    inner: GpuNode,
    id: NodeId,
    clock: std::sync::Arc<uhlc::HLC>,
}

/// A sample from `allocate_data_sample` (mod.rs:303-346, 434-503): host bytes the caller fills
/// (`Deref<Target = [u8]>`, as the reference's), uploaded into a device slot when sent.
pub struct DataSample {
    buf: Vec<u8>,
}

impl std::ops::Deref for DataSample {
    type Target = [u8];
    fn deref(&self) -> &[u8] {
        &self.buf
    }
}

impl std::ops::DerefMut for DataSample {
    fn deref_mut(&mut self) -> &mut [u8] {
        &mut self.buf
    }
}

impl std::fmt::Debug for DataSample {
    fn fmt(&self, f: &mut std::fmt::Formatter<'_>) -> std::fmt::Result {
        f.debug_struct("DataSample").field("len", &self.buf.len()).finish_non_exhaustive()
    }
}

/// `Event` (event.rs:10-26).
#[derive(Debug)]
#[non_exhaustive]
pub enum Event {
    Stop,
    Reload { operator_id: Option<OperatorId> },
    Input { id: DataId, metadata: Metadata, data: ArrowData },
    InputClosed { id: DataId },
    Error(String),
}

/// `EventStream` (event_stream/mod.rs:27): receives this node's events.
pub struct EventStream {
    node: SharedNode,
    clock: std::sync::Arc<uhlc::HLC>,
}

impl DoraNode {
    fn wrap(inner: GpuNode, id: NodeId) -> (Self, EventStream) {
        let clock = std::sync::Arc::new(uhlc::HLC::default());
        let events = EventStream { node: inner.shared(), clock: clock.clone() };
        (DoraNode { inner, id, clock }, events)
    }

    /// `init_from_env` (mod.rs:65-76).  The launcher of this data plane sets DORA_GPU_DATAFLOW
    /// (the dataflow's control region), DORA_NODE_ID and DORA_GPU_DEVICE instead of
    /// DORA_NODE_CONFIG.
    pub fn init_from_env() -> Result<(Self, EventStream)> {
        let id = std::env::var("DORA_NODE_ID")
            .wrap_err("env variable DORA_NODE_ID must be set. Are you sure you started the dataflow?")?;
        let inner = GpuNode::init_from_env().wrap_err("failed to init node")?;
        Ok(Self::wrap(inner, NodeId::from(id)))
    }

    /// `init_from_node_id` (mod.rs:87-110): a dynamic node (`path: dynamic`) of the running
    /// dataflow named by DORA_GPU_DATAFLOW, on DORA_GPU_DEVICE (default 0).
    pub fn init_from_node_id(node_id: NodeId) -> Result<(Self, EventStream)> {
        let dataflow = std::env::var("DORA_GPU_DATAFLOW")
            .wrap_err("env variable DORA_GPU_DATAFLOW must name the running dataflow")?;
        let device = std::env::var("DORA_GPU_DEVICE").ok().and_then(|d| d.parse().ok()).unwrap_or(0);
        let inner = GpuNode::init(&dataflow, node_id.as_ref(), device)
            .wrap_err_with(|| format!("Could not init node {node_id}"))?;
        Ok(Self::wrap(inner, node_id))
    }

    /// `init_flexible` (mod.rs:112-119).
    pub fn init_flexible(node_id: NodeId) -> Result<(Self, EventStream)> {
        if std::env::var("DORA_NODE_ID").is_ok() {
            Self::init_from_env()
        } else {
            Self::init_from_node_id(node_id)
        }
    }

    /// `send_output_raw` (mod.rs:180-196).
    pub fn send_output_raw<F>(
        &mut self,
        output_id: DataId,
        parameters: MetadataParameters,
        data_len: usize,
        data: F,
    ) -> Result<()>
    where
        F: FnOnce(&mut [u8]),
    {
        self.inner.send_output_raw(output_id.as_str(), parameters, data_len, data)
    }

    /// `send_output` (mod.rs:198-215): a host array, packed into a device sample.
    pub fn send_output(
        &mut self,
        output_id: DataId,
        parameters: MetadataParameters,
        data: impl Array,
    ) -> Result<()> {
        self.inner
            .send_output(output_id.as_str(), parameters, data)
            .wrap_err("failed to send output")
    }

    /// `send_output_bytes` (mod.rs:217-228).
    pub fn send_output_bytes(
        &mut self,
        output_id: DataId,
        parameters: MetadataParameters,
        data_len: usize,
        data: &[u8],
    ) -> Result<()> {
        if data.len() != data_len {
            bail!("send_output_bytes: data_len {data_len} but {} bytes given", data.len());
        }
        self.inner.send_output_bytes(output_id.as_str(), parameters, data)
    }

    /// `send_typed_output` (mod.rs:229-244): `data` fills `data_len` bytes laid out as
    /// `type_info` says.
    pub fn send_typed_output<F>(
        &mut self,
        output_id: DataId,
        type_info: ArrowTypeInfo,
        parameters: MetadataParameters,
        data_len: usize,
        data: F,
    ) -> Result<()>
    where
        F: FnOnce(&mut [u8]),
    {
        let mut sample = self.allocate_data_sample(data_len)?;
        data(&mut sample);
        self.send_output_sample(output_id, type_info, parameters, Some(sample))
    }

    /// `send_output_sample` (mod.rs:246-275): the sample's bytes go into a device slot (one
    /// H2D copy), sent with `type_info`.
    pub fn send_output_sample(
        &mut self,
        output_id: DataId,
        type_info: ArrowTypeInfo,
        parameters: MetadataParameters,
        sample: Option<DataSample>,
    ) -> Result<()> {
        let dev = match sample {
            Some(s) if !s.buf.is_empty() => {
                let mut d = self.inner.allocate_data_sample(s.buf.len())?;
                let st = self.inner.stream();
                check(unsafe {
                    sys::dora_gpu_memcpy_async(
                        d.as_mut_ptr() as *mut std::os::raw::c_void,
                        s.buf.as_ptr() as *const std::os::raw::c_void,
                        s.buf.len(),
                        st,
                    )
                })?;
                check(unsafe { sys::dora_gpu_stream_sync(st) })?;
                Some(d)
            }
            _ => None,
        };
        self.inner
            .send_output_sample(output_id.as_str(), parameters, dev, type_info)
            .wrap_err_with(|| format!("failed to send output {output_id}"))
    }

    /// `close_outputs` (mod.rs:277-289).
    pub fn close_outputs(&mut self, outputs: Vec<DataId>) -> Result<()> {
        let ids: Vec<&str> = outputs.iter().map(|o| o.as_str()).collect();
        self.inner.close_outputs(&ids).wrap_err("failed to report closed outputs to daemon")
    }

    /// `id` (mod.rs:291).
    pub fn id(&self) -> &NodeId {
        &self.id
    }

    /// `allocate_data_sample` (mod.rs:303): host bytes, uploaded by `send_output_sample`.
    pub fn allocate_data_sample(&mut self, data_len: usize) -> Result<DataSample> {
        Ok(DataSample { buf: vec![0u8; data_len] })
    }

    /// Extension: the device-first node (device samples, device-source sends).
    pub fn gpu(&mut self) -> &mut GpuNode {
        &mut self.inner
    }

    /// The clock that stamps this node's outputs.
    pub fn clock(&self) -> &uhlc::HLC {
        &self.clock
    }
}

/// The C library's nanosecond timestamp as the reference's `uhlc::Timestamp`.
fn timestamp(clock: &uhlc::HLC, ns: u64) -> uhlc::Timestamp {
    uhlc::Timestamp::new(uhlc::NTP64::from(Duration::from_nanos(ns)), *clock.get_id())
}

impl EventStream {
    /// The reference's `Event` from a device event: inputs staged to host `ArrowData`.
    fn convert(&self, ev: GpuEvent) -> Event {
        match ev {
            GpuEvent::Input { id, metadata, data } => match host_input(&data) {
                Ok((type_info, array)) => Event::Input {
                    id: DataId::from(id),
                    metadata: Metadata::from_parameters(
                        timestamp(&self.clock, metadata.timestamp_ns),
                        type_info,
                        metadata.parameters,
                    ),
                    data: ArrowData(array),
                },
                Err(e) => Event::Error(format!("input `{id}`: {e:?}")),
            },
            GpuEvent::InputClosed { id } => Event::InputClosed { id: DataId::from(id) },
            GpuEvent::Stop => Event::Stop,
            GpuEvent::Error(e) => Event::Error(e),
        }
    }

    /// One `dora_node_next_event` of at most `slice`: the node's lock is held only for that
    /// long, so a `DoraNode` on another thread keeps sending.
    fn poll(&mut self, slice: Duration) -> Result<Option<GpuEvent>, ()> {
        node::next_event(&self.node, slice.as_micros() as i64).map_err(|_| ())
    }

    /// `recv` (event_stream/mod.rs:121-124): the next event, None at the end of the stream.
    pub fn recv(&mut self) -> Option<Event> {
        self.recv_device().map(|e| self.convert(e))
    }

    /// `recv_timeout` (event_stream/mod.rs:126-128): as the reference, a timeout yields an
    /// `Event::Error`.
    pub fn recv_timeout(&mut self, dur: Duration) -> Option<Event> {
        match self.recv_device_timeout(dur) {
            Ok(e) => e.map(|e| self.convert(e)),
            Err(()) => Some(Event::Error("Receiver timed out".to_string())),
        }
    }

    /// `recv_async` (event_stream/mod.rs:130-132).
    pub async fn recv_async(&mut self) -> Option<Event> {
        loop {
            match self.poll(Duration::ZERO) {
                Ok(e) => return e.map(|e| self.convert(e)),
                Err(()) => YieldNow(false).await,
            }
        }
    }

    /// `recv_async_timeout` (event_stream/mod.rs:134-147).
    pub async fn recv_async_timeout(&mut self, dur: Duration) -> Option<Event> {
        let t0 = Instant::now();
        loop {
            match self.poll(Duration::ZERO) {
                Ok(e) => return e.map(|e| self.convert(e)),
                Err(()) if t0.elapsed() >= dur => {
                    return Some(Event::Error("Receiver timed out".to_string()))
                }
                Err(()) => YieldNow(false).await,
            }
        }
    }

    /// Extension: the next event with its input left in HBM (zero-copy `DeviceInput`).
    pub fn recv_device(&mut self) -> Option<GpuEvent> {
        loop {
            if let Ok(e) = self.poll(Duration::from_millis(1)) {
                return e;
            }
        }
    }

    /// Extension: `recv_device` bounded by `dur` (Err on a timeout).
    pub fn recv_device_timeout(&mut self, dur: Duration) -> Result<Option<GpuEvent>, ()> {
        let t0 = Instant::now();
        loop {
            let left = dur.saturating_sub(t0.elapsed());
            match self.poll(left.min(Duration::from_millis(1))) {
                Ok(e) => return Ok(e),
                Err(()) if t0.elapsed() >= dur => return Err(()),
                Err(()) => {}
            }
        }
    }
}

/// A device input as the reference's host `ArrayData` (`RawData::into_arrow_array`,
/// event.rs:35-91): its type info and a host copy; the input (and its token) goes with `data`.
fn host_input(data: &DeviceInput) -> Result<(ArrowTypeInfo, arrow::array::ArrayRef)> {
    let type_info = data.type_info()?;
    let (_, len) = data.raw()?;
    let array = if len == 0 {
        new_empty_array(&type_info.data_type) // RawData::Empty / Vec(empty)
    } else {
        make_array(data.to_host()?)
    };
    Ok((type_info, array))
}

/// Yield once to the executor (the C event call above never blocks in async mode).
struct YieldNow(bool);

impl Future for YieldNow {
    type Output = ();
    fn poll(mut self: Pin<&mut Self>, cx: &mut Context<'_>) -> Poll<()> {
        if self.0 {
            return Poll::Ready(());
        }
        self.0 = true;
        cx.waker().wake_by_ref();
        Poll::Pending
    }
}
