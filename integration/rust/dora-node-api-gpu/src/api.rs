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
use std::collections::{BTreeMap, BTreeSet, VecDeque};
use std::pin::Pin;
use std::sync::{Arc, Condvar, Mutex};
use std::task::{Context, Poll, Waker};
use std::thread::JoinHandle;
use std::time::{Duration, Instant};

use arrow::array::{make_array, new_empty_array, Array};
use dora_arrow_convert::ArrowData;
use dora_core::config::{DataId, NodeId, NodeRunConfig, OperatorId};
use dora_core::descriptor::Descriptor;
use dora_core::uhlc;
use dora_message::daemon_to_node::{DaemonCommunication, NodeConfig};
use dora_message::metadata::{ArrowTypeInfo, Metadata, MetadataParameters};
use dora_message::DataflowId;
use dora_gpu_sys as sys;
use eyre::{bail, Result, WrapErr};
use futures::Stream;

use crate::check;
use crate::node::{self, DeviceInput, GpuEvent, GpuNode, SharedNode};

/// `DoraNode` (mod.rs:42): sends outputs of this node.
pub struct DoraNode {
    inner: GpuNode,
    id: NodeId,
    dataflow_id: DataflowId,
    node_config: NodeRunConfig,
    dataflow_descriptor: Descriptor,
    clock: Arc<uhlc::HLC>,
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
    clock: Arc<uhlc::HLC>,
    // async readers (`recv_async*`, `Stream`): a thread that waits for events so the task
    // parks instead of spinning; started on the first async poll
    pump: Option<Pump>,
}

/// The GPU ordinal of this node: DORA_GPU_DEVICE, set by the launcher from the descriptor's
/// `_unstable_deploy.gpu` (default 0).
fn device_from_env() -> i32 {
    std::env::var("DORA_GPU_DEVICE").ok().and_then(|d| d.parse().ok()).unwrap_or(0)
}

impl DoraNode {
    fn wrap(inner: GpuNode, config: NodeConfig) -> (Self, EventStream) {
        let clock = Arc::new(uhlc::HLC::default());
        let events = EventStream { node: inner.shared(), clock: clock.clone(), pump: None };
        let node = DoraNode {
            inner,
            id: config.node_id,
            dataflow_id: config.dataflow_id,
            node_config: config.run_config,
            dataflow_descriptor: config.dataflow_descriptor,
            clock,
        };
        (node, events)
    }

    /// `init_from_env` (mod.rs:65-76): the `NodeConfig` in DORA_NODE_CONFIG, as the reference.
    /// This data plane's launcher (dora_amd/dataflow.py `node_config`) writes it in the
    /// reference's schema, naming its control region as the `Shmem` daemon communication.
    pub fn init_from_env() -> Result<(Self, EventStream)> {
        let node_config: NodeConfig = {
            let raw = std::env::var("DORA_NODE_CONFIG").wrap_err(
                "env variable DORA_NODE_CONFIG must be set. Are you sure your using `dora start`?",
            )?;
            serde_yaml::from_str(&raw).context("failed to deserialize operator config")?
        };
        Self::init(node_config)
    }

    /// `init_from_node_id` (mod.rs:87-110): a dynamic node (`path: dynamic`) of the running
    /// dataflow.  The reference asks the local daemon for the node's `NodeConfig` over TCP; this
    /// data plane's launcher hands it over in DORA_NODE_CONFIG for dynamic nodes too
    /// (`Dataflow.dynamic_env`), and without it the node attaches to the control region named
    /// by DORA_GPU_DATAFLOW with an empty run config.
    pub fn init_from_node_id(node_id: NodeId) -> Result<(Self, EventStream)> {
        if let Ok(raw) = std::env::var("DORA_NODE_CONFIG") {
            let config: NodeConfig =
                serde_yaml::from_str(&raw).context("failed to deserialize node config")?;
            if config.node_id == node_id {
                return Self::init(config);
            }
        }
        let dataflow = std::env::var("DORA_GPU_DATAFLOW")
            .wrap_err("failed to get node config from daemon: DORA_GPU_DATAFLOW is not set")?;
        let inner = GpuNode::init(&dataflow, node_id.as_ref(), device_from_env())
            .wrap_err_with(|| format!("Could not init node {node_id}"))?;
        let config = NodeConfig {
            dataflow_id: DataflowId::nil(),
            node_id,
            run_config: NodeRunConfig { inputs: BTreeMap::new(), outputs: BTreeSet::new() },
            daemon_communication: DaemonCommunication::Shmem {
                daemon_control_region_id: dataflow.clone(),
                daemon_drop_region_id: dataflow.clone(),
                daemon_events_region_id: dataflow.clone(),
                daemon_events_close_region_id: dataflow,
            },
            dataflow_descriptor: serde_yaml::from_str("nodes: []")
                .context("empty dataflow descriptor")?,
            dynamic: true,
        };
        Ok(Self::wrap(inner, config))
    }

    /// `init_flexible` (mod.rs:112-119).
    pub fn init_flexible(node_id: NodeId) -> Result<(Self, EventStream)> {
        if std::env::var("DORA_NODE_CONFIG").is_ok() {
            Self::init_from_env()
        } else {
            Self::init_from_node_id(node_id)
        }
    }

    /// `init` (mod.rs:122-156): attach to the dataflow the config names.  This data plane's
    /// daemon speaks over one shared-memory control region (requests, events and drop tokens
    /// in rings), named by the `Shmem` variant; the node's GPU is DORA_GPU_DEVICE.
    pub fn init(node_config: NodeConfig) -> eyre::Result<(Self, EventStream)> {
        let region = match &node_config.daemon_communication {
            DaemonCommunication::Shmem { daemon_control_region_id, .. } => {
                daemon_control_region_id.clone()
            }
            _ => bail!(
                "the device data plane's daemon is reached through a shared-memory control \
                 region (DaemonCommunication::Shmem)"
            ),
        };
        let inner = GpuNode::init(&region, node_config.node_id.as_ref(), device_from_env())
            .wrap_err("failed to init event stream")?;
        Ok(Self::wrap(inner, node_config))
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

    /// `dataflow_id` (mod.rs:295).
    pub fn dataflow_id(&self) -> &DataflowId {
        &self.dataflow_id
    }

    /// `node_config` (mod.rs:299): this node's inputs and outputs.
    pub fn node_config(&self) -> &NodeRunConfig {
        &self.node_config
    }

    /// `dataflow_descriptor` (mod.rs:376): the descriptor of the dataflow this node is part of.
    pub fn dataflow_descriptor(&self) -> &Descriptor {
        &self.dataflow_descriptor
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

    /// The next device event for an async reader: one queued by the pump, else the waker is
    /// registered and the pump asked for an event (woken also at `deadline`).
    fn poll_device(&mut self, cx: &Context<'_>, deadline: Option<Instant>) -> Poll<Option<GpuEvent>> {
        let node = self.node.clone();
        self.pump.get_or_insert_with(|| Pump::start(node)).poll(cx.waker(), deadline)
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

    /// `recv_async` (event_stream/mod.rs:130-132): parks the task until an event arrives (the
    /// pump thread waits for it and wakes the task), as the reference's awaited channel.
    pub async fn recv_async(&mut self) -> Option<Event> {
        let e = futures::future::poll_fn(|cx| self.poll_device(cx, None)).await;
        e.map(|e| self.convert(e))
    }

    /// `recv_async_timeout` (event_stream/mod.rs:134-147).
    pub async fn recv_async_timeout(&mut self, dur: Duration) -> Option<Event> {
        let deadline = Instant::now() + dur;
        let e = futures::future::poll_fn(|cx| match self.poll_device(cx, Some(deadline)) {
            Poll::Ready(e) => Poll::Ready(Ok(e)),
            Poll::Pending if Instant::now() >= deadline => Poll::Ready(Err(())),
            Poll::Pending => Poll::Pending,
        })
        .await;
        match e {
            Ok(e) => e.map(|e| self.convert(e)),
            Err(()) => Some(Event::Error("Receiver timed out".to_string())),
        }
    }

    /// Extension: the next event with its input left in HBM (zero-copy `DeviceInput`).
    pub fn recv_device(&mut self) -> Option<GpuEvent> {
        if let Some(p) = &self.pump {
            return p.wait(None).unwrap_or(None);  // keeps the order of events the pump holds
        }
        loop {
            if let Ok(e) = self.poll(Duration::from_millis(1)) {
                return e;
            }
        }
    }

    /// Extension: `recv_device` bounded by `dur` (Err on a timeout).
    pub fn recv_device_timeout(&mut self, dur: Duration) -> Result<Option<GpuEvent>, ()> {
        let t0 = Instant::now();
        if let Some(p) = &self.pump {
            return p.wait(Some(t0 + dur));
        }
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

/// `impl Stream for EventStream` (event_stream/mod.rs:201-214): `while let Some(event) =
/// events.next().await` works as with the reference.
impl Stream for EventStream {
    type Item = Event;

    fn poll_next(mut self: Pin<&mut Self>, cx: &mut Context<'_>) -> Poll<Option<Self::Item>> {
        let this = &mut *self;
        match this.poll_device(cx, None) {
            Poll::Ready(e) => Poll::Ready(e.map(|e| this.convert(e))),
            Poll::Pending => Poll::Pending,
        }
    }
}

impl Drop for EventStream {
    fn drop(&mut self) {
        if let Some(p) = self.pump.take() {
            p.stop();
        }
    }
}

/// Events fetched by the pump thread for async readers, and the reader it wakes.
#[derive(Default)]
struct PumpState {
    events: VecDeque<GpuEvent>,
    ended: bool,              // the stream ended (None was returned)
    wanted: bool,             // a reader waits: fetch an event
    waker: Option<Waker>,
    deadline: Option<Instant>, // wake the reader then even without an event (recv_async_timeout)
    stop: bool,
}

/// A thread that calls `dora_node_next_event` in 1 ms slices (the node's lock is free between
/// them, so sends on other threads proceed) while a reader wants an event, queues what it gets
/// and wakes the reader's task; it sleeps on a condition variable otherwise.  This replaces the
/// reference's event-stream thread + flume channel (event_stream/thread.rs) for async readers.
struct Pump {
    state: Arc<(Mutex<PumpState>, Condvar)>,
    thread: Option<JoinHandle<()>>,
}

impl Pump {
    fn start(node: SharedNode) -> Pump {
        let state = Arc::new((Mutex::new(PumpState::default()), Condvar::new()));
        let st = state.clone();
        let thread = std::thread::Builder::new()
            .name("dora-event-pump".into())
            .spawn(move || {
                let (m, cv) = &*st;
                loop {
                    {
                        let mut g = m.lock().unwrap();
                        while !g.stop && (!g.wanted || !g.events.is_empty() || g.ended) {
                            g = cv.wait(g).unwrap();
                        }
                        if g.stop {
                            return;
                        }
                    }
                    let got = node::next_event(&node, 1000);
                    let mut g = m.lock().unwrap();
                    match got {
                        Ok(Some(e)) => g.events.push_back(e),
                        Ok(None) => g.ended = true,
                        Err(_) => {
                            // no event in this slice: only a passed deadline wakes the reader
                            if !g.deadline.map_or(false, |d| Instant::now() >= d) {
                                continue;
                            }
                            g.deadline = None;
                        }
                    }
                    g.wanted = false;
                    if let Some(w) = g.waker.take() {
                        w.wake();
                    }
                    cv.notify_all();
                }
            })
            .expect("failed to spawn the event pump thread");
        Pump { state, thread: Some(thread) }
    }

    fn poll(&self, waker: &Waker, deadline: Option<Instant>) -> Poll<Option<GpuEvent>> {
        let (m, cv) = &*self.state;
        let mut g = m.lock().unwrap();
        if let Some(e) = g.events.pop_front() {
            return Poll::Ready(Some(e));
        }
        if g.ended {
            return Poll::Ready(None);
        }
        g.waker = Some(waker.clone());
        g.deadline = deadline;
        g.wanted = true;
        cv.notify_all();
        Poll::Pending
    }

    /// A blocking read through the pump (a synchronous `recv` after async ones): Err at
    /// `deadline`.
    fn wait(&self, deadline: Option<Instant>) -> Result<Option<GpuEvent>, ()> {
        let (m, cv) = &*self.state;
        let mut g = m.lock().unwrap();
        loop {
            if let Some(e) = g.events.pop_front() {
                return Ok(Some(e));
            }
            if g.ended {
                return Ok(None);
            }
            g.wanted = true;
            cv.notify_all();
            g = match deadline {
                None => cv.wait(g).unwrap(),
                Some(d) => {
                    let now = Instant::now();
                    if now >= d {
                        return Err(());
                    }
                    cv.wait_timeout(g, d - now).unwrap().0
                }
            };
        }
    }

    fn stop(mut self) {
        {
            let (m, cv) = &*self.state;
            m.lock().unwrap().stop = true;
            cv.notify_all();
        }
        if let Some(t) = self.thread.take() {
            let _ = t.join();
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

