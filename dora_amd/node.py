"""Python node API on the device data plane — mirrors the reference Python `Node`
(apis/python/node/src/lib.rs:29-185) and its event dicts (apis/python/operator/src/lib.rs:81-165).

    node = Node()                                   # from env (DORA_GPU_DATAFLOW, DORA_NODE_ID)
    for event in node:                              # or node.next(timeout)
        if event["type"] == "INPUT":
            arr = event["value"]                    # DeviceArray: zero-copy view of the HBM sample
            host = arr.to_pyarrow()                 # host staging for pyarrow consumers (F12)
    node.send_output("out", pa.array([...]), {"k": 1})   # host pyarrow: inline < 4096 B, else DMA
    node.send_output("out", device_array)                 # HBM array -> HIP pack kernel
    node.send_output("out", b"raw bytes")                 # ArrowTypeInfo::byte_array
"""
from __future__ import annotations

import ctypes
import os
import struct
import sys
import time
from ctypes import byref, c_double, c_size_t, c_uint8, c_uint64, c_void_p
from typing import Optional

from . import _lib
from ._lib import ARROW_DEVICE_CPU, ARROW_DEVICE_ROCM, DoraGpuError, call, load
from .arrow_c import ArrowArray, ArrowSchema, CArray

SEND_ASYNC = 1  # DORA_SEND_ASYNC (include/dora_gpu.h)
from .device import DeviceArray, DeviceBuffer
from .type_info import decode

try:
    from . import _dora_node as _fast
except ImportError as e:  # no fallback: the send path is native
    raise ImportError(f"dora_amd._dora_node is missing ({e}): build it with "
                      "`python -m dora_amd.build`") from e

# MetadataParameters bytes of a dict, natively (the send paths encode inside _fast)
encode_parameters = _fast.encode_parameters

EVENT_TYPES = {0: "STOP", 1: "INPUT", 2: "INPUT_CLOSED", 3: "ERROR", 4: "ALL_INPUTS_CLOSED"}


_U32 = struct.Struct("<I").pack
_U64 = struct.Struct("<Q").pack
_TAG_BOOL = struct.Struct("<BB").pack
_TAG_INT = struct.Struct("<Bq").pack
_TAG_STR = struct.Struct("<BQ").pack
_KEYS: dict = {}  # encoded key prefix by key (u64 length + utf-8)


def encode_parameters_py(metadata: Optional[dict]) -> bytes:
    """MetadataParameters encoding (pydict_to_metadata, apis/python/operator/src/lib.rs:165-186:
    bool / int / str, anything else stringified), in Python: the statement of the format that
    tests hold the native encoder (`encode_parameters`, csrc/pyext.cpp) to."""
    if not metadata:
        return b""
    out = [_U32(len(metadata))]
    for k in sorted(metadata):
        v = metadata[k]
        kp = _KEYS.get(k)
        if kp is None:
            kb = str(k).encode()
            kp = _U64(len(kb)) + kb
            if len(_KEYS) < 4096:
                _KEYS[k] = kp
        out.append(kp)
        t = type(v)
        if t is int:
            out.append(_TAG_INT(1, v))
        elif t is bool or isinstance(v, bool):
            out.append(_TAG_BOOL(0, int(v)))
        elif isinstance(v, int):
            out.append(_TAG_INT(1, v))
        else:
            sb = (v if isinstance(v, str) else str(v)).encode()
            out.append(_TAG_STR(2, len(sb)) + sb)
    return b"".join(out)


def decode_parameters(raw: bytes) -> dict:
    if len(raw) < 4:
        return {}
    (n,), i, out = struct.unpack_from("<I", raw), 4, {}
    for _ in range(n):
        (kl,) = struct.unpack_from("<Q", raw, i)
        i += 8
        key = raw[i:i + kl].decode()
        i += kl
        tag = raw[i]
        i += 1
        if tag == 0:
            out[key] = bool(raw[i])
            i += 1
        elif tag == 1:
            (out[key],) = struct.unpack_from("<q", raw, i)
            i += 8
        else:
            (sl,) = struct.unpack_from("<Q", raw, i)
            i += 8
            out[key] = raw[i:i + sl].decode()
            i += sl
    return out


def descriptor_path(region: str) -> str:
    """Where a dataflow's launcher leaves its parsed descriptor (JSON) for its nodes: beside its
    control region in /dev/shm, removed with it."""
    return "/dev/shm/" + region.lstrip("/") + ".descriptor.json"


def _is_pyarrow_array(data) -> bool:
    pa = sys.modules.get("pyarrow")  # an Array exists only once pyarrow is imported
    return pa is not None and isinstance(data, pa.Array)


class _EventHandle:
    """Owns a C dora_event; freeing it (explicitly or by GC) releases the drop token once no
    DeviceArray view references the sample any more."""

    def __init__(self, ptr):
        self.ptr = ptr
        self._lib = load()

    def free(self):
        if self.ptr:
            self._lib.dora_event_free(self.ptr)
            self.ptr = None

    def __del__(self):
        self.free()


class _Event(dict):
    """Event dict whose "type_info" (the input's ArrowTypeInfo, reference inline form) is
    decoded on first access: restoring bitmaps that travelled in the sample's validity tail
    reads them back from HBM, and a receiver that only uses "value" never pays for it."""

    def __missing__(self, key):
        if key != "type_info" or "_event" not in self:
            raise KeyError(key)
        p, n = ctypes.POINTER(c_uint8)(), c_size_t()
        call("dora_event_type_info", self["_event"].ptr, byref(p), byref(n))
        ti = decode(ctypes.string_at(p, n.value))
        self["type_info"] = ti
        return ti


class Node:
    """The reference's `Node` pyclass (apis/python/node/src/lib.rs:29-209): `Node(node_id=None)`,
    `next(timeout=None)`, iteration (`__iter__` / `__next__`), `send_output(output_id, data,
    metadata=None)`, `dataflow_descriptor()`, `dataflow_id()`, `merge_external_events(...)`.
    Added here: `dataflow` / `device` to join a dataflow by its region name on a given GPU (the
    reference finds a dynamic node's daemon by node id), and the device-side calls below."""

    def __init__(self, node_id: Optional[str] = None, dataflow: Optional[str] = None,
                 device: Optional[int] = None):
        self._lib = load()
        h = c_void_p()
        if node_id is None and dataflow is None:
            call("dora_node_init_from_env", byref(h))
        else:
            shm = dataflow or os.environ["DORA_GPU_DATAFLOW"]
            dev = device if device is not None else int(os.environ.get("DORA_GPU_DEVICE", "0"))
            call("dora_node_init", shm.encode(), node_id.encode(), dev, byref(h))
        self.handle = h.value
        self.id = self._lib.dora_node_id(self.handle).decode()
        self.device = device if device is not None else int(os.environ.get("DORA_GPU_DEVICE", "0"))
        self._region = dataflow or os.environ.get("DORA_GPU_DATAFLOW", "")

    # -------------------------------------------------------------------------------- sending
    def send_output(self, output_id: str, data, metadata: Optional[dict] = None, *,
                    asynchronous: bool = False):
        """send_output (apis/python/node/src/lib.rs:157-185).  Returns once the sample no longer
        needs `data`, as the reference (which copies inside the call): a device source's pack
        has read it.  `asynchronous=True` (DORA_SEND_ASYNC) returns as soon as the pack is
        queued; the caller then must not write a device source until `sync()`, or only by work
        queued on `stream` fetched after the send."""
        f = SEND_ASYNC if asynchronous else 0
        if isinstance(data, DeviceArray):
            a, s = data.send_addrs()
            rc = _fast.send_array(self.handle, output_id, a, s, ARROW_DEVICE_ROCM, metadata, f)
        elif isinstance(data, (bytes, bytearray, memoryview)):
            # read in place; the call copies them before it returns (inline below 4096 B)
            rc = _fast.send_buffer(self.handle, output_id, data, metadata)
        elif isinstance(data, DeviceBuffer):
            rc = _fast.send_bytes(self.handle, output_id, data.ptr, data.size, ARROW_DEVICE_ROCM,
                                  metadata, f)
        elif _is_pyarrow_array(data):
            # exported natively; the type's schema is exported once and lent to later sends
            rc = _fast.send_pyarrow(self.handle, output_id, data, metadata)
        elif hasattr(data, "_export_to_c"):
            with CArray.from_pyarrow(data) as c:
                rc = _fast.send_array(self.handle, output_id, ctypes.addressof(c.array),
                                      ctypes.addressof(c.schema), ARROW_DEVICE_CPU, metadata)
        else:
            raise TypeError("data must be bytes, a pyarrow.Array, a DeviceArray or a DeviceBuffer")
        if rc:
            _lib.check(rc)

    def send_output_async(self, output_id: str, data, metadata: Optional[dict] = None):
        """send_output(..., asynchronous=True)."""
        self.send_output(output_id, data, metadata, asynchronous=True)

    def set_async_sends(self, enable: bool = True):
        """Make every send of this node asynchronous (dora_node_set_async_sends)."""
        call("dora_node_set_async_sends", self.handle, int(enable))

    def set_event_thread(self, enable: bool = True):
        """Drain the daemon's events on a background thread (the reference's event-stream thread;
        dora_node_set_event_thread): inputs keep arriving, with the drop-oldest policy applied,
        while this node's user thread is busy elsewhere."""
        call("dora_node_set_event_thread", self.handle, int(enable))

    def send_output_device_bytes(self, output_id: str, ptr: int, n: int,
                                 metadata: Optional[dict] = None, *, asynchronous: bool = False):
        """send_output_raw with an HBM source: one pack kernel into a fresh device sample;
        returns once the pack has read the source unless `asynchronous` (send_output)."""
        rc = _fast.send_bytes(self.handle, output_id, ptr, n, ARROW_DEVICE_ROCM, metadata,
                              SEND_ASYNC if asynchronous else 0)
        if rc:
            _lib.check(rc)

    def set_compact(self, enable: bool = True):
        """Send device arrays with compacting plans (slices move only their own bytes)."""
        call("dora_node_set_compact", self.handle, int(enable))

    def forward(self, output_id: str, event: dict, metadata: Optional[dict] = None):
        """Re-send a received input on `output_id` with its type info (dora_node_forward): one
        copy, a cross-GPU input straight from the peer's slot.  Parameters default to the
        input's own."""
        params = encode_parameters(event.get("metadata") if metadata is None else metadata)
        call("dora_node_forward", self.handle, output_id.encode(), event["_event"].ptr,
             params, len(params))

    def close_outputs(self, outputs):
        arr = (ctypes.c_char_p * len(outputs))(*[o.encode() for o in outputs])
        call("dora_node_close_outputs", self.handle, arr, len(outputs))

    # ------------------------------------------------------------------------------ receiving
    def next(self, timeout: Optional[float] = None):
        """Next event dict, or None when the stream has ended (or on timeout)."""
        # one native call: the event's fields, its decoded parameters and its data's address
        r = _fast.next_event(self.handle, -1 if timeout is None else int(timeout * 1e6))
        if r.__class__ is int:
            if r in (-5, -6):   # closed / timeout
                return None
            _lib.check(r)
        ptr, t, eid, params, ts, dptr, dlen, on_dev, err = r
        ev = _EventHandle(ptr)
        kind = EVENT_TYPES.get(t, "UNKNOWN")
        if kind == "ALL_INPUTS_CLOSED":
            ev.free()
            return None
        out = _Event(type=kind, id=eid)
        if kind == "ERROR":
            out["error"] = err
        if kind == "INPUT":
            out["metadata"] = params
            out["timestamp_ns"] = ts
            out["_event"] = ev  # "type_info" is decoded on first access (_Event)
            out["data_ptr"], out["data_len"] = (dptr or None), dlen
            out["on_device"] = bool(on_dev)
            if dlen == 0:       # RawData::Vec(empty) -> ArrayData::new_empty(data_type)
                import pyarrow as pa
                out["value"] = pa.array([], type=out["type_info"].arrow_type())
            elif out["on_device"]:
                a, s = ArrowArray(), ArrowSchema()
                call("dora_event_array", ev.ptr, byref(a), byref(s))
                import pyarrow as pa
                t = pa.DataType._import_from_c(ctypes.addressof(s))
                # the array keeps the input alive; the event handle can go
                out["value"] = DeviceArray(a, t)
                out["value"]._device_id = self.device
            else:
                # an inline DataMessage::Vec sample (< 4096 B from a host source), or a host-only
                # producer's shared memory read in place: a host pyarrow array over its bytes,
                # as the reference's PyEvent::value; it keeps the input alive
                # (its type from a cache keyed by the schema: no schema import per event)
                r = _fast.export_typed(ev.ptr)
                if r.__class__ is int:
                    _lib.check(r)
                import pyarrow as pa
                try:
                    out["value"] = pa.Array._import_from_c(r[0], r[1])
                finally:
                    _fast.free_arrow(r[0], 0)
        out["_event"] = ev
        return out

    def wait_input(self, input_id: str, key: str, value, timeout: float = 60.0) -> dict:
        """Wait for an input event on `input_id` whose parameters have `key == value` and return
        its parameters; other events are skipped.  A control-message fast path: only the id and
        the parameters are decoded (no data mapping, no Arrow value), in one native call
        (_dora_node.wait_input), so the wait costs about one ring hop, not a Python event
        construction."""
        r = _fast.wait_input(self.handle, input_id, key, value, int(timeout * 1e6))
        if r.__class__ is int:
            if r == -6:
                raise TimeoutError(f"no `{input_id}` input with {key}={value!r}")
            _lib.check(r)
        return r

    def __iter__(self):
        return self

    def __next__(self):
        """`next(node)`: the next event (blocking); StopIteration once the stream has ended, as
        the reference's `__next__` returning None (lib.rs:118-120)."""
        ev = self.next()
        if ev is None:
            raise StopIteration
        return ev

    # ------------------------------------------------------------------------------ dataflow
    def dataflow_id(self) -> str:
        """The dataflow's id (lib.rs:196-202: DataflowId, a uuid): the one in the node's
        DORA_NODE_CONFIG, else the daemon's dataflow name as the inter-daemon wire maps it."""
        from .dataflow import dataflow_uuid
        cfg = self._node_config()
        if cfg and cfg.get("dataflow_id"):
            return str(cfg["dataflow_id"])
        return dataflow_uuid(self._lib.dora_node_dataflow_id(self.handle).decode())

    def dataflow_descriptor(self) -> dict:
        """The dataflow's descriptor as parsed from its YAML (lib.rs:186-194), written next to the
        dataflow's control region by its launcher (dora_amd.dataflow.Dataflow); else the
        descriptor of the node's DORA_NODE_CONFIG."""
        import json
        p = descriptor_path(self._region) if self._region else None
        if p and os.path.exists(p):
            with open(p) as f:
                return json.load(f)
        cfg = self._node_config()
        if cfg and "dataflow_descriptor" in cfg:
            return cfg["dataflow_descriptor"]
        raise RuntimeError(f"no descriptor for dataflow region `{self._region}`")

    def merge_external_events(self, subscription):
        """Merging an external event stream (lib.rs:204-209) exists in the reference only for
        ROS2 subscriptions (dora_ros2_bridge_python), which is outside this data plane: refused."""
        raise NotImplementedError(
            "merge_external_events takes a dora.Ros2Subscription; the ROS2 bridge is not part of "
            "the device data plane")

    def _node_config(self) -> Optional[dict]:
        raw = os.environ.get("DORA_NODE_CONFIG")
        if not raw:
            return None
        import yaml
        cfg = yaml.safe_load(raw)
        return cfg if isinstance(cfg, dict) and cfg.get("node_id") == self.id else None

    # -------------------------------------------------------------------------------- stats
    @property
    def stream(self) -> int:
        return self._lib.dora_node_stream(self.handle)

    def stats(self) -> dict:
        v = [c_uint64() for _ in range(4)]
        call("dora_node_stats", self.handle, *[byref(x) for x in v])
        out = dict(zip(["slots_created", "cache_hits", "in_flight", "dropped_inputs"],
                       [x.value for x in v]))
        c, b = c_uint64(), c_uint64()
        call("dora_node_peer_stats", self.handle, byref(c), byref(b))
        out["peer_copies"], out["peer_bytes"] = c.value, b.value
        call("dora_node_forward_stats", self.handle, byref(c), byref(b))
        out["zero_copy_forwards"], out["forwards_held"] = c.value, b.value
        return out

    def set_profiling(self, enable: bool = True):
        call("dora_node_set_profiling", self.handle, int(enable))

    def dataflow_counters(self, node_id: str) -> dict:
        """Slots created and IPC mappings opened by any node of the dataflow
        (dora_node_dataflow_counters)."""
        a, b, c = c_uint64(), c_uint64(), c_uint64()
        call("dora_node_dataflow_counters", self.handle, node_id.encode(), byref(a), byref(b),
             byref(c))
        return {"slots_created": a.value, "ipc_opens": b.value, "dropped_inputs": c.value}

    def plan_cache_stats(self) -> dict:
        """Device-array sends served by the node's plan cache (dora_node_plan_cache_stats)."""
        a, b = c_uint64(), c_uint64()
        call("dora_node_plan_cache_stats", self.handle, byref(a), byref(b))
        return {"hits": a.value, "entries": b.value}

    def fill_paths(self) -> dict:
        """Fills by dispatch path: raw AQL packets vs hipLaunchKernel (dora_node_fill_paths)."""
        a, h = c_uint64(), c_uint64()
        call("dora_node_fill_paths", self.handle, byref(a), byref(h))
        return {"aql": a.value, "hip": h.value}

    def host_paths(self) -> dict:
        """Host sources written into their slot by the CPU through the BAR, device samples this
        node (without a GPU) staged to host memory, and device samples this node packed straight
        into shared memory for receivers that all lack a GPU (dora_node_host_paths)."""
        a, b, c, d = c_uint64(), c_uint64(), c_uint64(), c_uint64()
        call("dora_node_host_paths", self.handle, byref(a), byref(b), byref(c), byref(d))
        return {"bar_fills": a.value, "staged": b.value, "staged_bytes": c.value,
                "host_packs": d.value}

    def host_bound_outputs(self) -> list:
        """The outputs the daemon named host-bound in AllNodesReady: all receivers lack a GPU
        (dora_node_host_bound_outputs)."""
        n = c_uint64()
        call("dora_node_host_bound_outputs", self.handle, None, 0, byref(n))
        buf = ctypes.create_string_buffer(n.value + 1)
        call("dora_node_host_bound_outputs", self.handle, buf, n.value + 1, byref(n))
        return buf.value.decode().split("\n")[:-1] if n.value else []

    def set_timing_period(self, period: int):
        """Stamp every `period`-th pack launch (0: the default, every 8th)."""
        call("dora_node_set_timing_period", self.handle, int(period))

    def pack_intervals(self, cap: int = 1 << 16):
        """[(start_ms, stop_ms)] of the stamped packs since profiling was enabled."""
        out, n = (c_double * (2 * cap))(), c_size_t()
        call("dora_node_pack_intervals", self.handle, out, cap, byref(n))
        k = min(n.value, cap)
        return [(out[2 * i], out[2 * i + 1]) for i in range(k)]

    def region_begin(self):
        """Start a device-timed run of sends (dora_node_region_begin)."""
        call("dora_node_region_begin", self.handle)

    def sync(self):
        """Wait for every fill of this node and its node stream (dora_node_sync)."""
        call("dora_node_sync", self.handle)

    def region_mark(self):
        """Record the region's stop events after the last send, without waiting on them."""
        call("dora_node_region_mark", self.handle)

    def region_end(self) -> dict:
        """Device span of the sends since region_begin: first pack start -> last pack end."""
        ms, packs, b = c_double(), c_uint64(), c_uint64()
        call("dora_node_region_end", self.handle, byref(ms), byref(packs), byref(b))
        return {"span_ms": ms.value, "packs": packs.value, "bytes": b.value}

    def pack_stats(self) -> dict:
        c, ms, b = c_uint64(), c_double(), c_uint64()
        call("dora_node_pack_stats", self.handle, byref(c), byref(ms), byref(b))
        return {"count": c.value, "total_ms": ms.value, "bytes": b.value}

    def send_profile(self) -> dict:
        out, cnt = (c_double * 4)(), c_uint64()
        call("dora_node_send_profile", self.handle, out, 4, byref(cnt))
        return {"alloc_us": out[0], "launch_us": out[1], "fill_us": out[2], "send_us": out[3],
                "count": cnt.value}

    def close(self):
        if self.handle:
            self._lib.dora_node_free(self.handle)
            self.handle = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


__all__ = ["Node", "encode_parameters", "decode_parameters", "DoraGpuError"]
