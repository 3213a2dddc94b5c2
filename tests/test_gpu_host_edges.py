"""The host side of the device data plane (verdict r05 items 1-3).

* A receiver without a GPU (DORA_GPU_DEVICE < 0) gets the reference's host ArrowData from a
  device producer (apis/rust/node/src/event_stream/event.rs:35-91; Python: a pyarrow array,
  apis/python/operator/src/lib.rs:135-144).  When every receiver of the output lacks a GPU, a
  sample <= 1 MiB is packed by the producer straight into shared memory and sent as the
  reference's DataMessage::SharedMemory; otherwise (larger, or a device receiver too) it is
  staged into pinned host memory on receipt and the producer's token goes back at once.
* Host-resident sources >= 4096 B from a device node (the reference benchmark's payloads,
  examples/benchmark/node/src/main.rs:38-70 via send_output_raw, mod.rs:180-215): up to 2 MiB the
  CPU writes the slot through the large BAR (no GPU dispatch), above that HIP DMAs them; both
  byte-identical to the oracle, and coherent with GPU fills of the same slots.
* The reference's zero-copy sample API (allocate_data_sample -> write -> send_output_sample,
  mod.rs:246-346) through the C ABI, with the sample written in place by a kernel on the node
  stream.
"""
import ctypes
import threading
import time
from ctypes import byref, c_size_t, c_void_p

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _nodes(df, spec):
    from dora_amd.node import Node
    out = {}

    def mk(i, dev):
        out[i] = Node(i, dataflow=df.shm, device=dev)
    ts = [threading.Thread(target=mk, args=(i, d)) for i, d in spec.items()]
    [t.start() for t in ts]
    [t.join(90) for t in ts]
    assert set(out) == set(spec)
    return out


def _device_bytes(ev, stream):
    from dora_amd._lib import call
    out = ctypes.create_string_buffer(max(ev["data_len"], 1))
    call("dora_gpu_memcpy_async", out, ev["data_ptr"], ev["data_len"], stream.handle)
    stream.sync()
    return out.raw[:ev["data_len"]]


def _settle(tx, rx, out="x"):
    """Let returned tokens reach the sender (handled on its next send)."""
    deadline = time.time() + 10
    while tx.stats()["in_flight"] and time.time() < deadline:
        tx.send_output(out, b"", {"settle": 1})
        rx.next(timeout=10)


def test_device_producer_to_host_only_python_receiver(launcher):
    """Device payloads of 8 B .. 40.96 MB, the C3 point cloud and every KAT reach a Python node
    without a GPU as pyarrow arrays equal to the oracle's, with the oracle's sample bytes and
    ArrowTypeInfo.  The tokens return on receipt: a second round creates no slot."""
    import pyarrow as pa
    from dora_amd import device
    from dora_amd.dataflow import Dataflow
    from dora_amd.device import DeviceArray, DeviceBuffer
    from dora_amd.workloads import point_cloud
    from oracle.checksum_ref import payload_seed, splitmix_bytes
    from oracle.pack_ref import pack, sample_regions
    from tests.golden import recipes
    desc = {"nodes": [
        {"id": "src", "path": "dynamic", "outputs": ["x"]},
        {"id": "dst", "path": "dynamic", "inputs": {"x": {"source": "src/x", "queue_size": 10}},
         "_unstable_deploy": {"gpu": -1}},
    ]}
    sizes = [8, 4096, 1 << 20, 6220800, 40960000]
    s = device.Stream()
    bufs = {}
    for z in sizes:
        b = DeviceBuffer(z)
        device.fill_splitmix(b.ptr, z, payload_seed(z), s)
        bufs[z] = b
    s.sync()
    arrays = {m: recipes.build(m) for m in recipes.KATS + recipes.CASES}
    arrays["c3_cloud"] = point_cloud()
    dev_arrays = {m: DeviceArray.from_pyarrow(a) for m, a in arrays.items()}
    with Dataflow(desc, launcher=launcher) as df:
        n = _nodes(df, {"src": 0, "dst": -1})
        tx, rx = n["src"], n["dst"]
        created = []
        for rep in range(2):
            for z in sizes:
                tx.send_output_device_bytes("x", bufs[z].ptr, z, {"z": z, "rep": rep})
                ev = rx.next(timeout=60)
                assert ev["type"] == "INPUT" and ev["metadata"] == {"z": z, "rep": rep}
                assert not ev["on_device"], z
                want = splitmix_bytes(z, payload_seed(z))
                assert ctypes.string_at(ev["data_ptr"], ev["data_len"]) == want, (z, rep)
                v = ev["value"]
                assert isinstance(v, pa.Array) and v.type == pa.uint8(), type(v)
                assert v.equals(pa.array(np.frombuffer(want, np.uint8))), z
                assert ev["type_info"].to_json() == pack(v)[1].to_json(), z
                del ev, v
            for m, a in arrays.items():
                tx.send_output("x", dev_arrays[m], {"m": m, "rep": rep})
                ev = rx.next(timeout=60)
                assert ev["metadata"] == {"m": m, "rep": rep}
                want, info = pack(a)
                assert ev["type_info"].to_json() == info.to_json(), m
                if ev["data_len"]:
                    assert not ev["on_device"], m
                    # every buffer region byte for byte (padding between them is not written,
                    # stale in a recycled slot as in the reference's recycled shared memory)
                    got = ctypes.string_at(ev["data_ptr"], ev["data_len"])
                    assert len(got) == len(want), m
                    assert sample_regions(got, info) == sample_regions(want, info), m
                assert isinstance(ev["value"], pa.Array), m
                # an empty sample is ArrayData::new_empty(data_type) (event.rs:65-67)
                assert ev["value"].equals(a if ev["data_len"] else pa.array([], type=a.type)), m
                del ev
            _settle(tx, rx)
            created.append(tx.stats()["slots_created"])
        assert created[1] == created[0], created  # tokens came back: every slot was reused
        # the output's only receiver lacks a GPU: samples <= 1 MiB were packed by the producer
        # straight into shared memory, larger ones staged by the receiver's copy engines
        assert tx.host_paths()["host_packs"] >= 2 * 3, tx.host_paths()
        assert rx.host_paths()["staged"] >= 2 * 2, rx.host_paths()
        # the edge's latency (device 4 KB -> host receiver, one process), for the record
        lat = []
        for k in range(200):
            t0 = time.perf_counter()
            tx.send_output_device_bytes("x", bufs[4096].ptr, 4096, {"k": k})
            ev = rx.next(timeout=30)
            lat.append((time.perf_counter() - t0) * 1e6)
            del ev
        lat.sort()
        print(f"device 4 KB -> host-only receiver: p50 {lat[100]:.2f} us, p99 {lat[198]:.2f} us")
        tx.close()
        rx.close()
        df.wait(30)
    for a in dev_arrays.values():
        a.close()
    for b in bufs.values():
        b.free()
    s.close()


def test_host_only_receiver_staging_stress(launcher):
    """600 device messages of 8 B .. 1 MiB, each with new bytes (the source is rewritten after
    every synchronous send), reach a receiver without a GPU byte for byte over both host paths:
    output `x`, whose only receiver lacks a GPU, is packed by the producer straight into recycled
    shared-memory regions; output `y` also feeds a device receiver, so its sample stays in HBM and
    the host receiver stages it with the copy engines into a recycled pinned buffer (a stale or
    reused region or buffer would show)."""
    from dora_amd import device
    from dora_amd.dataflow import Dataflow
    from dora_amd.device import DeviceBuffer
    from oracle.checksum_ref import csum64, splitmix_bytes
    desc = {"nodes": [
        {"id": "src", "path": "dynamic", "outputs": ["x", "y"]},
        {"id": "dst", "path": "dynamic",
         "inputs": {"x": {"source": "src/x", "queue_size": 10},
                    "y": {"source": "src/y", "queue_size": 10}},
         "_unstable_deploy": {"gpu": -1}},
        {"id": "gpu", "path": "dynamic", "inputs": {"y": {"source": "src/y", "queue_size": 10}}},
    ]}
    sizes = [8, 100, 4096, 4097, 65539, (1 << 20) - 1, 1 << 20]
    s = device.Stream()
    buf = DeviceBuffer(1 << 20)
    with Dataflow(desc, launcher=launcher) as df:
        n = _nodes(df, {"src": 0, "dst": -1, "gpu": 0})
        tx, rx, gx = n["src"], n["dst"], n["gpu"]
        # AllNodesReady names x only: y also has a receiver with a GPU
        assert tx.host_bound_outputs() == ["x"]
        for k in range(600):
            z = sizes[k % len(sizes)]
            out = "x" if k % 2 == 0 else "y"
            device.fill_splitmix(buf.ptr, z, 0xABC000 + k, s)
            s.sync()
            tx.send_output_device_bytes(out, buf.ptr, z, {"k": k})
            want = splitmix_bytes(z, 0xABC000 + k)
            ev = rx.next(timeout=60)
            assert ev["id"] == out and ev["metadata"] == {"k": k} and not ev["on_device"]
            assert ctypes.string_at(ev["data_ptr"], z) == want, (k, z, out)
            del ev
            if out == "y":
                ev = gx.next(timeout=60)
                assert ev["on_device"] and device.csum64(ev["data_ptr"], z, s) == csum64(want)
                del ev
        assert tx.host_paths()["host_packs"] >= 300, tx.host_paths()
        assert rx.host_paths()["staged"] >= 300, rx.host_paths()
        # the staging edge's latency (device 4 KB -> host-only receiver beside a device one), for
        # the record
        lat = []
        for k in range(200):
            t0 = time.perf_counter()
            tx.send_output_device_bytes("y", buf.ptr, 4096, {"k": k})
            ev = rx.next(timeout=30)
            lat.append((time.perf_counter() - t0) * 1e6)
            del ev
            ev = gx.next(timeout=30)  # the device receiver's copy of the same message
            del ev
        lat.sort()
        print(f"device 4 KB -> host-only receiver, staged: p50 {lat[100]:.2f} us, "
              f"p99 {lat[198]:.2f} us")
        tx.close()
        rx.close()
        gx.close()
        df.wait(30)
    buf.free()
    s.close()


def test_host_source_to_host_only_receiver_copied_into_shared_memory(launcher):
    """A device node's host-resident bytes (>= 4096 B) on an output read only on the host are
    copied by the CPU into shared memory, as a node without a GPU sends them (the reference's
    copy_array_into_sample): no BAR write into an HBM slot, nothing staged at the receiver."""
    from dora_amd.dataflow import Dataflow
    from oracle.checksum_ref import splitmix_bytes
    desc = {"nodes": [
        {"id": "src", "path": "dynamic", "outputs": ["x"]},
        {"id": "dst", "path": "dynamic", "inputs": {"x": {"source": "src/x", "queue_size": 10}},
         "_unstable_deploy": {"gpu": -1}},
    ]}
    sizes = [100, 4096, 65539, 3 << 20]
    with Dataflow(desc, launcher=launcher) as df:
        n = _nodes(df, {"src": 0, "dst": -1})
        tx, rx = n["src"], n["dst"]
        t0, r0 = tx.host_paths(), rx.host_paths()
        for k in range(40):
            z = sizes[k % len(sizes)]
            want = splitmix_bytes(z, 0x5EED00 + k)
            tx.send_output("x", want, {"k": k})
            ev = rx.next(timeout=60)
            assert ev["metadata"] == {"k": k} and not ev["on_device"]
            assert ctypes.string_at(ev["data_ptr"], ev["data_len"]) == want, (k, z)
            del ev
        t1, r1 = tx.host_paths(), rx.host_paths()
        assert t1["host_packs"] - t0["host_packs"] == 30, t1  # the 30 sends >= 4096 B
        assert t1["bar_fills"] == t0["bar_fills"] and r1["staged"] == r0["staged"], (t1, r1)
        tx.close()
        rx.close()
        df.wait(30)


def test_host_sources_bar_and_dma_paths_bit_exact(launcher):
    """Host bytes of 4096, 4097, 1 MiB + 3, 2 MiB, 2 MiB + 1 and 40.96 MB, and multi-buffer host
    pyarrow arrays (a 20k-point cloud on the BAR path, the 1M-point C3 cloud on the DMA path),
    reach a device receiver byte-identical to the oracle.  Device-source sends of the same sizes
    interleave with them, so slots alternate between GPU packs and CPU writes through the BAR;
    every message is also checksummed by a kernel on the receiving side."""
    import pyarrow as pa
    from dora_amd import device
    from dora_amd.dataflow import Dataflow
    from dora_amd.device import DeviceBuffer
    from dora_amd.workloads import point_cloud
    from oracle.checksum_ref import csum64, payload_seed, splitmix_bytes
    from oracle.pack_ref import pack, sample_regions
    desc = {"nodes": [
        {"id": "src", "path": "dynamic", "outputs": ["x"]},
        {"id": "dst", "path": "dynamic", "inputs": {"x": {"source": "src/x", "queue_size": 100}}},
    ]}
    sizes = [4096, 4097, (1 << 20) + 3, 2 << 20, (2 << 20) + 1, 40960000]
    payloads = {z: splitmix_bytes(z, payload_seed(z) ^ 0x55) for z in sizes}
    s = device.Stream()
    dev_src = {}
    for z in sizes:
        b = DeviceBuffer(z)
        device.fill_splitmix(b.ptr, z, payload_seed(z), s)
        dev_src[z] = b
    s.sync()
    dev_want = {z: splitmix_bytes(z, payload_seed(z)) for z in sizes}
    clouds = {"small": point_cloud(n_points=20000, n_lists=7, seed=11), "c3": point_cloud()}
    with Dataflow(desc, launcher=launcher) as df:
        n = _nodes(df, {"src": 0, "dst": 0})
        tx, rx = n["src"], n["dst"]
        bar0 = tx.host_paths()["bar_fills"]
        for rep in range(3):
            for z in sizes:
                for kind in ("host", "device"):
                    if kind == "host":
                        tx.send_output("x", payloads[z], {"z": z, "k": kind})
                        want = payloads[z]
                    else:
                        tx.send_output_device_bytes("x", dev_src[z].ptr, z, {"z": z, "k": kind})
                        want = dev_want[z]
                    ev = rx.next(timeout=60)
                    assert ev["metadata"] == {"z": z, "k": kind} and ev["on_device"], (z, kind)
                    assert device.csum64(ev["data_ptr"], z, s) == csum64(want), (z, kind, rep)
                    if z < (4 << 20) or rep == 0:
                        assert _device_bytes(ev, s) == want, (z, kind, rep)
                    del ev
        # 4096 .. 2 MiB host sends went through the BAR (3 rounds of 4 sizes), the larger ones not
        assert tx.host_paths()["bar_fills"] - bar0 == 12, tx.host_paths()
        for name, cloud in clouds.items():
            want, info = pack(cloud)
            for rep in range(2):
                tx.send_output("x", cloud, {"cloud": name})
                ev = rx.next(timeout=60)
                assert ev["on_device"], name
                assert ev["type_info"].to_json() == info.to_json(), name
                got = _device_bytes(ev, s)
                assert len(got) == len(want), name
                assert sample_regions(got, info) == sample_regions(want, info), (name, rep)
                assert ev["value"].to_pyarrow().equals(cloud), name
                ev["value"].close()
                del ev
        assert tx.host_paths()["bar_fills"] - bar0 == 14, tx.host_paths()
        # the BAR path's latency: 4 KB host bytes, send -> receipt (one process)
        lat = []
        for k in range(300):
            t0 = time.perf_counter()
            tx.send_output("x", payloads[4096], {"k": k})
            ev = rx.next(timeout=30)
            lat.append((time.perf_counter() - t0) * 1e6)
            del ev
        lat.sort()
        print(f"host 4 KB (BAR) send->receipt: p50 {lat[150]:.2f} us, p99 {lat[297]:.2f} us")
        tx.close()
        rx.close()
        df.wait(30)
    for b in dev_src.values():
        b.free()
    s.close()


def test_sample_api_written_in_place_by_a_kernel(launcher, lib):
    """allocate_data_sample -> a kernel on the node stream writes the slot -> send_output_sample
    with ArrowTypeInfo::byte_array, through the C ABI (the reference benchmark's own path, F7).
    The receiver's bytes equal the oracle's splitmix bytes at 4096 B, 4 MiB and 40.96 MB, the
    sender never synchronises, slots recycle, and a sample that was already sent or discarded
    is refused."""
    from dora_amd import device
    from dora_amd._lib import DoraGpuError, call
    from dora_amd.arrow_utils import Plan
    from dora_amd.dataflow import Dataflow
    from oracle.checksum_ref import csum64, payload_seed, splitmix_bytes
    desc = {"nodes": [
        {"id": "src", "path": "dynamic", "outputs": ["x"]},
        {"id": "dst", "path": "dynamic", "inputs": {"x": {"source": "src/x", "queue_size": 10}}},
    ]}
    sizes = [4096, 4 << 20, 40960000]
    s = device.Stream()
    with Dataflow(desc, launcher=launcher) as df:
        n = _nodes(df, {"src": 0, "dst": 0})
        tx, rx = n["src"], n["dst"]
        nst = tx.stream  # the node stream: the payload kernels run there
        tis = {}
        created = []
        for rep in range(3):
            for z in sizes:
                smp = c_void_p()
                call("dora_node_allocate_data_sample", tx.handle, z, byref(smp))
                assert lib.dora_sample_len(smp) == z
                ptr = lib.dora_sample_data(smp)
                if z not in tis:  # ArrowTypeInfo::byte_array(z) (metadata.rs:74-87)
                    with Plan.of_bytes(ptr, z, True) as p:
                        tis[z] = p.type_info_bytes()
                call("dora_gpu_fill_splitmix", ptr, z, payload_seed(z), nst)
                call("dora_node_send_output_sample", tx.handle, b"x", tis[z], len(tis[z]),
                     b"", 0, smp)
                ev = rx.next(timeout=60)
                assert ev["on_device"] and ev["data_len"] == z, z
                want = splitmix_bytes(z, payload_seed(z))
                assert device.csum64(ev["data_ptr"], z, s) == csum64(want), (z, rep)
                if z <= (4 << 20):
                    assert _device_bytes(ev, s) == want, (z, rep)
                assert ev["type_info"].to_json()["data_type"] == "C"  # UInt8
                # the reference's error: the sample is consumed by the send
                with pytest.raises(DoraGpuError, match="already sent or discarded"):
                    call("dora_node_send_output_sample", tx.handle, b"x", tis[z], len(tis[z]),
                         b"", 0, smp)
                del ev
            _settle(tx, rx)
            created.append(tx.stats()["slots_created"])
        assert created[2] == created[1] == created[0], created
        # an unsent sample discarded twice: the second is refused, nothing is freed twice
        smp = c_void_p()
        call("dora_node_allocate_data_sample", tx.handle, 4096, byref(smp))
        lib.dora_sample_discard(tx.handle, smp)
        lib.dora_sample_discard(tx.handle, smp)
        assert b"already sent or discarded" in lib.dora_gpu_last_error()
        with pytest.raises(DoraGpuError, match="already sent or discarded"):
            call("dora_node_send_output_sample", tx.handle, b"x", tis[4096], len(tis[4096]),
                 b"", 0, smp)
        tx.close()
        rx.close()
        df.wait(30)
    s.close()
