"""Host-resident samples on the device data plane (verdict r04 items 1 and 5).

* A device node's host-source payloads below the zero-copy threshold travel inline as
  `DataMessage::Vec` — the reference's allocate_data_sample (apis/rust/node/src/node/mod.rs:40,
  303-319): no slot, no H2D copy, no fill signal.  Every size 1..4095 class arrives byte-identical
  to the oracle's copy_array_into_sample (oracle/pack_ref.py), and 4096 B takes the device slot
  (written by the CPU through the BAR).
* A host-only node's samples >= 4096 B are `DataMessage::SharedMemory` regions (mod.rs:321-346);
  a device receiver pulls them into HBM by DMA and returns the token at once.
"""
import ctypes
import threading
import time

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _nodes(df, spec):
    """Start the dynamic nodes {id: device} of `df` concurrently (each init waits for
    AllNodesReady)."""
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


def test_host_small_payloads_go_inline_bit_exact(launcher):
    """Host bytes and host pyarrow arrays of 1..4095 B from a device node reach a device receiver
    as inline samples equal to the oracle's, with the oracle's ArrowTypeInfo; no pack runs for
    them, and 4096 B (the threshold itself) is a device sample."""
    import pyarrow as pa
    from dora_amd import device
    from dora_amd.dataflow import Dataflow
    from oracle.pack_ref import pack
    from tests.golden import recipes
    desc = {"nodes": [
        {"id": "src", "path": "dynamic", "outputs": ["x"]},
        {"id": "dst", "path": "dynamic", "inputs": {"x": {"source": "src/x", "queue_size": 100}}},
    ]}
    sizes = [1, 2, 3, 7, 8, 15, 16, 17, 63, 64, 65, 127, 128, 129, 511, 512, 1000, 2047, 2048,
             3001, 4000, 4094, 4095, 4096]
    rng = np.random.default_rng(5)
    s = device.Stream()
    with Dataflow(desc, launcher=launcher) as df:
        n = _nodes(df, {"src": 0, "dst": 0})
        tx, rx = n["src"], n["dst"]
        paths0 = tx.fill_paths()
        bar0 = tx.host_paths()["bar_fills"]
        for z in sizes:
            payload = rng.integers(0, 256, z, dtype=np.uint8).tobytes()
            want, info = pack(pa.array(np.frombuffer(payload, np.uint8), pa.uint8()))
            tx.send_output("x", payload, {"z": z})
            ev = rx.next(timeout=30)
            assert ev["type"] == "INPUT" and ev["metadata"] == {"z": z}
            assert ev["type_info"].to_json() == info.to_json(), z
            if z < 4096:
                assert not ev["on_device"], z
                assert ctypes.string_at(ev["data_ptr"], ev["data_len"]) == want, z
                assert np.asarray(ev["value"]).tobytes() == payload, z
            else:
                assert ev["on_device"], z
                assert _device_bytes(ev, s) == want, z
            del ev
        paths1 = tx.fill_paths()
        # nothing was packed: the 4096-B message went into its slot by CPU stores through the
        # BAR (node.cpp host_bar_fill), the rest inline
        assert paths1 == paths0, paths1
        assert tx.host_paths()["bar_fills"] - bar0 == 1, tx.host_paths()
        # host pyarrow arrays whose sample is < 4096 B (the reference's own KATs and fixtures)
        names = [m for m in recipes.KATS + recipes.CASES if len(pack(recipes.build(m))[0]) < 4096]
        assert len(names) >= 10, names
        for m in names:
            arr = recipes.build(m)
            want, info = pack(arr)
            tx.send_output("x", arr, {"m": m})
            ev = rx.next(timeout=30)
            assert ev["metadata"] == {"m": m}
            assert ev["type_info"].to_json() == info.to_json(), m
            if ev["data_len"]:
                assert not ev["on_device"], m
                assert ctypes.string_at(ev["data_ptr"], ev["data_len"]) == want, m
                assert ev["value"].equals(arr), m
            del ev
        assert tx.fill_paths() == paths1
        # the inline path's latency: 200 host 8-B messages, send -> receipt
        lat = []
        for k in range(200):
            t0 = time.perf_counter()
            tx.send_output("x", b"\x01" * 8, {"k": k})
            ev = rx.next(timeout=30)
            lat.append((time.perf_counter() - t0) * 1e6)
            del ev
        lat.sort()
        print(f"inline 8 B send->receipt (one process): p50 {lat[100]:.2f} us, p99 {lat[198]:.2f} us")
        tx.close()
        rx.close()
        df.wait(30)
    s.close()


def test_host_only_node_shared_memory_to_device_receiver(launcher):
    """A host-only node (DORA_GPU_DEVICE < 0) sends 4096 B, 1 MiB and 40.96 MB as shared-memory
    samples; a device receiver pulls each into HBM by DMA and the bytes equal the oracle's.  The
    tokens return on the pull, so a second round reuses the sender's regions."""
    import pyarrow as pa
    from dora_amd import device
    from dora_amd.dataflow import Dataflow
    from oracle.checksum_ref import payload_seed, splitmix_bytes
    from oracle.pack_ref import pack
    desc = {"nodes": [
        {"id": "src", "path": "dynamic", "outputs": ["x"], "_unstable_deploy": {"gpu": -1}},
        {"id": "dst", "path": "dynamic", "inputs": {"x": {"source": "src/x", "queue_size": 10}}},
    ]}
    sizes = [4096, 1 << 20, 40960000, 4099]
    payloads = {z: splitmix_bytes(z, payload_seed(z)) for z in sizes}
    wants = {z: pack(pa.array(np.frombuffer(payloads[z], np.uint8), pa.uint8())) for z in sizes}
    s = device.Stream()
    with Dataflow(desc, launcher=launcher) as df:
        n = _nodes(df, {"src": -1, "dst": 0})
        tx, rx = n["src"], n["dst"]
        for rep in range(2):
            for z in sizes:
                tx.send_output("x", payloads[z], {"z": z, "rep": rep})
                ev = rx.next(timeout=60)
                assert ev["type"] == "INPUT" and ev["metadata"] == {"z": z, "rep": rep}
                assert ev["on_device"], z
                want, info = wants[z]
                assert ev["type_info"].to_json() == info.to_json(), z
                assert _device_bytes(ev, s) == want, (z, rep)
                v = ev["value"]
                assert v.to_pyarrow().equals(pa.array(np.frombuffer(payloads[z], np.uint8))), z
                v.close()
                del ev, v
                time.sleep(0.05)  # the pull returned the token: let it reach the sender
        deadline = time.time() + 10
        while tx.stats()["in_flight"] and time.time() < deadline:
            tx.send_output("x", b"", {"z": 0, "rep": -1})  # handles the returned tokens
            rx.next(timeout=10)
        st = tx.stats()
        assert st["in_flight"] == 0, st
        # one region per size of the first round; 4099 B takes the best-fitting larger region,
        # and the second round creates none
        assert st["slots_created"] == 3 and st["cache_hits"] >= 5, st
        # the edge's latency (host-only 4 KB -> device receiver, pulled on receipt), for the record
        lat = []
        for k in range(200):
            t0 = time.perf_counter()
            tx.send_output("x", payloads[4096], {"k": k})
            ev = rx.next(timeout=30)
            lat.append((time.perf_counter() - t0) * 1e6)
            del ev
        lat.sort()
        print(f"host-only 4 KB -> device receiver, pulled: p50 {lat[100]:.2f} us, "
              f"p99 {lat[198]:.2f} us")
        tx.close()
        rx.close()
        df.wait(30)
    s.close()
