"""AQL argument slots and the region-end stamp reduction (aql.cpp aql_stamp_reduce).

A timed region's end reduces the stamp areas of its command-processor-signalled packs with one AQL
dispatch whose arguments sit in the host argument ring.  When the wait for it times out the packet
may still run later, so its argument slot must never be handed to another pack: a later pack's
arguments there would be read by the reduction (and the reduction would write stamps through
them).  The hook makes the wait time out at once while the packet is still in flight; then more
than a whole ring of packs (512 slots) runs through every queue and each must arrive intact.
"""
import ctypes
import threading

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


def _abandoned():
    from dora_amd._lib import call
    n = ctypes.c_uint32()
    call("dora_gpu_test_abandoned_slots", 0, ctypes.byref(n))
    return n.value


def test_timed_out_stamp_reduction_keeps_its_argument_slot(launcher):
    from dora_amd import device
    from dora_amd._lib import call
    from dora_amd.dataflow import Dataflow
    from dora_amd.device import DeviceBuffer
    from oracle.checksum_ref import csum64, payload_seed, splitmix_bytes
    desc = {"nodes": [
        {"id": "src", "path": "dynamic", "outputs": ["x"]},
        {"id": "dst", "path": "dynamic", "inputs": {"x": {"source": "src/x", "queue_size": 100}}},
    ]}
    sizes = [4096, 65536, 1 << 20, 3 << 20, (4 << 20) + 7]
    s = device.Stream()
    bufs = {}
    for z in sizes:
        bufs[z] = DeviceBuffer(z)
        device.fill_splitmix(bufs[z].ptr, z, payload_seed(z), s)
    s.sync()
    want = {z: csum64(splitmix_bytes(z, payload_seed(z))) for z in sizes}
    with Dataflow(desc, launcher=launcher) as df:
        n = _nodes(df, {"src": 0, "dst": 0})
        tx, rx = n["src"], n["dst"]
        tx.send_output_device_bytes("x", bufs[4096].ptr, 4096, {"k": -1})  # queues, stamp areas
        rx.next(timeout=30)
        before = _abandoned()
        call("dora_gpu_test_reduce_timeout", 1)  # 1 ns: the wait times out, the packet runs on
        try:
            tx.region_begin()
            for k in range(6):  # CP-signalled packs (1-32 MiB): each takes a stamp area
                tx.send_output_device_bytes("x", bufs[3 << 20].ptr, 3 << 20, {"k": k})
                ev = rx.next(timeout=30)
                assert device.csum64(ev["data_ptr"], 3 << 20, s) == want[3 << 20]
                del ev
            tx.sync()
            r = tx.region_end()  # the reduction "times out": the stamps are read via the BAR
        finally:
            call("dora_gpu_test_reduce_timeout", 0)
        assert _abandoned() == before + 1
        assert r["packs"] == 6 and r["span_ms"] > 0, r
        # more than a whole argument ring of packs, synchronous and asynchronous, every size
        for k in range(700):
            z = sizes[k % len(sizes)]
            tx.send_output_device_bytes("x", bufs[z].ptr, z, {"k": k}, asynchronous=k % 3 == 0)
            ev = rx.next(timeout=30)
            assert ev["metadata"] == {"k": k}
            assert device.csum64(ev["data_ptr"], z, s) == want[z], (k, z)
            del ev
        # a region with the default wait: its reduction completes, nothing more is abandoned
        tx.region_begin()
        for k in range(4):
            tx.send_output_device_bytes("x", bufs[3 << 20].ptr, 3 << 20, {"k": 1000 + k})
            rx.next(timeout=30)
        tx.sync()
        assert tx.region_end()["packs"] == 4
        assert _abandoned() == before + 1
        tx.close()
        rx.close()
        df.wait(30)
    for b in bufs.values():
        b.free()
    s.close()
