"""Armed lone dispatch (aql.cpp arm_locked).

A lone single-segment pack (a synchronous send, or one that finds every queue idle, < 1 MiB) can
leave through a pair written ahead on a queue of its own — a barrier-AND waiting on a host signal
and the pack's dispatch packet behind it — with its arguments written into the pair's slot and
the barrier released at send time.  Every message must arrive intact whichever way it left:
repeated sizes (the pair is used), alternating sizes (the pair is released unused), pipelined
bursts in between (a pipelined pack releases the pair), over more than one argument ring (the
pair's slot is skipped while armed), and with the mechanism switched off again.
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


def _stats():
    from dora_amd._lib import call
    v = (ctypes.c_uint64 * 3)()
    call("dora_gpu_test_arm_stats", 0, v)
    return {"hits": v[0], "misses": v[1], "arms": v[2]}


def test_armed_lone_packs_arrive_intact(launcher):
    from dora_amd import device
    from dora_amd._lib import call
    from dora_amd.dataflow import Dataflow
    from dora_amd.device import DeviceBuffer
    from oracle.checksum_ref import csum64, payload_seed, splitmix_bytes
    desc = {"nodes": [
        {"id": "src", "path": "dynamic", "outputs": ["x"]},
        {"id": "dst", "path": "dynamic", "inputs": {"x": {"source": "src/x", "queue_size": 100}}},
    ]}
    sizes = [8, 4093, 4096, 65536, 300001, (1 << 20) - 3]
    s = device.Stream()
    bufs = {}
    for z in sizes:
        bufs[z] = DeviceBuffer(z)
        device.fill_splitmix(bufs[z].ptr, z, payload_seed(z), s)
    s.sync()
    want = {z: csum64(splitmix_bytes(z, payload_seed(z))) for z in sizes}
    call("dora_gpu_test_armed", 1)
    try:
        with Dataflow(desc, launcher=launcher) as df:
            n = _nodes(df, {"src": 0, "dst": 0})
            tx, rx = n["src"], n["dst"]
            before = _stats()
            k = 0

            def one(z, asynchronous=False):
                nonlocal k
                tx.send_output_device_bytes("x", bufs[z].ptr, z, {"k": k},
                                            asynchronous=asynchronous)
                k += 1

            def drain(m):
                for _ in range(m):
                    ev = rx.next(timeout=30)
                    got = device.csum64(ev["data_ptr"], ev["data_len"], s)
                    assert got == want[ev["data_len"]], (ev["metadata"], ev["data_len"])
                    del ev

            # repeated sizes, one at a time: the pair is armed for the next message of the size
            for z in sizes:
                for _ in range(40):
                    one(z)
                    drain(1)
            # alternating sizes: every pair is released unused
            for r in range(60):
                one(sizes[r % len(sizes)])
                drain(1)
            # bursts of asynchronous sends between lone ones
            for r in range(30):
                one(4096)
                drain(1)
                for _ in range(8):
                    one(65536, asynchronous=True)
                drain(8)
                one(4096)
                drain(1)
            # more than one argument ring (512 slots) of lone packs
            for r in range(600):
                one(sizes[(r // 5) % len(sizes)])
                drain(1)
            st = _stats()
            assert st["hits"] - before["hits"] > 500, st
            assert st["misses"] - before["misses"] > 50, st
            tx.close()
            rx.close()
            df.wait(30)
    finally:
        call("dora_gpu_test_armed", 0)
    # off again: lone packs take the queues, and a pair is no longer written
    desc2 = {"nodes": [
        {"id": "src2", "path": "dynamic", "outputs": ["x"]},
        {"id": "dst2", "path": "dynamic",
         "inputs": {"x": {"source": "src2/x", "queue_size": 10}}},
    ]}
    with Dataflow(desc2, launcher=launcher) as df:
        n = _nodes(df, {"src2": 0, "dst2": 0})
        tx, rx = n["src2"], n["dst2"]
        a0 = _stats()["arms"]
        for r in range(20):
            tx.send_output_device_bytes("x", bufs[4096].ptr, 4096, {"k": r})
            ev = rx.next(timeout=30)
            assert device.csum64(ev["data_ptr"], 4096, s) == want[4096]
            del ev
        assert _stats()["arms"] == a0
        tx.close()
        rx.close()
        df.wait(30)
    for b in bufs.values():
        b.free()
    s.close()
