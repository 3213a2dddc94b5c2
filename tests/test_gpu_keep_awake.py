"""The keep-awake thread (aql.cpp warm_main, dora_gpu_set_keep_awake): while a node sends device
samples it publishes empty AQL packets whenever nothing was dispatched for one period, parks
100 ms after the last send, wakes with the next one, and stops when the period is set to 0.  A
slow periodic sender (three sends in a row > 5 ms apart) has it park 200 us after each send
instead, until a quicker send."""
import ctypes
import time

import pytest

pytestmark = pytest.mark.gpu


def _stats():
    from dora_amd._lib import call
    beats, parked = ctypes.c_uint64(), ctypes.c_int()
    call("dora_gpu_test_keep_awake_stats", 0, ctypes.byref(beats), ctypes.byref(parked))
    return beats.value, bool(parked.value)


def _wait_parked(limit=2.0):
    t = time.time() + limit
    while time.time() < t:
        if _stats()[1]:
            return True
        time.sleep(0.02)
    return False


def test_keep_awake_beats_while_sending_then_parks(tmp_path):
    from dora_amd import device
    from dora_amd.dataflow import Dataflow
    from dora_amd.node import Node
    desc = {"nodes": [
        {"id": "node", "path": "dynamic", "outputs": ["latency"], "inputs": {"ack": "sink/ack"}},
        {"id": "sink", "path": "dora-gpu-bench-sink", "outputs": ["ack"],
         "inputs": {"latency": {"source": "node/latency", "queue_size": 10}},
         "env": {"DORA_BENCH_RESULT": str(tmp_path / "sink.json")}},
    ]}
    device.set_keep_awake(25)
    try:
        with Dataflow(desc) as df:
            node = Node("node", dataflow=df.shm, device=0)
            buf = device.DeviceBuffer(4096)
            # the thread is the process's: quick sends first, whatever earlier tests sent
            for k in range(5):
                node.send_output_device_bytes("latency", buf.ptr, 4096, {"seq": 100 + k})
                time.sleep(0.001)
            node.send_output_device_bytes("latency", buf.ptr, 4096, {"seq": 0})
            b0, _ = _stats()
            time.sleep(0.03)
            b1, parked = _stats()
            # 30 ms at one packet per 25 us is ~1200; a loaded host wakes the thread late
            assert b1 - b0 > 50 and not parked, (b0, b1, parked)
            assert _wait_parked(), "still beating long after the last send"
            b2, _ = _stats()
            time.sleep(0.05)
            b3, parked = _stats()
            assert parked and b3 - b2 <= 2, (b2, b3)
            node.send_output_device_bytes("latency", buf.ptr, 4096, {"seq": 1})  # wakes it
            time.sleep(0.03)
            b4, parked = _stats()
            assert b4 - b3 > 50 and not parked, (b3, b4, parked)
            device.set_keep_awake(0)
            time.sleep(0.03)
            b5, _ = _stats()
            node.send_output_device_bytes("latency", buf.ptr, 4096, {"seq": 2})
            time.sleep(0.05)
            b6, _ = _stats()
            assert b6 - b5 <= 1, (b5, b6)
            node.send_output("latency", b"", {"seq": 3, "ack": True})
            node.wait_input("ack", "seq", 3, 30.0)
            buf.free()
            node.close()
            assert df.wait(30)["sink"] == 0, df.log("sink")
    finally:
        device.set_keep_awake(25)


def test_slow_periodic_sender_parks_after_each_send(tmp_path):
    from dora_amd import device
    from dora_amd.dataflow import Dataflow
    from dora_amd.node import Node
    desc = {"nodes": [
        {"id": "node", "path": "dynamic", "outputs": ["latency"], "inputs": {"ack": "sink/ack"}},
        {"id": "sink", "path": "dora-gpu-bench-sink", "outputs": ["ack"],
         "inputs": {"latency": {"source": "node/latency", "queue_size": 10}},
         "env": {"DORA_BENCH_RESULT": str(tmp_path / "sink.json")}},
    ]}
    device.set_keep_awake(25)
    with Dataflow(desc) as df:
        node = Node("node", dataflow=df.shm, device=0)
        buf = device.DeviceBuffer(4096)
        seq = 0
        for _ in range(5):  # 30 ms apart: slow from the fourth on
            node.send_output_device_bytes("latency", buf.ptr, 4096, {"seq": seq})
            seq += 1
            time.sleep(0.03)
        b0, _ = _stats()
        node.send_output_device_bytes("latency", buf.ptr, 4096, {"seq": seq})
        seq += 1
        time.sleep(0.03)
        b1, parked = _stats()
        # 200 us at one packet per 25 us is ~8; a whole 30 ms awake would be ~1200
        assert parked and b1 - b0 <= 60, (b0, b1, parked)
        for _ in range(6):  # 1 ms apart: the 100 ms window again
            node.send_output_device_bytes("latency", buf.ptr, 4096, {"seq": seq})
            seq += 1
            time.sleep(0.001)
        b2, _ = _stats()
        time.sleep(0.03)
        b3, parked = _stats()
        assert b3 - b2 > 50 and not parked, (b2, b3, parked)
        node.send_output("latency", b"", {"seq": seq, "ack": True})
        node.wait_input("ack", "seq", seq, 30.0)
        buf.free()
        node.close()
        assert df.wait(30)["sink"] == 0, df.log("sink")
