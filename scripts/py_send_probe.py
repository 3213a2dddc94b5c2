#!/usr/bin/env python3
"""The Python node's send and receive costs by data kind on the CPU (no GPU): an in-process
daemon, host-only sender and receiver in this process; 20,000 sends each of a UInt8 pyarrow
array (100 values), a Struct<x:f32,i:u8> array (50 rows) and 100 bytes, then the receiver's
next() over them.  us per message.

    python scripts/py_send_probe.py
"""
import sys, time, os
import pyarrow as pa
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
from test_dataflow_host import InProcessDaemon, _start_nodes
DESC = {"nodes": [
    {"id": "src", "outputs": ["out"]},
    {"id": "dst", "inputs": {"in": {"source": "src/out", "queue_size": 100000}}, "outputs": []},
]}
d = InProcessDaemon(DESC)
nodes = _start_nodes(d.shm, ["src", "dst"])
src, dst = nodes["src"], nodes["dst"]
N = 20000
arr = pa.array(list(range(100)), type=pa.uint8())
st = pa.StructArray.from_arrays([pa.array([1.0]*50, pa.float32()), pa.array([1]*50, pa.uint8())], names=["x","i"])
for name, a in (("uint8x100", arr), ("struct50", st), ("bytes100", bytes(100))):
    t0 = time.perf_counter()
    for i in range(N):
        src.send_output("out", a, {"seq": i})
    t1 = time.perf_counter()
    print(name, "send us/msg", round((t1 - t0) / N * 1e6, 2))
    got = 0
    t0 = time.perf_counter()
    while got < N:
        ev = dst.next(timeout=5)
        if ev is None: break
        got += ev["type"] == "INPUT"
    print(name, "next us/event", round((time.perf_counter() - t0) / N * 1e6, 2))
src.close(); dst.close(); d.join()
