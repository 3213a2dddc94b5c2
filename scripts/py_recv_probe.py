#!/usr/bin/env python3
"""The Python node's receive cost on the CPU (no GPU): an in-process daemon, a host-only sender
and receiver in this process; 20,000 inline 8-byte inputs drained with Node.next(), then 20,000
skipped by Node.wait_input.  us per event.

    python scripts/py_recv_probe.py
"""
import sys, time, os
import pyarrow
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
payload = b"12345678"
t0 = time.perf_counter()
for i in range(N):
    src.send_output("out", payload, {"seq": i})
t1 = time.perf_counter()
print("send us/msg", (t1 - t0) / N * 1e6)
time.sleep(0.5)
t0 = time.perf_counter()
got = 0
while got < N:
    ev = dst.next(timeout=5)
    if ev is None: break
    if ev["type"] == "INPUT": got += 1
t1 = time.perf_counter()
print("next() us/event", (t1 - t0) / got * 1e6, got)
for i in range(N):
    src.send_output("out", payload, {"seq": i})
time.sleep(0.5)
t0 = time.perf_counter()
m = dst.wait_input("in", "seq", N - 1, 30)
t1 = time.perf_counter()
print("wait_input skip us/event", (t1 - t0) / N * 1e6)
src.close(); dst.close(); d.join()
