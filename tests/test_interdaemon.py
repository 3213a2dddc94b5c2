"""Dataflows spanning machines: one daemon per machine, InterDaemonEvent::Output /
InputsClosed over TCP (libraries/message/src/daemon_to_daemon.rs:9-21, the remote branch of
send_out in binaries/daemon/src/lib.rs:955-1000), modelled on examples/multiple-daemons
(a source on one machine, its receivers on another).  CPU only: host-only nodes, inline and
shared-memory samples; the device-sample staging path is covered by tests/test_gpu_dataflow.py."""
import threading
import time

import numpy as np
import pytest

from dora_amd.dataflow import Dataflow, daemon_spec, parse_descriptor


def _desc(n_dst=1, queue_size=1000):
    nodes = [{"id": "src", "path": "dynamic", "outputs": ["data", "side"],
              "_unstable_deploy": {"machine": "A", "gpu": -1}},
             {"id": "local", "path": "dynamic", "inputs": {"side": "src/side"},
              "_unstable_deploy": {"machine": "A", "gpu": -1}}]
    for k in range(n_dst):
        nodes.append({"id": f"dst{k}", "path": "dynamic",
                      "inputs": {"data": {"source": "src/data", "queue_size": queue_size},
                                 "side": "src/side"},
                      "_unstable_deploy": {"machine": "B", "gpu": -1}})
    return {"nodes": nodes}


def test_spec_of_each_machine():
    nodes = parse_descriptor(_desc(2))
    a = daemon_spec(nodes, "A", {"A": ("127.0.0.1", 0), "B": ("127.0.0.1", 7000)}, "df")
    b = daemon_spec(nodes, "B", {"A": ("127.0.0.1", 7001), "B": ("127.0.0.1", 0)}, "df")
    assert "node src" in a and "node local" in a and "node dst0" not in a
    assert "remote src data B" in a and "remote src side B" in a
    assert "machine B 127.0.0.1 7000" in a and "listen 127.0.0.1 0" in a
    # B serves src as a proxy on the receivers' GPU (-1: host-only) with all its outputs
    assert "proxy src -1" in b and "output src data" in b and "output src side" in b
    assert "input dst1 data src data 1000" in b and "remote" not in b
    # single-machine descriptors are unchanged: every node local, no inter-daemon lines
    single = daemon_spec(parse_descriptor({"nodes": [{"id": "x", "outputs": ["o"]}]}))
    assert "proxy" not in single and "remote" not in single and "listen" not in single


def _open(df, nid):
    from dora_amd.node import Node
    return Node(nid, dataflow=df.shm, device=-1)


def test_two_daemons_deliver_in_order_and_close(tmp_path):
    """100 inline messages from machine A reach two receivers on machine B intact and in order,
    with their parameters and the producer's timestamps; closing the source's outputs on A
    closes the receivers' inputs on B, and both daemons finish."""
    desc = _desc(2)
    b = Dataflow(desc, machine="B", machines={"B": ("127.0.0.1", 0), "A": ("127.0.0.1", 1)},
                 dataflow_id="df-test", log_dir=str(tmp_path / "B")).start()
    a = Dataflow(desc, machine="A",
                 machines={"A": ("127.0.0.1", 0), "B": ("127.0.0.1", b.listen_port)},
                 dataflow_id="df-test", log_dir=str(tmp_path / "A")).start()
    got = {0: [], 1: []}
    closed = {0: [], 1: []}
    errs = []

    def receiver(k):
        try:
            n = _open(b, f"dst{k}")
            while True:
                ev = n.next(timeout=30)
                if ev is None:
                    break
                if ev["type"] == "INPUT":
                    got[k].append((ev["id"], ev["metadata"], ev["value"], ev["timestamp_ns"]))
                elif ev["type"] == "INPUT_CLOSED":
                    closed[k].append(ev["id"])
            n.close()
        except Exception as e:  # noqa: BLE001
            errs.append(e)
    ts = [threading.Thread(target=receiver, args=(k,)) for k in (0, 1)]
    for t in ts:
        t.start()
    try:
        box = {}
        lt = threading.Thread(target=lambda: box.update(local=_open(a, "local")))
        lt.start()
        src = _open(a, "src")
        lt.join(30)
        # receivers on another machine keep an output off the host-bound list of AllNodesReady
        # (daemon.cpp ready_payload): "side" also has a local host-only receiver
        assert src.host_bound_outputs() == []
        sent = []
        for i in range(100):
            # every tenth message >= 4096 B: a shared-memory sample on A (read by the
            # forwarder) and on B (written by the host-only proxy)
            n_b = 16 + 37 * i % 3000 if i % 10 else 4096 + 997 * i
            payload = bytes((i * 7 + j) & 0xFF for j in range(n_b))
            t0 = time.time_ns()
            src.send_output("data", payload, {"seq": i, "tag": f"m{i}"})
            sent.append((payload, t0))
        src.send_output("side", b"x" * 10, {"last": True})
        ev = box["local"].next(timeout=30)  # the same output's local receiver, unaffected
        assert ev["type"] == "INPUT" and ev["metadata"] == {"last": True}
        src.close()
        box["local"].close()
        for t in ts:
            t.join(60)
        codes = {"A": a.wait(30), "B": b.wait(30)}
    finally:
        a.stop()
        b.stop()
    assert not errs, errs
    for k in (0, 1):
        data = [g for g in got[k] if g[0] == "data"]
        assert [g[1]["seq"] for g in data] == list(range(100))
        for (pid, meta, value, ts_ns), (payload, t0) in zip(data, sent):
            assert np.asarray(value).tobytes() == payload and meta["tag"] == f"m{meta['seq']}"
            assert ts_ns >= t0 - 1000  # the producer's timestamp travels with the message
        side = [g for g in got[k] if g[0] == "side"]
        assert len(side) == 1 and side[0][1] == {"last": True}
        assert sorted(closed[k]) == ["data", "side"]
    assert codes["A"]["_daemon"] == 0 and codes["B"]["_daemon"] == 0, codes
    # one frame per message for machine B whatever its receiver count: 101 outputs + 2 closes
    assert '"forwarded": 103' in a.log("_daemon"), a.log("_daemon")
    assert '"remote_received": 103' in b.log("_daemon"), b.log("_daemon")


def test_wrong_dataflow_id_is_ignored(tmp_path):
    """A peer of another dataflow (different id) cannot inject messages."""
    desc = _desc(1)
    b = Dataflow(desc, machine="B", machines={"B": ("127.0.0.1", 0), "A": ("127.0.0.1", 1)},
                 dataflow_id="df-one", log_dir=str(tmp_path / "B")).start()
    a = Dataflow(desc, machine="A",
                 machines={"A": ("127.0.0.1", 0), "B": ("127.0.0.1", b.listen_port)},
                 dataflow_id="df-two", log_dir=str(tmp_path / "A")).start()
    try:
        box = {}
        lt = threading.Thread(target=lambda: box.update(local=_open(a, "local")))
        lt.start()
        rt = threading.Thread(target=lambda: box.update(dst=_open(b, "dst0")))
        rt.start()
        src = _open(a, "src")
        lt.join(30)
        rt.join(30)
        src.send_output("data", b"hello", {"seq": 1})
        assert box["dst"].next(timeout=2) is None  # nothing arrives (timeout)
        src.close()
        box["local"].close()
    finally:
        a.stop()
        b.stop()
    assert "ignored" in b.log("_daemon")


def test_crashed_peer_daemon_closes_remote_inputs(tmp_path, monkeypatch):
    """A remote daemon that dies without sending InputsClosed (killed) must not strand the
    local receivers: once every peer connection has been gone for the grace period
    (DORA_GPU_PEER_GRACE_MS) the proxy closes its outputs and the local dataflow finishes.
    The reference only ends the connection's read loop on EOF/reset
    (binaries/daemon/src/inter_daemon.rs:136-139) and leaves the receivers waiting; here the
    receivers see INPUT_CLOSED (a deliberate deviation)."""
    monkeypatch.setenv("DORA_GPU_PEER_GRACE_MS", "300")
    desc = _desc(1)
    b = Dataflow(desc, machine="B", machines={"B": ("127.0.0.1", 0), "A": ("127.0.0.1", 1)},
                 dataflow_id="df-crash", log_dir=str(tmp_path / "B")).start()
    a = Dataflow(desc, machine="A",
                 machines={"A": ("127.0.0.1", 0), "B": ("127.0.0.1", b.listen_port)},
                 dataflow_id="df-crash", log_dir=str(tmp_path / "A")).start()
    try:
        box = {}
        lt = threading.Thread(target=lambda: box.update(local=_open(a, "local")))
        lt.start()
        rt = threading.Thread(target=lambda: box.update(dst=_open(b, "dst0")))
        rt.start()
        src = _open(a, "src")
        lt.join(30)
        rt.join(30)
        for i in range(5):
            src.send_output("data", bytes([i]) * 100, {"seq": i})
        dst = box["dst"]
        seqs = []
        while len(seqs) < 5:
            ev = dst.next(timeout=30)
            assert ev is not None and ev["type"] == "INPUT", ev
            seqs.append(ev["metadata"]["seq"])
        assert seqs == list(range(5))
        a.daemon.kill()  # no InputsClosed ever leaves machine A
        t0 = time.time()
        closed = set()
        while closed != {"data", "side"}:
            ev = dst.next(timeout=30)
            assert ev is not None, "remote inputs never closed after the peer daemon died"
            if ev["type"] == "INPUT_CLOSED":
                closed.add(ev["id"])
        assert time.time() - t0 < 20
        dst.close()
        assert b.wait(30)["_daemon"] == 0, b.log("_daemon")
    finally:
        a.stop()
        b.stop()
    assert "gone; closing its outputs" in b.log("_daemon")


def test_oversized_frame_is_refused_per_message(tmp_path, monkeypatch):
    """A message whose frame exceeds the inter-daemon limit (DORA_GPU_MAX_FRAME_BYTES, lowered
    here to 2048 B) is refused by the forwarder with an error naming it: the link
    stays up, so the messages behind it and the InputsClosed still arrive."""
    monkeypatch.setenv("DORA_GPU_MAX_FRAME_BYTES", "2048")
    desc = _desc(1)
    b = Dataflow(desc, machine="B", machines={"B": ("127.0.0.1", 0), "A": ("127.0.0.1", 1)},
                 dataflow_id="df-big", log_dir=str(tmp_path / "B")).start()
    a = Dataflow(desc, machine="A",
                 machines={"A": ("127.0.0.1", 0), "B": ("127.0.0.1", b.listen_port)},
                 dataflow_id="df-big", log_dir=str(tmp_path / "A")).start()
    try:
        box = {}
        lt = threading.Thread(target=lambda: box.update(local=_open(a, "local")))
        lt.start()
        rt = threading.Thread(target=lambda: box.update(dst=_open(b, "dst0")))
        rt.start()
        src = _open(a, "src")
        lt.join(30)
        rt.join(30)
        src.send_output("data", b"a" * 100, {"seq": 0})
        src.send_output("data", b"b" * 3000, {"seq": 1})   # frame > 2048 B: refused
        src.send_output("data", b"c" * 100, {"seq": 2})
        src.close()
        box["local"].close()
        dst = box["dst"]
        seqs, closed = [], set()
        while True:
            ev = dst.next(timeout=30)
            if ev is None:
                break
            if ev["type"] == "INPUT":
                seqs.append(ev["metadata"]["seq"])
            elif ev["type"] == "INPUT_CLOSED":
                closed.add(ev["id"])
        dst.close()
        codes = {"A": a.wait(30), "B": b.wait(30)}
    finally:
        a.stop()
        b.stop()
    assert seqs == [0, 2] and closed == {"data", "side"}
    assert codes["A"]["_daemon"] == 0 and codes["B"]["_daemon"] == 0, codes
    assert "exceeds the inter-daemon frame limit" in a.log("_daemon")
    assert "refused" not in b.log("_daemon")
