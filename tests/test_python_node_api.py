"""The Python `Node` against the reference's (verdict r05 item 5): every method of the reference's
`#[pymethods] impl Node` (apis/python/node/src/lib.rs:41-210, restated as data in
tests/golden/python_node_api.json by tests/golden/make_python_api.py) exists on
dora_amd.node.Node with the same parameters in the same order and the same defaults present;
parameters added here are optional.  Iteration follows the reference (`__iter__` is the node,
`__next__` ends the loop when the stream has), and `dataflow_id()` / `dataflow_descriptor()`
answer on a running dataflow (host-only nodes, no GPU)."""
import inspect
import json
import os
import threading

import pytest

from dora_amd.node import Node

GOLDEN = os.path.join(os.path.dirname(__file__), "golden", "python_node_api.json")


def _params(fn):
    return [p for p in inspect.signature(fn).parameters.values() if p.name != "self"]


def test_node_has_every_reference_method_with_its_parameters():
    ref = json.load(open(GOLDEN))["methods"]
    assert set(ref) == {"__init__", "next", "__next__", "__iter__", "send_output",
                        "dataflow_descriptor", "dataflow_id", "merge_external_events"}
    for name, want in ref.items():
        assert hasattr(Node, name), name
        got = _params(getattr(Node, name))
        assert [p.name for p in got[:len(want)]] == [w["name"] for w in want], name
        for w, p in zip(want, got):
            if w["has_default"]:
                assert p.default is None, (name, p.name)  # every reference default is None
            else:
                assert p.default is inspect.Parameter.empty, (name, p.name)
        for p in got[len(want):]:  # ours only: optional
            assert p.default is not inspect.Parameter.empty or \
                p.kind in (p.VAR_KEYWORD, p.VAR_POSITIONAL), (name, p.name)


def test_iteration_follows_the_reference():
    n = Node.__new__(Node)
    events = [{"type": "INPUT", "id": "a"}, {"type": "INPUT", "id": "b"}, None]
    n.next = lambda timeout=None: events.pop(0)
    assert iter(n) is n
    assert next(n)["id"] == "a"
    assert [e["id"] for e in n] == ["b"]
    with pytest.raises(StopIteration):
        next(Node.__new__(Node) if False else _ended())


def _ended():
    n = Node.__new__(Node)
    n.next = lambda timeout=None: None
    return n


def test_merge_external_events_is_refused():
    with pytest.raises(NotImplementedError, match="ROS2"):
        Node.__new__(Node).merge_external_events(object())


def test_dataflow_id_and_descriptor_of_a_running_dataflow(tmp_path):
    from dora_amd.dataflow import Dataflow, dataflow_uuid
    desc = {"nodes": [
        {"id": "src", "path": "dynamic", "outputs": ["out"], "_unstable_deploy": {"gpu": -1}},
        {"id": "dst", "path": "dynamic", "inputs": {"in": {"source": "src/out", "queue_size": 3}},
         "_unstable_deploy": {"gpu": -1}},
    ]}
    with Dataflow(desc, log_dir=str(tmp_path), dataflow_id="camera-rig") as df:
        out = {}

        def mk(i):
            out[i] = Node(i, dataflow=df.shm, device=-1)
        ts = [threading.Thread(target=mk, args=(i,)) for i in ("src", "dst")]
        [t.start() for t in ts]
        [t.join(20) for t in ts]
        src, dst = out["src"], out["dst"]
        assert src.id == "src" and dst.id == "dst"
        assert src.dataflow_id() == dst.dataflow_id() == dataflow_uuid("camera-rig")
        assert src.dataflow_descriptor() == desc
        src.send_output("out", b"\x01\x02\x03", {"k": 1})
        ev = next(dst)
        assert ev["type"] == "INPUT" and ev["metadata"] == {"k": 1}
        src.close()
        assert [e["type"] for e in dst] == ["INPUT_CLOSED"]  # then the stream ends
        dst.close()
        df.wait(20)
