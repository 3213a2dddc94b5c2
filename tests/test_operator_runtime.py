"""Runtime nodes (the operator callers of the packing boundary,
binaries/runtime/src/operator/{shared_lib,python}.rs): a shared-library operator in
dora-gpu-runtime and a Python operator in dora_amd.operator_runtime, fed by a node of this
process and read back by another.  Host-only nodes here (inline samples, no GPU); the same
graphs with device samples run under -m gpu."""
import os
import subprocess
import threading

import pyarrow as pa
import pytest

from dora_amd.dataflow import Dataflow, parse_descriptor, shared_library_path
from dora_amd.node import Node
from dora_amd.operator_runtime import host_value

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OPS = os.path.join(ROOT, "tests", "operators")


def open_nodes(df, ids, gpu):
    """Attach several dynamic nodes of this process: each init waits for AllNodesReady, so they
    subscribe from threads of their own."""
    out, errs = {}, []

    def attach(i):
        try:
            out[i] = Node(i, dataflow=df.shm, device=gpu)
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    ts = [threading.Thread(target=attach, args=(i,)) for i in ids]
    for t in ts:
        t.start()
    for t in ts:
        t.join(90)
    if errs:
        raise errs[0]
    return [out[i] for i in ids]


def build_counter_op(tmp_path) -> str:
    """Compile tests/operators/counter_op.c against include/dora_operator_api.h."""
    so = tmp_path / "libcounter.so"
    subprocess.run(["gcc", "-shared", "-fPIC", "-O2", "-Wall", f"-I{ROOT}/include",
                    os.path.join(OPS, "counter_op.c"), "-o", str(so),
                    f"-L{ROOT}/dora_amd/lib", "-ldora_gpu"], check=True)
    return str(tmp_path / "counter")


def counter_desc(lib: str, gpu: int) -> dict:
    return {"nodes": [
        {"id": "src", "path": "dynamic", "outputs": ["message", "table", "stop"],
         "_unstable_deploy": {"gpu": gpu}},
        {"id": "rt", "operators": [
            {"id": "counter", "shared-library": lib,
             "inputs": {"message": "src/message", "table": "src/table", "stop": "src/stop"},
             "outputs": ["counter", "echo", "same"]}],
         "_unstable_deploy": {"gpu": gpu}},
        {"id": "sink", "path": "dynamic", "_unstable_deploy": {"gpu": gpu},
         "inputs": {"counter": "rt/counter/counter", "echo": "rt/counter/echo",
                    "same": "rt/counter/same"}},
    ]}


def _drain(sink):
    """Every input of `sink` as (host pyarrow array, metadata) per input id."""
    got = {}
    while True:
        ev = sink.next(timeout=30)
        if ev is None:
            return got
        if ev["type"] == "INPUT":
            got.setdefault(ev["id"], []).append((host_value(ev), ev["metadata"]))


def run_counter(tmp_path, gpu: int, payloads):
    lib = build_counter_op(tmp_path)
    table = pa.StructArray.from_arrays(
        [pa.array([1, None, 3], pa.int32()), pa.array(["a", "bb", None])], ["x", "s"])
    with Dataflow(counter_desc(lib, gpu)) as df:
        src, sink = open_nodes(df, ["src", "sink"], gpu)
        for k, p in enumerate(payloads):
            src.send_output("message", p, {"k": k})
        src.send_output("table", table)
        src.send_output("stop", b"")
        src.close()
        got = _drain(sink)
        sink.close()
        codes = df.wait(30)
    return got, codes, table


def test_shared_library_path_rule():
    # adjust_shared_library_path (libraries/core/src/lib.rs:14-31)
    assert shared_library_path("build/operator", "/x") == "/x/build/liboperator.so"
    with pytest.raises(ValueError):
        shared_library_path("build/libop", "/x")
    with pytest.raises(ValueError):
        shared_library_path("build/op.so", "/x")


def test_runtime_descriptor():
    nodes = parse_descriptor({"nodes": [
        {"id": "a", "path": "dynamic", "outputs": ["o"]},
        {"id": "one", "operator": {"python": "op.py", "inputs": {"i": "a/o"}, "outputs": ["r"]}},
        {"id": "b", "path": "dynamic", "inputs": {"x": "one/r"}}]})
    one = next(n for n in nodes if n.id == "one")
    assert one.outputs == ["op/r"] and one.inputs == {"op/i": ("a", "o", 10)}
    assert one.env["DORA_GPU_OPERATORS"].startswith("op=") and one.args[-1] == "dora_amd.operator_runtime"
    b = next(n for n in nodes if n.id == "b")
    assert b.inputs["x"] == ("one", "op/r", 10)  # `one/r` of a single-operator node


def test_shared_library_operator_host(tmp_path):
    payloads = [b"hello", b"world!", bytes(range(200))]
    check_counter(*run_counter(tmp_path, -1, payloads), payloads)


def as_bytes(arr) -> bytes:
    return arr.buffers()[1].to_pybytes()[arr.offset:arr.offset + len(arr)]


def check_counter(got, codes, table, payloads):
    assert codes["rt"] == 0, codes
    counters = [as_bytes(v) for v, _ in got["counter"]]
    assert counters == [f"The current counter value is {k}".encode() for k in (1, 2, 3)]
    assert [as_bytes(v) for v, _ in got["echo"]] == payloads
    assert all(md.get("open_telemetry_context") == "" for _, md in got["counter"])
    # the nested array came back unchanged through the operator's Arrow output
    (same, _), = got["same"]
    assert same.equals(table)


def python_desc(op_file: str, gpu: int) -> dict:
    return {"nodes": [
        {"id": "src", "path": "dynamic", "outputs": ["ints", "raw", "stop"],
         "_unstable_deploy": {"gpu": gpu}},
        {"id": "py", "operators": [
            {"id": "scale", "python": op_file,
             "inputs": {"ints": "src/ints", "raw": "src/raw", "stop": "src/stop"},
             "outputs": ["doubled", "length"]}],
         "_unstable_deploy": {"gpu": gpu}},
        {"id": "sink", "path": "dynamic", "_unstable_deploy": {"gpu": gpu},
         "inputs": {"doubled": "py/scale/doubled", "length": "py/scale/length"}},
    ]}


def run_python(gpu: int, ints, raw):
    with Dataflow(python_desc(os.path.join(OPS, "scale_op.py"), gpu)) as df:
        src, sink = open_nodes(df, ["src", "sink"], gpu)
        src.send_output("ints", ints, {"tag": "i"})
        src.send_output("raw", raw)
        src.send_output("stop", b"")
        src.close()
        got = _drain(sink)
        sink.close()
        codes = df.wait(60)
    return got, codes, df


def test_python_operator_host():
    got, codes, df = run_python(-1, pa.array([1, -2, 300], pa.int64()), b"abcdef")
    assert codes["py"] == 0, (codes, df.log("py"))
    check_python(got)


def check_python(got):
    (doubled, md), = got["doubled"]
    assert md["tag"] == "i" and md["open_telemetry_context"] == ""
    assert doubled.equals(pa.array([2, -4, 600], pa.int64()))
    (length, _), = got["length"]
    assert length.equals(pa.array([6, 2], pa.uint64()))


@pytest.mark.gpu
def test_shared_library_operator_device(tmp_path):
    """Device samples through a shared-library operator: inputs downloaded for the operator,
    its outputs packed into HBM slots; payloads above the inline threshold."""
    payloads = [bytes((k * 7 + i) & 255 for i in range(n)) for k, n in enumerate((5, 70000, 1 << 20))]
    check_counter(*run_counter(tmp_path, 0, payloads), payloads)


@pytest.mark.gpu
def test_python_operator_device():
    got, codes, df = run_python(0, pa.array(list(range(5000)), pa.int64()), bytes(9000))
    assert codes["py"] == 0, (codes, df.log("py"))
    (doubled, _), = got["doubled"]
    assert doubled.equals(pa.array([2 * k for k in range(5000)], pa.int64()))
    (length, _), = got["length"]
    assert length.equals(pa.array([9000, 2], pa.uint64()))


def test_send_stdout_as_host():
    """send_stdout_as (binaries/daemon/src/spawn.rs:280-437): a node's printed lines arrive as
    one-element Utf8 arrays on the named output, stdout and stderr alike; they still reach
    the node's log too."""
    import sys
    script = ("import sys\n"
              "from dora_amd.node import Node\n"
              "n = Node()\n"
              "print('hello from node')\n"
              "print('second line')\n"
              "sys.stderr.write('to stderr\\n')\n"
              "n.close()\n")
    desc = {"nodes": [
        {"id": "talker", "path": sys.executable, "args": ["-c", script], "outputs": ["logs"],
         "send_stdout_as": "logs", "env": {"PYTHONPATH": ROOT}, "_unstable_deploy": {"gpu": -1}},
        {"id": "sink", "path": "dynamic", "inputs": {"logs": "talker/logs"},
         "_unstable_deploy": {"gpu": -1}}]}
    with Dataflow(desc) as df:
        sink = Node("sink", dataflow=df.shm, device=-1)
        got = _drain(sink)
        sink.close()
        codes = df.wait(30)
        log = df.log("talker")
    assert codes["talker"] == 0, (codes, log)
    lines = sorted(v.to_pylist()[0] for v, _ in got["logs"])
    assert lines == ["hello from node\n", "second line\n", "to stderr\n"], got
    assert all(len(v) == 1 and v.type == pa.string() for v, _ in got["logs"])
    assert "hello from node" in log and "to stderr" in log


def test_send_stdout_as_must_be_an_output():
    with pytest.raises(ValueError):
        parse_descriptor({"nodes": [{"id": "a", "path": "x", "outputs": ["o"],
                                     "send_stdout_as": "logs"}]})
