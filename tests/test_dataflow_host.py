"""Control plane on the CPU (no GPU): daemon routing, AllNodesReady, drop-oldest input queues,
InputClosed / end of stream, metadata parameters, output checks — with host-only nodes, which
carry the reference's inline `DataMessage::Vec` samples (< 4096 B) and, from 4096 B, its
`DataMessage::SharedMemory` samples (POSIX shm regions, recycled through drop tokens)."""
import ctypes
import os
import threading
import time

import pytest

from dora_amd import _lib
from dora_amd.dataflow import daemon_spec, parse_descriptor
from dora_amd.node import Node, decode_parameters, encode_parameters, encode_parameters_py


class InProcessDaemon:
    def __init__(self, desc):
        self.lib = _lib.load()
        self.shm = f"/dora-gpu-test-{os.getpid()}-{id(self)}"
        h = ctypes.c_void_p()
        _lib.call("dora_daemon_create", self.shm.encode(),
                  daemon_spec(parse_descriptor(desc)).encode(), 1 << 20, ctypes.byref(h))
        self.h = h.value
        self.rc = None
        self.t = threading.Thread(target=self._run, daemon=True)
        self.t.start()

    def _run(self):
        self.rc = self.lib.dora_daemon_run(self.h, 20000)

    def join(self):
        self.t.join(25)
        assert not self.t.is_alive()
        self.lib.dora_daemon_free(self.h)


def _start_nodes(shm, ids):
    out = {}

    def mk(i):
        out[i] = Node(i, dataflow=shm, device=-1)
    ts = [threading.Thread(target=mk, args=(i,)) for i in ids]
    [t.start() for t in ts]
    [t.join(20) for t in ts]
    assert set(out) == set(ids)
    return out


def as_bytes(v) -> bytes:
    """The bytes of a received UInt8 value (a host pyarrow array, as the reference's value)."""
    import numpy as np
    return np.asarray(v).tobytes()


DESC = {"nodes": [
    {"id": "src", "outputs": ["out", "other"]},
    {"id": "dst", "inputs": {"in": {"source": "src/out", "queue_size": 3}}, "outputs": []},
]}


def test_parameters_roundtrip():
    p = {"a": True, "b": -5, "c": "hello", "d": 2.5}
    assert decode_parameters(encode_parameters(p)) == {"a": True, "b": -5, "c": "hello",
                                                       "d": "2.5"}
    assert encode_parameters(None) == b""


def test_native_parameter_encoding_matches_python():
    """The native encoder (csrc/pyext.cpp, used by every send) writes the same bytes as the
    Python statement of the format, for every value kind pydict_to_metadata handles
    (apis/python/operator/src/lib.rs:165-186) and for non-str keys / big ints."""
    class Odd:
        def __str__(self):
            return "odd\u00e9"
    cases = [None, {}, {"seq": 0}, {"b": False, "a": True, "c": -1},
             {"t_start": 1760000000123456789, "seq": 2 ** 63 - 1, "neg": -2 ** 63},
             {"s": "", "u": "h\u00e9llo \u2603", "f": 2.5, "l": [1, 2], "o": Odd(), "n": None},
             {"k" * 300: "v" * 5000}, {3: "int key", 1: "x"}]
    for p in cases:
        assert encode_parameters(p) == encode_parameters_py(p), p
    with pytest.raises(OverflowError):
        encode_parameters({"big": 2 ** 64})
    with pytest.raises(TypeError):
        encode_parameters([("a", 1)])


def test_native_receive_decodes_parameters_and_waits():
    """Node.next and Node.wait_input decode parameters natively (csrc/pyext.cpp next_event /
    wait_input): every value kind arrives as decode_parameters reads the same bytes; wait_input
    skips other inputs and ids, returns the matching parameters and raises TimeoutError."""
    d = InProcessDaemon({"nodes": [
        {"id": "a", "outputs": ["o", "p"]},
        {"id": "b", "inputs": {"i": {"source": "a/o", "queue_size": 100},
                               "j": {"source": "a/p", "queue_size": 100}}}]})
    nodes = _start_nodes(d.shm, ["a", "b"])
    a, b = nodes["a"], nodes["b"]
    cases = [None, {}, {"seq": 0}, {"b": False, "a": True, "c": -1},
             {"t_start": 1760000000123456789, "seq": 2 ** 63 - 1, "neg": -2 ** 63},
             {"s": "", "u": "héllo ☃", "f": 2.5}, {"k" * 300: "v" * 5000}]
    for k, p in enumerate(cases):
        a.send_output("o", bytes([k]) * 3, p)
    for k, p in enumerate(cases):
        ev = b.next(timeout=5)
        assert ev["type"] == "INPUT" and ev["id"] == "i"
        assert ev["metadata"] == decode_parameters(encode_parameters(p)), p
        assert as_bytes(ev["value"]) == bytes([k]) * 3
    for s in range(5):
        a.send_output("p", b"", {"seq": s})
        a.send_output("o", b"x", {"seq": s})
    assert b.wait_input("i", "seq", 3, 5.0) == {"seq": 3}
    assert b.wait_input("j", "seq", 4, 5.0) == {"seq": 4}   # the rest were consumed
    t0 = time.monotonic()
    with pytest.raises(TimeoutError):
        b.wait_input("i", "seq", 99, 0.2)
    assert time.monotonic() - t0 < 2.0
    a.close()
    b.close()
    d.join()


def test_native_pyarrow_send_matches_export_path():
    """send_output of a host pyarrow.Array goes through _dora_node.send_pyarrow (its type's
    schema exported once and lent to later sends): every input equals the one the generic
    _export_to_c path delivers for the same array — value and ArrowTypeInfo — for primitive,
    nullable, sliced, string, struct and list<struct> arrays, and for two struct types equal but
    for their field metadata sent alternately (the receiver's DataType cache, keyed by schema,
    must keep them apart too: the received types carry their own field metadata)."""
    import pyarrow as pa

    class Exported:  # not a pyarrow.Array: takes the generic CArray.from_pyarrow path
        def __init__(self, a):
            self.a = a

        def _export_to_c(self, *args):
            return self.a._export_to_c(*args)
    pts = pa.StructArray.from_arrays(
        [pa.array([1.5, None, 3.0], pa.float32()), pa.array([7, 8, 9], pa.uint8())],
        names=["x", "i"], mask=pa.array([False, False, True]))
    f1 = pa.struct([pa.field("a", pa.int32(), metadata={"u": "m"})])
    f2 = pa.struct([pa.field("a", pa.int32(), metadata={"u": "mm"})])
    arrays = [pa.array(list(range(100)), pa.uint8()),
              pa.array([1, None, -3, 2 ** 40], pa.int64()),
              pa.array(list(range(50)), pa.int16()).slice(7, 20),
              pa.array(["a", None, "héllo", ""]),
              pts, pa.array([[{"x": 1.0, "i": 2}], None, [], [{"x": None, "i": 5}] * 3],
                            pa.list_(pa.struct([("x", pa.float32()), ("i", pa.uint8())]))),
              pa.array([{"a": 1}, {"a": 2}], f1), pa.array([{"a": 3}], f2),
              pa.array([{"a": 4}], f1)]
    d = InProcessDaemon({"nodes": [
        {"id": "a", "outputs": ["o"]},
        {"id": "b", "inputs": {"i": {"source": "a/o", "queue_size": 1000}}}]})
    nodes = _start_nodes(d.shm, ["a", "b"])
    a, b = nodes["a"], nodes["b"]
    for k, arr in enumerate(arrays):
        a.send_output("o", arr, {"k": k, "native": True})
        a.send_output("o", Exported(arr), {"k": k, "native": False})
    got = {}
    for _ in range(2 * len(arrays)):
        ev = b.next(timeout=5)
        assert ev["type"] == "INPUT"
        m = ev["metadata"]
        got[(m["k"], m["native"])] = (ev["value"], ev["type_info"].to_json())
    for k, arr in enumerate(arrays):
        (v1, t1), (v0, t0) = got[(k, True)], got[(k, False)]
        assert t1 == t0, k
        assert v1.equals(v0) and v1.equals(arr), k
        assert v1.type.equals(arr.type, check_metadata=True), (k, v1.type, arr.type)
    a.close()
    b.close()
    d.join()


def test_descriptor_validation():
    with pytest.raises(ValueError, match="unknown output"):
        parse_descriptor({"nodes": [{"id": "a", "inputs": {"x": "b/y"}}, {"id": "b"}]})
    spec = daemon_spec(parse_descriptor(DESC))
    assert "input dst in src out 3" in spec


def test_routing_drop_oldest_and_close():
    d = InProcessDaemon(DESC)
    nodes = _start_nodes(d.shm, ["src", "dst"])
    src, dst = nodes["src"], nodes["dst"]
    for i in range(5):
        src.send_output("out", bytes([i]) * 10, {"seq": i})
    time.sleep(0.2)
    with pytest.raises(_lib.DoraGpuError, match="unknown dora node output"):
        src.send_output("nope", b"x")
    src.close()          # closes outputs -> InputClosed + end of stream for dst
    got = []
    closed = []
    while True:
        ev = dst.next(timeout=5)
        if ev is None:
            break
        if ev["type"] == "INPUT":
            got.append((ev["metadata"]["seq"], ev["value"]))
            assert ev["type_info"].to_json()["data_type"] == "C"
        elif ev["type"] == "INPUT_CLOSED":
            closed.append(ev["id"])
    # queue_size 3 (node_communication/mod.rs:320-359): the first next() takes the oldest
    # input — handed to the node, as the reference's event-stream thread takes events out of the
    # daemon's queue (event_stream/thread.rs:139-157) — and the three newest of the rest survive
    assert [s for s, _ in got] == [0, 2, 3, 4]
    assert as_bytes(got[0][1]) == bytes([0]) * 10
    assert as_bytes(got[1][1]) == bytes([2]) * 10
    assert closed == ["in"]
    dst.close()
    d.join()
    assert d.rc == 0


def test_zero_length_sample_and_ordering():
    d = InProcessDaemon({"nodes": [
        {"id": "a", "outputs": ["o"]},
        {"id": "b", "inputs": {"i": {"source": "a/o", "queue_size": 1000}}}]})
    nodes = _start_nodes(d.shm, ["a", "b"])
    n = 200
    for k in range(n):
        nodes["a"].send_output("o", b"" if k % 2 else bytes([k % 256]) * (k % 50), {"k": k})
    nodes["a"].close()
    seen = []
    for ev in nodes["b"]:
        if ev["type"] == "INPUT":
            seen.append(ev["metadata"]["k"])
            if ev["metadata"]["k"] % 2:   # empty sample -> ArrayData::new_empty(UInt8)
                assert len(ev["value"]) == 0 and str(ev["value"].type) == "uint8"
            elif ev["metadata"]["k"] % 50:
                assert as_bytes(ev["value"]) == bytes([ev["metadata"]["k"] % 256]) * (ev["metadata"]["k"] % 50)
    assert seen == list(range(n))
    nodes["b"].close()
    d.join()


def test_all_nodes_ready_names_host_bound_outputs():
    """AllNodesReady carries, for each node, the outputs whose every receiver is a running local
    node without a GPU (daemon.cpp ready_payload): a device producer packs those into shared
    memory instead of HBM.  An output nobody reads is not named; the consumer's own outputs go
    nowhere.  (Device receivers and receivers on another machine exclude an output: the first is
    covered by tests/test_gpu_host_edges.py, the second by tests/test_interdaemon.py.)"""
    d = InProcessDaemon({"nodes": [
        {"id": "a", "outputs": ["to_b", "unread", "to_both"]},
        {"id": "b", "inputs": {"x": "a/to_b", "y": "a/to_both"}, "outputs": ["back"]},
        {"id": "c", "inputs": {"y": "a/to_both", "z": "b/back"}}]})
    nodes = _start_nodes(d.shm, ["a", "b", "c"])
    assert nodes["a"].host_bound_outputs() == ["to_b", "to_both"]
    assert nodes["b"].host_bound_outputs() == ["back"]
    assert nodes["c"].host_bound_outputs() == []
    nodes["a"].close()
    for k in ("b", "c"):
        while nodes[k].next(timeout=5) is not None:
            pass
        nodes[k].close()
    d.join()
    assert d.rc == 0


def test_host_only_shared_memory_samples_recycle():
    """A host-only node sends samples >= 4096 B as DataMessage::SharedMemory (the reference's
    allocate_shared_memory, apis/rust/node/src/node/mod.rs:321-346): the receiver reads the
    region in place as a pyarrow array, its drop token returns the region to the sender's
    best-fit cache, and a steady stream of one size creates no new regions.  Sizes below 4096 B
    stay inline Vec samples (mod.rs:40)."""
    import glob
    d = InProcessDaemon({"nodes": [
        {"id": "a", "outputs": ["o"]},
        {"id": "b", "inputs": {"i": {"source": "a/o", "queue_size": 1000}}}]})
    nodes = _start_nodes(d.shm, ["a", "b"])
    a, b = nodes["a"], nodes["b"]
    sizes = [4095, 4096, 4097, 1 << 20, 5_000_001]
    seen = {}
    for rep in range(3):
        for z in sizes:
            payload = bytes((k * 131 + z + rep) % 251 for k in range(256)) * (z // 256 + 1)
            a.send_output("o", payload[:z], {"z": z, "rep": rep})
            ev = b.next(timeout=10)
            assert ev["type"] == "INPUT" and ev["metadata"] == {"z": z, "rep": rep}
            assert not ev["on_device"] and ev["data_len"] == z
            assert as_bytes(ev["value"]) == payload[:z], (z, rep)
            assert ev["type_info"].to_json()["data_type"] == "C"
            seen.setdefault(z, []).append(ev["data_ptr"])
            del ev  # the value goes: the token returns, the region is reusable
    st = a.stats()
    # one region per size >= 4096 (created in the first round, reused in the next two)
    assert st["slots_created"] == 4, st
    assert st["cache_hits"] >= 8, st
    mine = glob.glob(f"/dev/shm/dora-gpu-s-{os.getpid()}-*")
    assert len(mine) == 4, mine
    a.close()
    while b.next(timeout=5) is not None:
        pass
    b.close()
    d.join()
    assert d.rc == 0
    # the sender unlinks its regions when it goes
    assert not glob.glob(f"/dev/shm/dora-gpu-s-{os.getpid()}-*")


def test_host_only_receiver_holding_shared_memory_inputs():
    """A receiver that keeps several shared-memory inputs alive holds their regions (the sender
    allocates new ones meanwhile); releasing them returns every token, and a forward of such an
    input by a host-only relay is a CPU copy into the relay's own region."""
    d = InProcessDaemon({"nodes": [
        {"id": "a", "outputs": ["o"]},
        {"id": "r", "inputs": {"i": {"source": "a/o", "queue_size": 100}}, "outputs": ["f"]},
        {"id": "c", "inputs": {"i": {"source": "r/f", "queue_size": 100}}}]})
    nodes = _start_nodes(d.shm, ["a", "r", "c"])
    a, r, c = nodes["a"], nodes["r"], nodes["c"]
    held = []
    for k in range(5):
        a.send_output("o", bytes([k + 1]) * 70000, {"k": k})
        ev = r.next(timeout=10)
        r.forward("f", ev)
        held.append(ev)
        got = c.next(timeout=10)
        assert got["metadata"] == {"k": k} and as_bytes(got["value"]) == bytes([k + 1]) * 70000
        del got
    assert a.stats()["in_flight"] == 5 and a.stats()["slots_created"] == 5
    del ev
    held.clear()
    deadline = time.monotonic() + 5
    while a.stats()["in_flight"] and time.monotonic() < deadline:
        a.send_output("o", b"", {"k": -1})  # handles returned tokens
        r.next(timeout=5)
    assert a.stats()["in_flight"] == 0
    for n in (a, r):
        n.close()
    while c.next(timeout=5) is not None:
        pass
    c.close()
    d.join()


def test_event_thread_decouples_a_receiver_that_never_polls():
    """Verdict r04 item 3: a receiver whose event-stream thread runs (dora_node_set_event_thread,
    the reference's event_stream_loop) but whose user thread never calls next_event keeps taking
    events off the daemon and applies drop-oldest to them, as the reference's daemon-side queue
    does (node_communication/mod.rs:320-359): the producer's tokens come back (its in-flight
    samples stay bounded by that receiver's queue_size + the one its thread holds), the other
    receiver gets every message, and the producer's sends do not slow down.  Without the thread
    the same receiver holds every sample it was sent.  (An RCCL broadcast group posts its
    receives from this thread; a group needs >= 2 GPUs.)"""
    def run(thread):
        d = InProcessDaemon({"nodes": [
            {"id": "src", "outputs": ["o"]},
            {"id": "idle", "inputs": {"i": {"source": "src/o", "queue_size": 2}}},
            {"id": "busy", "inputs": {"i": {"source": "src/o", "queue_size": 1000}}}]})
        nodes = _start_nodes(d.shm, ["src", "idle", "busy"])
        src, idle, busy = nodes["src"], nodes["idle"], nodes["busy"]
        if thread:
            idle.set_event_thread(True)
        n, got, t_send = 40, [], []
        for k in range(n):
            t0 = time.perf_counter()
            src.send_output("o", bytes([k]) * 8192, {"k": k})  # shared-memory samples: tokens
            t_send.append(time.perf_counter() - t0)
            ev = busy.next(timeout=10)
            got.append(ev["metadata"]["k"])
            assert as_bytes(ev["value"]) == bytes([k]) * 8192
            del ev
        deadline = time.monotonic() + (5 if thread else 0.5)
        while time.monotonic() < deadline:
            src.send_output("o", b"", {"k": -1})  # the producer handles returned tokens
            busy.next(timeout=5)
            if src.stats()["in_flight"] <= 3:
                break
            time.sleep(0.01)
        in_flight = src.stats()["in_flight"]
        dropped = src.dataflow_counters("idle")["dropped_inputs"]
        # what the idle receiver finally reads: the event its thread held, then the newest ones
        seen = []
        while True:
            ev = idle.next(timeout=0.3)
            if ev is None:
                break
            if ev["type"] == "INPUT" and ev["metadata"]["k"] >= 0:
                seen.append(ev["metadata"]["k"])
            del ev
        for x in (src, idle, busy):
            x.close()
        d.join()
        return got, in_flight, dropped, seen, sorted(t_send)[len(t_send) // 2]
    got, in_flight, dropped, seen, t50 = run(thread=True)
    assert got == list(range(40))
    assert in_flight <= 3, in_flight
    assert dropped >= 37, dropped
    # the event its thread held (the oldest), then at most queue_size of the newest
    assert seen[0] == 0 and len(seen) <= 3 and set(seen[1:]) <= {38, 39}, seen
    got0, in_flight0, dropped0, seen0, t50_0 = run(thread=False)
    assert got0 == list(range(40))
    assert in_flight0 == 40 and dropped0 == 0, (in_flight0, dropped0)  # held until it polls
    print(f"send p50 with / without the idle receiver's thread: {t50 * 1e6:.1f} / "
          f"{t50_0 * 1e6:.1f} us")


def test_busy_stats_count_blocked_time():
    """dora_gpu_busy_stats: a receiver blocked on its empty event ring accumulates idle time
    (the diagnostics the bench tools report as busy = wall - idle)."""
    def idle_ns():
        idle, fill = ctypes.c_uint64(), ctypes.c_uint64()
        _lib.call("dora_gpu_busy_stats", ctypes.byref(idle), ctypes.byref(fill))
        return idle.value, fill.value

    d = InProcessDaemon(DESC)
    nodes = _start_nodes(d.shm, ["src", "dst"])
    src, dst = nodes["src"], nodes["dst"]
    i0, f0 = idle_ns()
    t0 = time.monotonic()
    threading.Timer(0.3, lambda: src.send_output("out", b"late", {"seq": 1})).start()
    ev = dst.next(timeout=5)
    waited = time.monotonic() - t0
    assert ev["type"] == "INPUT" and as_bytes(ev["value"]) == b"late"
    i1, f1 = idle_ns()
    # the daemon thread also idles in this process, so at least the receiver's wait is there
    assert i1 - i0 >= 0.8 * 0.3e9 and waited >= 0.29
    assert f1 == f0  # host-only samples have no fill flag to wait on
    src.close()
    while dst.next(timeout=5) is not None:
        pass
    dst.close()
    d.join()


def test_node_config_in_the_reference_schema():
    """DORA_NODE_CONFIG (the Rust facade's init_from_env / init(NodeConfig)) is the reference's
    NodeConfig (libraries/message/src/daemon_to_node.rs:20-27): run_config inputs/outputs, the
    Shmem daemon communication naming the control region, a descriptor whose nodes carry only
    fields the reference's `Node` accepts (descriptor/mod.rs:164-200, deny_unknown_fields;
    `_unstable_deploy` with `machine` only), and the dataflow UUID the daemon's wire uses."""
    import uuid

    import yaml

    from dora_amd.dataflow import Dataflow, dataflow_uuid, node_config_yaml, parse_descriptor
    desc = {"nodes": [
        {"id": "src", "path": "dynamic", "outputs": ["data"], "_unstable_deploy": {"gpu": 1}},
        {"id": "dst", "path": "/bin/true", "args": "-x 'a b'", "env": {"K": 3},
         "inputs": {"in": {"source": "src/data", "queue_size": 4}, "in2": "src/data"},
         "outputs": ["o"], "_unstable_deploy": {"machine": "B", "gpu": 2}}]}
    nodes = parse_descriptor(desc)
    c = yaml.safe_load(node_config_yaml(nodes, "dst", "df-test", "/dora-gpu-x"))
    assert set(c) == {"dataflow_id", "node_id", "run_config", "daemon_communication",
                      "dataflow_descriptor", "dynamic"}
    assert c["dataflow_id"] == dataflow_uuid("df-test") and uuid.UUID(c["dataflow_id"])
    assert c["node_id"] == "dst" and c["dynamic"] is False
    assert c["run_config"] == {"inputs": {"in": {"source": "src/data", "queue_size": 4},
                                          "in2": {"source": "src/data", "queue_size": 10}},
                               "outputs": ["o"]}
    assert c["daemon_communication"] == {"Shmem": {k: "/dora-gpu-x" for k in (
        "daemon_control_region_id", "daemon_drop_region_id", "daemon_events_region_id",
        "daemon_events_close_region_id")}}
    allowed = {"id", "name", "description", "env", "_unstable_deploy", "operators", "custom",
               "operator", "path", "args", "build", "send_stdout_as", "inputs", "outputs"}
    for n in c["dataflow_descriptor"]["nodes"]:
        assert set(n) <= allowed, n
        assert set(n.get("_unstable_deploy", {})) <= {"machine"}
    dst = c["dataflow_descriptor"]["nodes"][1]
    assert dst["args"] == "-x 'a b'" and dst["env"] == {"K": "3"}
    assert dst["_unstable_deploy"] == {"machine": "B"}
    # a UUID id is kept as it is; every node the launcher starts gets its config
    u = str(uuid.uuid4())
    assert dataflow_uuid(u) == u
    df = Dataflow(desc, machine=None)
    assert yaml.safe_load(df.dynamic_env("src")["DORA_NODE_CONFIG"])["dynamic"] is True
