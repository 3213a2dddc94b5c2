"""End-to-end device data plane on one MI355X: sender node (this process) -> daemon process ->
receiver node processes, with IPC-mapped HBM slots, drop-token recycling and bit-exact checks.

* C2: UInt8 payloads 4 KB..40 MB through the C++ benchmark sink, which checksums every received
  device sample (csum64 kernel) against the sender's checksum;
* C3: 1M-point List<Struct<x,y,z,intensity>> point clouds to a Python receiver that checksums
  every parity region on the GPU; compared with the CPU oracle's regions checksum;
* drop tokens: a zero-copy sink returns tokens, the sender's 20-slot cache serves every send;
* queue_size drop-oldest with a slow receiver returns tokens of dropped inputs.
"""
import json
import os
import sys
import threading
import time

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench_desc(result_path, queue_size=1000):
    return {"nodes": [
        {"id": "node", "path": "dynamic", "outputs": ["data"],
         "inputs": {"ack": "sink/ack"}},
        {"id": "sink", "path": "dora-gpu-bench-sink", "outputs": ["ack"],
         "inputs": {"data": {"source": "node/data", "queue_size": queue_size}},
         "env": {"DORA_BENCH_RESULT": result_path}},
    ]}


def test_bench_sink_bit_exact_c2(launcher, tmp_path):
    from dora_amd import device
    from dora_amd.dataflow import Dataflow
    from dora_amd.node import Node
    from dora_amd.verify import to_i64
    from dora_amd.workloads import payload_seed
    from oracle.checksum_ref import csum64, splitmix_bytes
    res = str(tmp_path / "sink.json")
    sizes = [4096, 16384, 40960, 409600, 4096000, 40960000]
    with Dataflow(_bench_desc(res), launcher=launcher) as df:
        node = Node("node", dataflow=df.shm, device=0)
        s = device.Stream()
        for size in sizes:
            buf = device.DeviceBuffer(size)
            device.fill_splitmix(buf.ptr, size, payload_seed(size), s)
            s.sync()
            c = device.csum64(buf.ptr, size, s)
            if size <= 409600:  # device generator == oracle bytes
                assert c == csum64(splitmix_bytes(size, payload_seed(size)))
            for k in range(5):
                node.send_output_device_bytes("data", buf.ptr, size,
                                              {"csum": to_i64(c), "verify": True, "seq": k})
            buf.free()
        stats = node.stats()
        paths = node.fill_paths()
        node.close()
        codes = df.wait(60)
        log = df.log("sink")
    assert codes["sink"] == 0, log
    out = json.load(open(res))
    assert out["errors"] == 0
    got = {s["size"]: s for s in out["series"]}
    for size in sizes:
        assert got[size]["n"] == 5
        assert got[size]["verified"] == 5
        assert got[size]["mismatches"] == 0
    assert stats["slots_created"] <= 5 * len(sizes), stats
    # every size went through raw AQL packets (40.96 MB in order per queue, aql.cpp)
    assert paths == {"aql": 30, "hip": 0}, paths


def test_payload_beyond_4_gib_bit_exact(launcher, tmp_path):
    """A maximum-size case: one UInt8 payload of 4.5 GiB + 13 bytes (offsets, lengths and chunk
    counts past 32 bits; a ragged tail) from a source 3 bytes past alignment, sent twice through
    the AQL path (the barrier policy of >= 32 MiB packs) to the sink, which checksums each
    delivered sample.  The source's bytes are the oracle generator's at three windows; the
    checksum of checksums holds for the whole payload (size-independent property)."""
    import numpy as np
    from dora_amd import device
    from dora_amd.dataflow import Dataflow
    from dora_amd.node import Node
    from dora_amd.verify import to_i64
    from oracle.checksum_ref import GOLDEN, MASK, fmix64_np
    res = str(tmp_path / "sink.json")
    size, mis, seed = (4 << 30) + (1 << 29) + 13, 3, 0xB16
    s = device.Stream()
    buf = device.DeviceBuffer(size + mis)
    try:
        device.fill_splitmix(buf.ptr + mis, size, seed, s)
        s.sync()
        csum = device.csum64(buf.ptr + mis, size, s)
        for w0 in (0, (size // 2) & ~7, (size - (1 << 20)) & ~7):   # word-aligned windows
            n = min(1 << 20, size - w0)
            got = buf.to_bytes(n, offset=mis + w0)
            k = np.arange(w0 // 8 + 1, w0 // 8 + 1 + (n + 7) // 8, dtype=np.uint64)
            with np.errstate(over="ignore"):
                want = fmix64_np(np.uint64(seed & MASK) + k * GOLDEN).astype("<u8").tobytes()[:n]
            assert got == want, w0
        with Dataflow(_bench_desc(res), launcher=launcher) as df:
            node = Node("node", dataflow=df.shm, device=0)
            for k in range(2):
                node.send_output_device_bytes("data", buf.ptr + mis, size,
                                              {"csum": to_i64(csum), "verify": True, "seq": k})
            paths = node.fill_paths()
            node.close()
            codes = df.wait(120)
            log = df.log("sink")
    finally:
        buf.free()
    assert codes["sink"] == 0, log
    out = json.load(open(res))
    assert out["errors"] == 0
    got = {x["size"]: x for x in out["series"]}
    assert got[size]["verified"] == 2 and got[size]["mismatches"] == 0, got
    assert paths["aql"] == 2, paths


def test_slots_recycle_through_drop_tokens(launcher, tmp_path):
    """The 20-entry slot cache (node/mod.rs:321-371) serves repeated sends once tokens return."""
    from dora_amd import device
    from dora_amd.dataflow import Dataflow
    from dora_amd.node import Node
    res = str(tmp_path / "sink.json")
    with Dataflow(_bench_desc(res), launcher=launcher) as df:
        node = Node("node", dataflow=df.shm, device=0)
        buf = device.DeviceBuffer(4 << 20)
        for k in range(100):
            node.send_output_device_bytes("data", buf.ptr, buf.size, {"seq": k})
            if k % 10 == 9:
                time.sleep(0.01)   # let tokens come back
        stats = node.stats()
        node.close()
        df.wait(60)
        buf.free()
    assert stats["slots_created"] + stats["cache_hits"] == 100
    assert stats["slots_created"] <= 40, stats
    assert stats["cache_hits"] >= 60, stats


def test_slot_cache_keeps_many_sizes(launcher, tmp_path):
    """r04: a sender whose message sizes change keeps its slots (up to 64 within 4 GiB, node.cpp
    slot_cache_bytes) instead of the reference's 20, so cycling through 30 sizes (30 slot
    capacities) a second and a third time creates no slot (the 20-entry cache evicted and
    re-created them on every pass: hipFree inside a send), and every delivered payload is still
    bit-exact."""
    from dora_amd import device
    from dora_amd.dataflow import Dataflow
    from dora_amd.node import Node
    from dora_amd.verify import to_i64
    res = str(tmp_path / "sink.json")
    sizes = [(2 * k + 1) << 20 for k in range(30)]  # 1..59 MiB: 30 slots of 2..60 MiB, 930 MiB
    src = device.DeviceBuffer(sizes[-1])
    s = device.Stream()
    device.fill_splitmix(src.ptr, src.size, 0x51075, s)
    sums = {z: to_i64(device.csum64(src.ptr, z, s)) for z in sizes}
    s.close()
    created = []
    with Dataflow(_bench_desc(res), launcher=launcher) as df:
        node = Node("node", dataflow=df.shm, device=0)
        seq = 0
        for rnd in range(3):
            before = node.stats()["slots_created"]
            for z in sizes:
                node.send_output_device_bytes("data", src.ptr, z,
                                              {"seq": seq, "csum": sums[z], "verify": True})
                seq += 1
                time.sleep(0.002)  # the token comes back: each send finds its best fit free
            node.send_output("data", b"", {"seq": seq, "ack": True})
            node.wait_input("ack", "seq", seq, 60.0)
            seq += 1
            created.append(node.stats()["slots_created"] - before)
        node.close()
        codes = df.wait(60)
        log = df.log("sink")
    src.free()
    assert codes["sink"] == 0, log
    out = json.load(open(res))
    assert out["errors"] == 0
    assert sum(x["verified"] for x in out["series"]) == 3 * len(sizes)
    assert sum(x["mismatches"] for x in out["series"]) == 0
    # round 1 creates the 30 slots; the 20-entry cache had to re-create at least 10 per later
    # round, now none (a token late by more than the 2 ms pause could cost one)
    assert created[0] >= 30, created
    assert created[1] <= 1 and created[2] <= 1, created


def test_python_receiver_c3_point_clouds(launcher):
    from dora_amd.dataflow import Dataflow
    from dora_amd.device import DeviceArray
    from dora_amd.node import Node
    from dora_amd.verify import to_u64
    from dora_amd.workloads import point_cloud
    from oracle.arrow_ffi import import_array
    from oracle.checksum_ref import regions_csum
    from oracle.pack_ref import node_regions, pack
    desc = {"nodes": [
        {"id": "src", "path": "dynamic", "outputs": ["pc"], "inputs": {"result": "recv/result"}},
        {"id": "recv", "path": sys.executable,
         "args": [os.path.join(ROOT, "examples", "verify_receiver.py")],
         "inputs": {"pc": {"source": "src/pc", "queue_size": 100}}, "outputs": ["result"]},
    ]}
    clouds = [point_cloud(37, 4, 7), point_cloud(20000, 16, 11), point_cloud()]
    with Dataflow(desc, launcher=launcher) as df:
        node = Node("src", dataflow=df.shm, device=0)
        want = []
        for seq, pc in enumerate(clouds):
            want.append(regions_csum(node_regions(import_array(pc))))
            sample, _ = pack(pc)
            with DeviceArray.from_pyarrow(pc) as da:
                node.send_output("pc", da, {"seq": seq})
        results = {}
        deadline = time.time() + 120
        while len(results) < len(clouds) and time.time() < deadline:
            ev = node.next(timeout=5)
            if ev is None:
                break
            if ev["type"] == "INPUT":
                results[ev["metadata"]["seq"]] = ev["metadata"]
        node.close()
        codes = df.wait(60)
        log = df.log("recv")
    assert codes["recv"] == 0, log
    for seq, pc in enumerate(clouds):
        r = results[seq]
        assert r["on_device"] is True
        assert to_u64(r["csum"]) == want[seq], seq
        assert r["data_type"] == "+l[item:?+s[x:?f,y:?f,z:?f,intensity:?C]]"
    assert results[0]["arrow_equal_len"] == 4


def test_c3_async_burst_batches_bit_exact(launcher):
    """Twelve point clouds (nested, validity bitmaps in the sample tail, 7 segments each) sent
    back to back with DORA_SEND_ASYNC from 12 distinct device arrays: the sends queued behind
    busy AQL queues leave as batch packs of whole clouds, and every cloud's parity regions
    checksum to the CPU oracle's at the receiver."""
    from dora_amd import device
    from dora_amd.dataflow import Dataflow
    from dora_amd.device import DeviceArray
    from dora_amd.node import Node
    from dora_amd.verify import to_u64
    from dora_amd.workloads import point_cloud
    from oracle.arrow_ffi import import_array
    from oracle.checksum_ref import regions_csum
    from oracle.pack_ref import node_regions
    desc = {"nodes": [
        {"id": "src", "path": "dynamic", "outputs": ["pc"], "inputs": {"result": "recv/result"}},
        {"id": "recv", "path": sys.executable,
         "args": [os.path.join(ROOT, "examples", "verify_receiver.py")],
         "inputs": {"pc": {"source": "src/pc", "queue_size": 100}}, "outputs": ["result"]},
    ]}
    clouds = [point_cloud(150000, 16, 100 + k) for k in range(12)]
    want = [regions_csum(node_regions(import_array(pc))) for pc in clouds]
    arrs = [DeviceArray.from_pyarrow(pc) for pc in clouds]
    with Dataflow(desc, launcher=launcher) as df:
        node = Node("src", dataflow=df.shm, device=0)
        node.set_async_sends(True)
        b0 = device.aql_batch_stats(0)
        device.aql_hold(0, True)   # every cloud waits in the backlog: batches of two clouds
        for seq, da in enumerate(arrs):
            node.send_output("pc", da, {"seq": seq})
        device.aql_hold(0, False)
        node.sync()
        b1 = device.aql_batch_stats(0)
        results = {}
        deadline = time.time() + 120
        while len(results) < len(clouds) and time.time() < deadline:
            ev = node.next(timeout=5)
            if ev is None:
                break
            if ev["type"] == "INPUT":
                results[ev["metadata"]["seq"]] = ev["metadata"]
        node.close()
        codes = df.wait(60)
        log = df.log("recv")
    for a in arrs:
        a.close()
    assert codes["recv"] == 0, log
    for seq in range(len(clouds)):
        assert to_u64(results[seq]["csum"]) == want[seq], seq
    print(f"c3 async burst: {b1['batches'] - b0['batches']} batches carried "
          f"{b1['batched_msgs'] - b0['batched_msgs']} of {len(clouds)} clouds")
    assert b1["batched_msgs"] - b0["batched_msgs"] == len(clouds), (b0, b1)


@pytest.mark.parametrize("peer_copy", ["kernel", "sdma"])
def test_c3_validity_tail_through_pulls_and_relay(launcher, peer_copy):
    """Point clouds (validity in the sample's tail) through a relay and a receiver with the
    cross-GPU pull path forced (DORA_GPU_EDGE_COPY=1): every pull and the relay's forward move
    the tail with the sample (ext_len), and the receiver's inline ArrowTypeInfo — restored from
    its local copy — checksums to the oracle's regions."""
    from dora_amd.dataflow import Dataflow
    from dora_amd.device import DeviceArray
    from dora_amd.node import Node
    from dora_amd.verify import to_u64
    from dora_amd.workloads import point_cloud
    from oracle.arrow_ffi import import_array
    from oracle.checksum_ref import regions_csum
    from oracle.pack_ref import node_regions
    env = {"DORA_GPU_EDGE_COPY": "1", "DORA_GPU_PEER_COPY": peer_copy}
    desc = {"nodes": [
        {"id": "src", "path": "dynamic", "outputs": ["pc"], "inputs": {"result": "recv/result"}},
        {"id": "relay", "path": "dora-gpu-relay", "outputs": ["pc"], "env": env,
         "inputs": {"pc": {"source": "src/pc", "queue_size": 100}}},
        {"id": "recv", "path": sys.executable, "env": env,
         "args": [os.path.join(ROOT, "examples", "verify_receiver.py")],
         "inputs": {"pc": {"source": "relay/pc", "queue_size": 100}}, "outputs": ["result"]},
    ]}
    clouds = [point_cloud(37, 4, 7), point_cloud(20000, 16, 11), point_cloud(300000, 16, 3)]
    with Dataflow(desc, launcher=launcher) as df:
        node = Node("src", dataflow=df.shm, device=0)
        want = []
        for seq, pc in enumerate(clouds):
            want.append(regions_csum(node_regions(import_array(pc))))
            with DeviceArray.from_pyarrow(pc) as da:
                node.send_output("pc", da, {"seq": seq})
        results = {}
        deadline = time.time() + 120
        while len(results) < len(clouds) and time.time() < deadline:
            ev = node.next(timeout=5)
            if ev is None:
                break
            if ev["type"] == "INPUT":
                results[ev["metadata"]["seq"]] = ev["metadata"]
        node.close()
        codes = df.wait(60)
        log = df.log("recv") + df.log("relay")
    assert codes["recv"] == 0 and codes["relay"] == 0, log
    for seq in range(len(clouds)):
        assert to_u64(results[seq]["csum"]) == want[seq], seq
    assert results[0]["arrow_equal_len"] == 4


@pytest.mark.parametrize("mode", ["sync", "async"])
def test_many_small_sends_bit_exact(launcher, tmp_path, mode):
    """More sends than the AQL argument ring holds (512 slots): every argument slot is reused
    after its launch signalled; 1200 messages of odd sizes from unaligned sources, each
    checksummed by the sink.  Async sends run ahead of the GPU: the sends that find every AQL
    queue busy leave as batch packs (dora_aql_packb_u4), several slots per dispatch."""
    from dora_amd import device
    from dora_amd.dataflow import Dataflow
    from dora_amd.node import Node
    from dora_amd.verify import to_i64
    res = str(tmp_path / "sink.json")
    sizes = [4096, 5003, 65537, 262139]
    n_msgs = 1200
    with Dataflow(_bench_desc(res), launcher=launcher) as df:
        node = Node("node", dataflow=df.shm, device=0)
        node.set_async_sends(mode == "async")
        b0 = device.aql_batch_stats(0)
        s = device.Stream()
        srcs = []
        for k in range(3):
            b = device.DeviceBuffer(262139 + 64)
            device.fill_splitmix(b.ptr, b.size, 0x5EED + k, s)
            srcs.append(b)
        s.sync()
        sums = {}
        for i in range(n_msgs):
            key = (i % 3, (5 * i) % 13, sizes[i % len(sizes)])
            if key not in sums:
                b = srcs[key[0]]
                sums[key] = device.csum64(b.ptr + key[1], key[2], s)
            b = srcs[key[0]]
            if mode == "async" and i % 10 == 0:
                device.aql_hold(0, True)   # the next 10 sends wait in the backlog ...
            node.send_output_device_bytes("data", b.ptr + key[1], key[2],
                                          {"csum": to_i64(sums[key]), "verify": True, "seq": i})
            if mode == "async" and i % 10 == 9:
                device.aql_hold(0, False)  # ... and leave as batch packs
        node.sync()
        b1 = device.aql_batch_stats(0)
        paths = node.fill_paths()
        node.close()
        codes = df.wait(60)
        log = df.log("sink")
        for b in srcs:
            b.free()
    assert codes["sink"] == 0, log
    out = json.load(open(res))
    assert out["errors"] == 0
    assert sum(x["verified"] for x in out["series"]) == n_msgs
    assert sum(x["mismatches"] for x in out["series"]) == 0
    batched = b1["batched_msgs"] - b0["batched_msgs"]
    print(f"{mode}: {b1['batches'] - b0['batches']} batches carried {batched} of {n_msgs} sends")
    if mode == "async":
        assert batched > 0, (b0, b1)
    assert paths["aql"] == n_msgs, paths


def test_host_pyarrow_send_to_device_receiver(launcher):
    """A Python node sending a host pyarrow array (reference Python path) -> device sample."""
    import pyarrow as pa
    from dora_amd.dataflow import Dataflow
    from dora_amd.node import Node
    from dora_amd.verify import to_u64
    from oracle.arrow_ffi import import_array
    from oracle.checksum_ref import regions_csum
    from oracle.pack_ref import node_regions
    from tests.golden import recipes
    desc = {"nodes": [
        {"id": "src", "path": "dynamic", "outputs": ["x"], "inputs": {"result": "recv/result"}},
        {"id": "recv", "path": sys.executable,
         "args": [os.path.join(ROOT, "examples", "verify_receiver.py")],
         "inputs": {"x": {"source": "src/x", "queue_size": 100}}, "outputs": ["result"]},
    ]}
    names = ["kat4", "kat5", "kat9", "struct_nulls_sliced", "dictionary", "map", "deep_nesting"]
    with Dataflow(desc, launcher=launcher) as df:
        node = Node("src", dataflow=df.shm, device=0)
        for seq, n in enumerate(names):
            node.send_output("x", recipes.build(n), {"seq": seq})
        results = {}
        deadline = time.time() + 60
        while len(results) < len(names) and time.time() < deadline:
            ev = node.next(timeout=5)
            if ev is None:
                break
            if ev["type"] == "INPUT":
                results[ev["metadata"]["seq"]] = ev["metadata"]
        node.close()
        df.wait(60)
    for seq, n in enumerate(names):
        arr = recipes.build(n)
        assert to_u64(results[seq]["csum"]) == regions_csum(node_regions(import_array(arr))), n
        assert results[seq]["arrow_equal_len"] == len(arr)


@pytest.mark.parametrize("peer_copy", ["kernel", "sdma"])
def test_pipeline_with_peer_copy_edges(launcher, tmp_path, peer_copy):
    """C5 shape on one GPU: node -> relay -> sink with the cross-GPU pull path forced
    (DORA_GPU_EDGE_COPY=1): the relay forwards each input straight from the producer's slot into
    its own (dora_node_forward, one copy per hop), the sink pulls it into a receive slot; every
    payload arrives bit-exact after two hops, with both pull engines."""
    from dora_amd import device
    from dora_amd.dataflow import Dataflow
    from dora_amd.node import Node
    from dora_amd.verify import to_i64
    from dora_amd.workloads import payload_seed
    res = str(tmp_path / "sink.json")
    env = {"DORA_GPU_EDGE_COPY": "1", "DORA_GPU_PEER_COPY": peer_copy}
    desc = {"nodes": [
        {"id": "node", "path": "dynamic", "outputs": ["data"], "inputs": {"ack": "sink/ack"}},
        {"id": "relay", "path": "dora-gpu-relay", "outputs": ["data"], "env": env,
         "inputs": {"data": {"source": "node/data", "queue_size": 100}}},
        {"id": "sink", "path": "dora-gpu-bench-sink", "outputs": ["ack"],
         "inputs": {"data": {"source": "relay/data", "queue_size": 100}},
         "env": dict(env, DORA_BENCH_RESULT=res)},
    ]}
    sizes = [4096, 409600, 40960000]
    with Dataflow(desc, launcher=launcher) as df:
        node = Node("node", dataflow=df.shm, device=0)
        s = device.Stream()
        for size in sizes:
            buf = device.DeviceBuffer(size)
            device.fill_splitmix(buf.ptr, size, payload_seed(size), s)
            s.sync()
            c = device.csum64(buf.ptr, size, s)
            for k in range(4):
                node.send_output_device_bytes("data", buf.ptr, size,
                                              {"csum": to_i64(c), "verify": True, "seq": k})
            s.sync()
            buf.free()
        node.close()
        codes = df.wait(120)
        relay_log = df.log("relay")
    assert codes["relay"] == 0 and codes["sink"] == 0, relay_log
    out = json.load(open(res))
    got = {x["size"]: x for x in out["series"]}
    for size in sizes:
        assert got[size]["verified"] == 4 and got[size]["mismatches"] == 0
    relay = json.loads(relay_log.strip().splitlines()[-1])
    assert relay["relay_peer_copies"] == 12 and relay["errors"] == 0


def test_python_forward(launcher, tmp_path):
    """Node.forward from Python: a relay written against the Python API keeps type info and
    parameters (C3 point cloud through two hops, checked by the sink's checksum)."""
    from dora_amd.dataflow import Dataflow
    from dora_amd.node import Node
    from dora_amd.verify import to_i64
    from dora_amd.device import DeviceArray
    from dora_amd.arrow_utils import Plan
    from dora_amd import device
    res = str(tmp_path / "sink.json")
    desc = {"nodes": [
        {"id": "node", "path": "dynamic", "outputs": ["data"]},
        {"id": "relay", "path": "dynamic", "outputs": ["data"], "inputs": {"data": "node/data"}},
        {"id": "sink", "path": "dora-gpu-bench-sink", "outputs": ["ack"],
         "inputs": {"data": {"source": "relay/data", "queue_size": 100}},
         "env": {"DORA_BENCH_RESULT": res}},
    ]}
    import threading
    from dora_amd.workloads import point_cloud
    cloud = point_cloud(n_points=20000)
    with Dataflow(desc, launcher=launcher) as df:
        relay_err = []

        def relay():
            try:
                r = Node("relay", dataflow=df.shm, device=0)
                for ev in r:
                    if ev["type"] == "INPUT":
                        r.forward("data", ev)
                        assert ev["type_info"].to_json()["len"] == len(cloud)
                st = r.stats()
                # same GPU: every forward re-sent the producer's slot in place (no new slot)
                assert st["zero_copy_forwards"] == 3 and st["slots_created"] == 0, st
                r.close()
            except Exception as e:  # noqa: BLE001
                relay_err.append(e)
        t = threading.Thread(target=relay)
        t.start()
        node = Node("node", dataflow=df.shm, device=0)
        s = device.Stream()
        with DeviceArray.from_pyarrow(cloud) as da, Plan.of(da) as p:
            ref = device.DeviceBuffer(p.size)
            p.pack(ref.ptr, p.size, s)
            s.sync()
            c = device.csum64(ref.ptr, p.size, s)
            ref.free()
            for k in range(3):
                node.send_output("data", da, {"csum": to_i64(c), "verify": True, "seq": k})
        # frees in this process (the cloud, the node's slots) race the sink's import of the
        # relay's newest slot: slots are whole 2 MiB allocations so that import cannot fail
        node.close()
        t.join(60)
        codes = df.wait(60)
        sink_log = df.log("sink")
    assert not relay_err, relay_err
    assert codes["sink"] == 0, (codes, sink_log)
    out = json.load(open(res))
    assert sum(x["verified"] for x in out["series"]) == 3
    assert sum(x["mismatches"] for x in out["series"]) == 0


def test_cross_gpu_bench_runs_on_one_gpu(launcher):
    """bench.py's C4 fan-out and C5 chain machinery with every stage on GPU 0 and the pull path
    forced: sources, relays and sinks finish, every verified payload is bit-exact."""
    sys.path.insert(0, ROOT)
    import bench
    out = bench.run_cross_gpu(
        3, launcher, timeout=180,
        runs=[("c4", bench.c4_descriptor, "kernel", {}),
              ("c5", bench.c5_descriptor, "kernel", {}),
              ("c5_sdma", bench.c5_descriptor, "sdma", {}),
              ("c4_rccl", bench.c4_descriptor, "kernel", {"fanout": "rccl"})],
        gpu=lambda g: 0, env={"DORA_GPU_EDGE_COPY": "1"}, tp_n=20)
    for name, r in out.items():
        assert r.get("ok"), (name, r)
        assert r["parity"]["mismatches"] == 0 and r["parity"]["verified_msgs"] > 0, r
        assert r["dropped_inputs"] == 0
    assert out["c4"]["receivers"] == 2
    assert set(out["c5"]["latency_us"]) == {"4096", "40960000"}
    # DORA_GPU_FANOUT=rccl with every receiver on the producer's GPU: the daemon admits no
    # broadcast group (one RCCL rank per device) and the receivers pull, bit-exact as before
    rc = out["c4_rccl"]
    assert rc["bcast"]["groups"] == 0 and rc["bcast"]["received"] == 0, rc
    assert "admitted no broadcast group" in rc["bcast"]["error"], rc
    assert rc["pulls"] > 0


@pytest.mark.gpu
def test_rccl_group_of_one_rank_broadcasts_in_place():
    """The RCCL fan-out path on one GPU (verdict r03 item 5): a broadcast group of one rank is
    formed (ncclGetUniqueId -> ncclCommInitRankConfig, non-blocking), one ncclBroadcast runs in
    place on a stream and the group is closed, all through the C ABI; the buffer's bytes are
    unchanged (the root's own data) and the communicator reports 1 rank, rank 0."""
    from ctypes import byref, c_int

    from dora_amd import device
    from dora_amd._lib import call
    from dora_amd.workloads import payload_seed
    size = 6220800  # one C4 frame (1920 x 1080 x 3)
    s = device.Stream()
    b = device.DeviceBuffer(size)
    try:
        device.fill_splitmix(b.ptr, size, payload_seed(size), s)
        s.sync()
        before = device.csum64(b.ptr, size, s)
        nranks, rank = c_int(-1), c_int(-1)
        call("dora_gpu_test_bcast_group", 0, b.ptr, size, byref(nranks), byref(rank))
        assert (nranks.value, rank.value) == (1, 0)
        assert device.csum64(b.ptr, size, s) == before
    finally:
        b.free()


def _distinct_sources(n, size):
    """n device buffers with distinct splitmix64 payloads and their checksums."""
    from dora_amd import device
    from dora_amd.verify import to_i64
    s = device.Stream()
    bufs, sums = [], []
    for k in range(n):
        b = device.DeviceBuffer(size)
        device.fill_splitmix(b.ptr, size, 0x5EED0000 + k, s)
        bufs.append(b)
    s.sync()
    for b in bufs:
        sums.append(to_i64(device.csum64(b.ptr, size, s)))
    s.close()
    return bufs, sums


def test_slow_receiver_drop_oldest_returns_tokens(launcher, tmp_path):
    """queue_size 2 (node_communication/mod.rs:320-359): a receiver that drains a burst of 60
    inputs at once is handed the oldest (the event its next() takes, like the one the reference's
    event-stream thread holds) and keeps exactly the newest 2 of the rest; every dropped input's
    token goes back at once, and the sender's close finds every token returned (no 10-s
    drop-token wait)."""
    import threading
    from dora_amd import device
    from dora_amd.dataflow import Dataflow
    from dora_amd.node import Node
    n_msgs, size = 60, 1 << 20
    desc = {"nodes": [
        {"id": "node", "path": "dynamic", "outputs": ["data"]},
        {"id": "recv", "path": "dynamic", "inputs": {"data": {"source": "node/data",
                                                               "queue_size": 2}}},
    ]}
    bufs, sums = _distinct_sources(n_msgs, size)
    with Dataflow(desc, launcher=launcher) as df:
        sent = threading.Event()
        got, err = [], []

        def receiver():
            try:
                r = Node("recv", dataflow=df.shm, device=0)
                sent.wait(60)
                s = device.Stream()
                for ev in r:
                    if ev["type"] != "INPUT":
                        continue
                    c = device.csum64(ev["data_ptr"], ev["data_len"], s)
                    got.append((ev["metadata"]["seq"], c, r.stats()["dropped_inputs"]))
                    del ev
                s.close()
                r.close()
            except Exception as e:  # noqa: BLE001
                err.append(e)
        t = threading.Thread(target=receiver)
        t.start()
        node = Node("node", dataflow=df.shm, device=0)
        for k in range(n_msgs):
            node.send_output_device_bytes("data", bufs[k].ptr, size, {"seq": k})
        # every fill complete before the receiver drains: the burst is fully "sent" in the
        # reference's sense (an input whose fill still runs is not queued for the policy yet)
        node.sync()
        sent.set()
        t_close = time.time()
        node_stats = node.stats()
        node.close()  # returns once every drop token is back
        close_s = time.time() - t_close
        t.join(60)
        df.wait(60)
    for b in bufs:
        b.free()
    assert not err, err
    # the handed-over input and exactly the newest queue_size of the rest survived, bit-exact;
    # the other 57 were dropped
    assert [g[0] for g in got] == [0, n_msgs - 2, n_msgs - 1], got
    from dora_amd.verify import to_i64
    assert [to_i64(g[1]) for g in got] == [sums[0]] + sums[-2:]
    assert got[0][2] == n_msgs - 3
    assert node_stats["slots_created"] + node_stats["cache_hits"] == n_msgs
    assert close_s < 5.0, close_s


def test_default_queue_keeps_up_with_async_burst(launcher, tmp_path):
    """A receiver with the reference's default queue_size (10) that keeps up with a back-to-back
    burst drops nothing: the sender keeps at most 10 samples in flight below 8 MiB (node.cpp
    max_in_flight), and inputs whose fill is still running are not yet queued for the drop
    policy (the reference fills before the message leaves the sender).  Every 50th input is
    checksummed against its source."""
    from dora_amd.dataflow import Dataflow
    from dora_amd.node import Node
    res = str(tmp_path / "sink.json")
    n_msgs, size, nsrc = 2000, 4096000, 16
    bufs, sums = _distinct_sources(nsrc, size)
    warm = 40  # slots created and mapped (milliseconds each) before the burst
    with Dataflow(_bench_desc(res, queue_size=10), launcher=launcher) as df:
        node = Node("node", dataflow=df.shm, device=0)
        node.set_async_sends(True)  # DORA_SEND_ASYNC: the contract under test
        for k in range(warm):
            node.send_output_device_bytes("data", bufs[k % nsrc].ptr, size, {"seq": k})
        node.send_output("data", b"", {"seq": warm, "ack": True})
        node.wait_input("ack", "seq", warm, 60.0)
        d0 = node.dataflow_counters("sink")["dropped_inputs"]
        for k in range(n_msgs):
            meta = {"seq": warm + 1 + k}
            if k % 50 == 0:
                meta.update({"csum": sums[k % nsrc], "verify": True})
            node.send_output_device_bytes("data", bufs[k % nsrc].ptr, size, meta)
        node.send_output("data", b"", {"seq": warm + 1 + n_msgs, "ack": True})
        node.wait_input("ack", "seq", warm + 1 + n_msgs, 60.0)
        dropped = node.dataflow_counters("sink")["dropped_inputs"] - d0
        node.close()
        codes = df.wait(60)
        log = df.log("sink")
    for b in bufs:
        b.free()
    assert codes["sink"] == 0, log
    out = json.load(open(res))
    assert out["errors"] == 0
    assert dropped == 0, (dropped, out["dropped_inputs"])
    assert sum(s["verified"] for s in out["series"]) == n_msgs // 50
    assert sum(s["mismatches"] for s in out["series"]) == 0


def test_queue_size_one_distinct_payloads_bit_exact(launcher, tmp_path):
    """A queue_size 1 receiver that checksums every input it keeps drops most of a fast
    sender's burst.  Dropped inputs return their tokens before their fills were waited on, so
    the sender refills recycled slots while earlier packs may still run: every payload is
    distinct and every delivered one must match its own checksum."""
    from dora_amd.dataflow import Dataflow
    from dora_amd.node import Node
    res = str(tmp_path / "sink.json")
    n_msgs, size, nsrc = 300, 4 << 20, 24
    bufs, sums = _distinct_sources(nsrc, size)
    with Dataflow(_bench_desc(res, queue_size=1), launcher=launcher) as df:
        node = Node("node", dataflow=df.shm, device=0)
        node.set_async_sends(True)  # DORA_SEND_ASYNC: the contract under test
        for k in range(n_msgs):
            node.send_output_device_bytes("data", bufs[k % nsrc].ptr, size,
                                          {"seq": k, "csum": sums[k % nsrc], "verify": True})
        stats = node.stats()
        node.close()
        codes = df.wait(60)
        log = df.log("sink")
    for b in bufs:
        b.free()
    assert codes["sink"] == 0, log
    out = json.load(open(res))
    assert out["errors"] == 0
    verified = sum(s["verified"] for s in out["series"])
    assert verified == sum(s["n"] for s in out["series"]) and verified > 0
    assert sum(s["mismatches"] for s in out["series"]) == 0
    assert verified + out["dropped_inputs"] == n_msgs, out
    assert stats["slots_created"] + stats["cache_hits"] == n_msgs


@pytest.mark.parametrize("mode", ["sync", "async"])
def test_cp_signalled_mid_size_sends_bit_exact(launcher, tmp_path, mode):
    """Mid-size single-segment packs sent alone are signalled by the command processor (the
    packet's completion signal in the flag's CpSignal line, shm.h) instead of the in-kernel flag
    store.  Sizes across the window (1-32 MiB: 2 MiB, 4 MiB + 13, misaligned sources, 16 MB) and
    past it (1 MiB - 16: in-kernel signals; 40.96 MB: in-kernel unless it runs alone, as every
    synchronous send does) interleave on the same slots' flags, so a flag goes from
    one completion rule to the other and back: every delivered payload must match its own
    checksum, and the sender must have used the CP path."""
    from dora_amd import device
    from dora_amd.dataflow import Dataflow
    from dora_amd.node import Node
    from dora_amd.verify import to_i64
    res = str(tmp_path / "sink.json")
    sizes = [(2 << 20, 0), ((4 << 20) + 13, 3), (4096000, 0), ((1 << 20) - 16, 0), (16 << 20, 7),
             (6 << 20, 1), (40960000, 0), ((2 << 20) - 1, 0)]
    nsrc = 6
    stride = 41 << 20
    s = device.Stream()
    bufs = []
    for k in range(nsrc):
        b = device.DeviceBuffer(stride)
        device.fill_splitmix(b.ptr, stride, 0xC0DE0000 + k, s)
        bufs.append(b)
    s.sync()
    plan = []
    n_msgs = 240
    for k in range(n_msgs):
        size, off = sizes[(k * 5 + k // len(sizes)) % len(sizes)]
        src = bufs[k % nsrc]
        plan.append((src.ptr + off, size, to_i64(device.csum64(src.ptr + off, size, s))))
    s.close()
    cp0 = device.aql_cp_signalled(0)
    with Dataflow(_bench_desc(res), launcher=launcher) as df:
        node = Node("node", dataflow=df.shm, device=0)
        node.set_async_sends(mode == "async")
        for k, (ptr, size, csum) in enumerate(plan):
            node.send_output_device_bytes("data", ptr, size,
                                          {"seq": k, "csum": csum, "verify": True})
        node.send_output("data", b"", {"seq": n_msgs, "ack": True})
        node.wait_input("ack", "seq", n_msgs, 60.0)
        node.close()
        codes = df.wait(60)
        log = df.log("sink")
    cp = device.aql_cp_signalled(0) - cp0
    for b in bufs:
        b.free()
    assert codes["sink"] == 0, log
    out = json.load(open(res))
    assert out["errors"] == 0
    assert sum(x["verified"] for x in out["series"]) == n_msgs
    assert sum(x["mismatches"] for x in out["series"]) == 0
    in_window = sum(1 for _, size, _ in plan if (1 << 20) <= size < (32 << 20))
    # a synchronous send runs its pack alone, so above the window too (aql.h `sync`)
    lone = sum(1 for _, size, _ in plan if size >= (1 << 20))
    print(f"{mode}: {cp} sends signalled by the command processor ({in_window} in the window, "
          f"{lone} at >= 1 MiB)")
    assert cp > 0
    if mode == "sync":  # one pack at a time: none waits in the backlog or goes out in a batch
        assert cp == lone, (cp, lone)


class _StreamHandle:
    def __init__(self, h):
        self.handle = h


@pytest.mark.parametrize("writer", ["kernel", "dma"])
@pytest.mark.parametrize("size", [256 << 10, (2 << 20) + 48])
def test_rewritten_source_each_send_bit_exact(launcher, tmp_path, writer, size):
    """One device source rewritten before every send (on the node stream, as
    dora_node_stream's contract says) — by a kernel, or by a host-to-device copy — and sent on
    the AQL path each time: every delivered sample must carry the bytes of its own rewrite.  The
    pack's workgroups may run on XCDs whose L2s still hold the buffer's lines from the previous
    pack; its agent-coherent loads (or the dispatch's acquire fence) must keep them from being
    served.  256 KiB: in-kernel-signalled packs behind the acquire fence; 2 MiB + 48: the
    CP-signalled mid-size packs, agent-coherent loads and no fence (aql.cpp mid_coherent)."""
    import ctypes
    from dora_amd import device
    from dora_amd._lib import call
    from dora_amd.dataflow import Dataflow
    from dora_amd.node import Node
    from dora_amd.verify import to_i64
    res = str(tmp_path / "sink.json")
    n_msgs = 200
    s = device.Stream()
    scratch = device.DeviceBuffer(size)
    sums, host = [], []
    for k in range(n_msgs):
        device.fill_splitmix(scratch.ptr, size, 0xC0FFEE00 + k, s)
        sums.append(to_i64(device.csum64(scratch.ptr, size, s)))
        if writer == "dma":
            host.append(scratch.to_bytes(stream=s))
    scratch.free()
    assert len(set(sums)) == n_msgs
    src = device.DeviceBuffer(size)
    with Dataflow(_bench_desc(res), launcher=launcher) as df:
        node = Node("node", dataflow=df.shm, device=0)
        node.set_async_sends(True)  # DORA_SEND_ASYNC: the contract under test
        for k in range(n_msgs):
            # dora_node_stream orders every fill launched so far (the previous pack still reading
            # `src`) before the work queued on it next: the rewrite
            ns = _StreamHandle(node.stream)
            if writer == "kernel":
                device.fill_splitmix(src.ptr, size, 0xC0FFEE00 + k, ns)
            else:
                hb = ctypes.create_string_buffer(host[k], size)
                call("dora_gpu_memcpy_async", src.ptr, hb, size, ns.handle)
            call("dora_gpu_stream_sync", ns.handle)  # node stream idle: the send takes AQL
            node.send_output_device_bytes("data", src.ptr, size,
                                          {"seq": k, "csum": sums[k], "verify": True})
        paths = node.fill_paths()
        node.close()
        codes = df.wait(60)
        log = df.log("sink")
    src.free()
    s.close()
    assert codes["sink"] == 0, log
    out = json.load(open(res))
    assert out["errors"] == 0
    assert sum(x["mismatches"] for x in out["series"]) == 0, out
    assert sum(x["verified"] for x in out["series"]) == n_msgs
    assert paths["aql"] >= n_msgs, paths


@pytest.mark.parametrize("mode,size,n_msgs", [("sync", 1 << 20, 200), ("async", 1 << 20, 200),
                                               ("sync", (3 << 20) + 5, 100),
                                               ("sync", 40960000, 60)])
def test_device_source_rewritten_on_unrelated_stream_after_send(launcher, tmp_path, mode, size,
                                                                n_msgs):
    """The reference copies inside send_output (arrow_utils.rs:48, node/mod.rs:206-209): the
    caller may rewrite its buffer as soon as the call returns.  Here the source is rewritten by
    a kernel on a stream the library knows nothing about, right after every send returns, with
    no synchronisation.  The default (synchronous) send must deliver every sample bit-exact —
    it returns when its read-signalled pack has every source byte in registers, while the
    stores still drain (aql_kernels.hip dora_aql_pack1r_u4; 1 MiB, a ragged 3 MiB + 5 B and the
    40.96 MB headline size); DORA_SEND_ASYNC makes no such promise (its contract: rewrite only
    via dora_node_stream or after dora_node_sync), and its count of corrupted samples is only
    reported."""
    from dora_amd import device
    from dora_amd.dataflow import Dataflow
    from dora_amd.node import Node
    from dora_amd.verify import to_i64
    res = str(tmp_path / "sink.json")
    s = device.Stream()
    scratch = device.DeviceBuffer(size)
    sums = []
    for k in range(n_msgs + 1):
        device.fill_splitmix(scratch.ptr, size, 0xFACE00 + k, s)
        sums.append(to_i64(device.csum64(scratch.ptr, size, s)))
    scratch.free()
    src = device.DeviceBuffer(size)
    other = device.Stream()   # unrelated to the node: no ordering with its fills
    device.fill_splitmix(src.ptr, size, 0xFACE00, other)
    other.sync()
    with Dataflow(_bench_desc(res), launcher=launcher) as df:
        node = Node("node", dataflow=df.shm, device=0)
        read0 = device.aql_dispatch_counts(0).get("dora_aql_pack1r_u4", 0)
        for k in range(n_msgs):
            # the rewrite launched after the previous send has finished before this send: a
            # source must be complete when it is sent (only what follows a send is under test)
            other.sync()
            node.send_output_device_bytes("data", src.ptr, size,
                                          {"seq": k, "csum": sums[k], "verify": True},
                                          asynchronous=mode == "async")
            device.fill_splitmix(src.ptr, size, 0xFACE00 + k + 1, other)  # no sync
        other.sync()
        reads = device.aql_dispatch_counts(0).get("dora_aql_pack1r_u4", 0) - read0
        node.close()
        codes = df.wait(60)
        log = df.log("sink")
    src.free()
    s.close()
    other.close()
    assert codes["sink"] == 0, log
    out = json.load(open(res))
    bad = sum(x["mismatches"] for x in out["series"])
    assert sum(x["verified"] for x in out["series"]) == n_msgs
    print(f"{mode} {size} B: {bad} of {n_msgs} samples corrupted by the rewrite; "
          f"{reads} read-signalled packs")
    if mode == "sync":
        assert bad == 0, out
        assert reads == n_msgs, reads


def test_device_array_send_waits_for_its_source(launcher):
    """send_output of a DeviceArray (the Python node API, a multi-segment pack) returns once the
    pack has read the array: both child buffers of a Struct<x,y:i64> are overwritten on an
    unrelated stream right after each send, and every array arrives with its own checksum."""
    import ctypes
    import numpy as np
    import pyarrow as pa
    from dora_amd import device
    from dora_amd._lib import call
    from dora_amd.dataflow import Dataflow
    from dora_amd.device import DeviceArray
    from dora_amd.node import Node
    from dora_amd.verify import to_u64
    from oracle.arrow_ffi import import_array
    from oracle.checksum_ref import regions_csum
    from oracle.pack_ref import node_regions
    desc = {"nodes": [
        {"id": "src", "path": "dynamic", "outputs": ["pc"], "inputs": {"result": "recv/result"}},
        {"id": "recv", "path": sys.executable,
         "args": [os.path.join(ROOT, "examples", "verify_receiver.py")],
         "inputs": {"pc": {"source": "src/pc", "queue_size": 100}}, "outputs": ["result"]},
    ]}
    n, k_msgs = 1 << 18, 16
    rng = np.random.default_rng(5)
    arrs = [pa.StructArray.from_arrays([pa.array(rng.integers(-2**62, 2**62, n)),
                                        pa.array(rng.integers(-2**62, 2**62, n))],
                                       names=["x", "y"]) for _ in range(k_msgs)]
    want = [regions_csum(node_regions(import_array(a))) for a in arrs]
    devs = [DeviceArray.from_pyarrow(a) for a in arrs]

    def child_values(da, c):
        child = da.array.children[c].contents
        return ctypes.cast(child.buffers, ctypes.POINTER(ctypes.c_void_p))[1]
    other = device.Stream()
    with Dataflow(desc, launcher=launcher) as df:
        node = Node("src", dataflow=df.shm, device=0)
        with DeviceArray.from_pyarrow(arrs[0]) as da:
            for seq in range(k_msgs):
                # the rewrite queued after the previous send has landed (it races that send's pack,
                # not this one's: the stream is not ordered with the node's packs)
                other.sync()
                node.send_output("pc", da, {"seq": seq})
                if seq + 1 < k_msgs:   # the next array's bytes into the sent one's buffers, no sync
                    for c in range(2):
                        call("dora_gpu_memcpy_async", child_values(da, c),
                             child_values(devs[seq + 1], c), 8 * n, other.handle)
            other.sync()
            results = {}
            deadline = time.time() + 120
            while len(results) < k_msgs and time.time() < deadline:
                ev = node.next(timeout=5)
                if ev is None:
                    break
                if ev["type"] == "INPUT":
                    results[ev["metadata"]["seq"]] = ev["metadata"]
        node.close()
        codes = df.wait(60)
        log = df.log("recv")
    for d in devs:
        d.close()
    other.close()
    assert codes["recv"] == 0, log
    for seq in range(k_msgs):
        assert to_u64(results[seq]["csum"]) == want[seq], seq


def test_big_multi_segment_async_sends_bit_exact(launcher):
    """Asynchronous 16 MiB Struct<x,y:i64> sends (two-segment packs >= 8 MiB, on the barrier
    queues with their arguments in the device ring): every array arrives with its own checksum."""
    import numpy as np
    import pyarrow as pa
    from dora_amd.dataflow import Dataflow
    from dora_amd.device import DeviceArray
    from dora_amd.node import Node
    from dora_amd.verify import to_u64
    from oracle.arrow_ffi import import_array
    from oracle.checksum_ref import regions_csum
    from oracle.pack_ref import node_regions
    desc = {"nodes": [
        {"id": "src", "path": "dynamic", "outputs": ["pc"], "inputs": {"result": "recv/result"}},
        {"id": "recv", "path": sys.executable,
         "args": [os.path.join(ROOT, "examples", "verify_receiver.py")],
         "inputs": {"pc": {"source": "src/pc", "queue_size": 100}}, "outputs": ["result"]},
    ]}
    n, k_msgs = 1 << 20, 12
    rng = np.random.default_rng(11)
    arrs = [pa.StructArray.from_arrays([pa.array(rng.integers(-2**62, 2**62, n)),
                                        pa.array(rng.integers(-2**62, 2**62, n))],
                                       names=["x", "y"]) for _ in range(k_msgs)]
    want = [regions_csum(node_regions(import_array(a))) for a in arrs]
    devs = [DeviceArray.from_pyarrow(a) for a in arrs]
    try:
        with Dataflow(desc, launcher=launcher) as df:
            node = Node("src", dataflow=df.shm, device=0)
            node.set_async_sends(True)
            for seq in range(k_msgs):
                node.send_output("pc", devs[seq], {"seq": seq})
            results = {}
            deadline = time.time() + 120
            while len(results) < k_msgs and time.time() < deadline:
                ev = node.next(timeout=5)
                if ev is None:
                    break
                if ev["type"] == "INPUT":
                    results[ev["metadata"]["seq"]] = ev["metadata"]
            node.close()
            codes = df.wait(60)
            log = df.log("recv")
    finally:
        for d in devs:
            d.close()
    assert codes["recv"] == 0, log
    for seq in range(k_msgs):
        assert to_u64(results[seq]["csum"]) == want[seq], seq


def test_host_source_reused_right_after_send_bit_exact(launcher, tmp_path):
    """send_output_raw semantics for host data (examples/benchmark/node/src/main.rs:46-48: the
    closure copies `data` before send returns): one host buffer overwritten with the next payload
    as soon as each send returns, through the C ABI as a Rust node would call it.  Every
    delivered sample must hold the payload of its own send."""
    import ctypes
    from dora_amd import device
    from dora_amd._lib import ARROW_DEVICE_CPU
    from dora_amd.dataflow import Dataflow
    from dora_amd.node import Node, _fast
    from dora_amd.verify import to_i64
    res = str(tmp_path / "sink.json")
    n_msgs, size = 120, 1 << 20
    payloads = [os.urandom(size) for _ in range(n_msgs)]
    s = device.Stream()
    sums = []
    for p in payloads:
        b = device.DeviceBuffer.from_bytes(p, s)
        sums.append(to_i64(device.csum64(b.ptr, size, s)))
        b.free()
    s.close()
    buf = ctypes.create_string_buffer(size)
    with Dataflow(_bench_desc(res), launcher=launcher) as df:
        node = Node("node", dataflow=df.shm, device=0)
        for k in range(n_msgs):
            ctypes.memmove(buf, payloads[k], size)
            rc = _fast.send_bytes(node.handle, "data", ctypes.addressof(buf), size,
                                  ARROW_DEVICE_CPU, {"seq": k, "csum": sums[k], "verify": True})
            assert rc == 0
            ctypes.memset(buf, 0xA5, size)  # the caller reuses its buffer at once
        node.close()
        codes = df.wait(60)
        log = df.log("sink")
    assert codes["sink"] == 0, log
    out = json.load(open(res))
    assert out["errors"] == 0
    assert sum(x["mismatches"] for x in out["series"]) == 0, out
    assert sum(x["verified"] for x in out["series"]) == n_msgs


def test_output_without_receivers_recycles_safely(launcher, tmp_path):
    """Sends on an output nobody subscribes to get their drop token back at once (the daemon's
    check_drop_token with no pending receiver), long before their packs finish.  The recycled
    slots then carry the next sends, here interleaved with verified sends on a connected
    output: every verified payload is bit-exact and no slot is created per send."""
    from dora_amd.dataflow import Dataflow
    from dora_amd.node import Node
    res = str(tmp_path / "sink.json")
    size, nsrc = 4 << 20, 16
    bufs, sums = _distinct_sources(nsrc, size)
    desc = {"nodes": [
        {"id": "node", "path": "dynamic", "outputs": ["void", "data"]},
        {"id": "sink", "path": "dora-gpu-bench-sink", "outputs": ["ack"],
         "inputs": {"data": {"source": "node/data", "queue_size": 1000}},
         "env": {"DORA_BENCH_RESULT": res}},
    ]}
    with Dataflow(desc, launcher=launcher) as df:
        node = Node("node", dataflow=df.shm, device=0)
        n_data = 0
        for k in range(400):
            if k % 8 == 7:
                node.send_output_device_bytes("data", bufs[k % nsrc].ptr, size,
                                              {"seq": k, "csum": sums[k % nsrc], "verify": True})
                n_data += 1
            else:
                node.send_output_device_bytes("void", bufs[k % nsrc].ptr, size, {"seq": k})
        stats = node.stats()
        t_close = time.time()
        node.close()
        close_s = time.time() - t_close
        codes = df.wait(60)
        log = df.log("sink")
    for b in bufs:
        b.free()
    assert codes["sink"] == 0, log
    out = json.load(open(res))
    assert out["errors"] == 0
    assert sum(s["verified"] for s in out["series"]) == n_data
    assert sum(s["mismatches"] for s in out["series"]) == 0
    assert stats["slots_created"] <= 40, stats
    assert close_s < 5.0, close_s


def _roundtrip_through_node(launcher, names, env=None):
    """Every fixture sent as a device array by one node and received by another node of this
    process: returns [(name, event type info json, oracle type info json, equal)]."""
    from dora_amd.dataflow import Dataflow
    from dora_amd.device import DeviceArray
    from dora_amd.node import Node
    from oracle.pack_ref import pack
    from tests.golden import recipes
    desc = {"nodes": [
        {"id": "src", "path": "dynamic", "outputs": ["x"]},
        {"id": "dst", "path": "dynamic", "inputs": {"x": {"source": "src/x", "queue_size": 1000}}},
    ]}
    out = []
    old = {k: os.environ.get(k) for k in (env or {})}
    os.environ.update(env or {})
    try:
        with Dataflow(desc, launcher=launcher) as df:
            # both nodes live in this process; each init waits for AllNodesReady
            import threading
            box = {}
            t = threading.Thread(target=lambda: box.update(dst=Node("dst", dataflow=df.shm,
                                                                    device=0)))
            t.start()
            src = Node("src", dataflow=df.shm, device=0)
            t.join(60)
            dst = box["dst"]
            for name in names:
                arr = recipes.build(name)
                _, info = pack(arr)
                with DeviceArray.from_pyarrow(arr) as da:
                    src.send_output("x", da, {"name": name})
                ev = dst.next(timeout=30)
                assert ev is not None and ev["type"] == "INPUT", ev
                assert ev["metadata"]["name"] == name
                if ev["data_len"] == 0:
                    # empty sample -> ArrayData::new_empty(data_type) (event.rs:65-67): a
                    # NullArray's length does not survive, as in the reference
                    import pyarrow as pa
                    equal = ev["value"].equals(pa.array([], type=arr.type))
                else:
                    equal = ev["value"].to_pyarrow().equals(arr)
                out.append((name, ev["type_info"].to_json(), info.to_json(), equal))
                del ev
            src.close()
            dst.close()
            df.wait(30)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    return out


def test_plan_cache_repeated_and_reused_addresses(launcher):
    """The node's plan cache: the same device array sent three times is planned once and every
    copy arrives intact; arrays allocated afterwards (possibly at the freed addresses, with
    other types, lengths and null counts) get plans of their own."""
    import threading
    from dora_amd.dataflow import Dataflow
    from dora_amd.device import DeviceArray
    from dora_amd.node import Node
    from tests.golden import recipes
    names = ["point_cloud_small", "struct_nulls_sliced", "list_i64_nulls", "i32_nulls_1000",
             "f64_sliced_nulls", "fixed_size_list", "deep_nesting", "point_cloud_small"]
    assert set(names) <= set(recipes.CASES)
    desc = {"nodes": [
        {"id": "src", "path": "dynamic", "outputs": ["x"]},
        {"id": "dst", "path": "dynamic", "inputs": {"x": {"source": "src/x", "queue_size": 1000}}},
    ]}
    with Dataflow(desc, launcher=launcher) as df:
        box = {}
        t = threading.Thread(target=lambda: box.update(dst=Node("dst", dataflow=df.shm, device=0)))
        t.start()
        src = Node("src", dataflow=df.shm, device=0)
        t.join(60)
        dst = box["dst"]
        for name in names:
            arr = recipes.build(name)
            with DeviceArray.from_pyarrow(arr) as da:
                for k in range(3):
                    src.send_output("x", da, {"name": name, "k": k})
                    ev = dst.next(timeout=30)
                    assert ev["metadata"] == {"name": name, "k": k}
                    assert ev["value"].to_pyarrow().equals(arr), (name, k)
                    del ev
        stats = src.plan_cache_stats()
        src.close()
        dst.close()
        df.wait(30)
    # arrays whose plan reads device bytes (slices exported with an unknown null count) are
    # planned every time; the others twice from the cache
    assert stats["entries"] >= 4 and stats["hits"] >= 2 * stats["entries"], stats


def test_in_sample_validity_type_info_and_roundtrip(launcher):
    """Device arrays sent by a node carry their validity bitmaps in the sample's tail (tag 2);
    the receiver's ArrowTypeInfo (dora_event_type_info, inline form restored from the slot) is
    identical to the oracle's and the zero-copy import equals the original array (nulls,
    nested, sliced, dictionary, strings)."""
    from tests.golden import recipes
    names = recipes.KATS + recipes.CASES
    for name, got, want, equal in _roundtrip_through_node(launcher, names):
        assert got == want, name
        assert equal, name


def test_two_daemons_device_samples_bit_exact(launcher, tmp_path):
    """A dataflow over two machines' daemons (here both on this box): machine A's forwarder
    waits for each device sample's fill, maps the slot, stages it to the host (validity tails
    folded back into the type info) and sends it over TCP; machine B's proxy uploads it into a
    slot of its own and re-sends it.  4 MB payloads are checksummed by B's sink; point clouds
    (nested, with nulls) arrive equal at a Python receiver."""
    import threading
    from dora_amd.dataflow import Dataflow
    from dora_amd.device import DeviceArray
    from dora_amd.node import Node
    from dora_amd.workloads import point_cloud
    res = str(tmp_path / "sink.json")
    desc = {"nodes": [
        {"id": "node", "path": "dynamic", "outputs": ["data", "pc"],
         "_unstable_deploy": {"machine": "A", "gpu": 0}},
        {"id": "sink", "path": "dora-gpu-bench-sink", "outputs": ["ack"],
         "inputs": {"data": {"source": "node/data", "queue_size": 1000}},
         "env": {"DORA_BENCH_RESULT": res}, "_unstable_deploy": {"machine": "B", "gpu": 0}},
        {"id": "recv", "path": "dynamic", "inputs": {"pc": {"source": "node/pc", "queue_size": 100}},
         "_unstable_deploy": {"machine": "B", "gpu": 0}},
    ]}
    size, n_msgs = 4 << 20, 20
    bufs, sums = _distinct_sources(4, size)
    clouds = [point_cloud(3000, 5, seed=s) for s in (1, 2, 3)]
    b = Dataflow(desc, machine="B", machines={"B": ("127.0.0.1", 0), "A": ("127.0.0.1", 1)},
                 dataflow_id="df-gpu", launcher=launcher, log_dir=str(tmp_path / "B")).start()
    a = Dataflow(desc, machine="A",
                 machines={"A": ("127.0.0.1", 0), "B": ("127.0.0.1", b.listen_port)},
                 dataflow_id="df-gpu", launcher=launcher, log_dir=str(tmp_path / "A")).start()
    got, errs = [], []

    def receiver():
        try:
            r = Node("recv", dataflow=b.shm, device=0)
            for ev in r:
                if ev["type"] == "INPUT":
                    got.append((ev["metadata"]["seq"], ev["value"].to_pyarrow()))
                    del ev
            r.close()
        except Exception as e:  # noqa: BLE001
            errs.append(e)
    t = threading.Thread(target=receiver)
    t.start()
    try:
        node = Node("node", dataflow=a.shm, device=0)
        for k in range(n_msgs):
            node.send_output_device_bytes("data", bufs[k % 4].ptr, size,
                                          {"seq": k, "csum": sums[k % 4], "verify": True})
        for k, pc in enumerate(clouds):
            with DeviceArray.from_pyarrow(pc) as da:
                node.send_output("pc", da, {"seq": k})
        node.close()
        t.join(60)
        codes = {"A": a.wait(60), "B": b.wait(60)}
        logs = {"A": a.log("_daemon"), "B": b.log("_daemon"), "sink": b.log("sink")}
    finally:
        a.stop()
        b.stop()
        for x in bufs:
            x.free()
    assert not errs, errs
    assert codes["B"]["sink"] == 0 and codes["A"]["_daemon"] == 0 and codes["B"]["_daemon"] == 0, \
        (codes, logs)
    out = json.load(open(res))
    assert sum(s["verified"] for s in out["series"]) == n_msgs, (out, logs)
    assert sum(s["mismatches"] for s in out["series"]) == 0
    assert [g[0] for g in got] == [0, 1, 2]
    for (_, arr), pc in zip(got, clouds):
        assert arr.equals(pc)
    assert f'"forwarded": {n_msgs + 3 + 2}' in logs["A"], logs["A"]


@pytest.mark.parametrize("mode", ["sync", "async"])
def test_full_size_samples_byte_identical_to_the_oracle(launcher, mode):
    """Byte-level parity at BASELINE's full sizes (verdict r03 weak 1: until now only checksums
    above 409,600 B): a 40,960,000-B UInt8 payload from an aligned source and from one 3 bytes
    past a 16-B boundary (BASELINE configs[1]), and a 1M-point cloud (configs[2]; validity tail
    included in the slot), sent through the daemon to a second node; every delivered byte is
    compared with the oracle's — splitmix64 payload bytes (oracle/checksum_ref.py) and the
    restated copy_array_into_sample sample (oracle/pack_ref.py, arrow_utils.rs:23-71)."""
    import ctypes

    from dora_amd import device
    from dora_amd._lib import call
    from dora_amd.dataflow import Dataflow
    from dora_amd.device import DeviceArray
    from dora_amd.node import Node
    from dora_amd.workloads import point_cloud
    from oracle.checksum_ref import payload_seed, splitmix_bytes
    from oracle.pack_ref import pack
    S = 40960000
    want_c2 = splitmix_bytes(S, payload_seed(S))
    cloud = point_cloud()
    want_c3, _ = pack(cloud)
    s = device.Stream()
    src = device.DeviceBuffer(S + 16)
    desc = {"nodes": [
        {"id": "src", "path": "dynamic", "outputs": ["out"]},
        {"id": "dst", "path": "dynamic", "inputs": {"in": {"source": "src/out", "queue_size": 8}}},
    ]}

    def host_copy(ev):
        out = ctypes.create_string_buffer(max(ev["data_len"], 1))
        call("dora_gpu_memcpy_async", out, ev["data_ptr"], ev["data_len"], s.handle)
        s.sync()
        return out.raw[:ev["data_len"]]
    try:
        with Dataflow(desc, launcher=launcher) as df:
            nodes = {}

            def mk(i):  # both dynamic nodes subscribe before either sees AllNodesReady
                nodes[i] = Node(i, dataflow=df.shm, device=0)
            ts = [threading.Thread(target=mk, args=(i,)) for i in ("src", "dst")]
            [t.start() for t in ts]
            [t.join(90) for t in ts]
            tx, rx = nodes["src"], nodes["dst"]
            tx.set_async_sends(mode == "async")
            got = []
            for off in (0, 3):
                device.fill_splitmix(src.ptr + off, S, payload_seed(S), s)
                s.sync()
                tx.send_output_device_bytes("out", src.ptr + off, S, {"off": off})
                if mode == "async":
                    tx.sync()  # the next fill rewrites the source
                ev = rx.next(timeout=30)
                assert ev is not None and ev["type"] == "INPUT" and ev["on_device"], ev
                got.append((ev["metadata"]["off"], host_copy(ev)))
                del ev
            with DeviceArray.from_pyarrow(cloud) as da:
                tx.send_output("out", da, {"c3": True})
                tx.sync()
            ev = rx.next(timeout=30)
            assert ev is not None and ev["metadata"] == {"c3": True}
            c3 = host_copy(ev)
            del ev
            tx.close()
            rx.close()
    finally:
        src.free()
        s.close()
    for off, b in got:
        assert len(b) == S
        assert b == want_c2, (off, next(i for i in range(S) if b[i] != want_c2[i]))
    assert len(c3) == len(want_c3) and c3 == bytes(want_c3)


@pytest.mark.parametrize("event_thread", [False, True])
def test_events_consumed_on_another_thread_bit_exact(event_thread):
    """The node is made on this thread; its events are taken, mapped and checksummed on a
    worker thread that never selected a HIP device — as a Rust EventStream moved to another
    thread, or the facade's async pump (node.cpp DeviceScope: every entry point makes the node's
    GPU current for the call).  With `event_thread` the node also drains on its event-stream
    thread.  One GPU cannot tell devices apart; this keeps the hand-over itself exact."""
    import ctypes

    from dora_amd import _lib, device
    from dora_amd.dataflow import daemon_spec, parse_descriptor
    from dora_amd.device import DeviceBuffer
    from dora_amd.node import Node
    lib = _lib.load()
    device.set_device(0)
    desc = {"nodes": [{"id": "src", "outputs": ["x"]},
                      {"id": "dst", "inputs": {"x": {"source": "src/x", "queue_size": 64}}}]}
    shm = f"/dora-gpu-xthread-{os.getpid()}-{int(event_thread)}"
    h = ctypes.c_void_p()
    _lib.call("dora_daemon_create", shm.encode(), daemon_spec(parse_descriptor(desc)).encode(),
              1 << 20, ctypes.byref(h))
    threading.Thread(target=lambda: lib.dora_daemon_run(h.value, 120000), daemon=True).start()
    nodes = {}
    ts = [threading.Thread(target=lambda i=i: nodes.update({i: Node(i, dataflow=shm, device=0)}))
          for i in ("src", "dst")]
    [t.start() for t in ts]
    [t.join(60) for t in ts]
    src, dst = nodes["src"], nodes["dst"]
    if event_thread:
        dst.set_event_thread(True)
    sizes = [4096, 65536, 1 << 20, 4 << 20, 13000068]
    s = device.Stream()
    bufs = {z: DeviceBuffer(z) for z in sizes}
    want = {}
    for k, z in enumerate(sizes):
        device.fill_splitmix(bufs[z].ptr, z, 0x7E + k, s)
        want[z] = device.csum64(bufs[z].ptr, z, s)
    got, errors = {}, []

    def consume():
        try:
            ws = device.Stream()  # created on this thread's current device
            for _ in range(3 * len(sizes)):
                ev = dst.next(timeout=30)
                assert ev is not None and ev["type"] == "INPUT", ev
                z = ev["metadata"]["n"]
                got.setdefault(z, []).append(device.csum64(ev["data_ptr"], z, ws))
                ev["value"].close()
                ev["_event"].free()
            ws.close()
        except Exception as e:  # noqa: BLE001 — reported below
            errors.append(repr(e))
    w = threading.Thread(target=consume)
    w.start()
    for r in range(3):
        for z in sizes:
            src.send_output_device_bytes("x", bufs[z].ptr, z, {"n": z, "r": r})
    w.join(120)
    src.close()
    dst.close()
    lib.dora_daemon_free(h.value)
    for b in bufs.values():
        b.free()
    s.close()
    assert not errors, errors
    for z in sizes:
        assert got.get(z) == [want[z]] * 3, (z, got.get(z), want[z])
