#!/usr/bin/env python3
"""bench.py — node->node device data plane on MI355X (BASELINE.json metric).

One rank per GPU.  Each rank runs its own local dataflow on its GPU (weak scaling: dataflow
graphs shard by node placement, SURVEY.md §8e — no data-path collective):

    node (this process, `path: dynamic`) --latency/throughput--> sink (dora-gpu-bench-sink)
         ^------------------------------------ ack ---------------------------------'

A step = one message of `--size` bytes (default 40,960,000 B, the top of the C2 ladder) sent
with `send_output_raw` semantics: allocate a device slot (20-entry recycled cache), HIP pack
kernel HBM->HBM from the node's device-resident source, descriptor through the daemon, IPC-mapped
zero-copy delivery at the sink, drop token back.  The timed region is K back-to-back steps
closed by the sink's ack of the last one, bracketed by barrier + device sync.

value = total payload bytes delivered by all ranks / max-over-ranks time (GB/s).
The JSON line also carries the per-size latency ladder (p50/p99, reference semantics: timestamp
after the fill), the pack-kernel roofline (HIP events on the node stream) and the CPU baseline
(C++ restatement of the reference shm path, oracle/build/shm_baseline, rank 0 at N=1).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
LADDER = [4096, 16384, 40960, 65536, 409600, 1 << 20, 4096000, 4 << 20, 16 << 20, 40960000]
# the rest of the reference ladder (examples/benchmark/node/src/main.rs:11-21): sizes the
# reference sends inline (< 4096 B, DataMessage::Vec); a device node sends them in slots too
LADDER_SMALL = [0, 8, 64, 512, 2048]
# host-resident sources of the latency ladder (output `latency_host`): below 4096 B they travel
# inline as the reference's DataMessage::Vec (no slot, no GPU), 4096 B is an H2D device sample
LADDER_HOST = [8, 512, 2048, 4096, 65536, 4 << 20, 6220800, 40960000]
# device-resident sources delivered to a node without a GPU (`hostsink`, DORA_GPU_DEVICE -1),
# the reference's host ArrowData (event.rs:35-91): `to_host` has no other receiver, so samples
# <= 1 MiB are packed by the producer straight into shared memory, larger ones staged to host
# memory on receipt
LADDER_D2H = [8, 4096, 65536, 1 << 20, 6220800, 40960000]


def host_lat_n(size, lat_n):
    """Latency-mode messages per host-source / host-receiver size: the full count up to 64 KB,
    200 above (a 40.96 MB message crosses PCIe in ~0.75 ms)."""
    return lat_n if size <= 65536 else min(lat_n, 200)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--size", type=int, default=40960000)
    ap.add_argument("--workload", choices=["c2", "c3"], default="c2",
                    help="c2: UInt8 payloads (BASELINE configs[1], default); c3: nested "
                         "List<Struct<x,y,z,intensity>> 1M-point clouds (configs[2])")
    ap.add_argument("--lat-n", type=int, default=1000,
                    help="latency-mode messages per size (SURVEY §8d: >= 1000 for a stable p99)")
    ap.add_argument("--lat-gap-us", type=int, default=1000)
    ap.add_argument("--no-ladder", action="store_true")
    ap.add_argument("--tp-n", type=int, default=200,
                    help="throughput ladder: back-to-back messages per size, at least 2000 up "
                         "to 4 MiB (0: skip)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--keep-awake-us", type=float, default=None,
                    help="period of the senders' keep-awake packets (dora_gpu_set_keep_awake; "
                         "0: off; default: the library's, 25)")
    ap.add_argument("--no-c3", action="store_true",
                    help="skip the C3 block the default C2 run reports beside the headline")
    ap.add_argument("--c3-steps", type=int, default=20)
    ap.add_argument("--sync-n", type=int, default=20,
                    help="default (synchronous) sends at the headline size after the timed "
                         "region (sync_send_headline; 0: skip)")
    ap.add_argument("--detail", default=os.path.join(ROOT, "gpurun_out", "bench_detail.json"),
                    help="file for the full result (stdout carries the compact line)")
    ap.add_argument("--sources", type=int, default=0, help="rotating source buffers (0: auto)")
    ap.add_argument("--c3-lists", type=int, default=0,
                    help="c3 diagnosis: lists per cloud (15: every buffer at 0 mod 16)")
    ap.add_argument("--src-offset", type=int, default=0,
                    help="c2 diagnosis: source bytes start this far past a 256-B boundary")
    ap.add_argument("--no-cross-gpu", action="store_true",
                    help="N>1: skip the C4 fan-out / C5 chain runs after the timed region")
    ap.add_argument("--no-kernel-timing", action="store_true",
                    help="skip the per-launch kernel stamps (roofline then unmeasured)")
    return ap.parse_args()


class Ranks:
    """Cross-rank control for the weak-scaled replicas: barrier and max/sum of scalars over a
    gloo (CPU) process group — the data path itself has no collective."""

    def __init__(self, world: int):
        self.dist = None
        if world > 1:
            import torch.distributed as dist
            if not dist.is_initialized():
                # gloo prints "[Gloo] Rank r is connected to ..." on fd 1: keep stdout for the
                # one JSON line (the banner goes to stderr instead)
                sys.stdout.flush()
                saved = os.dup(1)
                os.dup2(2, 1)
                try:
                    dist.init_process_group("gloo")
                finally:
                    os.dup2(saved, 1)
                    os.close(saved)
            self.dist = dist

    def barrier(self):
        if self.dist is not None:
            self.dist.barrier()

    def _reduce(self, x: float, op) -> float:
        if self.dist is None:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=op)
        return float(t.item())

    def max(self, x: float) -> float:
        return self._reduce(x, self.dist.ReduceOp.MAX) if self.dist else x

    def sum(self, x: float) -> float:
        return self._reduce(x, self.dist.ReduceOp.SUM) if self.dist else x


def box_copy_rate(size: int, stream, n_src: int = 8, reps: int = 24):
    """hipMemcpyAsync device-to-device of `size` bytes, `reps` back-to-back copies from `n_src`
    rotating sources (beyond the 256 MB Infinity Cache at the headline size), timed with events
    on one stream: the plain copy rate of this box right now, in 2·S bytes per second (TB/s)."""
    from dora_amd import device
    from dora_amd._lib import call
    srcs = [device.DeviceBuffer(size) for _ in range(n_src)]
    dst = device.DeviceBuffer(size)
    e0, e1 = device.Event(), device.Event()
    try:
        for k in range(3):
            call("dora_gpu_memcpy_async", dst.ptr, srcs[k % n_src].ptr, size, stream.handle)
        e0.record(stream)
        for k in range(reps):
            call("dora_gpu_memcpy_async", dst.ptr, srcs[k % n_src].ptr, size, stream.handle)
        e1.record(stream)
        e1.sync()
        us = e0.elapsed_ms(e1) * 1e3 / reps
        return {"bytes": size, "us_per_copy": round(us, 3),
                "TBps_2S": round(2 * size / (us * 1e-6) / 1e12, 3)}
    finally:
        e0.close(); e1.close(); dst.free()
        for b in srcs:
            b.free()


def box_h2d_rate(size: int, stream, reps: int = 10):
    """PCIe DMA of `size` bytes between pinned host memory and HBM on this box (hipMemcpyAsync,
    events on one stream), both directions: the H2D / D2H roofline the host paths are measured
    against (host sources, host-only receivers)."""
    from ctypes import c_void_p, byref
    from dora_amd import device
    from dora_amd._lib import call
    h = c_void_p()
    call("dora_gpu_host_alloc", byref(h), size)
    d = device.DeviceBuffer(size)
    e0, e1 = device.Event(), device.Event()
    out = {"bytes": size}
    try:
        for name, dst, src in (("h2d", d.ptr, h.value), ("d2h", h.value, d.ptr)):
            call("dora_gpu_memcpy_async", dst, src, size, stream.handle)
            e0.record(stream)
            for _ in range(reps):
                call("dora_gpu_memcpy_async", dst, src, size, stream.handle)
            e1.record(stream)
            e1.sync()
            us = e0.elapsed_ms(e1) * 1e3 / reps
            out[f"{name}_GBps"] = round(size / (us * 1e-6) / 1e9, 2)
        return out
    finally:
        e0.close(); e1.close(); d.free()
        call("dora_gpu_host_free", h.value)


def aql_kernel_name(workload: str, region_kernels=None) -> str:
    """The AQL pack kernel of a timed region: the one dispatched most there
    (dora_gpu_aql_dispatch_counts), else the one a pipelined send of this workload dispatches
    (aql.cpp dispatch_locked: one segment at offset 0 -> pack1, nested arrays -> pack)."""
    if region_kernels:
        return max(region_kernels, key=region_kernels.get) + " (AQL)"
    return ("dora_aql_pack1_u4" if workload == "c2" else "dora_aql_pack_u4") + " (AQL)"


def pmc_traffic(msg_bytes: int):
    """HBM bytes per pack launch from the newest committed PMC run for this message size
    (profiles/r*_pmc_traffic.json, FETCH_SIZE x2 + WRITE_SIZE per MI355X_MICROARCH.md)."""
    import glob
    best = None
    for p in sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_pmc_traffic.json"))):
        try:
            d = json.load(open(p))
        except (OSError, ValueError):
            continue
        if d.get("algorithmic_bytes_per_launch") == 2 * msg_bytes:
            best = (os.path.basename(p), d["traffic_bytes_per_launch"])
    return best


def cpu_share():
    """This box's CPU share: the cgroup's quota, its throttling counters and the load average
    (the boxes are a 16-CPU share of a shared host; a throttled period stalls every thread of
    the dataflow for the rest of the 100 ms period)."""
    out = {"nproc_affinity": len(os.sched_getaffinity(0))}
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        out["cpu_max"] = None if q == "max" else round(int(q) / int(per), 2)
        st = dict(line.split() for line in open("/sys/fs/cgroup/cpu.stat"))
        for k in ("nr_periods", "nr_throttled", "throttled_usec"):
            out[k] = int(st.get(k, 0))
    except (OSError, ValueError):
        pass
    try:
        out["loadavg_1m"] = float(open("/proc/loadavg").read().split()[0])
    except (OSError, ValueError):
        pass
    return out


def share_delta(a, b):
    return {k: b[k] - a[k] for k in ("nr_periods", "nr_throttled", "throttled_usec")
            if k in a and k in b}


def busy_union_ms(intervals):
    """Length of the union of [start, stop] intervals (ms)."""
    total, end = 0.0, None
    for a, b in sorted(intervals):
        if end is None or a > end:
            total += b - a
            end = b
        elif b > end:
            total += b - end
            end = b
    return total


def cpu_baseline(rank_cores):
    """Reference shm path restated in C++ (oracle/shm_baseline.cpp), bounded sample."""
    exe = os.path.join(ROOT, "oracle", "build", "shm_baseline")
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    cores = ",".join(str(c) for c in rank_cores[:3])
    sizes = "4096,40960,409600,4096000,40960000"
    out = subprocess.run([exe, "--sizes", sizes, "--lat-n", "100", "--lat-gap-us", "10000",
                          "--tp-n", "200", "--cores", cores], capture_output=True, text=True,
                         timeout=300, check=True).stdout
    return json.loads(out)


XGMI_LINK_GBPS = 153.0  # MI355X: 7 xGMI links x ~153 GB/s per GPU (one link per peer)
C4_FRAME = 1920 * 1080 * 3      # BASELINE configs C4: 6,220,800 B frames
C5_SIZES = [4096, 40960000]      # BASELINE configs C5: control message + tensor per stage


def _source_env(result, lat_sizes, tp_size, tp_n, acks, lat_n=30, gap_us=33333):
    return {"DORA_BENCH_RESULT": result, "DORA_BENCH_LAT_SIZES": ",".join(map(str, lat_sizes)),
            "DORA_BENCH_LAT_N": str(lat_n), "DORA_BENCH_LAT_GAP_US": str(gap_us),
            "DORA_BENCH_TP_SIZE": str(tp_size), "DORA_BENCH_TP_N": str(tp_n),
            "DORA_BENCH_ACKS": str(acks)}


def c4_descriptor(n_gpus, tmp, peer_copy="kernel", tp_n=200, gpu=lambda g: g, env=None,
                  fanout="pull"):
    """C4: one producer on GPU 0, a consumer on every other GPU (1 -> n_gpus-1 fan-out).
    fanout="pull": each consumer pulls the frame from the producer's slot over its own xGMI link
    (every receiver keeps its own queue and drop-oldest policy); fanout="rccl": the producer
    broadcasts each frame over an RCCL group of the output's receivers."""
    sinks = [f"sink{g}" for g in range(1, n_gpus)]
    env = dict(env or {}, DORA_GPU_PEER_COPY=peer_copy)
    src_env = _source_env(os.path.join(tmp, "source.json"), [C4_FRAME], C4_FRAME, tp_n,
                          len(sinks))
    if fanout == "rccl":
        src_env["DORA_GPU_FANOUT"] = "rccl"
    nodes = [{"id": "source", "path": "dora-gpu-bench-source",
              "outputs": ["latency", "throughput"],
              "inputs": {f"ack{k}": f"{s}/ack" for k, s in enumerate(sinks)},
              "env": src_env,
              "_unstable_deploy": {"gpu": gpu(0)}}]
    for g, s in zip(range(1, n_gpus), sinks):
        nodes.append({"id": s, "path": "dora-gpu-bench-sink", "outputs": ["ack"],
                      "inputs": {o: {"source": f"source/{o}", "queue_size": 1000}
                                 for o in ("latency", "throughput")},
                      "env": dict(env, DORA_BENCH_RESULT=os.path.join(tmp, f"{s}.json")),
                      "_unstable_deploy": {"gpu": gpu(g)}})
    return {"nodes": nodes}


def c5_descriptor(n_gpus, tmp, peer_copy="kernel", tp_n=100, gpu=lambda g: g, env=None):
    """C5: an n_gpus-stage chain, one node per GPU: source (GPU 0) -> relays -> sink (last GPU);
    each hop is one xGMI pull straight into the next stage's slot (dora_node_forward)."""
    env = dict(env or {}, DORA_GPU_PEER_COPY=peer_copy)
    stages = ["source"] + [f"relay{g}" for g in range(1, n_gpus - 1)] + ["sink"]
    outs = ("latency", "throughput")
    nodes = [{"id": "source", "path": "dora-gpu-bench-source", "outputs": list(outs),
              "inputs": {"ack0": "sink/ack"},
              "env": _source_env(os.path.join(tmp, "source.json"), C5_SIZES, C5_SIZES[1], tp_n,
                                 1),
              "_unstable_deploy": {"gpu": gpu(0)}}]
    for g in range(1, n_gpus):
        prev, me = stages[g - 1], stages[g]
        inputs = {o: {"source": f"{prev}/{o}", "queue_size": 1000} for o in outs}
        if me == "sink":
            nodes.append({"id": me, "path": "dora-gpu-bench-sink", "outputs": ["ack"],
                          "inputs": inputs,
                          "env": dict(env, DORA_BENCH_RESULT=os.path.join(tmp, "sink.json")),
                          "_unstable_deploy": {"gpu": gpu(g)}})
        else:
            nodes.append({"id": me, "path": "dora-gpu-relay", "outputs": list(outs),
                          "inputs": inputs, "env": env, "_unstable_deploy": {"gpu": gpu(g)}})
    return {"nodes": nodes}


def _load(path):
    try:
        return json.load(open(path))
    except (OSError, ValueError):
        return None


def run_cross_gpu(n_gpus, launcher, timeout=240.0, runs=None, **desc_kw):
    """Cross-GPU configurations C4 and C5 on this node's GPUs (rank 0, after the timed region;
    each stage is its own process).  Failures are reported, never raised: the headline line
    must not depend on them."""
    from dora_amd.dataflow import Dataflow
    out = {}
    runs = runs or [("c4_fanout_kernel", c4_descriptor, "kernel", {}),
                    ("c4_fanout_sdma", c4_descriptor, "sdma", {}),
                    ("c5_chain_kernel", c5_descriptor, "kernel", {}),
                    # last: RCCL runs only on distinct GPUs, so this is its first exercise on a
                    # real node; a shorter limit keeps a stuck group from holding the line back
                    ("c4_fanout_rccl", c4_descriptor, "kernel", {"fanout": "rccl"})]
    for name, fn, mode, kw in runs:
        tmp = tempfile.mkdtemp(prefix=f"dora-{name}-")
        try:
            df = Dataflow(fn(n_gpus, tmp, mode, **kw, **desc_kw), launcher=launcher).start()
            try:
                codes = df.wait(timeout if not kw else min(timeout, 120.0))
                logs = {k: df.log(k)[-400:] for k, c in codes.items() if c not in (0, None)}
            finally:
                df.stop()
            src = _load(os.path.join(tmp, "source.json")) or {}
            sinks = {f[:-5]: _load(os.path.join(tmp, f)) for f in sorted(os.listdir(tmp))
                     if f.endswith(".json") and f != "source.json"}
            out[name] = summarize_cross(name, src, sinks, codes, logs)
        except Exception as e:  # noqa: BLE001 — reported in the JSON line
            out[name] = {"error": repr(e)}
    return out


NATIVE_SIZES = [4096, 65536, 1 << 20, 4096000, 16 << 20, 40960000]


# extra environment of the bench sink (A/B of sink-side settings, e.g. its fill streams)
SINK_ENV = {k[len("DORA_BENCH_SINK_"):]: v for k, v in os.environ.items()
            if k.startswith("DORA_BENCH_SINK_DORA_")}


def native_ladder_msgs(size):
    """Messages per size of the native ladder: >= ~20 ms of back-to-back traffic, so one host
    hiccup does not set the rate (1000 x 4 KB took ~1 ms and varied 1.0-1.7 us per message)."""
    return 20000 if size <= 4096000 else 3000 if size <= (16 << 20) else 1000


# Resident sources of the native ladder's throughput mode: the reference node sends one buffer
# per size over and over (examples/benchmark/node/src/main.rs:28-36,59-69), and a 4 or 16 MB
# source read that way stays in the GPU's L2s (8 x 4 MB, each XCD reads its 1/8 of the source):
# only the sample writes reach HBM.  The HBM-resident ladder rotates copies past the L2s and,
# from 16 MB, past the 256 MB Infinity Cache (640 MB of sources, at most 64 copies).
NATIVE_RESIDENT_SIZES = [1 << 20, 4096000, 16 << 20]


def native_sources(size, resident=False):
    return 1 if resident else max(1, min(64, (640 << 20) // max(size, 1)))


# sizes of the sample-path ladder (allocate_data_sample -> kernel writes the slot -> send)
NATIVE_SAMPLE_SIZES = [4096, 65536, 1 << 20, 4 << 20, 40960000]


def run_native_ladder(launcher, gpu, n=None, timeout=120.0, resident=False, sample=False):
    """Throughput mode of the native benchmark node (dora-gpu-bench-source -> -sink, one GPU,
    zero-copy edge) per size: the data plane through its C ABI, as a Rust node would bind it,
    without the Python node's per-send cost.  Sources rotate past the caches unless `resident`
    (the reference's one buffer per size).  `sample`: the reference benchmark's own path,
    allocate_data_sample + a kernel writing the slot in place + send_output_sample (no pack;
    apis/rust/node/src/node/mod.rs:246-346), with 30 latency messages per size.  Reported,
    never raised."""
    from dora_amd.dataflow import Dataflow
    out = {}
    n_fixed = n
    sizes = (NATIVE_SAMPLE_SIZES if sample else
             NATIVE_RESIDENT_SIZES if resident else NATIVE_SIZES)
    for size in sizes:
        n = n_fixed or native_ladder_msgs(size)
        tmp = tempfile.mkdtemp(prefix="dora-native-")
        try:
            desc = c4_descriptor(2, tmp, "kernel", tp_n=n, gpu=lambda g: gpu)
            desc["nodes"][0]["env"].update({
                "DORA_BENCH_TP_SIZE": str(size), "DORA_BENCH_LAT_SIZES": str(size),
                "DORA_BENCH_LAT_N": "30" if sample else "5", "DORA_BENCH_LAT_GAP_US": "1000",
                "DORA_BENCH_TP_SOURCES": str(native_sources(size, resident))})
            if sample:
                desc["nodes"][0]["env"]["DORA_BENCH_SAMPLE_PATH"] = "1"
            df = Dataflow(desc, launcher=launcher).start()
            try:
                codes = df.wait(timeout)
            finally:
                df.stop()
            r = _load(os.path.join(tmp, "source.json")) or {}
            sk = _load(os.path.join(tmp, "sink1.json")) or {}
            gbps = r.get("tp_delivered_GBps")
            # the source counts messages sent; only delivered ones count (the sink's queue,
            # queue_size 10, drops its oldest inputs when it falls behind — any phase)
            dropped = sk.get("dropped_inputs", 0) or 0
            if gbps and dropped:
                gbps = round(gbps * (n - min(dropped, n - 1)) / n, 3)
            lat = [x for x in sk.get("series", []) if x.get("input") == "latency"]
            out[str(size)] = {"GBps": gbps, "msgs": n, "sink_dropped": dropped,
                              "lat_p50_us": lat[0]["p50_us"] if lat else None,
                              "lat_p50_incl_write_us": lat[0]["full_p50_us"] if lat else None,
                              "verified": sum(x.get("verified", 0) for x in sk.get("series", [])),
                              "mismatches": sum(x.get("mismatches", 0)
                                                for x in sk.get("series", [])),
                              "us_per_msg": round(size / (gbps * 1e3), 3) if gbps else None,
                              "hbm_frac_2S": round(2 * gbps / HBM_PEAK_GBPS, 4) if gbps else None,
                              "sources": native_sources(size, resident),
                              "send_phase_us": r.get("send_phase_us"), "ok": r.get("ok"),
                              "exit_codes": codes}
        except Exception as e:  # noqa: BLE001 — reported in the JSON line
            out[str(size)] = {"error": repr(e)}
    return out


def edge_rates(sinks):
    """Per receiving edge: payload GB/s of its back-to-back (throughput) series, from the sink's
    own first/last receipt stamps, and the bytes it pulled over xGMI or received by broadcast."""
    out = []
    for sname, r in sorted(sinks.items()):
        if not r:
            continue
        tp = [s for s in r.get("series", []) if s["input"] == "throughput" and s["n"] > 1]
        gbps = None
        if tp:
            s = max(tp, key=lambda x: x.get("burst_n", x["n"]))
            # the longest burst between two acks is the back-to-back phase (earlier receipts of
            # the same input and size, the warmup, would stretch the span over the latency phase)
            n, first, last = (s["burst_n"], s["burst_first_ns"], s["burst_last_ns"]) \
                if s.get("burst_n", 0) > 1 else (s["n"], s["first_ns"], s["last_ns"])
            span_ns = last - first
            # n receipts span n - 1 message intervals
            gbps = round((n - 1) * s["size"] / span_ns, 3) if span_ns > 0 else None
        moved = r.get("pull_bytes", 0) + (r.get("bcast_received", 0) and
                                          sum(x["n"] * x["size"] for x in r.get("series", [])))
        out.append({"sink": sname, "GBps": gbps, "pulls": r.get("pulls", 0),
                    "pull_bytes": r.get("pull_bytes", 0),
                    "bcast_received": r.get("bcast_received", 0),
                    "xgmi_frac": round(gbps / XGMI_LINK_GBPS, 4) if gbps and moved else None})
    return out


def summarize_cross(name, src, sinks, codes, logs):
    lat, verified, mismatches, dropped, errors = {}, 0, 0, 0, 0
    for sname, r in sinks.items():
        if not r:
            errors += 1
            continue
        dropped += r.get("dropped_inputs", 0)
        errors += r.get("errors", 0)
        for s in r.get("series", []):
            verified += s["verified"]
            mismatches += s["mismatches"]
            if s["input"] == "latency" and s["size"]:
                lat.setdefault(str(s["size"]), []).append(
                    {"sink": sname, "p50_us": s["p50_us"], "p99_us": s["p99_us"],
                     "e2e_p50_us": s["full_p50_us"], "e2e_p99_us": s["full_p99_us"], "n": s["n"]})
    per_rx = src.get("tp_per_receiver_GBps", 0.0)
    pulls = sum((r or {}).get("pulls", 0) for r in sinks.values())
    pull_bytes = sum((r or {}).get("pull_bytes", 0) for r in sinks.values())
    bcast_rx = sum((r or {}).get("bcast_received", 0) for r in sinks.values())
    # An xGMI roofline only when bytes crossed a link: with every stage on one GPU (a one-GPU
    # rehearsal without forced pulls) nothing did, and a fraction of the link peak means nothing.
    crossed = pulls > 0 or bcast_rx > 0
    roof = ({"bound": "xgmi", "achieved": per_rx, "peak": XGMI_LINK_GBPS, "unit": "GB/s",
             "frac": round(per_rx / XGMI_LINK_GBPS, 4)} if crossed else None)
    res = {"ok": bool(src.get("ok")) and errors == 0 and mismatches == 0,
           "receivers": src.get("receivers"), "msg_bytes": src.get("tp_size"),
           "tp_msgs": src.get("tp_n"), "delivered_GBps": src.get("tp_delivered_GBps"),
           "per_link_GBps": per_rx,
           "roofline": roof,
           "edges": edge_rates(sinks),
           "latency_us": lat, "parity": {"verified_msgs": verified, "mismatches": mismatches},
           "dropped_inputs": dropped, "errors": errors, "exit_codes": codes,
           "source_send_phase_us": src.get("send_phase_us"),
           # transfer path actually taken: pulls per receiver, or RCCL broadcast group traffic
           "pulls": pulls, "pull_bytes": pull_bytes,
           "bcast": {"groups": src.get("bcast_groups", 0), "ranks": src.get("bcast_ranks", 0),
                     "sent": src.get("bcast_sent", 0),
                     "received": bcast_rx,
                     "error": src.get("bcast_error") or next(
                         (r.get("bcast_error") for r in sinks.values()
                          if r and r.get("bcast_error")), "")}}
    if not crossed:
        res["note"] = "no byte crossed a GPU link (every stage on one GPU): roofline null"
    if logs:
        res["logs"] = logs
    return res


def run_sync_mid(node, wait_ack, seq, stream, size=4 << 20, n=200):
    """The default (synchronous) send at 4 MiB (verdict r05 weak 2: the line had no synchronous
    mid-size figure): `n` sends from four rotated device buffers, each returning once its pack
    has read the source (read-signalled, aql_kernels.hip dora_aql_pack1r_u4)."""
    from dora_amd import device
    from dora_amd.workloads import payload_seed
    bufs = [device.DeviceBuffer(size) for _ in range(4)]
    for b in bufs:
        device.fill_splitmix(b.ptr, size, payload_seed(size), stream)
    stream.sync()
    node.set_async_sends(False)
    node.send_output("throughput", b"", {"seq": seq, "ack": True})
    wait_ack(seq)
    seq += 1
    for k in range(2):  # this size's slots and the sink's mappings, untimed
        node.send_output_device_bytes("throughput", bufs[k].ptr, size, {"seq": seq})
        seq += 1
    t0 = time.perf_counter()
    for k in range(n):
        node.send_output_device_bytes("throughput", bufs[k % 4].ptr, size, {"seq": seq})
        seq += 1
    dt = time.perf_counter() - t0
    node.send_output("throughput", b"", {"seq": seq, "ack": True})
    wait_ack(seq)
    seq += 1
    node.set_async_sends(True)
    for b in bufs:
        b.free()
    us = dt / n * 1e6
    return seq, {"msg_bytes": size, "msgs": n, "us_per_msg": round(us, 2),
                 "hbm_frac_2S": round(2 * size / (us * 1e-6) / 8e12, 4)}


C3_GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "tests", "golden",
                         "c3_cloud.json")


def run_sync_leg(node, send, wait_ack, seq, S, n_sync):
    """The default (synchronous) send at the headline size: each send returns once its pack has
    read the source, as the reference's copy inside send_output (arrow_utils.rs:48; INTEGRATION
    §1).  A send that waits for its own pack runs it alone on the GPU (aql.h: signalled by the
    command processor, full grid).  Timed as a region: each pack's own device time from its
    stamps, and the host time between one pack's end and the next one's start."""
    from dora_amd import device
    node.set_async_sends(False)
    # the sink checksums the timed region's late messages after acking it: one ack round trip
    # first, so the GPU is idle, then two untimed synchronous sends (this path's first use)
    node.send_output("throughput", b"", {"seq": seq, "ack": True})
    wait_ack(seq)
    seq += 1
    for k in range(2):
        send(k, {"seq": seq})
        seq += 1
    node.set_profiling(False)  # resets the send-phase timers: they cover these sends
    cp0 = device.aql_cp_signalled(node.device)
    node.region_begin()
    t_calls = []
    t_s = time.perf_counter()
    for k in range(n_sync):
        t_calls.append(time.perf_counter())
        send(k, {"seq": seq})
        seq += 1
    t_calls.append(time.perf_counter())
    node.send_output("throughput", b"", {"seq": seq, "ack": True})
    wait_ack(seq)
    seq += 1
    dt_s = time.perf_counter() - t_s
    node.sync()
    region = node.region_end()
    iv = sorted(node.pack_intervals(4 * n_sync))
    phases = node.send_profile()
    cp1 = device.aql_cp_signalled(node.device)
    node.set_async_sends(True)
    own = [b - a for a, b in iv]
    gaps = [iv[i + 1][0] - iv[i][1] for i in range(len(iv) - 1)]
    med = (lambda v: sorted(v)[len(v) // 2] if v else None)
    own_us = sum(own) / len(own) * 1e3 if own else None
    return {"seq": seq, "msgs": n_sync, "GBps": round(n_sync * S / dt_s / 1e9, 1),
            "us_per_msg": round(dt_s / n_sync * 1e6, 2),
            "us_per_send_call": round((t_calls[-1] - t_calls[0]) / n_sync * 1e6, 2),
            "hbm_frac_2S": round(2 * S * n_sync / dt_s / 1e9 / HBM_PEAK_GBPS, 4),
            "pack_own_us": round(own_us, 3) if own_us else None,
            "pack_own_us_median": round(med(own) * 1e3, 3) if own else None,
            "pack_own_frac": round(2 * S / (own_us * 1e-6) / 1e9 / HBM_PEAK_GBPS, 4)
            if own_us else None,
            "gap_us_median": round(med(gaps) * 1e3, 3) if gaps else None,
            "region_packs": region["packs"],
            "cp_signalled": cp1 - cp0,
            "send_phase_us": {k: round(v, 3) for k, v in phases.items()},
            "send_calls_us": [round((t - t_calls[0]) * 1e6, 1) for t in t_calls]}


def run_c3_block(node, stream, wait_ack, seq, steps=20, nsrc=24, steady_steps=200):
    """BASELINE configs[2] beside the C2 headline: `send_output` of device-resident 1M-point
    clouds (List<Struct<x,y,z:f32,intensity:u8>>, 16 lists, validity bitmaps; one multi-segment
    AQL pack each), `steps` back-to-back sends from `nsrc` rotating clouds, device time from the
    packs' own stamps.  Parity: the last 4 timed clouds are held by the sink and checksummed
    against the CPU oracle's sample (tests/golden/c3_cloud.json, make_c3_golden.py), and so is
    a reference pack of the same cloud made before the clock.  `steady`: a second region of
    `steady_steps` sends, the pipeline's steady state."""
    from dora_amd import device
    from dora_amd.arrow_utils import Plan
    from dora_amd.device import DeviceArray
    from dora_amd.verify import to_i64
    from dora_amd.workloads import point_cloud
    golden = json.load(open(C3_GOLDEN))
    cloud = point_cloud()
    srcs = [DeviceArray.from_pyarrow(cloud) for _ in range(nsrc)]
    with Plan.of(srcs[0]) as p:
        S = p.size
        ref = device.DeviceBuffer(S)
        p.pack(ref.ptr, S, stream)
        stream.sync()
    ref_csum = device.csum64(ref.ptr, S, stream)
    ref.free()
    want = golden["csum64"]
    for k in range(2 * nsrc):  # slots of this size in the cache, the sink's mappings of them
        node.send_output("throughput", srcs[k % nsrc], {"seq": seq})
        seq += 1
    node.send_output("throughput", b"", {"seq": seq, "ack": True})
    wait_ack(seq)
    seq += 1
    # the same pipeline over `steady_steps` sends first: the steady state without the first
    # packs' ramp and the last ones' drain (reported beside the 20-step figure, which stays the
    # line's; before it, since the sink holds that region's late-verified clouds)
    steady = None
    if steady_steps > 0:
        node.region_begin()
        t_s = time.perf_counter()
        for k in range(steady_steps):
            node.send_output("throughput", srcs[k % nsrc],
                             {"seq": seq, "ack": True} if k == steady_steps - 1 else {"seq": seq})
            seq += 1
        node.region_mark()
        wait_ack(seq - 1)
        node.sync()
        dt_s = time.perf_counter() - t_s
        r2 = node.region_end()
        if r2["span_ms"] > 0 and r2["packs"]:
            a2 = 2.0 * S * r2["packs"] / (r2["span_ms"] * 1e-3) / 1e9
            steady = {"steps": steady_steps, "region_packs": r2["packs"],
                      "device_us_per_launch": round(r2["span_ms"] * 1e3 / r2["packs"], 3),
                      "achieved": round(a2, 1), "frac": round(a2 / HBM_PEAK_GBPS, 4),
                      "ms_per_step": round(dt_s / steady_steps * 1e3, 4)}
    late = min(4, steps)
    before = node.stats()
    node.sync()
    kern0, bs0 = device.aql_dispatch_counts(node.device), device.aql_batch_stats(node.device)
    node.region_begin()
    t0 = time.perf_counter()
    t_send = []
    for k in range(steps):
        meta = {"seq": seq}
        if k >= steps - late:
            meta.update({"csum": to_i64(want), "verify_late": True})
        if k == steps - 1:
            meta["ack"] = True
        t_send.append(time.perf_counter())
        node.send_output("throughput", srcs[k % nsrc], meta)
        seq += 1
    t_send.append(time.perf_counter())
    node.region_mark()
    wait_ack(seq - 1)
    node.sync()
    elapsed = time.perf_counter() - t0
    region = node.region_end()
    # each timed pack's own (start, end) stamps, us after the region's first start (sorted)
    intervals = sorted((round(a * 1e3, 2), round(b * 1e3, 2)) for a, b in node.pack_intervals(64))
    after = node.stats()
    kern1, bs1 = device.aql_dispatch_counts(node.device), device.aql_batch_stats(node.device)
    for a in srcs:
        a.close()
    span_ms, packs = region["span_ms"], region["packs"]
    achieved = 2.0 * S * packs / (span_ms * 1e-3) / 1e9 if span_ms > 0 else 0.0
    return seq, {
        "workload": "C3 (BASELINE configs[2]): send_output of device-resident 1M-point clouds, "
                    "List<Struct<x,y,z:f32,intensity:u8>> in 16 lists with validity bitmaps",
        "value": round(steps * S / elapsed / 1e9, 3), "unit": "GB/s", "steps": steps,
        "ms_per_step": round(elapsed / steps * 1e3, 4), "msg_bytes": S, "sources_rotated": nsrc,
        "slots_created_in_region": after["slots_created"] - before["slots_created"],
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                     "kernel": aql_kernel_name("c3", {k: kern1[k] - kern0.get(k, 0) for k in kern1
                                                      if kern1[k] - kern0.get(k, 0)}),
                     "device_us_per_launch": round(span_ms * 1e3 / max(packs, 1), 3),
                     "region_packs": packs, "algorithmic_bytes_per_launch": 2 * S,
                     "traffic": (pmc_traffic(S) or (None, None))[1],
                     "traffic_source": (pmc_traffic(S) or (None, None))[0],
                     "region_kernels": {k: kern1[k] - kern0.get(k, 0) for k in kern1
                                        if kern1[k] - kern0.get(k, 0)},
                     "batched_msgs": bs1["batched_msgs"] - bs0["batched_msgs"]},
        "steady": steady,
        "pack_intervals_us": intervals,
        "send_calls_us": [round((t - t_send[0]) * 1e6, 1) for t in t_send],
        "parity": {"oracle_sample_bytes": golden["sample_bytes"], "oracle_csum64": want,
                   "reference_pack_matches_oracle": ref_csum == want and S == golden["sample_bytes"],
                   "late_verified_msgs": late},
    }


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # DORA_BENCH_GPUS=k: rehearsal on a k-GPU box (rank / stage g runs on GPU g % k); unset on
    # the real node, where every rank and cross-GPU stage has a GPU of its own
    vis = int(os.environ.get("DORA_BENCH_GPUS", "0"))
    gpu_of = (lambda g: g % vis) if vis > 0 else (lambda g: g)
    local_rank = gpu_of(local_rank)
    affinity = sorted(os.sched_getaffinity(0))
    if args.keep_awake_us is not None:  # this process, and the native sources it spawns
        os.environ["DORA_BENCH_KEEP_AWAKE_US"] = str(args.keep_awake_us)
        from dora_amd import device as _device
        _device.set_keep_awake(args.keep_awake_us)

    # ---- CPU-only work and process spawning first: nothing below touches HIP until Node() ----
    base = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        base = cpu_baseline(affinity)

    launcher = None
    native_ladder = (world == 1 and rank == 0 and not args.no_ladder and args.tp_n > 0
                     and args.workload == "c2")
    if (world > 1 and rank == 0 and not args.no_cross_gpu) or native_ladder:
        from dora_amd.launcher import Launcher
        # spawns the cross-GPU stages / native ladder nodes after this process touched HIP
        launcher = Launcher()

    # The native ladder runs before this process opens the GPU: afterwards this process keeps
    # its HIP and AQL hardware queues, and the ladder's nodes then ran >= 16 MB ~1.4x slower
    # (DORA_BENCH_LADDER_LATE=1 keeps the old order for A/B).
    native = native_res = None
    ladder_late = os.environ.get("DORA_BENCH_LADDER_LATE") == "1"
    native_sample = None
    if native_ladder and not ladder_late:
        native = run_native_ladder(launcher, local_rank)
        native_res = run_native_ladder(launcher, local_rank, resident=True)
        native_sample = run_native_ladder(launcher, local_rank, sample=True)

    from dora_amd.dataflow import Dataflow
    result_path = os.path.join(tempfile.mkdtemp(prefix="dora-bench-"), "sink.json")
    host_result_path = os.path.join(os.path.dirname(result_path), "hostsink.json")
    desc = {"nodes": [
        {"id": "node", "path": "dynamic",
         "outputs": ["latency", "latency_host", "throughput", "to_host", "to_host_warm"],
         "inputs": {"ack": "sink/ack", "ack_host": "hostsink/ack"},
         "_unstable_deploy": {"gpu": local_rank}},
        # a receiver without a GPU: device samples reach it in host memory
        {"id": "hostsink", "path": "dora-gpu-bench-sink", "outputs": ["ack"],
         "inputs": {"to_host": {"source": "node/to_host", "queue_size": 10},
                    "to_host_warm": {"source": "node/to_host_warm", "queue_size": 10}},
         "env": {"DORA_BENCH_RESULT": host_result_path}, "_unstable_deploy": {"gpu": -1}},
        {"id": "sink", "path": "dora-gpu-bench-sink", "outputs": ["ack"],
         "inputs": {"latency": {"source": "node/latency", "queue_size": 10},
                    "latency_host": {"source": "node/latency_host", "queue_size": 10},
                    "throughput": {"source": "node/throughput", "queue_size": 10}},
         "env": dict({"DORA_BENCH_RESULT": result_path}, **SINK_ENV),
         "_unstable_deploy": {"gpu": local_rank}},
    ]}
    df = Dataflow(desc).start()

    ranks = Ranks(world)
    barrier, max_over_ranks, sum_over_ranks = ranks.barrier, ranks.max, ranks.sum

    from dora_amd import device
    from dora_amd.node import Node
    from dora_amd.verify import to_i64
    from dora_amd.workloads import payload_seed

    node = Node("node", dataflow=df.shm, device=local_rank)
    # the CPUs this process may run on once the node has placed itself (DORA_GPU_PIN)
    affinity_after_init = sorted(os.sched_getaffinity(0))
    # the benchmark node never rewrites its sources: every send returns as soon as its pack is
    # queued (DORA_SEND_ASYNC), so packs overlap; the default synchronous send is measured
    # beside it (sync_send_headline)
    sync_sends = os.environ.get("DORA_BENCH_SYNC_SENDS") == "1"
    node.set_async_sends(not sync_sends)
    stream = device.Stream()
    if args.workload == "c2":
        S = args.size
        nsrc = args.sources or max(2, min(16, (640 << 20) // max(S, 1)))
        srcs = []
        off = args.src_offset
        for _ in range(nsrc):  # rotate > 512 MiB of sources so the Infinity Cache cannot hold them
            b = device.DeviceBuffer(S + off)
            device.fill_splitmix(b.ptr + off, S, payload_seed(S), stream)
            srcs.append(b)
        stream.sync()
        csum = device.csum64(srcs[0].ptr + off, S, stream)

        def send(k, meta):
            node.send_output_device_bytes("throughput", srcs[k % nsrc].ptr + off, S, meta)
    else:
        # C3: List<Struct<x,y,z:f32,intensity:u8>> 1M-point clouds resident in HBM; each send is
        # plan (host DFS + validity read-back for the type info) + nested pack kernel
        from dora_amd.arrow_utils import Plan
        from dora_amd.device import DeviceArray
        from dora_amd.workloads import point_cloud
        cloud = point_cloud(n_lists=args.c3_lists) if args.c3_lists else point_cloud()
        nsrc = args.sources or 24
        srcs = [DeviceArray.from_pyarrow(cloud) for _ in range(nsrc)]
        with Plan.of(srcs[0]) as p:
            S = p.size
            ref = device.DeviceBuffer(S)
            p.pack(ref.ptr, S, stream)
            stream.sync()
        csum = device.csum64(ref.ptr, S, stream)
        ref.free()

        def send(k, meta):
            node.send_output("throughput", srcs[k % nsrc], meta)

    def wait_ack(seq, timeout=60.0):
        node.wait_input("ack", "seq", seq, timeout)

    # inputs the sink's queue (queue_size 10, the reference default) dropped, per phase of this
    # run (verdict r03 item 7): the timed and throughput phases must show 0
    drops = {}
    drop_mark = [node.dataflow_counters("sink")["dropped_inputs"]]

    # other processes with queues on this GPU at the end of each phase (dora_amd/tenants.py):
    # an HBM-bound rate that drops mid-run on a shared box is their traffic, not ours
    from dora_amd.tenants import gpu_tenants
    tenants = {}

    def phase_drops(name):
        now = node.dataflow_counters("sink")["dropped_inputs"]
        drops[name] = drops.get(name, 0) + now - drop_mark[0]
        drop_mark[0] = now
        t = gpu_tenants()
        if t.get("visible"):
            prev = tenants.get(name, (0, 0))
            tenants[name] = (max(prev[0], t["others"]), max(prev[1], t["other_queues"]))

    # Python's cyclic collector is paused from here to the end of the measurements, as timeit
    # does: a collection is the harness's pause, not the data plane's (a gen-0 collection of
    # ~40 us between two sends of the C3 burst took it from 0.74 to 0.53 once)
    import gc as _gc
    _gc.collect()
    _gc.disable()
    copy_cal = box_copy_rate(S, stream)
    h2d_cal = box_h2d_rate(40960000, stream) if not args.no_ladder else None
    # the same at the mid sizes, where per-message dispatch rather than HBM binds
    copy_mid = {str(z): box_copy_rate(z, stream) for z in (4 << 20, 16 << 20)
                if z != S and not args.no_ladder}

    # ---- cold start: the very first message (device queues, code object, the sink's first IPC
    # mapping), reported on its own so the ladders below measure a warm data plane ----
    seq = 0
    cold_buf = device.DeviceBuffer(4096)
    device.fill_splitmix(cold_buf.ptr, 4096, payload_seed(4096), stream)
    stream.sync()
    t_c = time.perf_counter()
    node.send_output_device_bytes("throughput", cold_buf.ptr, 4096, {"seq": seq, "ack": True})
    cold_send_us = (time.perf_counter() - t_c) * 1e6  # sender side: slot, queues, dispatch
    wait_ack(seq)
    cold_start_us = (time.perf_counter() - t_c) * 1e6
    seq += 1
    phase_drops("cold_start")

    # ---- warmup (the first messages are verified bit-exact by the sink's csum kernel) ----
    for k in range(args.warmup):
        meta = {"seq": seq, "t_start": time.time_ns()}
        if k < 3:
            meta.update({"csum": to_i64(csum), "verify": True})
        if k == args.warmup - 1:
            meta["ack"] = True
        send(k, meta)
        seq += 1
    if args.warmup <= 0:
        node.send_output("throughput", b"", {"seq": seq, "ack": True})
        seq += 1
    wait_ack(seq - 1)
    phase_drops("warmup")

    # ---- latency ladder (reference latency mode: spaced messages, output `latency`) ----
    ladder_bufs = {}
    share_lat0 = share_lat1 = None
    if not args.no_ladder:
        for size in LADDER:
            b = device.DeviceBuffer(size)
            device.fill_splitmix(b.ptr, size, payload_seed(size), stream)
            ladder_bufs[size] = b
        stream.sync()
        for size in LADDER_SMALL:  # prefixes of the 4 KB payload
            ladder_bufs[size] = ladder_bufs[4096]
        sizes = LADDER_SMALL + LADDER
        # every size once through the path untimed first (its slot, the sink's mapping of it)
        # the last message of a burst asks for the ack itself: a trailing empty marker has no
        # drop token, so it would not wait for the in-flight cap and could be the sink queue's
        # eleventh ready input (a drop, verdict r03 item 7)
        warm = [size for size in sizes for _ in range(2)]
        for k, size in enumerate(warm):
            meta = {"seq": seq, "ack": True} if k == len(warm) - 1 else {"seq": seq}
            node.send_output_device_bytes("throughput", ladder_bufs[size].ptr, size, meta)
            seq += 1
        wait_ack(seq - 1)
        phase_drops("latency_ladder_warm")
        share_lat0 = cpu_share()
        for size in sizes:
            for _ in range(args.lat_n):
                node.send_output_device_bytes("latency", ladder_bufs[size].ptr, size,
                                              {"seq": seq, "t_start": time.time_ns()})
                seq += 1
                time.sleep(args.lat_gap_us / 1e6)
        # host-resident sources (bytes objects): the reference's own latency case, whose sources
        # are host memory (examples/benchmark/node/src/main.rs:38-70)
        host_src = {z: bytes(range(256)) * (z // 256) + bytes(z % 256) for z in LADDER_HOST}
        for size in LADDER_HOST:
            node.send_output("throughput", host_src[size], {"seq": seq})  # untimed, once
            seq += 1
            time.sleep(args.lat_gap_us / 1e6)
            for _ in range(host_lat_n(size, args.lat_n)):
                node.send_output("latency_host", host_src[size],
                                 {"seq": seq, "t_start": time.time_ns()})
                seq += 1
                time.sleep(args.lat_gap_us / 1e6)
        node.send_output("throughput", b"", {"seq": seq, "ack": True})
        wait_ack(seq)
        seq += 1
        del host_src
        # device sources to the receiver without a GPU (staged to host memory there); the first
        # messages of each size carry their csum64, which the host sink checks on the host
        for size in LADDER_D2H:
            b = ladder_bufs.get(size)
            if b is None:
                b = ladder_bufs[size] = device.DeviceBuffer(size)
                device.fill_splitmix(b.ptr, size, payload_seed(size), stream)
                stream.sync()
            c = to_i64(device.csum64(b.ptr, size, stream))
            # untimed: the receiver's first staging buffer of this size, and the checksums (on
            # the host, ~10 ms at 40.96 MB: no timed message waits behind one); received before
            # the series starts
            for k in range(3):
                node.send_output_device_bytes("to_host_warm", b.ptr, size,
                                              {"seq": seq, "csum": c, "verify": True})
                seq += 1
                time.sleep(args.lat_gap_us / 1e6)
            node.send_output("to_host_warm", b"", {"seq": seq, "ack": True})
            node.wait_input("ack_host", "seq", seq, 60.0)
            seq += 1
            for k in range(host_lat_n(size, args.lat_n)):
                meta = {"seq": seq, "t_start": time.time_ns()}
                node.send_output_device_bytes("to_host", b.ptr, size, meta)
                seq += 1
                time.sleep(args.lat_gap_us / 1e6)
            node.send_output("to_host", b"", {"seq": seq, "ack": True})
            node.wait_input("ack_host", "seq", seq, 60.0)
            seq += 1
        phase_drops("latency_ladder")
        share_lat1 = cpu_share()
        for b in {id(b): b for b in ladder_bufs.values()}.values():
            b.free()

    # ---- throughput ladder (reference throughput mode: back-to-back messages per size) ----
    tp_ladder = {}
    # Python collections inside a ladder step (diagnosis of the bimodal 40.96 MB step)
    import gc
    gc_log, gc_t0 = [], [0.0]

    def gc_cb(phase, info):
        if phase == "start":
            gc_t0[0] = time.perf_counter()
        elif len(gc_log) < 64:
            gc_log.append((info.get("generation"), (time.perf_counter() - gc_t0[0]) * 1e6))
    gc.callbacks.append(gc_cb)
    if not args.no_ladder and args.tp_n > 0 and args.workload == "c2":
        for size in [z for z in LADDER_SMALL if z] + LADDER:
            nb = native_sources(size)  # rotated past the L2s / Infinity Cache, as the native ladder
            bufs = [device.DeviceBuffer(size) for _ in range(nb)]
            for b in bufs:
                device.fill_splitmix(b.ptr, size, payload_seed(size), stream)
            stream.sync()
            for k in range(24):  # warm the slot cache for this size (2x the in-flight cap)
                meta = {"seq": seq, "ack": True} if k == 23 else {"seq": seq}
                node.send_output_device_bytes("throughput", bufs[k % nb].ptr, size, meta)
                seq += 1
            wait_ack(seq - 1)
            phase_drops("throughput_ladder_warm")
            d0 = node.dataflow_counters("sink")["dropped_inputs"]
            bs0 = device.aql_batch_stats(local_rank)
            cp0 = device.aql_cp_signalled(local_rank)
            st0 = node.stats()
            node.set_profiling(False)  # resets the send-phase counters for this size
            # small sizes run ~1-2 us per message: >= 2000 of them, so a host hiccup does not
            # set the rate of a ~0.3 ms burst
            tp_n = args.tp_n if size > (4 << 20) else max(args.tp_n, 2000)
            # sizes from 16 MiB: the packs' own device time as a region (stamps), so a slow run
            # shows whether the GPU or the token path set its rate (the bimodal 40.96 MB ladder)
            dev_region = size >= (16 << 20) and not args.no_kernel_timing
            if dev_region:
                node.region_begin()
            gc_log.clear()
            t_a = time.perf_counter()
            t_first = t_a
            for k in range(tp_n):  # the last message asks for the ack (no trailing marker)
                meta = {"seq": seq, "ack": True} if k == tp_n - 1 else {"seq": seq}
                node.send_output_device_bytes("throughput", bufs[k % nb].ptr, size, meta)
                if k == 0:
                    t_first = time.perf_counter()
                    # the first send's own phases (one call; a slow first send shows where)
                    first_phases = node.send_profile() if dev_region else None
                seq += 1
            t_sent = time.perf_counter()
            wait_ack(seq - 1)
            dt = time.perf_counter() - t_a
            dev = None
            if dev_region:
                node.sync()
                reg = node.region_end()
                iv = sorted(node.pack_intervals(tp_n + 8))
                busy, end = 0.0, None
                for a0, b0 in iv:  # union of the packs' intervals, ms
                    if end is None or a0 > end:
                        busy += b0 - a0
                        end = b0
                    elif b0 > end:
                        busy += b0 - end
                        end = b0
                if reg["packs"]:
                    dev = {"device_us_per_pack": round(reg["span_ms"] * 1e3 / reg["packs"], 3),
                           "busy_us_per_pack": round(busy * 1e3 / reg["packs"], 3),
                           "packs": reg["packs"],
                           # host side of the same run: the first send call, the send loop,
                           # and last send -> ack (the device span explains the rest)
                           "host_us": {"first_send": round((t_first - t_a) * 1e6, 1),
                                       "send_loop": round((t_sent - t_a) * 1e6, 1),
                                       "close": round((t_a + dt - t_sent) * 1e6, 1),
                                       "total": round(dt * 1e6, 1),
                                       "device_span": round(reg["span_ms"] * 1e3, 1)},
                           # Python garbage collections during the run: [generation, us]
                           "gc": [[g, round(us, 1)] for g, us in gc_log],
                           "first_send_phases_us": ({k: round(v, 2) for k, v in
                                                     first_phases.items()}
                                                    if first_phases else None)}
            # the sink's queue (queue_size 10, the reference default) may drop inputs when it
            # falls behind: only delivered messages count
            dropped = node.dataflow_counters("sink")["dropped_inputs"] - d0
            phase_drops("throughput_ladder")
            bs1 = device.aql_batch_stats(local_rank)
            st1 = node.stats()
            phases = node.send_profile()
            got = tp_n - dropped
            tp_ladder[str(size)] = {"GBps": round(got * size / dt / 1e9, 2),
                                    "msgs_per_s": round(got / dt, 1),
                                    "us_per_msg": round(dt / got * 1e6, 2),
                                    "hbm_frac_2S": round(2 * got * size / dt / 1e9 /
                                                         HBM_PEAK_GBPS, 4),
                                    "dropped": dropped,
                                    # sends that left in batch packs (aql.cpp), and batches
                                    "batched_msgs": bs1["batched_msgs"] - bs0["batched_msgs"],
                                    "batches": bs1["batches"] - bs0["batches"],
                                    # packs the command processor signalled (CP window, lone)
                                    "cp_signalled": device.aql_cp_signalled(local_rank) - cp0,
                                    # where a send's host time goes, and whether its slots
                                    # came from the cache (verdict r02: the bimodal 40.96 MB
                                    # Python ladder)
                                    "send_phase_us": {k: round(v, 3) for k, v in phases.items()},
                                    "slots_created": st1["slots_created"] - st0["slots_created"],
                                    "cache_hits": st1["cache_hits"] - st0["cache_hits"],
                                    # from 16 MiB: device span / packs and the packs' busy time
                                    "device": dev}
            for b in bufs:
                b.free()
    if gc_cb in gc.callbacks:
        gc.callbacks.remove(gc_cb)

    cold_buf.free()

    # ---- refill: the ladders evicted the headline size's slots from the sender's 20-entry cache
    # (and the sink's mappings of them); send the in-flight cap's worth and more untimed, so the
    # timed region allocates and maps nothing ----
    for k in range(2 * 12):
        send(k, {"seq": seq})
        seq += 1
    node.send_output("throughput", b"", {"seq": seq, "ack": True})
    wait_ack(seq)
    seq += 1
    phase_drops("refill")

    # ---- timed region: K back-to-back steps, closed by the sink's ack ----
    # The last `late` messages are checksummed by the sink right after it acks the region (it
    # holds them until then), so parity covers timed traffic without a kernel inside the region.
    late = min(4, args.steps)
    node.set_profiling(False)  # resets the per-phase send timers: they cover the timed steps
    sink_before = node.dataflow_counters("sink")
    node_before = node.stats()
    barrier()
    device.set_device(local_rank)
    from dora_amd._lib import call
    presync = os.environ.get("DORA_BENCH_PRESYNC", "device")
    if presync == "device":
        call("dora_gpu_device_sync")
    elif presync == "node":
        node.sync()
    kern0 = device.aql_dispatch_counts(local_rank)
    if not args.no_kernel_timing:
        node.region_begin()  # setup (profiling signals) before the clock starts
    t0_ns = time.time_ns()
    t0 = time.perf_counter()
    region_first_seq = seq
    for k in range(args.steps):
        meta = {"seq": seq, "t_start": time.time_ns()}
        if k == 0:
            meta["mark"] = True  # the sink stamps its receipt: start of the region's pipeline
        if k >= args.steps - late:
            meta.update({"csum": to_i64(csum), "verify_late": True})
        if k == args.steps - 1:
            meta["ack"] = True  # the sink acks the region's last message on receipt
        send(k, meta)
        if k == 0:
            t_first = time.perf_counter()
            if os.environ.get("DORA_BENCH_FIRST_PHASES"):  # diagnosis: costs a call in the region
                first_phases = node.send_profile()
        seq += 1
    t_sent = time.perf_counter()
    t_sent_ns = time.time_ns()
    if not args.no_kernel_timing:
        node.region_mark()  # stop events after the last pack, while it is delivered
    wait_ack(seq - 1)
    t_acked = time.perf_counter()
    t_acked_ns = time.time_ns()
    region_ack_seq = seq - 1
    node.sync()  # every stream and AQL fill of this node complete (the ack implies it)
    elapsed = time.perf_counter() - t0
    barrier()
    region = node.region_end() if not args.no_kernel_timing else None
    kern1 = device.aql_dispatch_counts(local_rank)
    region_kernels = {k: kern1[k] - kern0.get(k, 0) for k in kern1 if kern1[k] - kern0.get(k, 0)}
    sink_after = node.dataflow_counters("sink")
    phase_drops("timed_region")
    node_after = node.stats()
    region_setup = {
        "slots_created_in_region": node_after["slots_created"] - node_before["slots_created"],
        "ipc_opens_in_region": sink_after["ipc_opens"] - sink_before["ipc_opens"],
        "sink_slots_created_in_region": sink_after["slots_created"] - sink_before["slots_created"],
        # every message counted in `value` was delivered: the sink's queue dropped none
        "sink_dropped_in_region": sink_after["dropped_inputs"] - sink_before["dropped_inputs"],
        "host_send_loop_us": round((t_sent - t0) * 1e6, 1),
        "first_send_us": round((t_first - t0) * 1e6, 1) if args.steps else None,
        "first_send_phases_us": ({k: round(v, 2) for k, v in first_phases.items()}
                                 if os.environ.get("DORA_BENCH_FIRST_PHASES") else None),
        "close_us": round((t_acked - t_sent) * 1e6, 1),
        "sync_us": round((t0 + elapsed - t_acked) * 1e6, 1),
        "late_verified_msgs": late}
    stats = node.stats()
    stats["send_phase_us"] = {k: round(v, 2) for k, v in node.send_profile().items()}
    stats["fill_paths"] = node.fill_paths()
    node_host_paths = node.host_paths()
    # the timed region's packs, each from its own stamps (first workgroup start -> fill signal)
    intervals = node.pack_intervals() if region else []
    # the default (synchronous) send at the headline size: each send returns once its pack has
    # read the source, as the reference's copy inside send_output
    sync_headline = sync_mid = None
    if not sync_sends and world == 1 and args.steps and args.sync_n > 0:
        sync_headline = run_sync_leg(node, send, wait_ack, seq, S, args.sync_n)
        seq = sync_headline.pop("seq")
        phase_drops("sync_leg")
        seq, sync_mid = run_sync_mid(node, wait_ack, seq, stream)
        phase_drops("sync_mid")
    c3 = None
    if args.workload == "c2" and not args.no_c3 and world == 1 and args.c3_steps > 0:
        seq, c3 = run_c3_block(node, stream, wait_ack, seq, steps=args.c3_steps)
        phase_drops("c3_block")
    node.close()
    codes = df.wait(120)
    df.stop()
    sink = json.load(open(result_path)) if os.path.exists(result_path) else {"series": []}
    hostsink = (json.load(open(host_result_path)) if os.path.exists(host_result_path)
                else {"series": []})
    # the close, split at the sink (realtime clocks of one host): last send -> the sink has the
    # last message (its fill complete) -> ack sent -> the ack is back here
    for a_seq, t_rx, t_ack in sink.get("acks", []):
        if a_seq == region_first_seq:
            region_setup["first_msg_receipt_us"] = round((t_rx - t0_ns) / 1e3, 1)
        if a_seq == region_ack_seq:
            region_setup["close_split_us"] = {
                "last_send_to_sink_receipt": round((t_rx - t_sent_ns) / 1e3, 1),
                "sink_receipt_to_ack_sent": round((t_ack - t_rx) / 1e3, 1),
                "ack_sent_to_node": round((t_acked_ns - t_ack) / 1e3, 1)}

    t_max = max_over_ranks(elapsed)
    total_bytes = sum_over_ranks(float(args.steps * S))
    cross = None
    if launcher is not None:
        if world > 1:
            cross = run_cross_gpu(world, launcher, gpu=gpu_of)
        if native_ladder and ladder_late:
            native = run_native_ladder(launcher, local_rank)
            native_res = run_native_ladder(launcher, local_rank, resident=True)
            native_sample = run_native_ladder(launcher, local_rank, sample=True)
        launcher.close()
    barrier()
    value = total_bytes / t_max / 1e9
    own_ms = [b - a for a, b in intervals]
    avg_pack_ms = sum(own_ms) / len(own_ms) if own_ms else 0.0
    busy_ms = busy_union_ms(intervals)
    # Packs of consecutive sends overlap (in flight on several queues), so one launch's own
    # duration is not the device time it costs: achieved = algorithmic bytes of the timed
    # region's packs / their device span (earliest pack start -> latest fill signal, from the
    # packs' own s_memrealtime stamps), i.e. device time per launch = span / packs.
    span_ms = region["span_ms"] if region else 0.0
    packs = region["packs"] if region else 0
    achieved = 2.0 * S * packs / (span_ms * 1e-3) / 1e9 if span_ms > 0 else 0.0

    if rank != 0:
        return
    traffic = pmc_traffic(S)
    lat = {}
    for s in sink.get("series", []):
        if s["input"] in ("latency", "latency_host"):
            key = str(s["size"]) if s["input"] == "latency" else f"host_{s['size']}"
            lat[key] = {"p50_us": s["p50_us"], "p99_us": s["p99_us"],
                        "p50_incl_pack_us": s["full_p50_us"],
                        "p99_incl_pack_us": s["full_p99_us"], "n": s["n"]}
    # (the checksummed messages of each size are its untimed warm-up, same path and bytes)
    warm = {s["size"]: s for s in hostsink.get("series", []) if s["input"] == "to_host_warm"}
    for s in hostsink.get("series", []):
        if s["input"] == "to_host" and s["size"]:
            w = warm.get(s["size"], {})
            lat[f"d2h_{s['size']}"] = {"p50_us": s["p50_us"], "p99_us": s["p99_us"],
                                       "p50_incl_pack_us": s["full_p50_us"],
                                       "p99_incl_pack_us": s["full_p99_us"], "n": s["n"],
                                       "verified": w.get("verified", 0),
                                       "mismatches": w.get("mismatches", 0)}
    # host paths as rates against this box's PCIe DMA (pinned <-> HBM, box_h2d): host sources
    # (BAR writes to 2 MiB, HIP's copy above) and device samples for a host-only receiver
    # (packed into shared memory to 1 MiB, staged on receipt above)
    host_rates = {}
    for key, z in ([(f"host_{z}", z) for z in LADDER_HOST if z >= 4096] +
                   [(f"d2h_{z}", z) for z in LADDER_D2H if z >= 4096]):
        if key in lat and lat[key]["p50_incl_pack_us"]:
            gbps = z / (lat[key]["p50_incl_pack_us"] * 1e3)
            peak = (h2d_cal or {}).get("h2d_GBps" if key.startswith("host") else "d2h_GBps")
            host_rates[key] = {"GBps_p50": round(gbps, 3),
                               "frac_of_box_dma": round(gbps / peak, 4) if peak else None}
    c2_series = [s for s in sink.get("series", []) if c3 is None or s["size"] != c3["msg_bytes"]]
    verified = sum(s["verified"] for s in c2_series)
    mismatches = sum(s["mismatches"] for s in c2_series)
    if args.workload == "c2":
        metric = f"node->node GB/s ({S:,} B UInt8 samples) + p50/p99 latency per msg size"
        workload = ("C2: examples/benchmark node->sink edge, device-resident UInt8 samples, "
                    "1 node + 1 sink per GPU")
        data = "synthetic (splitmix64 payloads, seed 0xD05A + size)"
    else:
        metric = "node->node GB/s (List<Struct<x,y,z:f32,intensity:u8>> 1M points) + latency"
        workload = ("C3: nested Arrow packing, 1M-point clouds in 16 lists with validity "
                    "bitmaps, node->sink edge per GPU")
        data = "synthetic (seeded point clouds, dora_amd.workloads.point_cloud)"
    line = {
        "metric": metric,
        "value": round(value, 3), "unit": "GB/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(t_max / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u8",
        "data": data,
        "config": {"workload": workload,
                   "msg_bytes": S, "parallelism": f"dp{world} (one dataflow per GPU)",
                   "sources_rotated": nsrc},
        "latency_us": lat,
        # the cgroup's CPU quota and how often it throttled the box during the latency ladder
        "cpu_share": dict(share_lat1 or cpu_share(),
                          during_latency_ladder=(share_delta(share_lat0, share_lat1)
                                                 if share_lat0 and share_lat1 else None)),
        "throughput_per_size": tp_ladder,
        # sources rotated past the L2s / Infinity Cache: every byte read and written in HBM
        "throughput_per_size_native": native,
        # the reference's one source buffer per size (L2-resident reads up to 16 MB)
        "throughput_per_size_native_resident_source": native_res,
        # the reference benchmark's path: allocate_data_sample, a kernel writes the slot, send
        "throughput_per_size_native_sample_path": native_sample,
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                     "vs_box_copy": (round(achieved / (copy_cal["TBps_2S"] * 1e3), 3)
                                     if copy_cal and copy_cal.get("TBps_2S") else None),
                     "traffic": traffic[1] if traffic else None,
                     "traffic_source": traffic[0] if traffic else None,
                     "kernel": (aql_kernel_name(args.workload, region_kernels)
                                if stats["fill_paths"]["aql"]
                                else "pack_kernel (HIP fill streams)"),
                     # AQL packets of the timed region per kernel (dora_gpu_aql_dispatch_counts)
                     "region_kernels": region_kernels,
                     "device_us_per_launch": round(span_ms * 1e3 / max(packs, 1), 3),
                     "region_packs": packs, "region_span_us": round(span_ms * 1e3, 1),
                     "timing": "every timed pack stamps its first workgroup's start and its "
                               "fill signal (s_memrealtime, 100 MHz) into its fill flag's line; "
                               "span = earliest start -> latest signal; achieved = 2 S x packs "
                               "/ span",
                     "per_pack": {"packs": len(intervals),
                                  "own_us": round(avg_pack_ms * 1e3, 3),
                                  "busy_us": round(busy_ms * 1e3 / max(len(intervals), 1), 3),
                                  "note": "own = one pack's start -> signal (concurrent packs "
                                          "overlap); busy = union of the intervals per pack"},
                     "algorithmic_bytes_per_launch": 2 * S},
        "parity": {"verified_msgs": verified, "mismatches": mismatches,
                   "timed_region_verified": verified - min(3, args.warmup)},
        "cold_start_us": round(cold_start_us, 1),
        # the same box's plain device copy of the message size, measured right before the run:
        # boxes differ (and GPUs are shared), so the pack's rate reads against this
        "box_copy": copy_cal,
        # PCIe DMA pinned <-> HBM of this box (the host paths' roofline) and the host paths' rates
        "box_h2d": h2d_cal,
        "host_path_rates": host_rates,
        "host_paths": node_host_paths,
        "box_copy_mid": copy_mid,
        "cold_start_send_us": round(cold_send_us, 1),
        "timed_region": region_setup,
        "sink_us": {"next_event": sink.get("next_event_us"), "free": sink.get("free_us")},
        # inputs the sink's queue (queue_size 10, the reference default) dropped, all phases;
        # `sink_dropped_by_phase` (added below) splits them.  The throughput ladders count only
        # delivered messages (their own `dropped`), and the timed region must show none
        "sink_dropped_inputs": sink.get("dropped_inputs"),
        "node_stats": stats, "exit_codes": codes,
    }
    line["send_mode"] = ("synchronous (DORA_BENCH_SYNC_SENDS=1)" if sync_sends else
                         "DORA_SEND_ASYNC: the benchmark node never rewrites its sources")
    if sync_headline is not None:
        line["sync_send_headline"] = sync_headline
    if sync_mid:
        line["sync_send_4mb"] = sync_mid
    if c3 is not None:
        s3 = [x for x in sink.get("series", []) if x["size"] == c3["msg_bytes"]]
        c3["parity"]["verified_msgs"] = sum(x["verified"] for x in s3)
        c3["parity"]["mismatches"] = sum(x["mismatches"] for x in s3)
        line["c3"] = c3
    if cross is not None:
        line["cross_gpu"] = cross
    if base is not None:
        tp = [s for s in base["series"] if s["mode"] == "throughput" and s["size"] == 40960000]
        line["cpu_baseline"] = {
            "value": tp[0]["GBps"] if tp else None, "unit": "GB/s", "cores": 3, "kind": "port",
            "sample": "reference shm path restated in C++ (sender/daemon/sink pinned to 3 cores,"
                      " TCP control, F8 daemon copy): 100 latency (10 ms apart) + 200 throughput "
                      "msgs per size in {4096, 40960, 409600, 4096000, 40960000}",
            "latency_us": {str(s["size"]): {"p50_us": s["p50_us"], "p99_us": s["p99_us"]}
                           for s in base["series"] if s["mode"] == "latency"},
            "wall_s": base["wall_s"], "nproc": base["nproc"], "cores_used": base["cores"]}
    import gc as _gc
    _gc.enable()
    line["sink_dropped_by_phase"] = drops
    # (other processes, their queues) on this GPU at each phase's end, when KFD sysfs is readable
    line["gpu_tenants_by_phase"] = {k: list(v) for k, v in tenants.items()}
    line["affinity_after_init"] = affinity_after_init
    line["affinity_at_start"] = affinity
    if args.detail:
        try:
            os.makedirs(os.path.dirname(os.path.abspath(args.detail)), exist_ok=True)
            with open(args.detail, "w") as f:
                json.dump(line, f)
        except OSError:
            pass
    print(json.dumps(compact_line(line, args.detail)), flush=True)


def _pick(d, *keys):
    return {k: d[k] for k in keys if d and k in d}


def compact_line(line, detail_path):
    """The stdout line: the contract's keys, the headline roofline, and one summary per target
    of BASELINE north_star (sync send, mid-size, C3, latency p50/p99), short enough to survive a
    2000-character log tail whole (verdict r03 item 4).  Everything else — ladders, per-size
    send phases, intervals — goes to the detail file."""
    out = {k: line[k] for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup",
                                "ms_per_step", "higher_is_better", "scaling", "vs_baseline",
                                "dtype", "data") if k in line}
    cfg = line.get("config", {})
    out["config"] = {"workload": cfg.get("workload", ""), "msg_bytes": cfg.get("msg_bytes"),
                     "parallelism": cfg.get("parallelism")}
    r = line.get("roofline", {})
    out["roofline"] = dict(_pick(r, "bound", "achieved", "peak", "unit", "frac", "traffic",
                                 "device_us_per_launch"),
                           kernel=(r.get("kernel") or "").split(" ")[0])
    out["parity"] = _pick(line.get("parity", {}), "verified_msgs", "mismatches")
    sh = line.get("sync_send_headline")
    if sh:
        out["sync_send"] = _pick(sh, "us_per_msg", "hbm_frac_2S", "pack_own_us", "pack_own_frac",
                                 "gap_us_median")
        # read-first packs hold their stores until every workgroup's loads are in:
        # own time counts that wait and the next pack starts before this one ends
        out["sync_send"]["note"] = "own incl. held-store wait; gap<0: packs overlap"
    if line.get("sync_send_4mb"):
        out["sync_send_4mb"] = _pick(line["sync_send_4mb"], "us_per_msg", "hbm_frac_2S")
    mid = {}
    tp = line.get("throughput_per_size") or {}
    nat = line.get("throughput_per_size_native") or {}
    for z in ("4194304", "4096000"):
        if z in tp and isinstance(tp[z], dict):
            mid[f"py_{z}"] = [tp[z].get("us_per_msg"), tp[z].get("hbm_frac_2S")]
        if z in nat and isinstance(nat[z], dict):
            mid[f"native_{z}"] = [nat[z].get("us_per_msg"), nat[z].get("hbm_frac_2S")]
    if mid:
        out["mid_us_frac"] = mid
    c3 = line.get("c3")
    if c3:
        out["c3"] = {"frac": c3["roofline"]["frac"],
                     "steady_frac": (c3.get("steady") or {}).get("frac"),
                     "us_per_launch": c3["roofline"]["device_us_per_launch"],
                     "mismatches": c3["parity"].get("mismatches")}
    drops = line.get("sink_dropped_by_phase") or {}
    out["sink_dropped"] = {"total": line.get("sink_dropped_inputs"),
                           "by_phase": {k: v for k, v in drops.items() if v}}
    lat = line.get("latency_us") or {}
    out["latency_summary"] = {z: [lat[z]["p50_us"], lat[z]["p99_us"], lat[z]["p99_incl_pack_us"]]
                              for z in ("host_8", "host_2048", "host_4096", "d2h_4096", "8",
                                        "4096", "4194304", "40960000") if z in lat}
    out["latency_summary_keys"] = "size: [p50, p99, p99 incl. pack] us"
    ten = line.get("gpu_tenants_by_phase")
    if ten:  # the most other processes seen on this GPU at any phase's end
        out["gpu_tenants_max"] = max(v[0] for v in ten.values())
    cross = line.get("cross_gpu")
    if cross:  # N > 1: each cross-GPU configuration in one short entry
        out["cross_gpu"] = {
            k: ({"ok": v.get("ok"), "link_GBps": v.get("per_link_GBps"),
                 "xgmi_frac": (v.get("roofline") or {}).get("frac"),
                 "bcast": [(v.get("bcast") or {}).get("groups"),
                           (v.get("bcast") or {}).get("ranks")]}
                if "error" not in v else {"error": v["error"][:60]})
            for k, v in cross.items()}
    out["detail"] = os.path.relpath(detail_path, ROOT) if detail_path else None
    cb = line.get("cpu_baseline")
    if cb:
        out["cpu_baseline"] = dict(_pick(cb, "value", "unit", "cores", "kind"),
                                   sample="oracle/shm_baseline (reference shm path in C++), 3 "
                                          "pinned cores: 100 latency + 200 throughput msgs per "
                                          "size, 4 KB-40.96 MB; value at 40.96 MB")
    return out


if __name__ == "__main__":
    main()
