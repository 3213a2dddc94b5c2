"""The N>1 path of bench.py on CPU: world_size-2 gloo ranks aggregate like the driver expects
(value = bytes of all ranks / max-over-ranks time), with rendezvous on 127.0.0.1."""
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank)})
    import bench
    r = bench.Ranks(world)
    r.barrier()
    elapsed = 1.0 + rank            # rank 1 is the slow one
    t_max = r.max(elapsed)
    total = r.sum(float(1000 * (rank + 1)))
    out[rank] = (t_max, total)
    r.barrier()


def test_two_rank_aggregation():
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(2, port, out), nprocs=2, join=True)
    assert out[0] == out[1] == (2.0, 3000.0)


def test_single_rank_is_identity():
    import bench
    r = bench.Ranks(1)
    r.barrier()
    assert r.max(3.5) == 3.5 and r.sum(2.0) == 2.0


def test_pmc_traffic_lookup():
    import bench
    t = bench.pmc_traffic(40960000)
    assert t is not None and abs(t[1] / 81920000 - 1) < 0.05
    assert bench.pmc_traffic(123) is None


@pytest.mark.parametrize("n", [2, 4, 8])
def test_cross_gpu_descriptors(n, tmp_path):
    """C4 fan-out / C5 chain dataflows of bench.py (N>1): valid descriptors, one stage per GPU."""
    import bench
    from dora_amd.dataflow import daemon_spec, parse_descriptor
    c4 = parse_descriptor(bench.c4_descriptor(n, str(tmp_path)))
    assert [x.gpu for x in c4] == list(range(n))
    assert len([x for x in c4 if x.id.startswith("sink")]) == n - 1
    assert c4[0].env["DORA_BENCH_ACKS"] == str(n - 1)
    assert c4[0].env["DORA_BENCH_TP_SIZE"] == str(1920 * 1080 * 3)
    c5 = parse_descriptor(bench.c5_descriptor(n, str(tmp_path), "sdma"))
    assert [x.gpu for x in c5] == list(range(n))
    assert [x.path for x in c5] == (["dora-gpu-bench-source"] + ["dora-gpu-relay"] * (n - 2)
                                    + ["dora-gpu-bench-sink"])
    for prev, cur in zip(c5, c5[1:]):
        assert cur.inputs["throughput"][0] == prev.id and cur.env["DORA_GPU_PEER_COPY"] == "sdma"
    assert "input source ack0 sink ack" in daemon_spec(c5)


def test_summarize_cross():
    import bench
    src = {"ok": True, "receivers": 2, "tp_size": 100, "tp_n": 10, "tp_delivered_GBps": 200.0,
           "tp_per_receiver_GBps": 100.0, "send_phase_us": {}}
    sink = {"errors": 0, "dropped_inputs": 0, "pulls": 13, "pull_bytes": 1300, "series": [
        {"input": "latency", "size": 100, "n": 5, "p50_us": 10.0, "p99_us": 20.0,
         "full_p50_us": 12.0, "full_p99_us": 22.0, "verified": 2, "mismatches": 0,
         "first_ns": 0, "last_ns": 500},
        {"input": "throughput", "size": 100, "n": 11, "p50_us": 1.0, "p99_us": 1.0,
         "full_p50_us": 0, "full_p99_us": 0, "verified": 0, "mismatches": 0,
         "first_ns": 1000, "last_ns": 2000}]}
    r = bench.summarize_cross("c4", src, {"sink1": sink, "sink2": sink}, {"source": 0}, {})
    assert r["ok"] and r["parity"]["verified_msgs"] == 4
    assert r["roofline"]["frac"] == round(100.0 / bench.XGMI_LINK_GBPS, 4)
    assert len(r["latency_us"]["100"]) == 2
    # per edge: 10 intervals of 100 B in 1000 ns = 1 GB/s, over a link (pulls > 0)
    assert [e["GBps"] for e in r["edges"]] == [1.0, 1.0]
    assert r["edges"][0]["xgmi_frac"] == round(1.0 / bench.XGMI_LINK_GBPS, 4)
    assert r["pull_bytes"] == 2600
    bad = dict(sink, series=[dict(sink["series"][0], mismatches=1)])
    assert not bench.summarize_cross("c4", src, {"s": bad}, {}, {})["ok"]


def test_summarize_cross_without_link_traffic_has_no_roofline():
    """A run whose stages all sat on one GPU (no pull, no broadcast) moved nothing over xGMI:
    its roofline is null and the edges carry no link fraction."""
    import bench
    src = {"ok": True, "receivers": 1, "tp_size": 100, "tp_n": 10, "tp_delivered_GBps": 900.0,
           "tp_per_receiver_GBps": 900.0, "send_phase_us": {}}
    sink = {"errors": 0, "dropped_inputs": 0, "pulls": 0, "pull_bytes": 0, "series": [
        {"input": "throughput", "size": 100, "n": 11, "p50_us": 1.0, "p99_us": 1.0,
         "full_p50_us": 0, "full_p99_us": 0, "verified": 1, "mismatches": 0,
         "first_ns": 1000, "last_ns": 2000}]}
    r = bench.summarize_cross("c4", src, {"sink1": sink}, {"source": 0}, {})
    assert r["roofline"] is None and "no byte crossed" in r["note"]
    assert r["edges"][0]["xgmi_frac"] is None


def test_edge_rate_uses_the_throughput_burst():
    """The sink's series of one (input, size) also holds the warmup receipts, seconds before the
    back-to-back phase; the edge rate comes from the longest burst between two acks (r02 N=2
    rehearsal: 1.25 GB/s over the whole series vs ~1300 GB/s delivered)."""
    import bench
    sink = {"pulls": 200, "pull_bytes": 200 * 100, "series": [
        {"input": "throughput", "size": 100, "n": 13, "first_ns": 0, "last_ns": 10 ** 9 + 2000,
         "burst_n": 11, "burst_first_ns": 10 ** 9 + 1000, "burst_last_ns": 10 ** 9 + 2000}]}
    e = bench.edge_rates({"sink1": sink})[0]
    assert e["GBps"] == 1.0 and e["xgmi_frac"] == round(1.0 / bench.XGMI_LINK_GBPS, 4)
    old = {"pulls": 0, "series": [dict(sink["series"][0], burst_n=0)]}  # older sinks: whole series
    assert bench.edge_rates({"s": old})[0]["GBps"] == round(12 * 100 / (10 ** 9 + 2000), 3)


def test_ladder_sources_rotate_past_the_caches():
    """The throughput ladders read every byte from HBM: rotated copies cover > 256 MB (the
    Infinity Cache) at 16 MB and up, > 32 MB (the eight L2s) from 1 MB, at most 64 copies; the
    resident-source ladder is the reference node's one buffer per size."""
    import bench
    for size in (1 << 20, 4096000, 16 << 20, 40960000):
        n = bench.native_sources(size)
        assert 1 < n <= 64
        assert n * size > 32 << 20
        if size >= 16 << 20:
            assert n * size > 256 << 20
        assert bench.native_sources(size, resident=True) == 1
    assert bench.native_sources(0) == 64 and bench.native_sources(4096) == 64


def test_aql_kernel_name_is_the_region_kernel():
    import bench
    assert bench.aql_kernel_name("c2") == "dora_aql_pack1_u4 (AQL)"
    assert bench.aql_kernel_name("c3") == "dora_aql_pack_u4 (AQL)"
    assert bench.aql_kernel_name("c2", {"dora_aql_pack1_u4": 18, "dora_aql_pack1c_u4": 2}) == \
        "dora_aql_pack1_u4 (AQL)"
    assert bench.aql_kernel_name("c2", {"dora_aql_pack1c_u4": 20}) == "dora_aql_pack1c_u4 (AQL)"


def test_compact_line_fits_the_driver_tail():
    """The stdout line keeps the contract's keys and the north_star summaries (latency p50/p99 at
    4 KB / 4 MiB / 40.96 MB, sync send, mid-size, C3, drops) within a 2000-character log tail
    (verdict r03 item 4), from a full r03 line with every ladder filled in."""
    import json
    import os

    import bench
    full = json.load(open(os.path.join(os.path.dirname(__file__), "..", "profiles",
                                       "r03_final_bench_1.json")))
    full["sink_dropped_by_phase"] = {"warmup": 0, "latency_ladder": 2, "timed_region": 0}
    full["config"]["workload"] = ("C2: examples/benchmark node->sink edge, device-resident UInt8 "
                                  "samples, 1 node + 1 sink per GPU")
    for z in ("host_8", "host_512", "host_2048", "host_4096", "d2h_4096"):
        full["latency_us"][z] = dict(full["latency_us"]["8"])
    full["sync_send_headline"].update({"hbm_frac_2S": 0.19, "pack_own_us": 17.9,
                                       "pack_own_frac": 0.57, "gap_us_median": 6.3})
    c = bench.compact_line(full, os.path.join(bench.ROOT, "gpurun_out", "bench_detail.json"))
    text = json.dumps(c)
    assert len(text) < 1900, len(text)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
              "roofline", "cpu_baseline"):
        assert k in c, k
    assert list(c)[-1] == "cpu_baseline"
    assert set(c["latency_summary"]) == {"host_8", "host_2048", "host_4096", "d2h_4096", "8",
                                         "4096", "4194304", "40960000"}
    assert c["config"]["workload"] == full["config"]["workload"]  # whole, not cut
    assert c["roofline"]["frac"] == full["roofline"]["frac"]
    assert c["sink_dropped"]["by_phase"] == {"latency_ladder": 2}
    assert c["c3"]["frac"] == full["c3"]["roofline"]["frac"]


def test_compact_line_with_cross_gpu_block():
    """N > 1: the compact line carries one short entry per cross-GPU configuration (link GB/s,
    xGMI fraction, RCCL groups and the ranks RCCL formed) and still fits the driver's tail."""
    import json

    import bench
    cross = {"c4_fanout_kernel": {"ok": True, "per_link_GBps": 120.5,
                                  "roofline": {"frac": 0.7876}, "bcast": {"groups": 0, "ranks": 0}},
             "c4_fanout_rccl": {"ok": True, "per_link_GBps": 98.1, "roofline": {"frac": 0.641},
                                "bcast": {"groups": 1, "ranks": 8}},
             "c5_chain_kernel": {"error": "RuntimeError('daemon failed to start: ...')" * 3}}
    full = {"metric": "m", "value": 1.0, "unit": "GB/s", "n_gpus": 8, "steps": 20, "warmup": 5,
            "ms_per_step": 0.1, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "u8", "data": "synthetic", "config": {"workload": "C2", "msg_bytes": 1,
                                                           "parallelism": "dp8"},
            "roofline": {"bound": "hbm", "frac": 0.8, "kernel": "dora_aql_pack1_u4 (AQL)"},
            "parity": {"verified_msgs": 3, "mismatches": 0}, "latency_us": {},
            "cross_gpu": cross, "sink_dropped_inputs": 0}
    c = bench.compact_line(full, None)
    assert c["cross_gpu"]["c4_fanout_rccl"] == {"ok": True, "link_GBps": 98.1, "xgmi_frac": 0.641,
                                                "bcast": [1, 8]}
    assert len(c["cross_gpu"]["c5_chain_kernel"]["error"]) <= 60
    assert len(json.dumps(c)) < 1900
