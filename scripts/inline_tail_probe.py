#!/usr/bin/env python3
"""Where the inline small-message tail comes from (verdict r05 item 4).

The bench's `latency_host` series, alone and traced: a Python node sends host bytes at a fixed
spacing to the native bench sink (dora-gpu-bench-sink), with DORA_GPU_TRACE on, so every message
is stamped at the sender (after its request is pushed; TP_SENT_RANG when it had to wake the
daemon), at the daemon (routed; TP_ROUTED_WOKE right after a futex sleep) and at the receiver
(popped; TP_POPPED_WOKE when its wait slept).  Inline samples are keyed by their metadata
timestamp.  Per size it prints the sink's p50/p99 and, for the messages above the p90, which
stage took the time and which process had been asleep.

    python scripts/inline_tail_probe.py --sizes 8,4096 --n 2000 --gap-us 1000 --out gpurun_out/x
"""
import argparse
import csv
import glob
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SENT, ROUTED, POPPED = 5, 7, 9
SENT_RANG, ROUTED_WOKE, POPPED_WOKE = 14, 15, 16


def load_traces(d):
    per = {}  # key -> {stage: (t, woke)}
    for f in glob.glob(os.path.join(d, "*.trace.csv")):
        for row in csv.DictReader(open(f)):
            p, k, t = int(row["point"]), row["token"], int(row["t_ns"])
            cpu = int(row.get("cpu", -1))
            stage = {SENT: ("sent", 0), SENT_RANG: ("sent", 1), ROUTED: ("routed", 0),
                     ROUTED_WOKE: ("routed", 1), POPPED: ("popped", 0),
                     POPPED_WOKE: ("popped", 1)}.get(p)
            if stage:
                per.setdefault(k, {})[stage[0]] = (t, stage[1], cpu)
    return per


def interrupts():
    """{(irq, name): [count per CPU]} from /proc/interrupts."""
    out = {}
    try:
        lines = open("/proc/interrupts").read().splitlines()
    except OSError:
        return out
    ncpu = len(lines[0].split())
    for ln in lines[1:]:
        f = ln.split()
        if not f:
            continue
        cnt = []
        for x in f[1:1 + ncpu]:
            if not x.isdigit():
                break
            cnt.append(int(x))
        out[(f[0].rstrip(":"), " ".join(f[1 + len(cnt):])[-40:])] = cnt
    return out


def irq_delta(a, b, cpus):
    """Interrupts each of `cpus` took between snapshots a and b, by source (nonzero only)."""
    res = {}
    for k, cb in b.items():
        ca = a.get(k, [0] * len(cb))
        for c in cpus:
            if c < len(cb) and c < len(ca) and cb[c] - ca[c]:
                res.setdefault(str(c), {})[f"{k[0]} {k[1]}"] = cb[c] - ca[c]
    return res


def ts_of_key(k):
    return int.from_bytes(bytes.fromhex(k[:16]), "little") if k.endswith("f" * 16) else None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="8,4096")
    ap.add_argument("--n", type=int, default=2000)
    ap.add_argument("--gap-us", type=int, default=1000)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "inline_tail"))
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    tdir = tempfile.mkdtemp(prefix="dora-trace-")
    os.environ["DORA_GPU_TRACE"] = tdir
    from dora_amd.dataflow import Dataflow
    from dora_amd.launcher import Launcher
    launcher = Launcher()
    res = os.path.join(tdir, "sink.json")
    desc = {"nodes": [
        {"id": "node", "path": "dynamic", "outputs": ["latency_host", "throughput"],
         "inputs": {"ack": "sink/ack"}},
        {"id": "sink", "path": "dora-gpu-bench-sink", "outputs": ["ack"],
         "inputs": {"latency_host": {"source": "node/latency_host", "queue_size": 10},
                    "throughput": {"source": "node/throughput", "queue_size": 10}},
         "env": {"DORA_BENCH_RESULT": res}},
    ]}
    from dora_amd.node import Node
    sizes = [int(x) for x in a.sizes.split(",")]
    irq0 = None
    with Dataflow(desc, launcher=launcher) as df:
        node = Node("node", dataflow=df.shm, device=0)
        seq = 0
        for z in sizes:
            src = bytes(range(256)) * (z // 256) + bytes(z % 256)
            for _ in range(20):  # warm
                node.send_output("throughput", src, {"seq": seq})
                seq += 1
                time.sleep(a.gap_us / 1e6)
            if irq0 is None:
                irq0, t_irq0 = interrupts(), time.time()
            for _ in range(a.n):
                node.send_output("latency_host", src, {"seq": seq, "t_start": time.time_ns()})
                seq += 1
                time.sleep(a.gap_us / 1e6)
        irq1, t_irq1 = interrupts(), time.time()
        node.send_output("throughput", b"", {"seq": seq, "ack": True})
        node.wait_input("ack", "seq", seq, 60)
        node.close()
        df.wait(60)
        daemon_done = [json.loads(ln) for ln in df.log("_daemon").splitlines()
                       if ln.startswith("{") and '"done"' in ln]
    launcher.close()
    sink = json.load(open(res))
    per = load_traces(tdir)
    out = {"gap_us": a.gap_us, "n": a.n, "sizes": {},
           "pin": os.environ.get("DORA_GPU_PIN", "default"),
           "sink_sched": sink.get("sched"),
           "daemon_sched": daemon_done[0].get("sched") if daemon_done else None}
    for z in sizes:
        s = [x for x in sink["series"] if x["input"] == "latency_host" and x["size"] == z]
        out["sizes"][str(z)] = {"sink_p50_us": s[0]["p50_us"] if s else None,
                                "sink_p99_us": s[0]["p99_us"] if s else None}
    # per message: ts -> sent (the send's request pushed) -> routed -> popped
    rows = []
    for k, st in per.items():
        if not all(x in st for x in ("sent", "routed", "popped")):
            continue
        ts = ts_of_key(k)
        base = ts if ts else st["sent"][0]
        rows.append({"t0": base, "total": (st["popped"][0] - base) / 1e3,
                     "send": (st["sent"][0] - base) / 1e3,
                     "route": (st["routed"][0] - st["sent"][0]) / 1e3,
                     "deliver": (st["popped"][0] - st["routed"][0]) / 1e3,
                     "rang": st["sent"][1], "daemon_woke": st["routed"][1],
                     "recv_woke": st["popped"][1], "inline": ts is not None,
                     "cpu_daemon": st["routed"][2], "cpu_recv": st["popped"][2]})
    # the measured series only: each size's first 20 (warm-up) and the closing ack go
    rows.sort(key=lambda r: r["t0"])
    rows = [r for r in rows if r["t0"]]
    groups = {True: [r for r in rows if r["inline"]], False: [r for r in rows if not r["inline"]]}
    for k in groups:
        groups[k] = groups[k][20:20 + a.n]
    out["rows"] = {("inline" if k else "slot"): v for k, v in groups.items()}
    for inline in (True, False):
        rr = sorted(groups[inline], key=lambda r: r["total"])
        if not rr:
            continue
        tail = rr[int(0.9 * len(rr)):]
        pct = lambda v, q: sorted(v)[int(q * (len(v) - 1))]
        summ = {"msgs": len(rr),
                "total_p50_us": pct([r["total"] for r in rr], .5),
                "total_p99_us": pct([r["total"] for r in rr], .99),
                "tail_msgs": len(tail)}
        for f in ("send", "route", "deliver"):
            summ[f"{f}_p50_us"] = pct([r[f] for r in rr], .5)
            summ[f"tail_{f}_mean_us"] = sum(r[f] for r in tail) / len(tail)
        for f in ("rang", "daemon_woke", "recv_woke"):
            summ[f"{f}_frac_all"] = sum(r[f] for r in rr) / len(rr)
            summ[f"{f}_frac_tail"] = sum(r[f] for r in tail) / len(tail)
        out["inline" if inline else "slot"] = summ
        out[("inline" if inline else "slot") + "_worst"] = rr[-12:]
    cpus = sorted({r["cpu_daemon"] for g in groups.values() for r in g} |
                  {r["cpu_recv"] for g in groups.values() for r in g})
    out["cpus_daemon"] = sorted({r["cpu_daemon"] for g in groups.values() for r in g})
    out["cpus_recv"] = sorted({r["cpu_recv"] for g in groups.values() for r in g})
    out["irqs_on_those_cpus"] = irq_delta(irq0 or {}, irq1, cpus)
    out["irq_window_s"] = round(t_irq1 - t_irq0, 3) if irq0 else None
    print(json.dumps({k: v for k, v in out.items() if k != "rows"}, indent=1))
    json.dump(out, open(os.path.join(a.out, "inline_tail.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
