"""Per-CPU busy share between two /proc/stat snapshots (scripts/lat_tail_ab.sh).

`snap` prints {cpu: [busy_ticks, total_ticks]}; busy() reduces two snapshots to the busy share
of every CPU plus the CPUs of L3 domain 0 of NUMA node 0 (where DORA_GPU_PIN=fixed puts the
dataflow of GPU 0) and of the whole box.
"""
import json
import sys


def snap():
    out = {}
    with open("/proc/stat") as f:
        for ln in f:
            if ln.startswith("cpu") and ln[3].isdigit():
                p = ln.split()
                v = [int(x) for x in p[1:]]
                idle = v[3] + v[4]
                out[p[0][3:]] = [sum(v) - idle, sum(v)]
    return out


def _cpus(path):
    s = set()
    try:
        txt = open(path).read().strip()
    except OSError:
        return s
    for part in txt.split(","):
        if "-" in part:
            a, b = part.split("-")
            s.update(range(int(a), int(b) + 1))
        elif part:
            s.add(int(part))
    return s


def busy(a, b):
    share = {}
    for c in a:
        if c in b:
            dt = b[c][1] - a[c][1]
            share[int(c)] = (b[c][0] - a[c][0]) / dt if dt > 0 else 0.0
    l3 = _cpus("/sys/devices/system/cpu/cpu0/cache/index3/shared_cpu_list")
    node0 = _cpus("/sys/devices/system/node/node0/cpulist")

    def mean(cs):
        v = [share[c] for c in cs if c in share]
        return round(sum(v) / len(v), 3) if v else None

    return {"box": mean(share), "numa0": mean(node0), "l3_of_cpu0": mean(l3),
            "l3_of_cpu0_cpus": sorted(l3),
            "l3_of_cpu0_each": {c: round(share[c], 3) for c in sorted(l3) if c in share},
            "busiest": sorted(((round(v, 3), c) for c, v in share.items()), reverse=True)[:8]}


if __name__ == "__main__":
    if sys.argv[1:] == ["snap"]:
        print(json.dumps(snap()))
