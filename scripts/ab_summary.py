#!/usr/bin/env python3
"""One JSON line per bench run of an interleaved A/B directory (b_<tag>_<rep>.json lines and
d_<tag>_<rep>.json detail files, as scripts/r05_probe7.sh / r05_probe8.sh write them): the
headline, the pack's roofline fraction, the synchronous send, C3, latency p50s and the Python
throughput ladder at 64 KB / 4 MB.

    python scripts/ab_summary.py gpurun_out/r5j > profiles/r05_queue_ring_ab.jsonl
"""
import glob
import json
import os
import re
import sys


def main(d):
    for f in sorted(glob.glob(os.path.join(d, "b_*_*.json"))):
        m = re.match(r"b_(.+)_(\d+)\.json$", os.path.basename(f))
        if not m:
            continue
        tag, rep = m.group(1), int(m.group(2))
        try:
            line = json.loads(open(f).read().strip().splitlines()[-1])
        except (ValueError, IndexError):
            print(json.dumps({"tag": tag, "rep": rep, "error": "no bench line"}))
            continue
        det_path = os.path.join(d, f"d_{tag}_{rep}.json")
        det = json.load(open(det_path)) if os.path.exists(det_path) else {}
        lat = line.get("latency_summary") or {}
        tp = det.get("throughput_per_size") or {}
        sync = line.get("sync_send") or {}
        print(json.dumps({
            "tag": tag, "rep": rep, "GBps": line.get("value"),
            "pack_frac": (line.get("roofline") or {}).get("frac"),
            "sync_us_per_msg": sync.get("us_per_msg"), "sync_gap_us": sync.get("gap_us_median"),
            "c3_frac": (line.get("c3") or {}).get("frac"),
            "c3_steady": (line.get("c3") or {}).get("steady_frac"),
            "p50_us": {k: (v or [None])[0] for k, v in lat.items()},
            "tp_us_per_msg": {k: (tp.get(k) or {}).get("us_per_msg") for k in ("65536", "4194304")},
        }))


if __name__ == "__main__":
    main(sys.argv[1])
