#!/usr/bin/env python3
"""Per-message cost of ordering a sample written on the node stream (dora_node_send_output_sample
-> order_fill, hipStreamWriteValue64 into the fill flag): dora_gpu_test_stream_order_probe, a
kernel per message alone / + hipStreamWriteValue64 / + an 8-byte kernel, three rounds.

    python scripts/stream_order_probe.py --n 2000
"""
import argparse
import ctypes
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=2000)
    ap.add_argument("--sizes", default="4096,1048576")
    a = ap.parse_args()
    from dora_amd._lib import call
    out = (ctypes.c_uint64 * 2)()
    for r in range(3):
        for z in [int(x) for x in a.sizes.split(",")]:
            for mode in (0, 1, 2):
                call("dora_gpu_test_stream_order_probe", 0, mode, z, a.n, out)
                print(json.dumps({"round": r, "bytes": z,
                                  "mode": ["kernel", "kernel+write_value", "kernel+kernel"][mode],
                                  "enqueue_us": out[0] / 1e3, "per_msg_us": out[1] / 1e3}),
                      flush=True)


if __name__ == "__main__":
    main()
