#!/usr/bin/env python3
"""Host-side cost of a C3 send, piece by piece (1M-point List<Struct<x,y,z,intensity>> cloud
resident in HBM): schema export, device plan (host DFS + validity gather), pack launch + sync.
Prints one JSON line of mean microseconds per call."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from dora_amd import device
    from dora_amd.arrow_c import release_schema
    from dora_amd.arrow_utils import Plan
    from dora_amd.device import DeviceArray
    from dora_amd.workloads import point_cloud
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    da = DeviceArray.from_pyarrow(point_cloud())
    st = device.Stream()
    out = {}

    def timeit(name, fn):
        fn()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        out[name] = round((time.perf_counter() - t0) / n * 1e6, 2)

    timeit("export_schema_us", lambda: release_schema(da.export_schema()))
    timeit("plan_us", lambda: Plan.of(da).close())
    cloud = point_cloud()
    timeit("plan_host_array_us", lambda: Plan.of(cloud).close())  # same walk, no device reads
    p = Plan.of(da)
    timeit("type_info_us", lambda: p.type_info())
    buf = device.DeviceBuffer(p.size)

    def pack_sync():
        p.pack(buf.ptr, p.size, st)
        st.sync()
    timeit("pack_sync_us", pack_sync)
    out["sample_bytes"] = p.size
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
