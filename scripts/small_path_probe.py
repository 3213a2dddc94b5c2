#!/usr/bin/env python3
"""The alternatives to a pack kernel for a device-resident sample < 4096 B (verdict r04 item 1,
DESIGN §10.1): what it costs the host to get such a sample's bytes out of HBM without a kernel
dispatch, from an idle GPU (1 ms between reads, as the bench's latency ladder).

  * copy:  hipMemcpyAsync device -> pinned host + stream synchronize (the runtime's engine);
  * bar:   host loads straight from device memory through the PCIe BAR (memory of the
           coarse-grained pool made host-accessible, dora_gpu_test_bar_alloc).

    python scripts/small_path_probe.py --n 300 > small_path.jsonl
"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=300)
    ap.add_argument("--gap-us", type=int, default=1000)
    a = ap.parse_args()
    from dora_amd import _lib, device
    from dora_amd.device import DeviceBuffer
    device.set_device(0)
    s = device.Stream()
    src = DeviceBuffer(4096)
    hp = ctypes.c_void_p()
    _lib.call("dora_gpu_host_alloc", ctypes.byref(hp), 4096)
    pattern = bytes((i * 131 + 7) & 255 for i in range(4096))
    ctypes.memmove(hp.value, pattern, 4096)
    _lib.call("dora_gpu_memcpy_async", src.ptr, hp.value, 4096, s.handle)
    s.sync()
    bp = ctypes.c_void_p()
    _lib.call("dora_gpu_test_bar_alloc", 0, 4096, ctypes.byref(bp))
    _lib.call("dora_gpu_test_bar_write", 0, bp.value, hp.value, 4096)  # the same bytes in both
    out = ctypes.create_string_buffer(4096)
    for path in ("copy", "bar"):
        for z in (8, 4096):
            ts = []
            for k in range(a.n + 5):
                time.sleep(a.gap_us / 1e6)
                t0 = time.perf_counter()
                if path == "copy":
                    _lib.call("dora_gpu_memcpy_async", hp.value, src.ptr, z, s.handle)
                    s.sync()
                    ctypes.memmove(out, hp.value, z)
                else:
                    ctypes.memmove(out, bp.value, z)
                ts.append((time.perf_counter() - t0) * 1e6)
            assert out.raw[:z] == pattern[:z], path
            ts = sorted(ts[5:])
            print(json.dumps({"path": path, "bytes": z, "n": a.n, "gap_us": a.gap_us,
                              "p50_us": round(statistics.median(ts), 3),
                              "p99_us": round(ts[int(0.99 * (len(ts) - 1))], 3)}), flush=True)
    _lib.load_testing().dora_gpu_test_bar_free(bp.value)
    _lib.call("dora_gpu_host_free", hp.value)
    src.free()
    s.close()


if __name__ == "__main__":
    main()
