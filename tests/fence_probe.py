"""Acquire-fence probe (run as a subprocess by tests/test_gpu_fence.py; the AQL knobs it tests
are read once per process).

Per trial: every CU reads the whole source (`dora_gpu_l2_touch`: the lines sit in every XCD's
L2), WARM packs of the source in this configuration leave its lines in the L1s of the CUs they
ran on, the source is rewritten with a fresh pattern by an engine that runs no
kernel on the GPU's CUs (or a HIP copy), and the source is
sent (`send_output_raw` of a device buffer: one single-segment AQL pack) to a receiver node in
this process, which compares the received sample with the new pattern.  A pack that reads a
stale L2 line delivers bytes of an earlier pattern.

Engines: `bar` (the source lives in the GPU's coarse-grained pool and the host writes it
directly through the PCIe BAR: stores + HDP flush, nothing on the GPU runs), `h2d`
(hipMemcpyAsync from pinned host memory), `d2d` (hipMemcpyAsync from another device buffer).
The negative control's writer is `bar`.  Prints one JSON line: trials,
mismatched trials and the kernels dispatched.
"""
import ctypes
import json
import os
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


WARM = 256


def main():
    import numpy as np

    from dora_amd import _lib, device
    from dora_amd.dataflow import daemon_spec, parse_descriptor
    from dora_amd.device import DeviceBuffer
    from dora_amd.node import Node

    engine = sys.argv[1]
    trials = int(sys.argv[2])
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 16 << 10
    lib = _lib.load()
    device.set_device(0)
    desc = {"nodes": [
        {"id": "src", "outputs": ["raw", "warm"]},
        {"id": "dst", "outputs": [], "inputs": {"raw": {"source": "src/raw", "queue_size": 4}}},
    ]}
    shm = f"/dora-gpu-fence-{os.getpid()}"
    h = ctypes.c_void_p()
    _lib.call("dora_daemon_create", shm.encode(), daemon_spec(parse_descriptor(desc)).encode(),
              1 << 20, ctypes.byref(h))
    t = threading.Thread(target=lambda: lib.dora_daemon_run(h.value, 120000), daemon=True)
    t.start()
    nodes = {}

    def mk(i):
        nodes[i] = Node(i, dataflow=shm, device=0)
    ts = [threading.Thread(target=mk, args=(i,)) for i in ("src", "dst")]
    [x.start() for x in ts]
    [x.join(60) for x in ts]
    src, dst = nodes["src"], nodes["dst"]

    s = device.Stream()
    if engine == "bar":
        bp = ctypes.c_void_p()
        _lib.call("dora_gpu_test_bar_alloc", 0, n, ctypes.byref(bp))
        S = DeviceBuffer.__new__(DeviceBuffer)
        S.ptr, S.size = bp.value, n
    else:
        S = DeviceBuffer(n)
    stage = DeviceBuffer(n)
    hp = ctypes.c_void_p()
    _lib.call("dora_gpu_host_alloc", ctypes.byref(hp), n)
    host = (ctypes.c_uint8 * n).from_address(hp.value)
    got = ctypes.create_string_buffer(n)
    rng = np.random.default_rng(1234)
    bad = 0
    stale_bytes = 0
    for k in range(trials):
        pat = rng.integers(0, 256, n, dtype=np.uint8)
        ctypes.memmove(host, pat.ctypes.data, n)
        # every XCD's L2 holds the source's current lines ...
        _lib.call("dora_gpu_l2_touch", S.ptr, n, s.handle)
        s.sync()
        # ... and so do the L1s of the CUs that ran WARM packs of it (AQL dispatches of this
        # configuration, no release fence: nothing at their end invalidates a CU's L1; sent on
        # an output without receivers, whose tokens come back at once)
        for _ in range(WARM):
            src.send_output_device_bytes("warm", S.ptr, n)
        src.sync()
        if engine == "bar":
            _lib.call("dora_gpu_test_bar_write", 0, S.ptr, hp.value, n)
        elif engine == "h2d":
            _lib.call("dora_gpu_memcpy_async", S.ptr, hp.value, n, s.handle)
        elif engine == "d2d":
            _lib.call("dora_gpu_memcpy_async", stage.ptr, hp.value, n, s.handle)
            s.sync()
            _lib.call("dora_gpu_memcpy_async", S.ptr, stage.ptr, n, s.handle)
        else:
            raise SystemExit(f"unknown engine {engine}")
        s.sync()
        src.send_output_device_bytes("raw", S.ptr, n, {"seq": k})
        while True:
            ev = dst.next(timeout=30)
            if ev is None:
                raise SystemExit("receiver timed out")
            if ev["type"] == "INPUT":
                break
        _lib.call("dora_gpu_memcpy_async", got, ev["data_ptr"], n, None)
        _lib.call("dora_gpu_device_sync")
        ev["value"].close()
        ev["_event"].free()
        diff = np.frombuffer(got.raw, np.uint8) != pat
        if diff.any():
            bad += 1
            stale_bytes += int(diff.sum())
    c = (ctypes.c_uint64 * 16)()
    m = ctypes.c_size_t()
    _lib.call("dora_gpu_aql_dispatch_counts", 0, c, 16, ctypes.byref(m))
    kernels = {lib.dora_gpu_aql_kernel_name(i).decode(): c[i] for i in range(m.value) if c[i]}
    src.close()
    dst.close()
    t.join(30)
    lib.dora_daemon_free(h.value)
    if engine == "bar":
        lib.dora_gpu_test_bar_free(S.ptr)
    else:
        S.free()
    stage.free()
    _lib.call("dora_gpu_host_free", hp.value)
    print(json.dumps({"engine": engine, "trials": trials, "bytes": n, "mismatched": bad,
                      "stale_bytes": stale_bytes, "kernels": kernels,
                      "coherent": os.environ.get("DORA_GPU_AQL_COHERENT", "default"),
                      "acquire": os.environ.get("DORA_GPU_AQL_ACQUIRE", "agent")}), flush=True)


if __name__ == "__main__":
    main()
