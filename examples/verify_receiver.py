"""A Python receiver node: for every input, checksum the received device sample (every parity
region, on the GPU) and report it on the `result` output.  Used by the end-to-end parity tests
(the pyarrow-assert role of node-hub/pyarrow-assert/pyarrow_assert/main.py:52-55)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from dora_amd.device import DeviceBuffer  # noqa: E402
from dora_amd.node import Node  # noqa: E402
from dora_amd.verify import regions_csum, to_i64  # noqa: E402


def main():
    node = Node()
    for ev in node:
        if ev["type"] != "INPUT":
            continue
        ptr, tmp = ev["data_ptr"], None
        if ev["data_len"] and not ev["on_device"]:
            # an inline Vec sample (< 4096 B from a host source): its bytes into HBM, then the
            # same device checksum
            tmp = DeviceBuffer.from_bytes(ctypes.string_at(ptr, ev["data_len"]))
            ptr = tmp.ptr
        c = regions_csum(ptr, ev["type_info"]) if ev["data_len"] else 0
        if tmp is not None:
            tmp.free()
        meta = {"seq": ev["metadata"].get("seq", -1), "csum": to_i64(c), "len": ev["data_len"],
                "on_device": ev["on_device"], "data_type": ev["type_info"].data_type}
        v = ev["value"]
        if ev["data_len"] and ev["data_len"] <= 1 << 16:
            meta["arrow_equal_len"] = len(v.to_pyarrow() if hasattr(v, "to_pyarrow") else v)
        if hasattr(v, "close"):
            v.close()
        node.send_output("result", b"", meta)
    node.close()


if __name__ == "__main__":
    main()
