"""Runtime node hosting Python operators: `python -m dora_amd.operator_runtime`.

The counterpart of binaries/runtime/src/operator/python.rs.  Every operator is a
file defining `class Operator` with `on_event(self, dora_event, send_output) -> DoraStatus`
(examples/python-operator-dataflow/*.py).  Events are dicts `{"type", "id", "value",
"metadata"}` whose `value` is a host pyarrow array, as in the reference — a device input is
downloaded first (pyarrow cannot import ROCm arrays); `send_output(output_id, data,
metadata=None)` takes bytes or a pyarrow array and sends it as `<operator>/<output>` through the
node's device data plane (python.rs:340-385: bytes as `byte_array`, arrays packed).

    DORA_GPU_OPERATORS="op=/path/op.py|out1,out2;op2=..."   (+ the node env; set by Dataflow)
"""
from __future__ import annotations

import enum
import importlib.util
import os
import sys
import types


class DoraStatus(enum.Enum):
    """apis/rust/operator/types/src/lib.rs:139-146."""
    CONTINUE = 0
    STOP = 1
    STOP_ALL = 2


def _provide_dora_module():
    """Operators written for the reference do `from dora import DoraStatus`: provide that name
    when no `dora` package is importable (it is not part of this build)."""
    try:
        import dora  # noqa: F401
        return
    except ImportError:
        pass
    m = types.ModuleType("dora")
    m.DoraStatus = DoraStatus
    sys.modules["dora"] = m


def _status(ret) -> int:
    if ret is None:
        return 0
    return int(getattr(ret, "value", ret))


def host_value(ev: dict):
    """The input of a node event as a host pyarrow array (what a reference operator receives)."""
    from .device import DeviceArray
    v = ev.get("value")
    if isinstance(v, DeviceArray):
        return v.to_pyarrow()
    return v  # an inline Vec or shared-memory sample: a host pyarrow array already (node.py)


class _Operator:
    def __init__(self, oid: str, path: str, outputs):
        self.id = oid
        self.outputs = [f"{oid}/{o}" for o in outputs if o]
        d = os.path.dirname(os.path.abspath(path))
        if d not in sys.path:
            sys.path.insert(0, d)  # operators import their sibling modules
        spec = importlib.util.spec_from_file_location(f"dora_operator_{oid}", path)
        if spec is None or spec.loader is None:
            raise ImportError(f"operator `{oid}`: cannot load {path}")
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        self.instance = mod.Operator()
        self.running = True


def parse_spec(spec: str):
    for item in filter(None, spec.split(";")):
        oid, _, rest = item.partition("=")
        path, _, outs = rest.partition("|")
        yield oid, path, outs.split(",") if outs else []


def main() -> int:
    from .node import Node
    _provide_dora_module()
    ops = {oid: _Operator(oid, path, outs)
           for oid, path, outs in parse_spec(os.environ["DORA_GPU_OPERATORS"])}
    node = Node()

    def stop(op: _Operator):
        if not op.running:
            return
        op.running = False
        if op.outputs:
            node.close_outputs(op.outputs)
        op.instance = None  # drop_operator

    def deliver(op: _Operator, event: dict) -> bool:
        def send_output(output_id, data, metadata=None):
            md = dict(metadata or {})
            md.setdefault("open_telemetry_context", "")
            node.send_output(f"{op.id}/{output_id}", data, md)

        try:
            status = _status(op.instance.on_event(event, send_output))
        except Exception as e:  # noqa: BLE001 — reported like the reference's on_event error
            print(f"runtime: operator `{op.id}` on_event failed: {e!r}", file=sys.stderr)
            return False
        if status == DoraStatus.STOP.value:
            stop(op)
        elif status == DoraStatus.STOP_ALL.value:
            for o in ops.values():
                stop(o)
        return True

    rc = 0
    while rc == 0 and any(o.running for o in ops.values()):
        ev = node.next()
        if ev is None:
            break
        kind = ev["type"]
        oid, _, local = ev.get("id", "").partition("/")
        op = ops.get(oid)
        if kind == "INPUT" and op and op.running:
            event = {"type": "INPUT", "id": local, "value": host_value(ev),
                     "metadata": ev.get("metadata", {})}
            rc = 0 if deliver(op, event) else 1
        elif kind == "INPUT_CLOSED" and op and op.running:
            rc = 0 if deliver(op, {"type": "INPUT_CLOSED", "id": local}) else 1
        elif kind in ("STOP", "ERROR"):
            event = {"type": kind}
            if kind == "ERROR":
                event["error"] = ev.get("error", "")
            for o in ops.values():
                if o.running and not deliver(o, dict(event)):
                    rc = 1
                    break
    for o in ops.values():
        stop(o)
    node.close()
    return rc


if __name__ == "__main__":
    sys.exit(main())
