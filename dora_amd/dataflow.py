"""Local dataflow launcher: descriptor -> daemon process + node processes.

The descriptor follows the reference YAML (libraries/core/src/descriptor/mod.rs:25-200):
`nodes: [{id, path, args, inputs: {in: "node/out" | {source, queue_size}}, outputs, env,
_unstable_deploy: {gpu: N}}]`.  Input queue_size defaults to 10 (binaries/daemon/src/spawn.rs:56).
`path: dynamic` nodes are not spawned: the caller attaches them (e.g. the benchmark process).
GPU placement: `_unstable_deploy.gpu` (new, next to `machine`) sets DORA_GPU_DEVICE.
Runtime nodes (`operators: [{id, shared-library | python, inputs, outputs}]`, or `operator:` with
the default id `op`, descriptor/mod.rs:35-100) run every operator in one process —
`dora-gpu-runtime` for shared libraries, `python -m dora_amd.operator_runtime` for Python
operators — with inputs and outputs named `<operator>/<id>`.

Processes are spawned either directly (the caller has not touched the GPU yet) or through a
`dora_amd.launcher.Launcher` started before the caller initialised HIP.
"""
from __future__ import annotations

import itertools
import os
import shlex
import sys
import subprocess
import tempfile
import time
from dataclasses import dataclass, field
from typing import Dict, List, Optional

from ._lib import LIB_DIR

DEFAULT_QUEUE_SIZE = 10
_counter = itertools.count()


@dataclass
class NodeSpec:
    id: str
    path: str = "dynamic"
    args: List[str] = field(default_factory=list)
    inputs: Dict[str, tuple] = field(default_factory=dict)  # input -> (src_node, src_out, queue)
    outputs: List[str] = field(default_factory=list)
    env: Dict[str, str] = field(default_factory=dict)
    gpu: int = 0          # -1: host-only node
    machine: str = ""     # `_unstable_deploy.machine` ("" = the default machine)


SINGLE_OPERATOR_DEFAULT_ID = "op"  # descriptor/mod.rs:35


def shared_library_path(source: str, base: str) -> str:
    """`adjust_shared_library_path` (libraries/core/src/lib.rs:14-31): `dir/name` ->
    `dir/libname.so`; the name must carry neither the prefix nor an extension."""
    name = os.path.basename(source)
    if name.startswith("lib"):
        raise ValueError("Shared library file name must not start with `lib`, prefix is added "
                         "automatically")
    if os.path.splitext(name)[1]:
        raise ValueError("Shared library file name must have no extension, it is added "
                         "automatically")
    path = os.path.join(os.path.dirname(source), f"lib{name}.so")
    return path if os.path.isabs(path) else os.path.join(base, path)


def _runtime_node(n: dict, base: str) -> dict:
    """A runtime node (`operators` / `operator`) as a plain node spawning the runtime."""
    ops = n.get("operators")
    if ops is None:
        ops = [dict(n["operator"], id=n["operator"].get("id", SINGLE_OPERATOR_DEFAULT_ID))]
    inputs, outputs, items, kinds, stdout_as = {}, [], [], set(), None
    for op in ops:
        oid = op["id"]
        for inp, src in (op.get("inputs") or {}).items():
            inputs[f"{oid}/{inp}"] = src
        outs = [str(o) for o in op.get("outputs", [])]
        outputs += [f"{oid}/{o}" for o in outs]
        if "shared-library" in op:
            kinds.add("shared-library")
            target = shared_library_path(op["shared-library"], base)
        elif "python" in op:
            kinds.add("python")
            src = op["python"]
            target = src if os.path.isabs(src) else os.path.join(base, src)
        else:
            raise ValueError(f"operator `{n['id']}/{oid}` needs `shared-library` or `python`")
        items.append(f"{oid}={target}|{','.join(outs)}")
        if op.get("send_stdout_as"):
            stdout_as = f"{oid}/{op['send_stdout_as']}"
    if len(kinds) > 1:
        raise ValueError(f"runtime node `{n['id']}` mixes shared-library and Python operators")
    env = dict(n.get("env") or {}, DORA_GPU_OPERATORS=";".join(items))
    r = {k: v for k, v in n.items() if k not in ("operators", "operator")}
    if stdout_as:
        r["send_stdout_as"] = stdout_as
    r.update(inputs=inputs, outputs=outputs, env=env)
    if kinds == {"python"}:
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        env["PYTHONPATH"] = os.pathsep.join(
            p for p in (root, os.environ.get("PYTHONPATH", "")) if p)
        r.update(path=sys.executable, args=["-m", "dora_amd.operator_runtime"])
    else:
        r.update(path="dora-gpu-runtime")
    return r


def dataflow_uuid(dataflow_id: str) -> str:
    """The dataflow's `DataflowId` (uuid::Uuid): the id itself when it is a UUID, else the
    name-derived UUID the daemon puts on the inter-daemon wire (csrc/bincode.cpp dataflow_uuid:
    two FNV-1a-64 passes, version 8 / RFC 4122 variant bits)."""
    import uuid
    try:
        return str(uuid.UUID(dataflow_id)) if len(dataflow_id) == 36 else _fnv_uuid(dataflow_id)
    except ValueError:
        return _fnv_uuid(dataflow_id)


def _fnv_uuid(name: str) -> str:
    import uuid
    m = (1 << 64) - 1
    h1, h2 = 0xcbf29ce484222325, 0x84222325cbf29ce4
    for c in name.encode():
        h1 = ((h1 ^ c) * 0x100000001b3) & m
        h2 = ((h2 ^ c) * 0x100000001b3) & m
    u = bytearray(h1.to_bytes(8, "little") + h2.to_bytes(8, "little"))
    u[6] = (u[6] & 0x0F) | 0x80
    u[8] = (u[8] & 0x3F) | 0x80
    return str(uuid.UUID(bytes=bytes(u)))


def node_config(nodes: List[NodeSpec], node_id: str, dataflow_id: str, shm: str) -> dict:
    """The reference's `NodeConfig` (libraries/message/src/daemon_to_node.rs:20-27) of one node,
    as `dora start` hands it over in DORA_NODE_CONFIG (apis/rust/node/src/node/mod.rs:65-76):
    the Rust facade's `DoraNode::init_from_env` / `init(NodeConfig)` (integration/rust) read it.
    `daemon_communication` is the `Shmem` variant naming this data plane's control region (one
    region carries the control, drop and event channels); the descriptor is restated in the
    reference's schema (descriptor/mod.rs:25-200) — `_unstable_deploy` keeps `machine` only,
    since the reference's `Deploy` denies unknown fields; the GPU ordinal travels in
    DORA_GPU_DEVICE."""
    def inputs(n):
        return {k: {"source": f"{src}/{out}", "queue_size": q}
                for k, (src, out, q) in n.inputs.items()}

    def desc_node(n):
        d = {"id": n.id, "inputs": inputs(n), "outputs": list(n.outputs)}
        if n.path != "dynamic":
            d["path"] = n.path
            if n.args:
                d["args"] = " ".join(shlex.quote(a) for a in n.args)
        else:
            d["path"] = "dynamic"
        env = {k: v for k, v in n.env.items() if k != "DORA_GPU_SEND_STDOUT_AS"}
        if env:
            d["env"] = env
        if n.env.get("DORA_GPU_SEND_STDOUT_AS"):
            d["send_stdout_as"] = n.env["DORA_GPU_SEND_STDOUT_AS"]
        if n.machine:
            d["_unstable_deploy"] = {"machine": n.machine}
        return d
    me = next(x for x in nodes if x.id == node_id)
    return {"dataflow_id": dataflow_uuid(dataflow_id), "node_id": node_id,
            "run_config": {"inputs": inputs(me), "outputs": list(me.outputs)},
            "daemon_communication": {"Shmem": {"daemon_control_region_id": shm,
                                               "daemon_drop_region_id": shm,
                                               "daemon_events_region_id": shm,
                                               "daemon_events_close_region_id": shm}},
            "dataflow_descriptor": {"nodes": [desc_node(n) for n in nodes]},
            "dynamic": me.path == "dynamic"}


def node_config_yaml(nodes: List[NodeSpec], node_id: str, dataflow_id: str, shm: str) -> str:
    import yaml
    return yaml.safe_dump(node_config(nodes, node_id, dataflow_id, shm), sort_keys=False)


def _load_descriptor(desc) -> dict:
    """The descriptor as a plain dict (a path is read as YAML), JSON-safe."""
    import json
    if isinstance(desc, str):
        import yaml
        with open(desc) as f:
            desc = yaml.safe_load(f)
    return json.loads(json.dumps(desc, default=str))


def parse_descriptor(desc) -> List[NodeSpec]:
    base = os.getcwd()
    if isinstance(desc, str):
        import yaml
        base = os.path.dirname(os.path.abspath(desc))
        with open(desc) as f:
            desc = yaml.safe_load(f)
    single_op = {n["id"] for n in desc["nodes"] if "operator" in n}
    nodes = []
    for n in desc["nodes"]:
        if "operators" in n or "operator" in n:
            n = _runtime_node(n, base)
        spec = NodeSpec(id=n["id"], path=n.get("path", "dynamic"))
        args = n.get("args", [])
        spec.args = shlex.split(args) if isinstance(args, str) else list(args)
        spec.outputs = list(n.get("outputs", []))
        spec.env = {str(k): str(v) for k, v in (n.get("env") or {}).items()}
        if n.get("send_stdout_as"):
            # the node library sends its stdout / stderr lines on this output (spawn.rs:280-437)
            if n["send_stdout_as"] not in spec.outputs:
                raise ValueError(f"node `{n['id']}`: send_stdout_as `{n['send_stdout_as']}` is "
                                 f"not one of its outputs")
            spec.env["DORA_GPU_SEND_STDOUT_AS"] = str(n["send_stdout_as"])
            spec.env.setdefault("PYTHONUNBUFFERED", "1")  # lines, not blocks, through the pipe
        deploy = n.get("_unstable_deploy") or {}
        spec.gpu = int(deploy.get("gpu", 0))
        spec.machine = str(deploy.get("machine", ""))
        for inp, src in (n.get("inputs") or {}).items():
            q = DEFAULT_QUEUE_SIZE
            if isinstance(src, dict):
                q = int(src.get("queue_size", DEFAULT_QUEUE_SIZE))
                src = src["source"]
            node, out = src.split("/", 1)
            if node in single_op and "/" not in out:  # `node/out` of a single-operator node
                out = f"{SINGLE_OPERATOR_DEFAULT_ID}/{out}"
            spec.inputs[inp] = (node, out, q)
        nodes.append(spec)
    ids = [n.id for n in nodes]
    if len(set(ids)) != len(ids):
        raise ValueError("duplicate node ids")
    outs = {(n.id, o) for n in nodes for o in n.outputs}
    for n in nodes:
        for inp, (src, out, _) in n.inputs.items():
            if (src, out) not in outs:
                raise ValueError(f"input `{n.id}/{inp}` maps unknown output `{src}/{out}`")
    return nodes


def daemon_spec(nodes: List[NodeSpec], machine: Optional[str] = None,
                machines: Optional[Dict[str, tuple]] = None, dataflow_id: str = "local") -> str:
    """The daemon's spec for the nodes deployed on `machine` (None: every node is local).

    A dataflow spanning machines (`_unstable_deploy.machine`, one daemon per machine): remote
    nodes that feed local inputs become proxies of the local daemon, local outputs with remote
    receivers get a `remote` line per machine, `machines` = {name: (host, port)} of the peer
    daemons (this machine's entry is where it listens)."""
    local = [n for n in nodes if machine is None or n.machine == machine]
    local_ids = {n.id for n in local}
    by_id = {n.id: n for n in nodes}
    proxies = {}  # remote source node -> GPU of its first local receiver
    for n in local:
        for _, (src, _, _) in n.inputs.items():
            if src not in local_ids:
                proxies.setdefault(src, n.gpu)
    lines = [f"dataflow {dataflow_id}"]
    if machine is not None and machines:
        for name, (host, port) in sorted(machines.items()):
            if name == machine:
                lines.append(f"listen {host} {port}")
            else:
                lines.append(f"machine {name} {host} {port}")
    lines += [f"node {nid}" for nid in [n.id for n in local] + sorted(proxies)]
    for nid in [n.id for n in local] + sorted(proxies):
        lines += [f"output {nid} {o}" for o in by_id[nid].outputs]
    for src, gpu in sorted(proxies.items()):
        lines.append(f"proxy {src} {gpu}")
    for n in local:
        lines += [f"input {n.id} {i} {s} {o} {q}" for i, (s, o, q) in n.inputs.items()]
    remote = {}  # (src, out, machine) -> receivers' (node, input) there (InputsClosed)
    for n in nodes:
        if n.id in local_ids:
            continue
        for inp, (src, out, _) in n.inputs.items():
            if src in local_ids:
                remote.setdefault((src, out, n.machine), set()).add((n.id, inp))
    lines += [" ".join([f"remote {s} {o} {m}"] + [f"{r}/{i}" for r, i in sorted(ins)])
              for (s, o, m), ins in sorted(remote.items())]
    return "\n".join(lines) + "\n"


def resolve(path: str) -> str:
    cand = os.path.join(LIB_DIR, path)
    return cand if os.path.exists(cand) else path


class _Proc:
    """A spawned process, direct (Popen) or through a Launcher."""

    def __init__(self, argv, env, out, launcher=None):
        self.launcher = launcher
        if launcher is not None:
            self.id = launcher.spawn(argv, env, out)
            if self.id < 0:
                raise RuntimeError(f"launcher could not spawn {argv}")
            self.p = None
        else:
            f = open(out, "w") if out else subprocess.DEVNULL
            self.p = subprocess.Popen(argv, env=env, stdout=f,
                                      stderr=subprocess.STDOUT if out else None)

    def poll(self):
        return self.launcher.poll(self.id) if self.p is None else self.p.poll()

    def wait(self, timeout: float):
        deadline = time.time() + timeout
        while time.time() < deadline:
            rc = self.poll()
            if rc is not None:
                return rc
            time.sleep(0.01)
        return None

    def kill(self):
        if self.p is None:
            self.launcher.kill(self.id)
        elif self.p.poll() is None:
            self.p.kill()
            self.p.wait()


class Dataflow:
    def __init__(self, descriptor, ring_bytes: int = 4 << 20, name: Optional[str] = None,
                 launcher=None, log_dir: Optional[str] = None, machine: Optional[str] = None,
                 machines: Optional[Dict[str, tuple]] = None, dataflow_id: str = "local"):
        """`machine`: run only the nodes deployed on this machine (`_unstable_deploy.machine`)
        under this daemon; `machines` maps machine names to the (host, port) their daemons
        listen on (port 0 for this machine: any free port, see `listen_port`)."""
        self.all_nodes = parse_descriptor(descriptor)
        self.descriptor = _load_descriptor(descriptor)
        self.machine, self.machines, self.dataflow_id = machine, machines, dataflow_id
        self.nodes = [n for n in self.all_nodes if machine is None or n.machine == machine]
        self.listen_port: Optional[int] = None
        self.shm = name or f"/dora-gpu-{os.getpid()}-{next(_counter)}"
        self.ring_bytes = ring_bytes
        self.launcher = launcher
        self.log_dir = log_dir or tempfile.mkdtemp(prefix="dora-gpu-logs-")
        os.makedirs(self.log_dir, exist_ok=True)
        self.daemon: Optional[_Proc] = None
        self.procs: Dict[str, _Proc] = {}
        self._spec_file = None

    def node_env(self, node: NodeSpec) -> dict:
        env = dict(os.environ)
        env.update(node.env)
        env.update(self.dynamic_env(node.id))
        return env

    def dynamic_env(self, node_id: str) -> dict:
        """Environment a node runs with (set it before Node() for `path: dynamic` nodes)."""
        n = next(x for x in self.nodes if x.id == node_id)
        return {"DORA_GPU_DATAFLOW": self.shm, "DORA_NODE_ID": n.id,
                "DORA_GPU_DEVICE": str(n.gpu),
                "DORA_NODE_CONFIG": node_config_yaml(self.all_nodes, n.id, self.dataflow_id,
                                                     self.shm)}

    @staticmethod
    def _ready_port(log: str) -> Optional[int]:
        import json
        for line in log.splitlines():
            if '"ready"' in line:
                try:
                    p = json.loads(line).get("listen_port", -1)
                    return p if p >= 0 else None
                except ValueError:
                    return None
        return None

    def log(self, name: str) -> str:
        p = os.path.join(self.log_dir, f"{name}.log")
        return open(p).read() if os.path.exists(p) else ""

    def start(self, timeout: float = 30.0):
        # the parsed descriptor, for Node.dataflow_descriptor (apis/python/node/src/lib.rs:186)
        import json
        from .node import descriptor_path
        with open(descriptor_path(self.shm), "w") as f:
            json.dump(self.descriptor, f)
        fd, self._spec_file = tempfile.mkstemp(prefix="dora-gpu-spec-", suffix=".txt")
        with os.fdopen(fd, "w") as f:
            f.write(daemon_spec(self.all_nodes, self.machine, self.machines, self.dataflow_id))
        dlog = os.path.join(self.log_dir, "_daemon.log")
        self.daemon = _Proc([resolve("dora-gpu-daemon"), "--shm", self.shm, "--spec",
                             self._spec_file, "--ring-bytes", str(self.ring_bytes)],
                            dict(os.environ), dlog, self.launcher)
        deadline = time.time() + timeout
        while '"ready"' not in self.log("_daemon"):
            if self.daemon.poll() is not None or time.time() > deadline:
                raise RuntimeError(f"daemon failed to start: {self.log('_daemon')!r}")
            time.sleep(0.005)
        self.listen_port = self._ready_port(self.log("_daemon"))
        for n in self.nodes:
            if n.path == "dynamic":
                continue
            self.procs[n.id] = _Proc([resolve(n.path), *n.args], self.node_env(n),
                                     os.path.join(self.log_dir, f"{n.id}.log"), self.launcher)
        return self

    def wait(self, timeout: float = 60.0) -> Dict[str, Optional[int]]:
        deadline = time.time() + timeout
        codes = {}
        for nid, p in self.procs.items():
            codes[nid] = p.wait(max(0.1, deadline - time.time()))
            if codes[nid] is None:
                p.kill()
        if self.daemon:
            codes["_daemon"] = self.daemon.wait(max(0.1, deadline - time.time()))
        return codes

    def stop(self):
        for p in self.procs.values():
            if p.poll() is None:
                p.kill()
        if self.daemon and self.daemon.poll() is None:
            self.daemon.kill()
        if self._spec_file and os.path.exists(self._spec_file):
            os.unlink(self._spec_file)
        shm_path = "/dev/shm" + self.shm
        if os.path.exists(shm_path):
            os.unlink(shm_path)
        from .node import descriptor_path
        if os.path.exists(descriptor_path(self.shm)):
            os.unlink(descriptor_path(self.shm))

    def __enter__(self):
        return self.start()

    def __exit__(self, *exc):
        self.stop()
