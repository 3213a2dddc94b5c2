"""A process launcher started BEFORE the caller initialises the GPU.

A process that has initialised HIP must not fork+exec new programs itself on this platform, so
long-lived drivers (the pytest session, the benchmark) start this small server first and ask it
to spawn the daemon and node processes.  Protocol: one JSON object per line on stdin/stdout.
    {"op": "spawn", "argv": [...], "env": {...}, "out": path|null}  -> {"id": n, "pid": p}
    {"op": "poll", "id": n}                                         -> {"rc": int|null}
    {"op": "kill", "id": n}                                         -> {"ok": true}
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import threading


class Launcher:
    def __init__(self):
        self.p = subprocess.Popen([sys.executable, "-m", "dora_amd.launcher"],
                                  stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True,
                                  cwd=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        self._lock = threading.Lock()

    def _rpc(self, msg: dict) -> dict:
        with self._lock:
            self.p.stdin.write(json.dumps(msg) + "\n")
            self.p.stdin.flush()
            line = self.p.stdout.readline()
        if not line:
            raise RuntimeError("launcher died")
        return json.loads(line)

    def spawn(self, argv, env=None, out=None) -> int:
        return self._rpc({"op": "spawn", "argv": list(argv), "env": env or dict(os.environ),
                          "out": out})["id"]

    def poll(self, pid_id: int):
        return self._rpc({"op": "poll", "id": pid_id})["rc"]

    def kill(self, pid_id: int):
        self._rpc({"op": "kill", "id": pid_id})

    def close(self):
        if self.p.poll() is None:
            self.p.stdin.close()
            self.p.wait(10)


_default = None


def default() -> Launcher:
    """Process-wide launcher; call this before any GPU work."""
    global _default
    if _default is None:
        _default = Launcher()
    return _default


def _serve():
    procs = {}
    files = {}
    n = 0
    for line in sys.stdin:
        msg = json.loads(line)
        op = msg["op"]
        if op == "spawn":
            out = open(msg["out"], "w") if msg.get("out") else subprocess.DEVNULL
            try:
                p = subprocess.Popen(msg["argv"], env=msg["env"], stdout=out,
                                     stderr=subprocess.STDOUT if msg.get("out") else None)
                n += 1
                procs[n] = p
                files[n] = out
                reply = {"id": n, "pid": p.pid}
            except OSError as e:
                reply = {"id": -1, "error": str(e)}
        elif op == "poll":
            p = procs.get(msg["id"])
            reply = {"rc": None if p is None or p.poll() is None else p.returncode}
            if p is None:
                reply = {"rc": -999}
        elif op == "kill":
            p = procs.get(msg["id"])
            if p is not None and p.poll() is None:
                p.kill()
                p.wait()
            reply = {"ok": True}
        else:
            reply = {"error": f"unknown op {op}"}
        sys.stdout.write(json.dumps(reply) + "\n")
        sys.stdout.flush()
    for p in procs.values():
        if p.poll() is None:
            p.kill()
            p.wait()


if __name__ == "__main__":
    _serve()
