"""dora_amd.tenants (bench diagnostics): other processes with queues on this process's GPU, read
from a KFD sysfs tree — here a fake one, since the container has no GPU."""
import os

from dora_amd import tenants


def _queue(root, pid, qid, gpuid):
    d = os.path.join(root, str(pid), "queues", str(qid))
    os.makedirs(d)
    with open(os.path.join(d, "gpuid"), "w") as f:
        f.write(f"{gpuid}\n")


def test_counts_other_processes_on_our_gpu_only(tmp_path, monkeypatch):
    root = str(tmp_path)
    me = os.getpid()
    _queue(root, me, 0, 1234)           # our queues: GPU 1234
    _queue(root, 999001, 0, 1234)       # a tenant with two queues on our GPU
    _queue(root, 999001, 1, 1234)
    _queue(root, 999002, 0, 5678)       # a process on another GPU
    os.makedirs(os.path.join(root, "999003"))  # a KFD process with no queues
    monkeypatch.setattr(tenants, "KFD_PROC", root)
    monkeypatch.setattr(tenants, "_ppid", lambda pid: 1)  # none of them descends from us
    t = tenants.gpu_tenants()
    assert t == {"visible": True, "kfd_processes": 4, "gpuids": [1234], "others": 1,
                 "other_queues": 2}


def test_descendants_are_ours(tmp_path, monkeypatch):
    root = str(tmp_path)
    me = os.getpid()
    _queue(root, me, 0, 7)
    _queue(root, 999011, 0, 7)          # our sink (a grandchild)
    parents = {999011: 999010, 999010: me}
    monkeypatch.setattr(tenants, "KFD_PROC", root)
    monkeypatch.setattr(tenants, "_ppid", lambda pid: parents.get(pid, 1))
    assert tenants.gpu_tenants()["others"] == 0


def test_unreadable_tree_is_reported_invisible(tmp_path, monkeypatch):
    monkeypatch.setattr(tenants, "KFD_PROC", str(tmp_path / "missing"))
    assert tenants.gpu_tenants() == {"visible": False}
