"""Other processes using this process's GPU, from the KFD sysfs tree (diagnostics for the bench:
an HBM-bound rate that drops mid-run on a shared box is another tenant's traffic, not ours).

/sys/class/kfd/kfd/proc/<pid>/queues/<qid>/gpuid names the GPU of each user queue a process
holds.  The GPU of this process is the one its own queues sit on (it has created them by the
time the bench asks); a process holding a queue on that GPU whose pid is not ours nor a descendant
of ours is a tenant.  Everything here is best effort: unreadable entries are skipped."""
import os

KFD_PROC = "/sys/class/kfd/kfd/proc"


def _gpuids(pid):
    out = set()
    qdir = os.path.join(KFD_PROC, str(pid), "queues")
    try:
        qs = os.listdir(qdir)
    except OSError:
        return out
    for q in qs:
        try:
            with open(os.path.join(qdir, q, "gpuid")) as f:
                out.add(int(f.read().strip() or 0))
        except (OSError, ValueError):
            pass
    return out


def _ppid(pid):
    try:
        with open(f"/proc/{pid}/stat") as f:
            return int(f.read().rsplit(")", 1)[1].split()[1])
    except (OSError, ValueError, IndexError):
        return 0


def _descends_from(pid, root):
    for _ in range(16):
        pid = _ppid(pid)
        if pid <= 1:
            return False
        if pid == root:
            return True
    return False


def gpu_tenants(own_pids=()):
    """{"visible": bool, "gpuids": [...], "others": n, "other_queues": n} for the GPUs this
    process (or any pid in `own_pids`) has queues on."""
    try:
        pids = [int(p) for p in os.listdir(KFD_PROC) if p.isdigit()]
    except OSError:
        return {"visible": False}
    me = os.getpid()
    ours = {me, *own_pids}
    mine = set()
    for p in ours:
        mine |= _gpuids(p)
    others, queues = 0, 0
    for p in pids:
        if p in ours or _descends_from(p, me):
            continue
        g = _gpuids(p)
        if mine and g & mine:
            others += 1
            try:
                queues += len(os.listdir(os.path.join(KFD_PROC, str(p), "queues")))
            except OSError:
                pass
    return {"visible": True, "kfd_processes": len(pids), "gpuids": sorted(mine),
            "others": others, "other_queues": queues}
