"""The N>1 path of bench.py on CPU: world_size-2 gloo ranks aggregate like the driver expects
(value = bytes of all ranks / max-over-ranks time), with rendezvous on 127.0.0.1."""
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank)})
    import bench
    r = bench.Ranks(world)
    r.barrier()
    elapsed = 1.0 + rank            # rank 1 is the slow one
    t_max = r.max(elapsed)
    total = r.sum(float(1000 * (rank + 1)))
    out[rank] = (t_max, total)
    r.barrier()


def test_two_rank_aggregation():
    port = _free_port()
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(2, port, out), nprocs=2, join=True)
    assert out[0] == out[1] == (2.0, 3000.0)


def test_single_rank_is_identity():
    import bench
    r = bench.Ranks(1)
    r.barrier()
    assert r.max(3.5) == 3.5 and r.sum(2.0) == 2.0


def test_pmc_traffic_lookup():
    import bench
    t = bench.pmc_traffic(40960000)
    assert t is not None and abs(t[1] / 81920000 - 1) < 0.05
    assert bench.pmc_traffic(123) is None
