"""CPU: the multi-GPU harness of bench.py at world size 2 over gloo (the GPU box uses RCCL):
max-over-ranks time, summed frames, and the all-gather of every rank's pose array (ragged)."""
import os
import socket
import sys

import numpy as np
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path.insert(0, ROOT)
    import torch.distributed as dist
    import bench
    dist.init_process_group("gloo", init_method="env://", rank=rank, world_size=world)
    poses = np.arange(7 * (3 + rank), dtype=np.float64).reshape(-1, 7) + 100 * rank
    el, frames, allp = bench.reduce_results(dist, 1.0 + rank, 10 + rank, poses, "cpu")
    out[rank] = (el, frames, [a.tolist() for a in allp])
    dist.destroy_process_group()


def test_reduce_results_gloo_world2():
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(2, port, out), nprocs=2, join=True)
        res = dict(out)
    for rank in (0, 1):
        el, frames, allp = res[rank]
        assert el == 2.0 and frames == 21
        assert len(allp) == 2
        for r in (0, 1):
            exp = np.arange(7 * (3 + r), dtype=np.float64).reshape(-1, 7) + 100 * r
            np.testing.assert_array_equal(np.array(allp[r]), exp)
