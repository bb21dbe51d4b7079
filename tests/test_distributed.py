"""Multi-process glue of bench.py (one clip per GPU, RCCL only for the
barrier and the max-over-ranks time), rehearsed with gloo on CPU, world 2."""
import os
import socket

import pytest
import torch.multiprocessing as mp

import bench


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world),
                      RANK=str(rank), LOCAL_RANK=str(rank))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    w, r, local, seed, device = bench.rank_setup()
    dist.barrier()
    dt = 1.0 + r                      # rank 1 is the slow one
    dt_max = bench.max_over_ranks(dt, dist, "cpu")
    out[r] = (w, r, local, seed, device, dt_max, bench.job_value(w, 10, dt_max))
    dist.destroy_process_group()


def test_rank_setup_single_process():
    assert bench.rank_setup({}) == (1, 0, 0, 0, 0)
    assert bench.rank_setup({"WORLD_SIZE": "8", "RANK": "5", "LOCAL_RANK": "5"}) == (8, 5, 5, 5, 5)


def test_max_over_ranks_gloo_world2():
    world = 2
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    res = dict(out)
    assert sorted(res) == [0, 1]
    for r in range(world):
        w, rr, local, seed, device, dt_max, value = res[r]
        assert (w, rr, local, seed, device) == (world, r, r, r, r)   # distinct clip per rank
        assert dt_max == 2.0                                          # slowest rank
        assert value == pytest.approx(world * 10 / 2.0)              # whole-job it/s
