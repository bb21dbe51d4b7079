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


@pytest.mark.gpu
def test_bench_two_ranks_on_the_engine(tmp_path):
    """bench.py's multi-rank path end to end on the GPU box: two ranks launched
    by torch.distributed.run, each building and running its own clip on the
    engine (ranks share the one card; gloo for the barrier / max-over-ranks,
    the RCCL path differs only in the backend name), one JSON line from rank 0
    with the whole-job value."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, FASST_BENCH_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--T", "400", "--no-cpu-baseline"]
    r = subprocess.run(cmd, env=env, cwd=str(tmp_path), capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 3 and d["scaling"] == "weak"
    assert d["value"] > 0 and d["value"] == pytest.approx(2 * 3 / (d["ms_per_step"] * 3e-3), rel=1e-3)
