"""Multi-process glue of bench.py (one clip per GPU; RCCL / gloo only for the
barrier, the max-over-ranks time and the clips' allgather), rehearsed with
gloo on CPU, world 2, and through bench.py's own launcher."""
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
    # eight GPUs: one clip per card; one GPU (the rehearsal box): the ranks share it
    assert bench.rank_setup({"WORLD_SIZE": "8", "RANK": "5", "LOCAL_RANK": "5"}, ndev=8) == \
        (8, 5, 5, 5, 5)
    assert bench.rank_setup({"WORLD_SIZE": "2", "RANK": "1", "LOCAL_RANK": "1"}, ndev=1) == \
        (2, 1, 1, 1, 0)


def test_choose_backend():
    assert bench.choose_backend(8, 8, {}) == "nccl"          # RCCL, one GPU per rank
    assert bench.choose_backend(1, 1, {}) == "nccl"
    assert bench.choose_backend(2, 1, {}) == "gloo"          # ranks share a card
    assert bench.choose_backend(8, 8, {"FASST_BENCH_BACKEND": "gloo"}) == "gloo"
    with pytest.raises(SystemExit):
        bench.choose_backend(2, 1, {"FASST_BENCH_BACKEND": "nccl"})


def test_check_clips():
    bench.check_clips([[0, 0, 0, -1.5, 1.0], [1, 1, 1, -1.25, 1.1]])
    with pytest.raises(RuntimeError):      # two ranks ran the same clip
        bench.check_clips([[0, 0, 0, -1.5, 1.0], [1, 0, 1, -1.5, 1.1]])
    with pytest.raises(RuntimeError):      # a rank is missing
        bench.check_clips([[0, 0, 0, -1.5, 1.0], [0, 1, 1, -1.25, 1.1]])


def _bench_cmd(*args):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    return [sys.executable, os.path.join(root, "bench.py")] + list(args)


def _clean_env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR",
                        "MASTER_PORT", "FASST_BENCH_BACKEND")}
    env.update(kw)
    return env


def test_launcher_two_ranks_without_torchrun(tmp_path):
    """`python bench.py --gpus 2` with no WORLD_SIZE starts the two ranks
    itself; rank 0 prints one line with n_gpus 2 and two distinct clips
    (the control plane on the CPU: --dry-run)."""
    import json
    import subprocess
    r = subprocess.run(_bench_cmd("--gpus", "2", "--steps", "3", "--dry-run"), env=_clean_env(),
                       cwd=str(tmp_path), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 3
    assert sorted(c["rank"] for c in d["clips"]) == [0, 1]
    assert len({c["data_seed"] for c in d["clips"]}) == 2
    assert len({c["loglik"] for c in d["clips"]}) == 2
    assert d["value"] == pytest.approx(2 * 3 / (d["ms_per_step"] * 3e-3), rel=1e-6)


def test_launcher_refuses_world_size_mismatch(tmp_path):
    import subprocess
    r = subprocess.run(_bench_cmd("--gpus", "2", "--steps", "1", "--dry-run"),
                       env=_clean_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"),
                       cwd=str(tmp_path), capture_output=True, text=True, timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE=1 but --gpus 2" in r.stderr


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
def test_bench_gpus2_self_launched(tmp_path):
    """`python bench.py --gpus 2` exactly as the driver invokes it (no
    torchrun): two ranks, two distinct clips on the engine, one JSON line.
    On the one-GPU box the ranks share the card (gloo control plane)."""
    import json
    import subprocess
    import torch
    r = subprocess.run(_bench_cmd("--gpus", "2", "--steps", "3", "--warmup", "1", "--warm-s", "0",
                                  "--T", "400", "--no-cpu-baseline"),
                       env=_clean_env(), cwd=str(tmp_path), capture_output=True, text=True,
                       timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 3
    assert d["control_plane"] == ("nccl" if torch.cuda.device_count() >= 2 else "gloo")
    clips = d["clips"]
    assert sorted(c["rank"] for c in clips) == [0, 1]
    assert len({c["loglik"] for c in clips}) == 2          # distinct clips
    assert d["value"] == pytest.approx(2 * 3 / (d["ms_per_step"] * 3e-3), rel=1e-3)


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
