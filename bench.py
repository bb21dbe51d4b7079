"""bench.py -- EM iterations/sec of the FASST GEM loop on MI355X.

Workload (BASELINE.json configs[2] / [3]): synthetic stereo STFT-domain clip,
F=2049 bins x T=10000 frames, J=4 convolutive sources of spatial rank 2,
K=32 NMF components (MultiChanNMFConv + makeItConvolutive).  One clip per
GPU (config 4 = 8 independent clips): weak scaling, no collective in the
data path; torch.distributed (RCCL when every rank has its own GPU, gloo
when ranks share one) provides the start/stop barrier, the max-over-ranks
time and the final allgather of the per-clip logliks / times.

`python bench.py --gpus N` with no WORLD_SIZE in the environment starts the
N ranks itself (launch_local: one worker process per GPU, started before
anything in the parent touches a GPU); under torchrun WORLD_SIZE must equal
N.

A "step" is one GEM iteration (audioModel.py:384-428) on the GPU, inputs
resident in HBM.  Prints ONE JSON line on rank 0.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu-baseline] [--dry-run]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

F_BINS, T_FRAMES, J_SRC, RANK, K_NMF = 2049, 10000, 4, 2, 32
FP64_MFMA_PEAK = 78.6e12   # MI355X dense FP64 matrix, FLOP/s (spec)
FP64_VALU_PEAK = 78.6e12   # MI355X FP64 vector, FLOP/s (spec)
HBM_PEAK = 8.0e12          # B/s (spec)


def kernel_work(F, T, J, R, K):
    """ALGORITHMIC FLOPs / bytes per launch of the GEM-iteration kernels
    (SURVEY.md §8(d) accounting: every quantity counted once per iteration,
    however often a kernel chooses to recompute it; `exec_flops` is what the
    kernel actually issues, for reference only).

    k_estep:       the single-pass E-step: V tiles 2JK (the only algorithmic V
                   before the E-step), Sigma_x 8J, the guarded 2x2 inverse,
                   loglik, P and N ~70, the cross and pair statistics
                   2 (8J + 4 J(J+1)/2), hat_W ~8J per (f,t); bytes 32 (Cx
                   read) + 8J (rho write) per (f,t)
    k_estep_part1 / k_estep_part2: the round-1 two-pass E-step (A/B only,
                   FASST_ESTEP_SPLIT=1); part 2's V tiles are a recompute
    k_fb_contract: FB numerator 2K per (f,t,j); bytes 8 (rho) per (f,t,j)
    k_tw_contract: V after the FB update 2K + TW numerator 2K + denominator
                   2K per (f,t,j) (its V_old tiles are a recompute); bytes 8
                   (rho re-read, counted in B_alg as hat_W's re-read) per (f,t,j)
    """
    ft = float(F) * T
    np_ = J * (J + 1) / 2
    estep = ft * (2 * J * K + 8 * J + 70 + 2 * (8 * J + 4 * np_) + 8 * J)
    return {
        "k_estep": dict(flops=estep, exec_flops=estep, bytes=ft * (32 + 8 * J)),
        "k_estep_part1": dict(flops=ft * (2 * J * K + 8 * J + 70 + 9 * np_),
                              exec_flops=ft * (2 * J * K + 8 * J + 70 + 9 * np_),
                              bytes=ft * (32 + 8 * J)),
        "k_estep_part2": dict(flops=ft * (17 * J + 10 * R),
                              exec_flops=ft * (2 * J * K + 17 * J + 10 * R), bytes=0.0),
        "k_fb_contract": dict(flops=ft * J * 2 * K, exec_flops=ft * J * 2 * K, bytes=ft * J * 8),
        "k_tw_contract": dict(flops=ft * J * 6 * K, exec_flops=ft * J * 8 * K, bytes=ft * J * 8),
    }


def iteration_work(F, T, J, R, K):
    """per GEM iteration, B_alg = 8 F T (4 + 2J) bytes,
    F_mfma = 10 J F K T, F_valu = F T (8 R^2 + 40 R); t_ideal = max(B_alg / BW,
    F_mfma / P_mfma + F_valu / P_valu)."""
    ft = float(F) * T
    b_alg = 8.0 * ft * (4 + 2 * J)
    f_mfma = 10.0 * J * K * ft
    f_valu = ft * (8 * R * R + 40 * R)
    t_ideal = max(b_alg / HBM_PEAK, f_mfma / FP64_MFMA_PEAK + f_valu / FP64_VALU_PEAK)
    return dict(B_alg=b_alg, F_mfma=f_mfma, F_valu=f_valu, t_ideal_s=t_ideal)


# the kernels one GEM iteration launches (each once), for the PMC traffic sum
ITERATION_KERNELS = ("k_w_from_fb", "k_fwh_t", "k_tw_rowsum", "k_inst_A", "k_estep_part1",
                     "k_estep_part2", "k_estep", "k_loglik", "k_mix", "k_mix_inst",
                     "k_fb_contract", "k_fb_update", "k_tw_contract", "k_tw_contract_lds",
                     "k_tw_update",
                     "k_renorm_stats", "k_renorm_apply", "k_renorm_final", "k_renorm_scales",
                     "k_renorm_rows", "k_renorm_tail")


def pmc_bytes(pmc, k):
    """HBM bytes per launch of kernel k in a summarize_prof.py record (the
    single-component TW contraction is profiled as k_tw_contract_lds)."""
    for name in (k, k + "_lds"):
        if pmc and name in pmc and pmc[name].get("hbm_bytes_per_launch"):
            return pmc[name]["hbm_bytes_per_launch"]
    return None


PROF_STEPS = 64   # iterations of the per-kernel timing pass (two event rings)


def pmc_file(J, K, T, rounds=range(9, 0, -1)):
    """The newest committed rocprofv3 FETCH / WRITE summary of THIS
    configuration (tools/gpu_prof.sh + tools/summarize_prof.py):
    profiles/rN_bench.json for the headline, rN_bench_J<J>K<K>.json for a
    structure variant; None if there is none."""
    if T != T_FRAMES:
        return None
    default_cfg = (J, K) == (J_SRC, K_NMF)
    for r in rounds:
        name = "r%d_bench.json" % r if default_cfg else "r%d_bench_J%dK%d.json" % (r, J, K)
        p = os.path.join(ROOT, "profiles", name)
        if os.path.exists(p):
            return p
    return None


def build_model(seed, device, T=T_FRAMES, J=J_SRC, K=K_NMF):
    import pyfasst_amd.audioModel as am
    from pyfasst_amd import synthetic
    from pyfasst_amd.audioObject import SpectralAudio
    X = synthetic.stereo_mixture(F_BINS, T, J=J, K_true=8, rank=RANK, seed=seed)
    np.random.seed(1)
    m = am.MultiChanNMFConv(SpectralAudio(X=X), nbComps=J, nbNMFComps=K,
                            spatial_rank=RANK, iter_num=1, wlen=4096, hopsize=512,
                            device=device)
    m.makeItConvolutive()
    return m


def psd_schedule(m, n):
    N = m.iter_num = max(n, 1)
    return np.array([m._annealed_psd(i % N) for i in range(n)])


def cpu_baseline(T_sample=T_FRAMES):
    """The oracle (NumPy restatement keeping the reference's operation
    structure: the R x R pair loop over full F x T arrays, per-bin Python
    loops) timed for ONE GEM iteration of the same C3 workload, at the full
    T = 10000 by default (the reference's 5.2 GB temporaries do not scale
    linearly from a smaller sample).  Also reports the restatement / reference
    time ratio measured in the build container (profiles/r2_cpu_ratio.json)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import fasst_ref as R
    from pyfasst_amd import synthetic
    X = synthetic.stereo_mixture(F_BINS, T_sample, J=J_SRC, K_true=8, rank=RANK, seed=0)
    o = R.RefFASST(iter_num=1)
    o.set_transform([X[0], X[1]])
    del X
    np.random.seed(1)
    R.init_nmf_inst(o, J_SRC, K_NMF, RANK)
    R.make_convolutive(o)
    o.noise['PSD'] = o.annealed_psd(0)
    t0 = time.perf_counter()
    o.GEM_iteration()
    dt = time.perf_counter() - t0
    try:
        from threadpoolctl import threadpool_info
        info = threadpool_info()
        cores = max([p.get('num_threads', 1) for p in info] + [1])
        blas = ",".join(sorted(set("%s %s" % (p.get('internal_api'), p.get('version'))
                                   for p in info)))
    except Exception:
        cores, blas = 1, "unknown"
    scale = T_FRAMES / float(T_sample)
    out = {"value": 1.0 / (dt * scale), "unit": "EM it/s", "cores": int(cores), "kind": "port",
           "sample": "oracle/fasst_ref.py, 1 GEM iteration at F=%d T=%d J=%d r=%d K=%d: %.2f s%s; "
                     "BLAS %s with %d threads, elementwise NumPy single-threaded"
                     % (F_BINS, T_sample, J_SRC, RANK, K_NMF, dt,
                        "" if scale == 1 else " (scaled x%.1f to T=%d)" % (scale, T_FRAMES),
                        blas, cores)}
    rp = os.path.join(ROOT, "profiles", "r2_cpu_ratio.json")
    if os.path.exists(rp):
        r = json.load(open(rp))
        out["oracle_over_reference_time"] = r.get("ratio")
        out["ratio_source"] = os.path.relpath(rp, ROOT)
    return out


def rank_setup(env=None, ndev=None):
    """(world, rank, local_rank, data_seed, device) of this process: one clip per
    GPU, data seed = global rank, device = local rank (torchrun env vars).  With
    fewer visible GPUs than local ranks (the one-GPU rehearsal box) the ranks
    share the cards round-robin."""
    env = os.environ if env is None else env
    world = int(env.get("WORLD_SIZE", "1"))
    rank = int(env.get("RANK", "0"))
    local = int(env.get("LOCAL_RANK", "0"))
    device = local if not ndev else local % ndev
    return world, rank, local, rank, device


def choose_backend(world, ndev, env=None):
    """Control-plane backend: RCCL ('nccl') when every rank has a GPU of its
    own, as north_star names it; gloo when ranks share a card (RCCL refuses two
    ranks on one device).  FASST_BENCH_BACKEND overrides; forcing nccl onto
    shared cards is refused."""
    env = os.environ if env is None else env
    forced = env.get("FASST_BENCH_BACKEND")
    if forced:
        if forced == "nccl" and ndev < world:
            raise SystemExit("bench.py: FASST_BENCH_BACKEND=nccl needs one GPU per rank "
                             "(%d ranks, %d GPUs)" % (world, ndev))
        return forced
    return "nccl" if ndev >= world else "gloo"


def launch_local(n, argv, env=None):
    """`python bench.py --gpus N` without a launcher: start N worker processes
    of this script, one per GPU (RANK = LOCAL_RANK = i, WORLD_SIZE = N, a
    rendezvous on 127.0.0.1), before anything in this process touches a GPU;
    rank 0's stdout (the JSON line) passes through.  A failing worker stops
    the others (by their own handles).  Returns the job's exit code."""
    import signal
    import socket
    import subprocess
    env = dict(os.environ if env is None else env)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        e = dict(env, WORLD_SIZE=str(n), RANK=str(r), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE=str(n),
                 MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv),
                                      env=e, stdout=None if r == 0 else subprocess.DEVNULL))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                for q in live:
                    q.send_signal(signal.SIGTERM)
        if live:
            time.sleep(0.05)
    return rc if rc >= 0 else 128 - rc


def max_over_ranks(dt, dist=None, device="cpu"):
    """Wall time of the slowest rank (the whole job's time)."""
    if dist is None:
        return dt
    import torch
    t = torch.tensor([dt], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_clips(rec, dist=None, device="cpu"):
    """SURVEY.md §8(e)1's final allgather: every rank's (rank, data seed,
    device, last loglik, own timed seconds) -> list over ranks."""
    if dist is None:
        return [list(rec)]
    import torch
    t = torch.tensor(rec, dtype=torch.float64, device=device)
    out = [torch.zeros_like(t) for _ in range(dist.get_world_size())]
    dist.all_gather(out, t)
    return [o.cpu().tolist() for o in out]


def check_clips(clips):
    """Distinct ranks must have run distinct clips (distinct data seeds and
    logliks); raises otherwise."""
    ranks = [int(c[0]) for c in clips]
    seeds = [int(c[1]) for c in clips]
    lls = [c[3] for c in clips]
    if sorted(ranks) != list(range(len(clips))):
        raise RuntimeError("clip records from ranks %s" % ranks)
    if len(set(seeds)) != len(seeds) or len(set(lls)) != len(lls):
        raise RuntimeError("ranks did not run distinct clips: seeds %s, logliks %s" % (seeds, lls))


def dry_run(args, world, rank, seed):
    """--dry-run: the multi-rank control plane of main() on the CPU (gloo),
    around a host stand-in for one clip (the mean log power of a small
    synthetic mixture drawn from the rank's data seed); rank 0 prints the
    JSON line."""
    import torch.distributed as dist
    from pyfasst_amd import synthetic
    dist.init_process_group("gloo")
    dist.barrier()
    t0 = time.perf_counter()
    X = synthetic.stereo_mixture(65, 32 * max(args.steps, 1), J=2, K_true=2, rank=2, seed=seed)
    ll = float(np.mean(np.log(np.abs(X) ** 2 + 1e-300)))
    dist.barrier()
    dt_own = time.perf_counter() - t0
    dt = max_over_ranks(dt_own, dist, "cpu")
    clips = gather_clips([rank, seed, -1, ll, dt_own], dist, "cpu")
    check_clips(clips)
    if rank == 0:
        print(json.dumps({"metric": "dry run (control plane only)", "value": job_value(world, args.steps, dt),
                          "n_gpus": world, "steps": args.steps, "control_plane": "gloo",
                          "ms_per_step": dt / max(args.steps, 1) * 1e3,
                          "clips": [{"rank": int(c[0]), "data_seed": int(c[1]), "loglik": c[3]}
                                    for c in clips]}), flush=True)
    dist.destroy_process_group()
    return 0


def job_value(world, steps, dt_max):
    """Whole-job throughput: iterations of all clips / slowest rank's time."""
    return world * steps / dt_max


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--warm-s", type=float, default=1.0,
                    help="untimed GEM iterations for at least this long before the W warm-up "
                         "steps (the GPU clock ramps over the first ~20 iterations)")
    ap.add_argument("--T", type=int, default=T_FRAMES)
    # structure variants (the headline is J=4, K=32): the J > 4 E-step runs
    # at one wave per SIMD, K up to 64 per source on the HIP path
    ap.add_argument("--J", type=int, default=J_SRC)
    ap.add_argument("--K", type=int, default=K_NMF)
    ap.add_argument("--cpu-T", type=int, default=T_FRAMES,
                    help="frames of the CPU-baseline sample (default: the full T)")
    ap.add_argument("--dry-run", action="store_true",
                    help="control plane only, on the CPU: launcher, gloo barrier, max-over-ranks "
                         "and the clips' allgather around a tiny host stand-in for the clip "
                         "(tests/test_distributed.py); no GPU is touched")
    args = ap.parse_args(argv)

    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        # no launcher: this process only starts the ranks (no GPU call here)
        return launch_local(args.gpus, sys.argv[1:] if argv is None else argv)
    if env_world is not None and int(env_world) != args.gpus:
        sys.stderr.write("bench.py: WORLD_SIZE=%s but --gpus %d\n" % (env_world, args.gpus))
        return 2

    import torch
    ndev = 0 if args.dry_run else torch.cuda.device_count()   # does not initialise the GPU
    world, rank, local, seed, device = rank_setup(ndev=ndev)
    if args.dry_run:
        return dry_run(args, world, rank, seed)
    dist = None
    backend = None
    # control plane only (start/stop barrier, max-over-ranks time, the clips'
    # allgather): RCCL when each rank has its own GPU (choose_backend).
    # FASST_BENCH_DIST=1 initialises the process group even for one rank (the
    # barrier / max-over-ranks path exercised on a one-GPU box)
    if world > 1 or os.environ.get("FASST_BENCH_DIST") == "1":
        import torch.distributed as dist
        backend = choose_backend(world, ndev)
        torch.cuda.set_device(device)
        if backend == "nccl":
            # eager communicator (device_id), then one barrier: RCCL's setup
            # finishes before the engine exists and long before the timed loop
            dist.init_process_group(backend, device_id=torch.device("cuda", device))
        else:
            dist.init_process_group(backend)
        dist.barrier()
    coll_dev = "cuda:%d" % device if backend == "nccl" else "cpu"

    m = build_model(seed=seed, device=device, T=args.T, J=args.J, K=args.K)
    eng = m._engine
    order, Ks, conv = m._upload()
    rows_w = psd_schedule(m, max(args.warmup, 1))
    state = {"upl": (order, Ks, conv)}

    def run_rows(rows):
        """GEM iterations over the PSD rows; a random TW restart (host RNG)
        is performed and the run resumed, as the product does.  Returns the
        last iteration's loglik."""
        done, last = 0, float("nan")
        while done < len(rows):
            ll, n, mask = eng.run(rows[done:], m.nmfUpdateCoeff)
            done += n
            if n:
                last = float(ll[n - 1])
            if mask:
                m._download(*state["upl"])
                m._restart_tw(mask, state["upl"][0])
                state["upl"] = m._upload()
        return last

    # clock ramp: the first ~20 iterations of a process run while the GPU
    # clock rises (tools/ramp_probe.py); iterate untimed until it has settled,
    # so that the K timed steps measure the steady state
    if args.warm_s > 0:
        rows_r = psd_schedule(m, 10)
        t_w = time.perf_counter()
        while time.perf_counter() - t_w < args.warm_s:
            run_rows(rows_r)
    if args.warmup:
        run_rows(rows_w[:args.warmup])

    def barrier_sync():
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()
            torch.cuda.synchronize()

    rows = psd_schedule(m, args.steps)
    barrier_sync()
    t0 = time.perf_counter()
    ll_last = run_rows(rows)
    barrier_sync()
    dt_own = time.perf_counter() - t0
    dt = max_over_ranks(dt_own, dist, coll_dev)
    clips = gather_clips([rank, seed, device, ll_last, dt_own], dist, coll_dev)
    if world > 1:
        check_clips(clips)

    # per-kernel HIP-event timing in the timed loop's own schedule (separate,
    # untimed pass): the side stream stays forked, each kernel's events sit
    # on the stream it runs on, and the host syncs once per 32 iterations
    eng.set_profiling(True)
    run_rows(psd_schedule(m, PROF_STEPS))
    times = eng.kernel_times()
    eng.set_profiling(False)

    if rank == 0:
        R = sum(m.rank)
        F, T = m.nbFreqsSigRepr, m.nbFramesSigRepr
        work = kernel_work(F, T, args.J, R, args.K)
        itw = iteration_work(F, T, args.J, R, args.K)
        dom = max(times, key=lambda k: times[k][0])
        rl = None
        pmc = None
        # PMC traffic of THIS configuration's own rocprofv3 passes
        # (tools/gpu_prof.sh; BENCH_ARGS="--J 8" -> profiles/r4_bench_J8K32.json)
        pmc_path = os.environ.get("FASST_PMC_JSON") or pmc_file(args.J, args.K, args.T) or ""
        if os.path.exists(pmc_path):
            try:
                pmc = json.load(open(pmc_path))["kernels"]
            except Exception:
                pmc = None
        step_s = dt / args.steps
        iter_traffic = None
        if pmc:
            # each kernel weighted by its launches per E-step launch (k_fwh_t /
            # k_tw_rowsum run only where k_tw_update's prep does not)
            n_it = pmc.get("k_estep", {}).get("calls") or None
            tot = [pmc[k]["hbm_bytes_per_launch"] *
                   (min(1.0, pmc[k]["calls"] / n_it) if n_it and pmc[k].get("calls") else 1.0)
                   for k in ITERATION_KERNELS
                   if k in pmc and pmc[k].get("hbm_bytes_per_launch")]
            iter_traffic = float(sum(tot)) if tot else None
        if dom in work:
            sec = times[dom][0] * 1e-3
            achieved = work[dom]["flops"] / sec / 1e12
            traffic = pmc_bytes(pmc, dom)
            # the binding roofline of the kernel: HBM when its algorithmic
            # bytes take longer at HBM_PEAK than its flops at the FP64 MFMA peak
            hbm_bound = work[dom]["bytes"] / HBM_PEAK > work[dom]["flops"] / FP64_MFMA_PEAK
            if hbm_bound:
                achieved = work[dom]["bytes"] / sec / 1e9
                rl = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK / 1e9,
                      "unit": "GB/s", "frac": round(achieved * 1e9 / HBM_PEAK, 4),
                      "tflops": round(work[dom]["flops"] / sec / 1e12, 3)}
            else:
                rl = {"bound": "mfma", "achieved": round(achieved, 3),
                      "peak": FP64_MFMA_PEAK / 1e12, "unit": "TFLOP/s",
                      "frac": round(achieved * 1e12 / FP64_MFMA_PEAK, 4)}
            rl.update({
                  "traffic": traffic, "kernel": dom, "kernel_ms": round(times[dom][0], 4),
                  "dtype": "f64", "algorithmic_flops": work[dom]["flops"],
                  "executed_flops": work[dom]["exec_flops"],
                  "executed_tflops": round(work[dom]["exec_flops"] / sec / 1e12, 3),
                  "algorithmic_bytes": work[dom]["bytes"],
                  "traffic_source": os.path.relpath(pmc_path, ROOT) if traffic else None,
                  # whole GEM iteration against SURVEY.md §8(d)'s ideal time
                  "iteration": {
                      "t_ideal_ms": round(itw["t_ideal_s"] * 1e3, 4),
                      "t_measured_ms": round(step_s * 1e3, 4),
                      "frac": round(itw["t_ideal_s"] / step_s, 4),
                      "B_alg": itw["B_alg"], "F_mfma": itw["F_mfma"], "F_valu": itw["F_valu"],
                      "traffic": iter_traffic,
                      "traffic_ratio": round(iter_traffic / itw["B_alg"], 3) if iter_traffic
                      else None}})
        if rl is not None:
            # every timed kernel of the iteration on its algorithmic work (the
            # dominant one above; the TW contraction is the kernel VERDICT names)
            rl["kernels"] = {
                k: {"ms": round(times[k][0], 4),
                    "tflops": round(work[k]["flops"] / (times[k][0] * 1e-3) / 1e12, 3),
                    "frac": round(work[k]["flops"] / (times[k][0] * 1e-3) / FP64_MFMA_PEAK, 4),
                    "gbps": round(work[k]["bytes"] / (times[k][0] * 1e-3) / 1e9, 1),
                    "hbm_frac": round(work[k]["bytes"] / (times[k][0] * 1e-3) / HBM_PEAK, 4),
                    "bound": "hbm" if work[k]["bytes"] / HBM_PEAK
                    > work[k]["flops"] / FP64_MFMA_PEAK else "mfma",
                    "traffic": pmc_bytes(pmc, k)}
                for k in ("k_estep", "k_tw_contract", "k_fb_contract") if k in times and k in work}
        out = {
            "metric": "EM iterations/sec (F=2049, T=10000, 2ch, 4src) at 1/2/4/8 MI355X",
            "value": round(job_value(world, args.steps, dt), 4),
            "unit": "EM it/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (STFT-domain stereo NMF mixture, RandomState(rank); init seed 1)",
            "config": {"workload": "C3/C4: MultiChanNMFConv GEM, F=%d T=%d J=%d spatial_rank=%d "
                                   "K=%d, one clip per GPU" % (m.nbFreqsSigRepr, m.nbFramesSigRepr,
                                                              args.J, RANK, args.K),
                       "parallelism": "clip-per-GPU x%d" % world},
            "control_plane": backend or "none (one process)",
            "clips": [{"rank": int(c[0]), "data_seed": int(c[1]), "device": int(c[2]),
                       "loglik": c[3], "timed_s": round(c[4], 6)} for c in clips],
            "roofline": rl,
            "kernels_ms": {k: round(v[0], 4) for k, v in sorted(times.items())},
            "kernels_schedule": "in situ: %d iterations, side stream forked, HIP events on each "
                                "kernel's own stream, one host sync per 32 iterations" % PROF_STEPS,
        }
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(args.cpu_T)
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
