"""Secondary benchmarks of the §8 rows next to the headline (bench.py):

  --workload simm   Stereo_SIMM iterations/s at config 5 (F=2049, T=20000,
                    NF0=1092, P=30, K=4, R=40), SIMM.py:613-941
  --workload nmf    NMF_decomposition iterations/s at config 2 (F=1025,
                    T=2000, K=64), tools/nmf.py:34-59
  --workload cqt    MinQT front end (tftransforms/minqt.py:471-646, 1410-1450)
                    as FASST builds it at 44.1 kHz (transf='mqt', wlen 4096,
                    hop 512: FFTLen 8192, 5 octaves x 48 bins + 1980 linear
                    bins) on a signal of T = 10000 STFT frames (the C3 clip
                    length): forward and inverse transforms/s, device time
  --workload wf0    SIMM source dictionary generate_WF0_TR_chirped at config
                    5 (44.1 kHz, NFT 4096, 1092 KLGLOTT88 combs, STFT middle
                    frame): device time per dictionary
  --workload viterbi  melody tracking (_tracking.pyx:11-93) at config 5:
                    S = 1092 F0 states, N = 20000 frames (runViterbi's
                    transitions, stepNotes 16): tracks/s, device time

Inputs are synthetic and resident in HBM before the timed region; the timed
region is `steps` iterations of the update loop (simm_run / nmf_run, which
synchronise at the end).  Prints one JSON line.  Not part of the driver
contract; the headline metric is bench.py's.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

FP64_PEAK = 78.6e12


NO_CPU = False


def bench_simm(steps, warmup, F=2049, N=20000, NF0=1092, P=30, K=4, R=40, seed=0):
    from pyfasst_amd import _lib
    from pyfasst_amd.SeparateLeadStereo.SIMM.SIMM import _SimmContext, _c
    rs = np.random.RandomState(seed)
    SXR = rs.gamma(0.8, 1.0, size=(F, N))
    SXL = rs.gamma(0.8, 1.0, size=(F, N))
    WF0 = rs.gamma(1.0, 1.0, size=(F, NF0))
    WG = rs.gamma(1.0, 1.0, size=(F, P))
    HG, HPHI, HF0 = np.abs(rs.randn(P, K)), np.abs(rs.randn(K, N)), np.abs(rs.randn(NF0, N))
    HM, WM = np.abs(rs.randn(R, N)), np.abs(rs.randn(F, R))
    ctx = _SimmContext(F, N, NF0, P, K, R, True, _lib.default_device())
    _lib.check(_lib.lib.simm_set_data(ctx.ptr, _lib.dptr(SXR), _lib.dptr(SXL), _lib.dptr(WF0),
                                      _lib.dptr(WG)), "set_data")
    alpha, bR = np.array([.5, .5]), rs.rand(R)
    _lib.check(_lib.lib.simm_set_params(ctx.ptr, *[_lib.dptr(_c(a)) for a in
                                                   (HG, HPHI, HF0, HM, WM, alpha, bR)], None),
               "set_params")
    if warmup:
        _lib.check(_lib.lib.simm_run(ctx.ptr, warmup, 1.0, 1, None), "run")
    t0 = time.perf_counter()
    _lib.check(_lib.lib.simm_run(ctx.ptr, steps, 1.0, 1, None), "run")
    dt = time.perf_counter() - t0
    # GEMM flops per iteration: WF0^T{num,den} (2), SF0 recompute (1) on F x NF0 x N;
    # the R-sized products (HM: 4, WM: 4, beta: 4, SM refreshes: 2 x 3) on F x R x N
    flops = 2.0 * F * N * (3 * NF0 + 18 * R)
    achieved = flops / (dt / steps) / 1e12
    # CPU baseline: the oracle restatement (SIMM.py's operation order), ONE
    # iteration at the full size (all N frames: no scaling)
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import simm_ref
    n_cpu = N
    np.random.seed(1)
    t1 = time.perf_counter()
    if not NO_CPU:
        simm_ref.stereo_simm(SXR, SXL, WF0, WG, K, R, numberOfIterations=1)
    cpu_s = max(time.perf_counter() - t1, 1e-9)
    return {"metric": "Stereo_SIMM iterations/sec (config 5)", "value": round(steps / dt, 4),
            "unit": "SIMM it/s", "ms_per_step": round(dt / steps * 1e3, 3), "steps": steps,
            "warmup": warmup, "dtype": "f64", "data": "synthetic gamma spectrograms, RandomState(0)",
            "config": {"workload": "Stereo_SIMM F=%d N=%d NF0=%d P=%d K=%d R=%d" % (F, N, NF0, P, K, R)},
            "roofline": {"bound": "mfma", "achieved": round(achieved, 2), "peak": FP64_PEAK / 1e12,
                         "unit": "TFLOP/s", "frac": round(achieved * 1e12 / FP64_PEAK, 4),
                         "traffic": None, "scope": "whole iteration, GEMM flops 2FN(3 NF0 + 18 R)"},
            "gemm_tflops_per_s": round(achieved, 2),
            "cpu_baseline": {"value": round(1.0 / cpu_s, 5), "unit": "SIMM it/s", "cores": _blas_threads(),
                             "kind": "port", "sample": "oracle/simm_ref.py stereo_simm, 1 iteration "
                             "at the full size, %d frames (%.2f s)" % (n_cpu, cpu_s)},
            "reference_cpu": "14.27 s/iter = 0.070 it/s (BASELINE/SURVEY §6, measured on CPU)"}


def _blas_threads():
    try:
        from threadpoolctl import threadpool_info
        return int(max([p.get('num_threads', 1) for p in threadpool_info()] + [1]))
    except Exception:
        return 1


def bench_separate(steps, warmup):
    """Wiener separation + iSTFT at C3 (audioModel.py:1088-1233): the device-
    resident path (fasst_separate_waveforms, only the 8 waveforms cross PCIe)
    vs the images path (fasst_wiener_images: J x 2 x F x T complex images to
    the host, the per-image iSTFT after).  Host-inclusive wall times."""
    sys.path.insert(0, ROOT)
    import bench as B
    m = B.build_model(seed=0, device=0)
    eng = m._engine
    m._upload()
    nfft, hop = 4096, 512
    w = np.hanning(nfft)
    psd = np.full(m.nbFreqsSigRepr, 1e-6)
    for _ in range(max(warmup, 1)):
        eng.separate_waveforms(psd, w, w, nfft, hop)
    t0 = time.perf_counter()
    for _ in range(steps):
        Y = eng.separate_waveforms(psd, w, w, nfft, hop)
    dt = (time.perf_counter() - t0) / steps
    eng.wiener_images(psd)
    t1 = time.perf_counter()
    for _ in range(steps):
        S = eng.wiener_images(psd)
    di = (time.perf_counter() - t1) / steps
    J = Y.shape[0]
    # front end as FASST runs it (comp_transf_Cx, audioModel.py:250-302):
    # fasst_set_audio uploads the 2-channel signal, STFTs it on the device and
    # builds Cx there (the channel STFTs stay resident for the separation)
    L = hop * (m.nbFramesSigRepr - 2)
    x = np.random.RandomState(0).randn(L, 2)
    eng.set_audio(x, w, nfft, hop)
    t2 = time.perf_counter()
    for _ in range(steps):
        eng.set_audio(x, w, nfft, hop)
    ds = (time.perf_counter() - t2) / steps
    return {"metric": "FASST separation (Wiener images + iSTFT) per clip, host-inclusive",
            "value": round(dt * 1e3, 3), "unit": "ms", "higher_is_better": False,
            "steps": steps, "warmup": warmup, "dtype": "f64",
            "data": "synthetic C3 model (bench.py build_model, seed 0)",
            "config": {"workload": "J=%d sources x 2 channels, F=%d, T=%d, nfft %d hop %d"
                                   % (J, m.nbFreqsSigRepr, m.nbFramesSigRepr, nfft, hop)},
            "waveform_bytes_to_host": int(Y.nbytes),
            "images_path_ms": round(di * 1e3, 3), "image_bytes_to_host": int(S.nbytes),
            "front_end_ms": round(ds * 1e3, 3), "front_end": "fasst_set_audio: %d x 2 samples -> "
            "resident STFTs + Cx, host-inclusive" % L}


def bench_nmf(steps, warmup, F=1025, N=2000, K=64, seed=0):
    from pyfasst_amd import _lib
    from pyfasst_amd.tools.nmf import _NmfContext
    rs = np.random.RandomState(seed)
    SX = rs.gamma(0.7, 1.0, size=(F, N))
    W = rs.randn(F, K) ** 2
    H = rs.randn(K, N) ** 2
    W /= W.sum(axis=0)
    ctx = _NmfContext(F, N, K, _lib.default_device())
    _lib.check(_lib.lib.nmf_set_data(ctx.ptr, _lib.dptr(SX)), "set_data")
    _lib.check(_lib.lib.nmf_set_params(ctx.ptr, _lib.dptr(W), _lib.dptr(H)), "set_params")
    if warmup:
        _lib.check(_lib.lib.nmf_run(ctx.ptr, warmup, 1, 1), "run")
    t0 = time.perf_counter()
    _lib.check(_lib.lib.nmf_run(ctx.ptr, steps, 1, 1), "run")
    dt = time.perf_counter() - t0
    flops = 2.0 * F * N * K * 6
    achieved = flops / (dt / steps) / 1e12
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import fasst_ref
    n_cpu = 20
    t1 = time.perf_counter()
    if not NO_CPU:
        fasst_ref.nmf_decomp_init(SX, nbComps=K, niter=n_cpu, Winit=W.copy(), Hinit=H.copy())
    cpu_s = max((time.perf_counter() - t1) / n_cpu, 1e-9)
    return {"metric": "NMF_decomposition iterations/sec (config 2)", "value": round(steps / dt, 3),
            "unit": "NMF it/s", "ms_per_step": round(dt / steps * 1e3, 4), "steps": steps,
            "warmup": warmup, "dtype": "f64", "data": "synthetic gamma spectrogram, RandomState(0)",
            "config": {"workload": "IS-NMF F=%d T=%d K=%d" % (F, N, K)},
            "roofline": {"bound": "mfma", "achieved": round(achieved, 2), "peak": FP64_PEAK / 1e12,
                         "unit": "TFLOP/s", "frac": round(achieved * 1e12 / FP64_PEAK, 4),
                         "traffic": None, "scope": "whole iteration, GEMM flops 12FTK"},
            "gemm_tflops_per_s": round(achieved, 2),
            "cpu_baseline": {"value": round(1.0 / cpu_s, 3), "unit": "NMF it/s", "cores": _blas_threads(),
                             "kind": "port", "sample": "oracle/fasst_ref.py nmf_decomp_init, %d "
                             "iterations at the full size" % n_cpu},
            "reference_cpu": "0.0318 s/iter = 31.4 it/s (SURVEY §6, measured on CPU)"}


def bench_cqt(steps, warmup, fs=44100, wlen=4096, hop=512, T=10000, seed=0):
    from pyfasst_amd import _lib
    from pyfasst_amd.tftransforms import minqt
    L = hop * (T - 2)
    rs = np.random.RandomState(seed)
    x = rs.randn(L) * (1 + np.sin(np.arange(L) / 7000.0))
    t = minqt.MinQTransfo(fmin=25, fmax=18000, bins=48, fs=fs, perfRast=1, linFTLen=wlen,
                          atomHopFactor=hop / float(wlen))
    fwd, inv = [], []
    for i in range(warmup + steps):
        t.computeTransform(x)
        sp = t.transfo
        y = t.invertTransform()
        f, b = ctypes.c_double(), ctypes.c_double()
        _lib.check(_lib.lib.cqt_device_ms(t._context(), ctypes.byref(f), ctypes.byref(b)), "ms")
        if i >= warmup:
            fwd.append(f.value)
            inv.append(b.value)
    k = t.cqtkernel
    fm, im = float(np.median(fwd)), float(np.median(inv))
    return {"metric": "MinQT forward transforms/sec (device time)", "value": round(1e3 / fm, 3),
            "unit": "transforms/s", "forward_ms": round(fm, 3), "inverse_ms": round(im, 3),
            "msamples_per_s_forward": round(L / fm / 1e3, 1), "steps": steps, "warmup": warmup,
            "dtype": "f64", "data": "synthetic modulated noise, RandomState(0)",
            "config": {"workload": "MinQT fs=%d linFTLen=%d hop=%d bins=48 fmin=25: %d samples "
                                   "(T=%d frames), spCQT %dx%d, FFTLen %d, %d octaves, "
                                   "kernel band %s" % (fs, wlen, hop, L, T, sp.shape[0],
                                                       sp.shape[1], int(k.FFTLen),
                                                       int(t.octaveNr), "n/a")},
            "roundtrip_rel_err": float(np.abs(y - x).max() / np.abs(x).max())}


def bench_wf0(steps, warmup):
    import tempfile
    from pyfasst_amd import _lib
    from pyfasst_amd.SeparateLeadStereo import separateLeadFunctions as slf
    from pyfasst_amd.tftransforms.stft import STFT
    from pyfasst_amd.tools.utils import sqrt_blackmanharris
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import dict_ref as D
    os.chdir(tempfile.mkdtemp())
    t = STFT(linFTLen=4096, atomHopFactor=0.25, winFunc=sqrt_blackmanharris, fs=44100)
    ms = []
    for i in range(warmup + steps):
        F0Table, WF0, _ = slf.generate_WF0_TR_chirped(t, 39, 2000, stepNotes=16, loadWF0=False)
        m = ctypes.c_double()
        _lib.lib.dict_last_ms(ctypes.byref(m))
        if i >= warmup:
            ms.append(m.value)
    dm = float(np.median(ms))
    ab = ctypes.c_int()
    _lib.lib.viterbi_fallback_count(ctypes.byref(ab))
    # CPU: the oracle (the reference's outer-product synthesis) on 8 of the 1092 F0s
    idx = np.linspace(0, F0Table.size - 1, 8).astype(int)
    t0 = time.perf_counter()
    for i in idx:
        D.stft_mid_frame_power(D.generate_odgd(F0Table[i], 44100, lengthOdgd=8192), t.window,
                               t.fthop, 4096, 44100)
    cpu_s = (time.perf_counter() - t0) / idx.size * F0Table.size
    partials = sum(int(np.floor(22050.0 / f)) for f in F0Table)
    return {"metric": "SIMM WF0 dictionaries/sec (config 5, device time)",
            "value": round(1e3 / dm, 3), "unit": "dictionaries/s", "device_ms": round(dm, 3),
            "steps": steps, "warmup": warmup, "dtype": "f64",
            "config": {"workload": "generate_WF0_TR_chirped STFT NFT=4096 fs=44100 minF0=39 "
                                   "maxF0=2000 stepNotes=16: %d combs, %d partials, 4096-sample "
                                   "frames" % (F0Table.size, partials)},
            "partial_samples_per_s": round(partials * 4096 / (dm * 1e-3) / 1e9, 2),
            "cpu_baseline": {"value": round(1.0 / cpu_s, 5), "unit": "dictionaries/s",
                             "cores": 1, "kind": "port",
                             "sample": "oracle/dict_ref.py on 8 of the %d F0s, scaled"
                                       % F0Table.size}}


def bench_nnls(steps, warmup, frames=1000, seed=0):
    """initHF00='nnls' on one pipeline chunk at config-5 scale: the C5 STFT
    dictionary (1092 combs, F=2049) and 1000 frames of synthetic spectra
    (a few combs + noise), one batched GPU solve per step; the CPU baseline
    is scipy.optimize.nnls (the reference's call) on a sample of frames."""
    import tempfile
    from pyfasst_amd.SeparateLeadStereo import separateLeadFunctions as slf
    from pyfasst_amd.tftransforms.stft import STFT
    from pyfasst_amd.tools.nnls import nnls_columns
    from pyfasst_amd.tools.utils import sqrt_blackmanharris
    os.chdir(tempfile.mkdtemp())
    t = STFT(linFTLen=4096, atomHopFactor=0.25, winFunc=sqrt_blackmanharris, fs=44100)
    F0Table, WF0, _ = slf.generate_WF0_TR_chirped(t, 39, 2000, stepNotes=16, loadWF0=False)
    rs = np.random.RandomState(seed)
    F, n = WF0.shape
    H = np.zeros((n, frames))
    for q in range(frames):
        H[rs.choice(n, 4, replace=False), q] = rs.rand(4)
    SX = WF0.dot(H) + 1e-3 * WF0.max() * rs.rand(F, frames)
    ms = []
    for i in range(warmup + steps):
        t0 = time.perf_counter()
        X = nnls_columns(WF0, SX)
        if i >= warmup:
            ms.append((time.perf_counter() - t0) * 1e3)
    dm = float(np.median(ms))
    out = {"metric": "NNLS frames/sec (initHF00='nnls', one 1000-frame chunk, host-inclusive)",
           "value": round(frames / (dm * 1e-3), 2), "unit": "frames/s", "ms_per_chunk": round(dm, 2),
           "steps": steps, "warmup": warmup, "dtype": "f64",
           "config": {"workload": "nnls(WF0 %d x %d, 1000 frames)" % (F, n)},
           "active_mean": round(float(np.mean(np.sum(X > 0, axis=0))), 1)}
    if not NO_CPU:
        from scipy.optimize import nnls
        t0 = time.perf_counter()
        k = 4
        ref = [nnls(WF0, SX[:, q])[0] for q in range(k)]
        cpu = (time.perf_counter() - t0) / k
        out["vs_scipy"] = {"max_rel": float(max(np.max(np.abs(X[:, q] - ref[q])) /
                                              max(np.max(np.abs(ref[q])), 1e-300)
                                              for q in range(k))),
                           "same_support": bool(all(np.array_equal(X[:, q] > 0, ref[q] > 0)
                                                    for q in range(k)))}
        out["cpu_baseline"] = {"value": round(1.0 / cpu, 3), "unit": "frames/s", "cores": 1,
                               "kind": "reference",
                               "sample": "scipy.optimize.nnls (the reference's call) on 4 frames"}
    return out


def bench_viterbi(steps, warmup, S=1092, N=20000, seed=0):
    from pyfasst_amd import _lib
    from pyfasst_amd.SeparateLeadStereo.tracking._tracking import viterbiTracking
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import viterbi_ref as V
    rs = np.random.RandomState(seed)
    logD = np.log(rs.gamma(0.3, 1.0, size=(S + 1, N)))
    logT, prior = V.melody_transitions(S, 16)
    ms = []
    for i in range(warmup + steps):
        viterbiTracking(S, N, logD, prior, logT)
        m, k = ctypes.c_double(), ctypes.c_int()
        _lib.lib.viterbi_last_timing(ctypes.byref(m), ctypes.byref(k))
        if i >= warmup:
            ms.append(m.value)
    dm = float(np.median(ms))
    ab = ctypes.c_int()
    _lib.lib.viterbi_fallback_count(ctypes.byref(ab))
    # CPU: the oracle restatement of the pyx recursion on a bounded sample
    n_cpu = 40
    t0 = time.perf_counter()
    V.viterbi_tracking(S, n_cpu, logD, prior, logT)
    cpu_s = (time.perf_counter() - t0) / (n_cpu - 1) * (N - 1)
    return {"metric": "Viterbi melody tracks/sec (config 5 size, device time)",
            "value": round(1e3 / dm, 3), "unit": "tracks/s", "device_ms": round(dm, 2),
            "us_per_frame": round(dm * 1e3 / N, 3), "steps": steps, "warmup": warmup,
            "dtype": "f64", "data": "synthetic log-gamma densities, RandomState(0)",
            "config": {"workload": "viterbiTracking S=%d N=%d (max-plus S^2 per frame)" % (S, N)},
            "maxplus_gops": round(float(S) * S * (N - 1) / (dm * 1e-3) / 1e9, 1),
            # persistent launches rerun on the per-frame path (results taken
            # on the slower fallback are identifiable)
            "path_kind": k.value, "persistent_aborts": ab.value,
            "cpu_baseline": {"value": round(1.0 / cpu_s, 5), "unit": "tracks/s", "cores": 1,
                             "kind": "port", "sample": "oracle/viterbi_ref.py, %d frames, "
                             "scaled to N=%d" % (n_cpu, N)}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", choices=("simm", "nmf", "cqt", "viterbi", "wf0", "separate",
                                           "nnls"),
                    required=True)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--no-cpu-baseline", action="store_true",
                    help="skip the CPU baseline (profiling passes)")
    a = ap.parse_args()
    global NO_CPU
    NO_CPU = a.no_cpu_baseline
    fn = {"simm": bench_simm, "nmf": bench_nmf, "cqt": bench_cqt, "viterbi": bench_viterbi,
          "wf0": bench_wf0, "separate": bench_separate, "nnls": bench_nnls}[a.workload]
    out = fn(a.steps, a.warmup)
    if NO_CPU:
        out["cpu_baseline"] = None   # not measured (the sample above timed nothing)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
