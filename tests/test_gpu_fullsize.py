"""BASELINE-size parity on the MI355X: the HIP path at the configurations the
bench is quoted on, against the oracle's outputs on identical seeded inputs.

The fixtures (tests/golden/{c3_full,c3_t1000,c1_50,c5_full}.npz) are written
by tests/golden/make_fullsize.py, which runs oracle/fasst_ref.py and
oracle/simm_ref.py at these sizes in the build container (the oracle is
pinned bit-exactly to the reference on the small golden cases); the box
regenerates the seeded inputs (pyfasst_amd/synthetic.py).  Outputs are
compared on the fixture's subsample (every 7th bin, ~40 frames) and through
full-array sums.

Tolerances: 1e-8 relative (max-normalised) after 1-3 iterations; the C1-shaped
50-iteration run holds the north-star bar, 1e-4 relative on the separated
magnitude spectrograms, and reports the drift it actually shows (SURVEY.md §7
measured 7.4e-5 for a 1e-7 input perturbation after 50 iterations).
"""
import threading

import numpy as np
import pytest

from helpers import FULL_CASES, load, rel, rel_elem, sub_f, sub_t

pytestmark = pytest.mark.gpu

BAR = 1e-4


def _fasst_model(name, **over):
    import pyfasst_amd.audioModel as am
    from pyfasst_amd import synthetic
    from pyfasst_amd.audioObject import SpectralAudio
    c = dict(FULL_CASES[name], **over)
    X = synthetic.stereo_mixture(c["F"], c["T"], J=c["J"], K_true=c["K_true"],
                                 rank=c["data_rank"], seed=c["data_seed"])
    np.random.seed(c["init_seed"])
    cls = am.MultiChanNMFConv if c["conv"] else am.MultiChanNMFInst_FASST
    m = cls(SpectralAudio(X=X), nbComps=c["J"], nbNMFComps=c["K"], spatial_rank=c["rank"],
            iter_num=c["iters"], wlen=2 * (c["F"] - 1), hopsize=(c["F"] - 1) // 4)
    if c["conv"]:
        m.makeItConvolutive()
    return m


def _drift(m, g, name):
    """max relative deviation from the oracle fixture per output group"""
    c = FULL_CASES[name]
    fs, ts = sub_f(c["F"]), sub_t(c["T"])
    d = {"params": 0.0, "FB": 0.0, "TW": 0.0, "sums": 0.0}
    for j in range(c["J"]):
        p = m.spat_comps[j]['params']
        d["params"] = max(d["params"], rel(p[..., fs] if c["conv"] else p, g["params_%d" % j]))
        fac = m.spec_comps[j]['factor'][0]
        d["FB"] = max(d["FB"], rel(fac['FB'][fs], g["FB_%d" % j]))
        d["TW"] = max(d["TW"], rel(fac['TW'][:, ts], g["TW_%d" % j]))
        d["sums"] = max(d["sums"], abs(fac['FB'].sum() / g["FB_sum_%d" % j] - 1),
                        abs(fac['TW'].sum() / g["TW_sum_%d" % j] - 1))
    S = np.abs(m.separated_images())
    d["absS"] = rel(S[:, :, fs][:, :, :, ts], g["absS"])
    # every kept point against its own magnitude (floored at 1e-6 max)
    d["absS_elem"] = rel_elem(S[:, :, fs][:, :, :, ts], g["absS"])
    d["absS_sum"] = rel(S.sum(axis=(2, 3)), g["absS_sum"])
    return d


@pytest.mark.parametrize("name", ["c3_full", "c3_t1000", "j8k128_t1000", "j4k128_t1000"])
def test_config3_full_size_vs_oracle(name):
    """BASELINE configs[2] (F=2049, T=10000, J=4, r=2, K=32) at its real size:
    the production launch shapes (several E-step / FB chunks, TW bin splits,
    ragged last chunks) against the oracle's GEM iterations."""
    g = load(name)
    m = _fasst_model(name)
    ll = m.estim_param_a_post_model()
    assert rel(ll, g["logliks"]) < 1e-10, (ll, g["logliks"])
    assert rel(m.noise['PSD'], g["final_psd"]) < 1e-14
    d = _drift(m, g, name)
    print(name, "drift", d)
    for k, v in d.items():
        # elementwise |S|: low-power points carry the reordered sums' rounding
        # relative to their own (tiny) magnitude
        assert v < (1e-6 if k == "absS_elem" else 1e-8), (k, v)


def test_config3_every_point_vs_live_oracle(tmp_path):
    """BASELINE configs[2] at its real size, one GEM iteration and the Wiener
    images, compared at EVERY bin and frame with the live oracle
    (tests/oracle_c3_every_point.py, oracle/fasst_ref.py on bin slices in a
    process pool; started first, so it computes while the GPU runs).  The
    production launch shapes (15 E-step chunks, 19 FB chunks, 4 TW bin
    splits, ragged last chunks) are pinned point by point, not through the
    c3_full fixture's subsample: logliks 1e-10, PSD 1e-14, mixing filters /
    FB / TW max-normalised 1e-8 and elementwise 1e-6, |S| elementwise 1e-6
    (each point against its own magnitude, floored at 1e-6 of the max)."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    out = str(tmp_path / "oracle")
    proc = subprocess.Popen([sys.executable, os.path.join(here, "oracle_c3_every_point.py"), out,
                             str(min(16, os.cpu_count() or 1))],
                            stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    try:
        m = _fasst_model("c3_full", iters=1)
        ll = m.estim_param_a_post_model()
        S = np.abs(m.separated_images())
        log, _ = proc.communicate(timeout=900)
    finally:
        if proc.poll() is None:
            proc.kill()
            proc.wait()
    print(log)
    assert proc.returncode == 0, log
    g = lambda n: np.load(os.path.join(out, n + ".npy"))
    assert rel(ll, g("logliks")) < 1e-10
    assert rel(m.noise['PSD'], g("psd")) < 1e-14
    worst = {}
    for j in range(4):
        fac = m.spec_comps[j]['factor'][0]
        for key, a in (("params", m.spat_comps[j]['params']), ("FB", fac['FB']), ("TW", fac['TW']),
                       ("FW", fac['FW'])):
            b = g("%s_%d" % (key, j))
            assert a.shape == b.shape, (key, a.shape, b.shape)
            worst[key] = max(worst.get(key, 0.0), rel(a, b))
            if key != "FW":
                worst[key + "_elem"] = max(worst.get(key + "_elem", 0.0), rel_elem(a, b))
    Sr = g("absS")
    assert S.shape == Sr.shape
    worst["absS"] = rel(S, Sr)
    worst["absS_elem"] = rel_elem(S, Sr)
    print("c3 every point, worst relative deviation:", worst)
    for k, v in worst.items():
        assert v < (1e-6 if k.endswith("_elem") else 1e-8), (k, v)


def test_chunk_overrides_vs_oracle(monkeypatch):
    """Forced multi-chunk reductions (E-step chunks 3, FB chunks 3, TW bin
    splits 2, ragged last chunks) on a small case against the live oracle."""
    import fasst_ref as R
    from test_gpu_parity import _c3_like
    monkeypatch.setenv("FASST_NCHUNK_E", "3")
    monkeypatch.setenv("FASST_NCHUNK_B", "3")
    monkeypatch.setenv("FASST_NSPLIT_T", "2")
    m, o, X = _c3_like(129, 301, 4, 32, 2, 3)
    ll = m.estim_param_a_post_model()
    llo = o.estim_param_a_post_model()
    assert rel(ll, llo) < 1e-10
    for j in range(4):
        assert rel(m.spat_comps[j]['params'], o.spat_comps[j]['params']) < 1e-8
        assert rel(m.spec_comps[j]['factor'][0]['FB'], o.spec_comps[j]['factor'][0]['FB']) < 1e-8
        assert rel(m.spec_comps[j]['factor'][0]['TW'], o.spec_comps[j]['factor'][0]['TW']) < 1e-8
    assert rel(np.abs(m.separated_images()), np.abs(o.separated_images(X))) < 1e-8
    del R


def test_config1_shape_50_iterations_drift():
    """C1-shaped run (MultiChanNMFInst_FASST J=2, rank 1, K=32, F=1025,
    T=1122, 50 GEM iterations) against the oracle: the north-star 1e-4 bar on
    the separated magnitude spectrograms after the full iteration count."""
    name = "c1_50"
    g = load(name)
    m = _fasst_model(name)
    ll = m.estim_param_a_post_model()
    d = _drift(m, g, name)
    d["logliks"] = rel(ll, g["logliks"])
    print("c1_50 drift after 50 iterations:", d)
    # the north-star bar, max-normalised AND elementwise (each kept bin/frame of
    # |S| against its own magnitude, floored at 1e-6 max: SURVEY.md §7's metric)
    assert d["absS"] < BAR and d["absS_sum"] < BAR and d["absS_elem"] < BAR
    # the FP64 path holds far tighter than the bar (recorded, asserted loosely)
    assert d["logliks"] < 1e-8
    assert max(d["params"], d["FB"], d["TW"]) < 1e-5


@pytest.mark.parametrize("name", ["c5_full", "c5_10"])
@pytest.mark.parametrize("gemm", ["0", "2"])
def test_config5_full_size_vs_oracle(monkeypatch, gemm, name):
    """BASELINE configs[4]: Stereo_SIMM at F=2049, N=20000, NF0=1092, P=30,
    K=4, R=40 against oracle/simm_ref.py (SIMM.py:613-941), one iteration and
    the pipeline's default 10 (SeparateLeadStereoTF.py:264), with the
    NF0-sized products on the hand-written k_dgemm2 (FASST_SIMM_GEMM=0, the
    default) and on the generic k_gemm (=2)."""
    monkeypatch.setenv("FASST_SIMM_GEMM", gemm)
    from pyfasst_amd.SeparateLeadStereo.SIMM import SIMM as S
    c = FULL_CASES[name]
    g = load(name)
    F, N, NF0, P, K, Rr = (c[k] for k in ("F", "N", "NF0", "P", "K", "R"))
    rs = np.random.RandomState(c["data_seed"])
    SXR = rs.gamma(0.8, 1.0, size=(F, N))
    SXL = rs.gamma(0.8, 1.0, size=(F, N))
    WF0 = rs.gamma(1.0, 1.0, size=(F, NF0))
    WG = rs.gamma(1.0, 1.0, size=(F, P))
    np.random.seed(c["init_seed"])
    import ctypes
    from pyfasst_amd import _lib

    def counts():
        d2, kg = ctypes.c_long(0), ctypes.c_long(0)
        _lib.check(_lib.lib.simm_nf0_product_counts(ctypes.byref(d2), ctypes.byref(kg)),
                   "simm_nf0_product_counts")
        return d2.value, kg.value
    before = counts()
    res = S.Stereo_SIMM(SXR, SXL, WF0, WG, numberOfFilters=K,
                        numberOfAccompanimentSpectralShapes=Rr, numberOfIterations=c["iters"],
                        computeError=True, verbose=False)
    after = counts()
    # the selected kernel ran, and only it: at least two NF0-sized products
    # per iteration (SF0 and WF0^T [num | den]) plus the model rebuilds
    ran = (after[0] - before[0], after[1] - before[1])
    used, other = ran if gemm == "0" else ran[::-1]
    assert used >= 2 * c["iters"] and other == 0, (gemm, ran)
    names = ['alphaR', 'alphaL', 'HGAMMA', 'HPHI', 'HF0', 'betaR', 'betaL', 'HM', 'WM',
             'recoError']
    fs, ts = sub_f(F), sub_t(N)
    worst = {}
    for n, v in zip(names, res):
        v = np.asarray(v)
        s = v.sum()
        worst[n + "_sum"] = abs(s - g[n + "_sum"]) / max(abs(g[n + "_sum"]), 1e-300)
        if n in ('HPHI', 'HM'):
            v = v[:, ts]
        elif n == 'HF0':
            v = v[::8][:, ts]
        elif n == 'WM':
            v = v[fs]
        worst[n] = rel(v, g[n])
    print(name, "drift:", worst)
    for k, v in worst.items():
        assert v < 1e-8, (k, v)


def test_config4_independent_contexts_concurrent():
    """Config 4 semantics in one process: two contexts on distinct seeded
    clips, run concurrently from two host threads on one GPU, each bit-equal
    to its solo run (fresh state per clip)."""
    over = dict(F=513, T=1200, iters=4)
    solo = []
    for seed in (0, 1):
        m = _fasst_model("c3_full", data_seed=seed, **over)
        ll = m.estim_param_a_post_model()
        solo.append((ll, [m.spec_comps[j]['factor'][0]['TW'].copy() for j in range(4)],
                     [m.spat_comps[j]['params'].copy() for j in range(4)]))
        del m
    models = [_fasst_model("c3_full", data_seed=s, **over) for s in (0, 1)]
    out = [None, None]
    err = []

    def work(i):
        try:
            out[i] = models[i].estim_param_a_post_model()
        except Exception as e:   # surfaced below
            err.append(e)

    th = [threading.Thread(target=work, args=(i,)) for i in (0, 1)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not err, err
    for i in (0, 1):
        np.testing.assert_array_equal(out[i], solo[i][0])
        for j in range(4):
            np.testing.assert_array_equal(models[i].spec_comps[j]['factor'][0]['TW'], solo[i][1][j])
            np.testing.assert_array_equal(models[i].spat_comps[j]['params'], solo[i][2][j])
    # and the two clips really differ
    assert rel(out[0], out[1]) > 1e-6
