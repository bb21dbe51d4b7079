"""BASELINE configs[3] (C4) at its real workload on one MI355X: eight
independent full-size C3 clips (F=2049, T=10000, J=4, spatial rank 2, K=32;
data seeds 0..7), one model context each (~2.2 GB of HBM per clip, ~18 GB
together), run CONCURRENTLY from eight host threads.

Each clip must come out bit-equal to its solo run (no state shared between
contexts: SURVEY.md §8(e)1, quirk N2), and clip 0 -- the c3_full input --
within the C3 bar of the oracle fixture tests/golden/c3_full.npz.  The
driver's 8-GPU run shards the same clips one per GPU (bench.py); this test is
the data-path half of that claim on the one-GPU box.

The clips are generated on the host in spawned worker processes (22 s of
NumPy each), written as .npy files and memory-mapped back.
"""
import multiprocessing as mp
import os
import threading

import numpy as np
import pytest

from helpers import FULL_CASES, load, rel

pytestmark = pytest.mark.gpu

NCLIP = 8


def _gen_clip(args):
    seed, path = args
    from pyfasst_amd import synthetic
    c = FULL_CASES["c3_full"]
    X = synthetic.stereo_mixture(c["F"], c["T"], J=c["J"], K_true=c["K_true"],
                                 rank=c["data_rank"], seed=seed)
    np.save(path, X)
    return path


def _model(X):
    import pyfasst_amd.audioModel as am
    from pyfasst_amd.audioObject import SpectralAudio
    c = FULL_CASES["c3_full"]
    np.random.seed(c["init_seed"])
    m = am.MultiChanNMFConv(SpectralAudio(X=np.asarray(X)), nbComps=c["J"], nbNMFComps=c["K"],
                            spatial_rank=c["rank"], iter_num=c["iters"],
                            wlen=2 * (c["F"] - 1), hopsize=(c["F"] - 1) // 4)
    m.makeItConvolutive()
    return m


def _state(m, ll):
    J = FULL_CASES["c3_full"]["J"]
    return dict(ll=np.array(ll),
                TW=[m.spec_comps[j]['factor'][0]['TW'].copy() for j in range(J)],
                FB=[m.spec_comps[j]['factor'][0]['FB'].copy() for j in range(J)],
                A=[m.spat_comps[j]['params'].copy() for j in range(J)])


def test_config4_eight_full_size_clips_concurrent(tmp_path):
    paths = [str(tmp_path / ("clip%d.npy" % s)) for s in range(NCLIP)]
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env_pp = os.environ.get("PYTHONPATH", "")
    os.environ["PYTHONPATH"] = os.pathsep.join([root, os.path.join(root, "tests"), env_pp])
    try:
        with mp.get_context("spawn").Pool(min(NCLIP, 8)) as pool:
            pool.map(_gen_clip, [(s, p) for s, p in zip(range(NCLIP), paths)])
    finally:
        os.environ["PYTHONPATH"] = env_pp
    clips = [np.load(p, mmap_mode="r") for p in paths]

    # all eight contexts resident at once, iterated concurrently
    models = [_model(X) for X in clips]
    out = [None] * NCLIP
    err = []

    def work(i):
        try:
            out[i] = models[i].estim_param_a_post_model()
        except Exception as e:   # surfaced below
            err.append((i, e))

    th = [threading.Thread(target=work, args=(i,)) for i in range(NCLIP)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not err, err
    conc = [_state(m, ll) for m, ll in zip(models, out)]
    S0 = np.abs(models[0].separated_images())
    for m in models:
        m._engine.close()
    del models

    # clip 0 against the oracle fixture (the c3_full input and init)
    g = load("c3_full")
    assert rel(conc[0]["ll"], g["logliks"]) < 1e-10
    from helpers import sub_f, sub_t
    fs, ts = sub_f(2049), sub_t(10000)
    for j in range(4):
        assert rel(conc[0]["TW"][j][:, ts], g["TW_%d" % j]) < 1e-8
        assert rel(conc[0]["FB"][j][fs], g["FB_%d" % j]) < 1e-8
        assert rel(conc[0]["A"][j][..., fs], g["params_%d" % j]) < 1e-8
    assert rel(S0[:, :, fs][:, :, :, ts], g["absS"]) < 1e-8

    # each clip bit-equal to its solo run
    for i in range(NCLIP):
        m = _model(clips[i])
        solo = _state(m, m.estim_param_a_post_model())
        m._engine.close()
        np.testing.assert_array_equal(conc[i]["ll"], solo["ll"])
        for j in range(4):
            for k in ("TW", "FB", "A"):
                np.testing.assert_array_equal(conc[i][k][j], solo[k][j], err_msg="clip %d %s" % (i, k))
    # the clips really differ
    assert min(rel(conc[0]["ll"], conc[i]["ll"]) for i in range(1, NCLIP)) > 1e-6
