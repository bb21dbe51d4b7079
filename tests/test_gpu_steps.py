"""The GEM step methods as device calls (fasst_steps.hip, include/fasst_hip.h
"GEM step methods") against the oracle's restatement of the same methods
(oracle/fasst_ref.py, pinned to the reference by the golden EM cases):
retrieve_subsrc_params, compute_suff_stat, update_mix_matrix,
update_spectral_components, compute_sigma_comp_2d, compute_inv_sigma_mix_2d,
compute_Wiener_gain_2d (audioModel.py:384-428, 514-889, 1327-1978).

Tolerances: FP64 with reductions ordered differently from NumPy's, so
relative to the array's max-abs: 1e-11 for pointwise algebra, 1e-9 for the
frame-summed statistics, 1e-8 for the NMF updates (as the fused-path tests).
"""
import numpy as np
import pytest

import fasst_ref as R
from helpers import rel
from test_gpu_parity import _c3_like, _split_spec

pytestmark = pytest.mark.gpu


def _inst_model(F=65, T=90, J=3, K=6, rank=2, seed=4, fixed=None):
    from pyfasst_amd import synthetic
    from pyfasst_amd.audioObject import SpectralAudio
    import pyfasst_amd.audioModel as am
    X = synthetic.stereo_mixture(F, T, J=J, K_true=3, rank=1, seed=seed)
    np.random.seed(3)
    m = am.MultiChanNMFInst_FASST(SpectralAudio(X=X), nbComps=J, nbNMFComps=K,
                                  spatial_rank=rank, iter_num=2, wlen=128, hopsize=32)
    o = R.RefFASST(iter_num=2)
    o.set_transform([X[0], X[1]])
    np.random.seed(3)
    R.init_nmf_inst(o, J, K, rank)
    if fixed is not None:
        for mod in (m, o):
            mod.spat_comps[fixed]['frdm_prior'] = 'fixed'
    return m, o, X


def _model(which):
    if which == "conv":   # every component free 'conv', mixed ranks
        m, o, X = _c3_like(97, 130, 3, 20, [1, 2, 1], 1)
    else:                 # 'inst', one component fixed (the 'other' subtraction)
        m, o, X = _inst_model(fixed=2)
    for mod in (m, o):
        mod.noise['PSD'] = mod.noise['ann_PSD_lim'][0]
    return m, o


@pytest.mark.parametrize("which", ["conv", "inst+fixed"])
def test_estep_statistics_vs_oracle(which):
    m, o = _model(which)
    V, mix, parts = m.retrieve_subsrc_params()
    Vo, mixo, partso = o.retrieve_subsrc_params()
    assert rel(V, Vo) < 1e-12
    assert rel(mix, mixo) == 0.0
    assert all(np.array_equal(parts[j], partso[j]) for j in partso)
    out = m.compute_suff_stat(Vo, mixo)
    ref = o.compute_suff_stat(Vo, mixo)
    names = ("hat_Rxx", "hat_Rxs", "hat_Rss", "hat_Ws", "loglik")
    for name, a, b, tol in zip(names, out, ref, (1e-13, 1e-9, 1e-9, 1e-11, 1e-12)):
        assert np.shape(a) == np.shape(b), name
        assert rel(a, b) < tol, (name, rel(a, b))
    # hat_Rss is Hermitian per bin, as the reference enforces (:733-740)
    rss = out[2]
    assert np.array_equal(rss, np.conj(np.transpose(rss, (0, 2, 1))))


@pytest.mark.parametrize("which", ["conv", "inst+fixed"])
def test_mix_update_vs_oracle(which):
    m, o = _model(which)
    Vo, mixo, parts = o.retrieve_subsrc_params()
    _, rxs, rss, _, _ = o.compute_suff_stat(Vo, mixo)
    mix_m = mixo.copy()
    m.update_mix_matrix(rxs.copy(), rss.copy(), mix_m, parts)
    o.update_mix_matrix(rxs.copy(), rss.copy(), mixo, parts)
    assert rel(mix_m, mixo) < 1e-10
    for j in o.spat_comps:
        assert m.spat_comps[j]['params'].shape == o.spat_comps[j]['params'].shape
        assert rel(m.spat_comps[j]['params'], o.spat_comps[j]['params']) < 1e-10


def test_mix_update_singular_raises_linalgerror():
    m, o, X = _c3_like(33, 40, 2, 8, 1, 1)
    Vo, mixo, parts = o.retrieve_subsrc_params()
    rss = np.zeros((33, 2, 2), dtype=complex)
    rxs = np.ones((33, 2, 2), dtype=complex)
    before = mixo.copy()
    with pytest.raises(np.linalg.LinAlgError):
        m.update_mix_matrix(rxs, rss, mixo, parts)
    assert np.array_equal(mixo, before)


@pytest.mark.parametrize("case", ["single", "multi", "lambda"])
def test_spectral_update_vs_oracle(case):
    """update_spectral_components from the oracle's hat_W, on the fused path's
    single-component kernels, the multi-block path and lambdaCorr."""
    m, o, X = _c3_like(97, 130, 3, 24, 2, 1)
    for mod in (m, o):
        if case != "single":
            _split_spec(mod, {0: [10, 14], 1: [8, 8, 8], 2: [24]}, ((3, 'TW'),))
        if case == "lambda":
            mod.lambdaCorr = 0.4
        mod.noise['PSD'] = mod.noise['ann_PSD_lim'][0]
    Vo, mixo, parts = o.retrieve_subsrc_params()
    _, rxs, rss, ws, _ = o.compute_suff_stat(Vo, mixo)
    hat_W = np.array([np.mean(ws[parts[j]], axis=0) for j in range(len(parts))])
    m.update_spectral_components(hat_W)
    o.update_spectral_components(hat_W)
    for k in sorted(o.spec_comps):
        for key in ('FB', 'FW', 'TW'):
            assert rel(m.spec_comps[k]['factor'][0][key], o.spec_comps[k]['factor'][0][key]) < 1e-9, \
                (k, key)


def test_piecewise_iteration_matches_fused():
    """retrieve -> suff_stat -> mix -> spectral -> renormalize through the
    step methods reproduces the fused GEM_iteration (fasst_run)."""
    m1, o, X = _c3_like(65, 77, 2, 16, 2, 1)
    m2, _, _ = _c3_like(65, 77, 2, 16, 2, 1)
    for mod in (m1, m2):
        mod.noise['PSD'] = mod.noise['ann_PSD_lim'][0]
    ll_fused = m1.GEM_iteration()
    V, mix, parts = m2.retrieve_subsrc_params()
    _, rxs, rss, ws, ll = m2.compute_suff_stat(V, mix)
    m2.update_mix_matrix(rxs, rss, mix, parts)
    hat_W = np.array([np.mean(ws[parts[j]], axis=0) for j in range(len(parts))])
    m2.update_spectral_components(hat_W)
    m2.renormalize_parameters()
    assert abs(ll - ll_fused) <= 1e-12 * abs(ll_fused)
    for j in range(2):
        assert rel(m2.spat_comps[j]['params'], m1.spat_comps[j]['params']) < 1e-9
        for key in ('FB', 'TW'):
            assert rel(m2.spec_comps[j]['factor'][0][key], m1.spec_comps[j]['factor'][0][key]) < 1e-9


def test_wiener_pieces_vs_oracle():
    m, o, X = _c3_like(97, 130, 3, 24, 2, 1)
    for mod in (m, o):
        _split_spec(mod, {0: [10, 14], 1: [8, 8, 8], 2: [24]})
        mod.noise['PSD'] = mod.noise['ann_PSD_lim'][0]
    sds, sos = [], []
    for j, keys in ((0, []), (1, [4]), (2, [5]), (1, [1, 5])):
        sd, so = m.compute_sigma_comp_2d(j, keys)
        sdo, soo = o.compute_sigma_comp_2d(j, keys)
        assert rel(sd, sdo) < 1e-12 and rel(so, soo) < 1e-12, (j, keys)
        sds.append(sdo)
        sos.append(soo)
    isd, iso = m.compute_inv_sigma_mix_2d(np.array(sds), np.array(sos))
    isdo, isoo = o.compute_inv_sigma_mix_2d(np.array(sds), np.array(sos))
    assert rel(isd, isdo) < 1e-11 and rel(iso, isoo) < 1e-11
    WG = m.compute_Wiener_gain_2d(sds[0], sos[0], isdo, isoo)
    WGo = R.RefFASST.compute_Wiener_gain_2d(sds[0], sos[0], isdo, isoo)
    assert WG.shape == WGo.shape
    assert rel(WG, WGo) < 1e-13
    # timeInvariant gains: [2, 2, F]
    WG = m.compute_Wiener_gain_2d(sds[0][:, :, 0], sos[0][:, 0], isdo[:, :, 0], isoo[:, 0],
                                  timeInvariant=True)
    assert WG.shape == (2, 2, 97)
    assert rel(WG, WGo[:, :, :, 0]) < 1e-13


def test_step_methods_leave_fused_state_usable():
    """Step calls between fused iterations: the context buffers the step
    kernels reuse (the rho planes, (FW H)^T, TW row sums) are rebuilt by the
    next fused iteration."""
    m, o, X = _c3_like(65, 77, 2, 16, 2, 2)
    for mod in (m, o):
        mod.noise['PSD'] = mod.noise['ann_PSD_lim'][0]
    lls = [m.GEM_iteration()]
    V, mix, parts = m.retrieve_subsrc_params()
    _, _, _, ws, _ = m.compute_suff_stat(V, mix)
    m.compute_sigma_comp_2d(0, [])
    lls.append(m.GEM_iteration())
    llo = [o.GEM_iteration(), o.GEM_iteration()]
    assert rel(np.array(lls), np.array(llo)) < 1e-10
    for j in range(2):
        assert rel(m.spec_comps[j]['factor'][0]['TW'], o.spec_comps[j]['factor'][0]['TW']) < 1e-8


def test_column_sets_past_64_vs_oracle():
    """K > 64 (padded to 128 columns): the column sets of compute_sigma_comp_2d,
    the source powers and the separation sources are 128-bit, so a spectral
    component whose columns pass 64 (here 40..79 of source 0) is selected
    exactly (a 64-bit mask kept only its low columns)."""
    m, o, X = _c3_like(49, 60, 2, 80, 1, 1)
    for mod in (m, o):
        _split_spec(mod, {0: [40, 40], 1: [80]})
        mod.noise['PSD'] = mod.noise['ann_PSD_lim'][0]
    for j, keys in ((0, [2]), (0, [0]), (0, []), (1, [])):
        sd, so = m.compute_sigma_comp_2d(j, keys)
        sdo, soo = o.compute_sigma_comp_2d(j, keys)
        assert rel(sd, sdo) < 1e-12 and rel(so, soo) < 1e-12, (j, keys)
    # one separation source per spectral component (columns 40..79 of source 0)
    groups = {n: [k] for n, k in enumerate(sorted(m.spec_comps))}
    S = m.separated_images(groups)
    So = o.separated_images(X, groups)
    assert S.shape == So.shape
    assert rel(np.abs(S), np.abs(So)) < 1e-11


def test_suff_stat_refuses_a_context_without_observation():
    """fasst_suff_stat on a context that never received Cx returns
    FASST_ERR_SHAPE (ValueError) before any launch, like the other step entry
    points' host-side guards."""
    from pyfasst_amd.engine import Engine
    F, T, Rk = 9, 11, 2
    e = Engine(F, T)
    try:
        V = np.ones((Rk, F, T))
        mix = np.ones((Rk, 2, F), complex)
        with pytest.raises(ValueError, match="no observation"):
            e.suff_stat(V, mix, 1.0)
    finally:
        e.close()
