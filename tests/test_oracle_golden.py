"""The CPU oracle (oracle/fasst_ref.py) against the reference's own outputs.

Golden vectors were produced by running the reference itself
(tests/golden/make_golden.py); inv_herm.npz holds the known-answer data of
the reference test pyfasst_tests/pyfasst/tools/test_signalTools.py:27-64.
"""
import numpy as np
import pytest

import fasst_ref as R
from helpers import CASES, CQT_CASES, load, oracle_model_from_golden, rel, spec_keys


def test_inv_herm_known_answer():
    g = load("inv_herm")
    d, o, det = R.inv_herm_mat_2d(g['sigma_x_diag'], g['sigma_x_off'])
    # the reference test's own assertions (A A^-1 = I to 6 decimals)
    np.testing.assert_array_almost_equal(d[0] * g['sigma_x_diag'][0] + g['sigma_x_off'] * np.conj(o),
                                         np.ones_like(o))
    np.testing.assert_array_almost_equal(d[0] * np.conj(g['sigma_x_off']) +
                                         g['sigma_x_diag'][1] * np.conj(o), np.zeros_like(o))
    np.testing.assert_array_equal(d, g['inv_diag_run'])
    np.testing.assert_array_equal(o, g['inv_off_run'])
    # (the test file's inv_*_ref literals are not asserted by the reference
    # test itself: its inputs are printed to 8 digits and near-singular)


def test_stft_istft_golden():
    g = load("stft")
    for nfft, hop in ((256, 64), (512, 128), (1024, 256)):
        X = R.stft(g['x'], np.hanning(nfft), hop, nfft)
        np.testing.assert_array_equal(X, g['X_%d_%d' % (nfft, hop)])
        y = R.istft(X, np.hanning(nfft), np.hanning(nfft), hop, nfft)[:g['x'].size]
        np.testing.assert_array_equal(y, g['y_%d_%d' % (nfft, hop)])


@pytest.mark.parametrize("name,kind,kw", CQT_CASES, ids=[c[0] for c in CQT_CASES])
def test_cqt_golden(name, kind, kw):
    """CQTransfo / MinQTransfo forward + inverse (tftransforms/minqt.py), perfRast=1."""
    import cqt_ref
    g = load("cqt")
    t = cqt_ref.RefCQT(kind, **kw)
    X = t.forward(g['x'])
    np.testing.assert_array_equal(X, g['X_' + name])
    np.testing.assert_array_equal(np.array(t.nframes), g['nframes_' + name])
    np.testing.assert_array_equal(t.freq_stamps(), g['freqs_' + name])
    np.testing.assert_array_equal(t.inverse(X), g['y_' + name])


def test_nmf_golden():
    g = load("nmf")
    rng = np.random.RandomState(1)
    W, H = R.nmf_decomposition(g['SX'], nbComps=6, niter=7, rng=rng)
    np.testing.assert_array_equal(W, g['W'])
    np.testing.assert_array_equal(H, g['H'])
    np.random.seed(2)
    W, H = R.nmf_decomp_init(g['SX'], nbComps=5, niter=6)
    np.testing.assert_array_equal(W, g['di_W'])
    np.testing.assert_array_equal(H, g['di_H'])
    np.random.seed(3)
    W, H = R.nmf_decomp_init(g['SX'], nbComps=4, niter=5, Winit=g['Winit'], updateW=False)
    np.testing.assert_array_equal(W, g['dw_W'])
    np.testing.assert_array_equal(H, g['dw_H'])
    np.random.seed(4)
    W, H = R.nmf_decomp_init(g['SX'], nbComps=4, niter=5, Hinit=g['Hinit'])
    np.testing.assert_array_equal(W, g['dh_W'])
    np.testing.assert_array_equal(H, g['dh_H'])


@pytest.mark.parametrize("case", sorted(CASES))
def test_em_golden(case):
    g = load(case)
    m, X = oracle_model_from_golden(g, case)
    J = CASES[case][0]
    np.testing.assert_array_equal(m.Cx, g['Cx'])
    for j in range(J):
        np.testing.assert_array_equal(np.array(m.spat_comps[j]['params']), g['init_params_%d' % j])
    for j in spec_keys(g, J):
        np.testing.assert_array_equal(m.spec_comps[j]['factor'][0]['FB'], g['init_FB_%d' % j])
        np.testing.assert_array_equal(m.spec_comps[j]['factor'][0]['TW'], g['init_TW_%d' % j])
        np.testing.assert_array_equal(m.spec_comps[j]['factor'][0]['FW'], g['init_FW_%d' % j])
        if 'init_TB_%d' % j in g:
            np.testing.assert_array_equal(m.spec_comps[j]['factor'][0]['TB'], g['init_TB_%d' % j])
    ll = m.estim_param_a_post_model()
    np.testing.assert_array_equal(ll, g['logliks'])
    for j in range(J):
        np.testing.assert_array_equal(np.array(m.spat_comps[j]['params']), g['final_params_%d' % j])
    for j in spec_keys(g, J):
        np.testing.assert_array_equal(m.spec_comps[j]['factor'][0]['FB'], g['final_FB_%d' % j])
        np.testing.assert_array_equal(m.spec_comps[j]['factor'][0]['TW'], g['final_TW_%d' % j])
        np.testing.assert_array_equal(m.spec_comps[j]['factor'][0]['FW'], g['final_FW_%d' % j])
        if 'final_TB_%d' % j in g:
            np.testing.assert_array_equal(m.spec_comps[j]['factor'][0]['TB'], g['final_TB_%d' % j])
    S = m.separated_images(X)
    assert rel(np.abs(S), np.abs(g['images'])) == 0.0


def _simm_check(g, prefix, out, names):
    for n, v in zip(names, out):
        np.testing.assert_array_equal(np.asarray(v), g[prefix + n], err_msg=prefix + n)


def test_simm_golden():
    import simm_ref
    g = load("simm")
    st_names = ['alphaR', 'alphaL', 'HGAMMA', 'HPHI', 'HF0', 'betaR', 'betaL', 'HM', 'WM',
                'recoError']
    mono_names = ['HGAMMA', 'HPHI', 'HF0', 'HM', 'WM', 'recoError']
    K, R = g['st_HGAMMA'].shape[1], g['st_HM'].shape[0]
    np.random.seed(1)
    out = simm_ref.stereo_simm(g['SXR'], g['SXL'], g['WF0'], g['WGAMMA'], K, R,
                               numberOfIterations=4)
    _simm_check(g, 'st_', out, st_names)
    np.random.seed(2)
    _simm_check(g, 'mono_', simm_ref.simm(g['SXR'], g['WF0'], g['WGAMMA'], K, 1,
                                          numberOfIterations=4), mono_names)
    np.random.seed(3)
    out = simm_ref.stereo_simm(g['SXR'], g['SXL'], g['WF0'], g['WGAMMA'], K, R,
                               numberOfIterations=3, updateRulePower=0.7, updateHGAMMA=False,
                               computeError=True)
    _simm_check(g, 'st2_', out, st_names)
    np.random.seed(4)
    N = g['SXR'].shape[1]
    _simm_check(g, 'monoN_', simm_ref.simm(g['SXR'], g['WF0'], g['WGAMMA'], K, N,
                                           numberOfIterations=3), mono_names)


def test_lead_golden():
    """SIMM-pipeline stft/istft and the writeSeparatedSignals masks."""
    import simm_ref as S
    g = load("lead")
    for (wlen, hop, nfft, start, stop) in ((128, 32, 128, 0, None), (256, 64, 512, 3, 17),
                                           (100, 25, 128, 0, None)):
        tag = '%d_%d_%d' % (wlen, hop, nfft)
        X, F, N = S.slf_stft(g['x'], S.sinebell(wlen), float(hop), float(nfft), fs=8000.,
                             start=start, stop=stop)
        np.testing.assert_array_equal(X, g['X_' + tag])
        np.testing.assert_array_equal(F, g['F_' + tag])
        np.testing.assert_array_equal(N, g['N_' + tag])
        np.testing.assert_array_equal(
            S.slf_istft(X, window=S.sinebell(wlen), hopsize=float(hop), nfft=float(nfft)),
            g['y_' + tag])
        np.testing.assert_array_equal(
            S.slf_istft(X, analysisWindow=np.hanning(wlen), window=S.sinebell(wlen),
                        hopsize=float(hop), nfft=float(nfft), originalDataLen=1000),
            g['yh_' + tag])
    s = load("simm")
    P = {'WF0': s['WF0'], 'HF0': s['st_HF0'], 'WGAMMA': s['WGAMMA'], 'HGAMMA': s['st_HGAMMA'],
         'HPHI': s['st_HPHI'], 'HM': s['st_HM'], 'WM': s['st_WM'], 'alphaR': s['st_alphaR'],
         'alphaL': s['st_alphaL'], 'betaR': s['st_betaR'], 'betaL': s['st_betaL']}
    masks = S.lead_masks(P, g['XR'], g['XL'])
    for name, m in zip(('vR', 'vL', 'mR', 'mL'), masks):
        np.testing.assert_array_equal(m, g['mask_' + name])
        y = S.slf_istft(m, window=S.sinebell(128), hopsize=32., nfft=128)
        np.testing.assert_array_equal(y, g['est_' + name])
    voc = np.array(np.round(np.array([g['est_vR'], g['est_vL']]).T), dtype=np.int16)
    np.testing.assert_array_equal(voc, g['voc_wav'])


def test_viterbi_golden():
    """Viterbi tracker (tracking.py / _tracking.pyx) and runViterbi's inputs."""
    import viterbi_ref as V
    g = load("viterbi")
    for p in ('r', 't'):
        S, N = g[p + '_logD'].shape
        path = V.viterbi_tracking(S, N, g[p + '_logD'], g[p + '_prior'], g[p + '_logT'])
        np.testing.assert_array_equal(path, g[p + '_path'])
        np.testing.assert_array_equal(path, g[p + '_path_naive'])
    logT, prior = V.melody_transitions(64, 4)
    np.testing.assert_array_equal(logT, g['m_logT'])
    np.testing.assert_array_equal(prior, g['m_prior'])
    np.testing.assert_array_equal(V.melody_log_density(g['m_HF0']), g['m_logD'])
    S = int(g['m_S'])
    path = V.viterbi_tracking(S, g['m_HF0'].shape[1], g['m_logD'], g['m_prior'], g['m_logT'])
    np.testing.assert_array_equal(path, g['m_path'])


def test_wf0_dictionaries_golden():
    """generate_WF0_TR_chirped (STFT transform) and generateHannBasis."""
    import dict_ref as D
    from cqt_ref import sqrt_blackmanharris
    g = load("wf0")
    for tag, (fs, nft, minF0, maxF0, stepNotes, perF0) in {
            'a': (8000, 256, 100, 800, 4, 1), 'b': (8000, 512, 150, 600, 2, 3),
            'c': (16000, 256, 60, 1000, 1, 1)}.items():
        F0Table, WF0 = D.generate_wf0_tr_chirped_stft(
            nft, int(nft * 0.25), sqrt_blackmanharris(nft), fs, minF0, maxF0, stepNotes,
            perF0=perF0)
        np.testing.assert_array_equal(F0Table, g['F0Table_' + tag])
        np.testing.assert_array_equal(WF0, g['WF0_' + tag])
    for tag, (F, nft, fs, P, ov) in {'h1': (129, 256, 8000, 10, 0.75),
                                     'h2': (257, 512, 16000, 30, 0.5),
                                     'h3': (2049, 4096, 44100, 30, 0.75)}.items():
        np.testing.assert_array_equal(D.generate_hann_basis(F, nft, fs, numberOfBasis=P, overlap=ov),
                                      g['WGAMMA_' + tag])


@pytest.mark.parametrize("tag", ["m1", "m2", "c1"])
def test_wf0_cqt_dictionaries_golden(tag):
    """generate_WF0_TR_chirped on a MinQT / CQT transform (the complex comb
    through the transform, separateLeadFunctions.py:742-886) vs the reference
    run (tests/golden/wf0_cqt.npz)."""
    import cqt_ref
    import dict_ref as D
    g = load("wf0_cqt")
    fs, nft, fmin, fmax, bins, minF0, maxF0, stepNotes, perF0 = g['cfg_' + tag]
    kind = 'cqt' if tag[0] == 'c' else 'mqt'
    t = cqt_ref.RefCQT(kind, fmin=fmin, fmax=fmax, bins=int(bins), fs=fs, linFTLen=int(nft))
    F0Table, WF0 = D.generate_wf0_tr_chirped_cqt(t, minF0, maxF0, stepNotes, perF0=int(perF0))
    np.testing.assert_array_equal(F0Table, g['F0Table_' + tag])
    ref = g['WF0_' + tag]
    assert WF0.shape == ref.shape
    assert float(np.max(np.abs(WF0 - ref) / np.max(ref, axis=0))) < 1e-12


@pytest.mark.parametrize("same", [True, False])
def test_nmf_init_golden(same):
    """initialize_all_spec_comps_with_NMF (audioModel.py:2091-2222), then EM."""
    name = "nmfinit_same" if same else "nmfinit_indiv"
    g = load(name)
    x, _ = R.read_scaled(g['wav'])
    X = [R.stft(x[:, c], np.hanning(256), 64, 256) for c in range(2)]
    m = R.RefFASST(iter_num=2)
    m.set_transform(X)
    np.random.seed(0)
    R.init_nmf_inst(m, 3, 4, 2)
    R.make_convolutive(m)
    np.random.seed(5)
    if same:
        R.init_nmf_same(m, niter=4)
    else:
        R.init_nmf_indiv(m, niter=4)
    for k in range(3):
        np.testing.assert_array_equal(m.spec_comps[k]['factor'][0]['FB'], g['init_FB_%d' % k])
        np.testing.assert_array_equal(m.spec_comps[k]['factor'][0]['TW'], g['init_TW_%d' % k])
        np.testing.assert_array_equal(np.array(m.spat_comps[k]['params']), g['init_params_%d' % k])
    np.testing.assert_array_equal(m.estim_param_a_post_model(), g['logliks'])
    for k in range(3):
        np.testing.assert_array_equal(m.spec_comps[k]['factor'][0]['FB'], g['final_FB_%d' % k])


def test_conv_rand_init_golden():
    """initializeConvParams(initMethod='rand') (audioModel.py:2224-2294): the
    steering vectors' RNG order and the 'conv' parameters, then EM."""
    g = load("convinit_rand")
    x, _ = R.read_scaled(g['wav'])
    X = [R.stft(x[:, c], np.hanning(256), 64, 256) for c in range(2)]
    m = R.RefFASST(iter_num=3)
    m.set_transform(X)
    np.random.seed(0)
    R.init_nmf_inst(m, 3, 4, [1, 2, 1])
    np.random.seed(9)
    R.init_conv_rand(m)
    for j in range(3):
        assert m.spat_comps[j]['mix_type'] == str(g['mix_type_%d' % j])
        np.testing.assert_array_equal(m.spat_comps[j]['params'], g['init_params_%d' % j])
    np.testing.assert_array_equal(m.estim_param_a_post_model(), g['logliks'])
    for j in range(3):
        np.testing.assert_array_equal(m.spat_comps[j]['params'], g['final_params_%d' % j])


def test_nnls_oracle_matches_reference_run():
    """initHF00='nnls' (SeparateLeadStereoTF.py:982-993): the oracle's per-frame
    scipy.optimize.nnls reproduces the HF00 the reference handed to SIMM."""
    import nnls_ref
    g = load("pipeline_nnls")
    for i in range(int(g['nchunks'])):
        np.testing.assert_array_equal(nnls_ref.nnls_hf00(g['WF0'], g['SX_%d' % i]),
                                      g['nnls_HF00_%d' % i])
