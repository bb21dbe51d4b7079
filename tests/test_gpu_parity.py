"""HIP path vs the oracle / the reference's golden vectors (run on MI355X).

Every compute call goes through the C ABI of libfasst_hip.so.  Tolerances:
the BASELINE bar is 1e-4 relative on reconstructed magnitude spectrograms;
the FP64 HIP path is held to much tighter bounds below (its reductions are
ordered differently from NumPy/OpenBLAS, so bit-equality is not expected).
"""
import os

import numpy as np
import pytest
import scipy.io.wavfile as wf

import fasst_ref as R
from helpers import CASES, apply_setup, load, oracle_model_from_golden, rel, spec_keys

pytestmark = pytest.mark.gpu

BAR = 1e-4          # north_star: magnitude spectrograms, relative
TIGHT = 1e-9        # what the FP64 path actually holds on the golden cases
# em_multi's conv mixing filters amplify rounding ~50x more than em_conv's: the
# oracle itself moves its final params by 1.1e-11 (em_conv: 2.2e-13) when Cx is
# perturbed by 1e-15 relative noise, and the GPU's reordered FP64 sums land at
# 4e-9 (em_conv 6e-11): the same ratio to that sensitivity (tools/relcheck.py)
TIGHT_CASE = {'em_multi': 2e-8}


def _am():
    import pyfasst_amd.audioModel as am
    return am


def _product_model(case, g, tmp_path):
    am = _am()
    J, K, rank, conv, kw = CASES[case]
    kw = dict(kw)
    setup = kw.pop('_setup', None)
    wav = os.path.join(str(tmp_path), case + ".wav")
    wf.write(wav, int(g['fs']), g['wav'])
    np.random.seed(0)
    cls = am.MultiChanNMFConv if conv else am.MultiChanNMFInst_FASST
    m = cls(wav, nbComps=J, nbNMFComps=K, spatial_rank=rank, **kw)
    if conv:
        m.makeItConvolutive()
    if setup:
        apply_setup(m, setup)
    return m


def test_native_library_is_loaded():
    from pyfasst_amd import _lib
    assert _lib.device_count() >= 1
    assert os.path.exists(_lib.LIB_PATH)


def test_inv_herm_known_answer_gpu():
    from pyfasst_amd.tools.signalTools import inv_herm_mat_2d
    g = load("inv_herm")
    d, o, det = inv_herm_mat_2d(g['sigma_x_diag'], g['sigma_x_off'])
    # the reference test's assertions (test_signalTools.py:55-64)
    np.testing.assert_array_almost_equal(d[0] * g['sigma_x_diag'][0] + g['sigma_x_off'] * np.conj(o),
                                         np.ones_like(o))
    np.testing.assert_array_almost_equal(d[0] * np.conj(g['sigma_x_off']) +
                                         g['sigma_x_diag'][1] * np.conj(o), np.zeros_like(o))
    # these matrices are near-singular (det ~ 1e-5 of d0*d1): the cancellation
    # amplifies the last-bit differences of |o|^2 (hypot vs re^2+im^2, FMA)
    assert rel(d, g['inv_diag_run']) < 1e-12
    assert rel(o, g['inv_off_run']) < 1e-12
    assert rel(det, g['det_run']) < 1e-12


def test_inv_herm_guards_gpu():
    from pyfasst_amd.tools.signalTools import inv_herm_mat_2d
    rs = np.random.RandomState(0)
    d = rs.randn(2, 7, 33)
    o = rs.randn(7, 33) + 1j * rs.randn(7, 33)
    d[:, 0, :5] = 0.0
    o[0, :5] = 0.0            # det == 0 -> floored to +eps
    d[0, 1, :3] = 1e-6
    d[1, 1, :3] = -1e-6       # negative det below eps -> -eps
    o[1, :3] = 0.0
    a = inv_herm_mat_2d(d, o)
    b = R.inv_herm_mat_2d(d, o)
    for x, y in zip(a, b):
        assert rel(x, y) < 1e-13


def test_stft_istft_golden_gpu():
    from pyfasst_amd.tftransforms import stft as S
    g = load("stft")
    for nfft, hop in ((256, 64), (512, 128), (1024, 256)):
        tr = S.STFT(linFTLen=nfft, atomHopFactor=hop / float(nfft))
        tr.computeTransform(g['x'])
        X = g['X_%d_%d' % (nfft, hop)]
        assert tr.transfo.shape == X.shape
        assert rel(tr.transfo, X) < 1e-13
        y = tr.invertTransform()
        assert rel(y, g['y_%d_%d' % (nfft, hop)]) < 1e-13


def test_stft_edge_lengths_gpu():
    from pyfasst_amd.tftransforms.stft import stft, istft
    rs = np.random.RandomState(5)
    for L, nfft, hop in ((1, 64, 16), (63, 64, 16), (64, 64, 64), (1000, 128, 48), (4097, 4096, 1024)):
        x = rs.randn(L)
        X, _, _ = stft(x, window=np.hanning(nfft), hopsize=hop, nfft=nfft)
        Xr = R.stft(x, np.hanning(nfft), hop, nfft)
        assert X.shape == Xr.shape
        assert rel(X, Xr) < 1e-13
        y = istft(X, window=np.hanning(nfft), hopsize=hop, nfft=nfft)
        yr = R.istft(Xr, np.hanning(nfft), np.hanning(nfft), hop, nfft)
        assert y.shape == yr.shape
        assert rel(y, yr) < 1e-12


@pytest.mark.parametrize("case", sorted(CASES))
def test_em_end_to_end_vs_reference(case, tmp_path):
    """WAV -> GPU STFT/Cx -> GPU GEM iterations -> GPU Wiener images, vs the
    reference's own outputs on the same file and seed."""
    g = load(case)
    J = CASES[case][0]
    m = _product_model(case, g, tmp_path)
    assert rel(m.Cx, g['Cx']) < 1e-13
    for j in range(J):
        assert rel(m.spat_comps[j]['params'], g['init_params_%d' % j]) < 1e-14
    for j in spec_keys(g, J):
        assert rel(m.spec_comps[j]['factor'][0]['FB'], g['init_FB_%d' % j]) < 1e-14
        assert rel(m.spec_comps[j]['factor'][0]['TW'], g['init_TW_%d' % j]) < 1e-14
        assert rel(m.spec_comps[j]['factor'][0]['FW'], g['init_FW_%d' % j]) < 1e-14
    ll = m.estim_param_a_post_model()
    assert abs(ll[0] - g['e_loglik'].real) <= 1e-12 * abs(ll[0])
    assert rel(ll, g['logliks']) < TIGHT
    tight = TIGHT_CASE.get(case, TIGHT)
    for j in range(J):
        # (the reference leaves a fixed 'inst' component's real params real)
        assert np.iscomplexobj(m.spat_comps[j]['params']) == \
            np.iscomplexobj(g['final_params_%d' % j])
        assert rel(m.spat_comps[j]['params'], g['final_params_%d' % j]) < tight
    for j in spec_keys(g, J):
        assert rel(m.spec_comps[j]['factor'][0]['FB'], g['final_FB_%d' % j]) < tight
        assert rel(m.spec_comps[j]['factor'][0]['TW'], g['final_TW_%d' % j]) < tight
        assert rel(m.spec_comps[j]['factor'][0]['FW'], g['final_FW_%d' % j]) < tight
        if 'final_TB_%d' % j in g:
            assert rel(m.spec_comps[j]['factor'][0]['TB'], g['final_TB_%d' % j]) < tight
    assert rel(m.noise['PSD'], g['final_psd']) < 1e-14
    groups = _spatial_groups(m)   # the golden images: separate_spat_comps
    S = m.separated_images(groups)
    assert rel(np.abs(S), np.abs(g['images'])) < tight
    assert rel(np.abs(S), np.abs(g['images'])) < BAR
    # the device-resident separation (images never leave HBM) is the per-image
    # iSTFT of those images, bit for bit (same kernels, same order)
    Y = m.separated_waveforms(groups) if m.tft.transformname == 'stft' else None
    for n in range(S.shape[0] if Y is not None else 0):
        for c in range(2):
            m.tft.transfo = S[n, c]
            np.testing.assert_array_equal(Y[n, c], m.tft.invertTransform())
            del m.tft.transfo
    if len(m.spec_comps) > J and Y is not None:
        # separate_comps' default, one source per spectral component (the
        # source-table kernel), device-resident as well
        S2 = m.separated_images()
        Y2 = m.separated_waveforms()
        assert S2.shape[0] == Y2.shape[0] == len(m.spec_comps)
        for n in range(S2.shape[0]):
            for c in range(2):
                m.tft.transfo = S2[n, c]
                np.testing.assert_array_equal(Y2[n, c], m.tft.invertTransform())
                del m.tft.transfo
    # separated WAV files: int16 after iSTFT, identical up to 1 LSB
    m.separate_spat_comps(dir_results=str(tmp_path))
    for n, fn in enumerate(m.files['spat_comp']):
        y = wf.read(fn)[1].astype(np.int64)
        ref = g['sep_wav_%d' % n].astype(np.int64)
        assert y.shape == ref.shape
        assert np.max(np.abs(y - ref)) <= 1


def _spatial_groups(m):
    """spec_comp_ind of separate_spat_comps: one source per spatial component
    (audioModel.py:1063-1086)."""
    groups = {}
    for j in range(len(m.spat_comps)):
        groups[j] = [k for k in sorted(m.spec_comps) if m.spec_comps[k]['spat_comp_ind'] == j]
    return groups


def _c3_like(F, T, J, K, rank, iters, seed=0):
    """STFT-domain synthetic model: product and oracle on identical inputs."""
    from pyfasst_amd import synthetic
    from pyfasst_amd.audioObject import SpectralAudio
    am = _am()
    X = synthetic.stereo_mixture(F, T, J=J, K_true=4, rank=rank if np.isscalar(rank) else 2,
                                 seed=seed)
    np.random.seed(1)
    m = am.MultiChanNMFConv(SpectralAudio(X=X), nbComps=J, nbNMFComps=K, spatial_rank=rank,
                            iter_num=iters, wlen=2 * (F - 1), hopsize=(F - 1) // 2)
    m.makeItConvolutive()
    o = R.RefFASST(iter_num=iters)
    o.set_transform([X[0], X[1]])
    np.random.seed(1)
    R.init_nmf_inst(o, J, K, rank)
    R.make_convolutive(o)
    return m, o, X


@pytest.mark.parametrize("F,T,J,K,rank,iters", [
    (129, 301, 4, 32, 2, 3),     # config-3 structure (R = 8, K = 32), ragged T
    (65, 77, 2, 20, 1, 4),       # K not a multiple of 16, R = 2
    (33, 17, 3, 5, 2, 2),        # tiny F and T (one tile), odd K
    (97, 203, 3, 40, [1, 2, 1], 3),  # mixed ranks (general-rank E-step), K padded to 64
    (161, 250, 4, 16, 1, 3),     # rank 1 everywhere, K = 16 (one MFMA k block)
    (65, 77, 6, 8, 2, 3),        # 6 sources, total rank 12
    (49, 60, 8, 4, 1, 2),        # 8 sources of rank 1
    (33, 40, 8, 16, 2, 2),       # 8 sources of rank 2: total rank 16 (the k_mix LU maximum)
    (57, 70, 5, 36, [3, 2, 3, 2, 3], 2),  # 5 sources, mixed ranks 13, K padded to 64
    # K > 64 per source (padded to 128: the E-step's NKS = 32 instantiation,
    # NKC = 8 contractions, FW read from L2 by its staging kernels)
    (97, 150, 2, 100, 2, 3),     # K = 100
    (65, 77, 4, 128, 1, 2),      # K = 128 on 4 sources
    (129, 90, 3, 72, [1, 2, 1], 3),  # K = 72, mixed ranks
    # K > 64 with more than 4 sources (the VR E-step with its W operand from L2)
    (65, 77, 8, 128, 1, 2),      # J = 8, K = 128
    (33, 40, 5, 70, 2, 2),       # J = 5, K = 70, total rank 10
    (49, 52, 6, 100, [1, 2, 1, 2, 1, 2], 2),  # J = 6, K = 100, mixed ranks
    # more than 8 sources (the two-pass E-step, k_egen_point / k_egen_stats;
    # k_wiener's runtime-bounded kMaxJ form)
    (49, 60, 12, 8, 1, 2),       # J = 12
    (33, 40, 16, 4, 1, 2),       # J = 16, total rank 16
    (65, 77, 10, 100, 1, 2),     # J = 10, K = 100 (KP = 128)
    (40, 45, 9, 20, [2, 1, 2, 1, 2, 1, 2, 1, 2], 2),  # J = 9, mixed ranks, total 14
    (33, 40, 12, 6, 2, 2),       # J = 12 'conv' at rank 2: total rank 24 (k_mix's 32-rank form)
    (33, 36, 16, 4, 2, 2),       # J = 16 at rank 2: total rank 32
    # the full F = 2049 of BASELINE config 3, every point compared (the
    # golden full-size fixtures keep a subsample): the production launch
    # shapes -- E-step frame chunks, FB / TW splits, XCD block order -- of the
    # headline structure and of 8 sources (oracle ~30 s / ~15 s on the host)
    (2049, 1000, 4, 32, 2, 2),
    (2049, 500, 8, 32, 1, 2),
    # the fused many-source E-step (k_egen_fused) at the full F: 129 bin
    # tiles, the production frame chunks, J = 16 at rank 2 (total rank 32)
    (2049, 96, 16, 32, 2, 1),
    # ... its KP = 16 form with an odd J, ragged T, rank 1
    (1025, 77, 11, 12, 1, 2),
])
def test_em_stft_domain_vs_oracle(F, T, J, K, rank, iters):
    m, o, X = _c3_like(F, T, J, K, rank, iters)
    for j in range(J):
        assert rel(m.spec_comps[j]['factor'][0]['TW'], o.spec_comps[j]['factor'][0]['TW']) < 1e-14
    ll = m.estim_param_a_post_model()
    llo = o.estim_param_a_post_model()
    assert rel(ll, llo) < 1e-10
    for j in range(J):
        assert rel(m.spat_comps[j]['params'], o.spat_comps[j]['params']) < 1e-8
        assert rel(m.spec_comps[j]['factor'][0]['FB'], o.spec_comps[j]['factor'][0]['FB']) < 1e-8
        assert rel(m.spec_comps[j]['factor'][0]['TW'], o.spec_comps[j]['factor'][0]['TW']) < 1e-8
    S = m.separated_images()
    So = o.separated_images(X)
    assert rel(np.abs(S), np.abs(So)) < 1e-8


def test_k_above_128_fails_loudly():
    """More than 128 NMF columns on one spatial component is outside the HIP
    path: it raises instead of running (no CPU fallback)."""
    with pytest.raises(NotImplementedError):
        m, o, X = _c3_like(33, 40, 2, 130, 1, 1)
        m.estim_param_a_post_model()


@pytest.mark.parametrize("what", ["free_fw", "multi", "multi_free_fw", "lambda", "time_blobs"])
def test_k_above_64_every_structure_vs_oracle(what):
    """K > 64 (KP = 128: the NKC = 8 forms of k_multi_prep, the DEN FB
    contraction, the FW contraction and the BLK / LAM / TBQ TW contractions,
    k_fw_reduce on 32-bin chunks) on every structure, not only the
    single-component path: free FW, several spectral components, free FW on
    some of them, lambdaCorr, time blobs; against the oracle."""
    m, o, X = _c3_like(65, 77, 2, 100, 1, 2)
    tb = {}
    for mod in (m, o):
        if what in ("free_fw", "multi_free_fw"):
            keys = [0] if what == "free_fw" else [0, 2]
            if what == "multi_free_fw":
                _split_spec(mod, {0: [40, 60], 1: [100]})
            for k in keys:
                fac = mod.spec_comps[k]['factor'][0]
                n = fac['FW'].shape[0]
                fac['FW'] = fac['FW'] + 0.2 * np.abs(np.random.RandomState(80 + k).randn(n, n))
                fac['FW_frdm_prior'] = 'free'
        elif what == "multi":
            _split_spec(mod, {0: [40, 60], 1: [30, 70]}, ((3, 'FB'),))
        elif what == "lambda":
            mod.lambdaCorr = 0.3
            _split_spec(mod, {0: [100], 1: [50, 50]})
        else:
            _split_spec(mod, {0: [40, 60], 1: [100]})
            tb = {0: (6, 'free', 'free'), 1: (4, 'free', 'free'), 2: (3, 'fixed', 'free')}
            _time_blobs(mod, tb)
    ll = m.estim_param_a_post_model()
    llo = o.estim_param_a_post_model()
    assert rel(ll, llo) < 1e-10
    for k in sorted(o.spec_comps):
        keys = ('FB', 'FW', 'TW', 'TB') if k in tb else ('FB', 'FW', 'TW')
        for key in keys:
            assert rel(m.spec_comps[k]['factor'][0][key], o.spec_comps[k]['factor'][0][key]) < 1e-8, \
                (k, key)
    for j in range(2):
        assert rel(m.spat_comps[j]['params'], o.spat_comps[j]['params']) < 1e-8
    groups = _spatial_groups(m)
    assert rel(np.abs(m.separated_images(groups)), np.abs(o.separated_images(X, groups))) < 1e-8


@pytest.mark.parametrize("what", ["multi_fw", "lambda_tb"])
def test_many_sources_every_structure_vs_oracle(what):
    """J = 10 (the two-pass E-step) with several spectral components per
    spatial component, free FW, lambdaCorr and time blobs, against the
    oracle."""
    m, o, X = _c3_like(49, 60, 10, 12, 1, 2)
    tb = {}
    for mod in (m, o):
        _split_spec(mod, {0: [5, 7], 3: [6, 6], **{j: [12] for j in (1, 2, 4, 5, 6, 7, 8, 9)}})
        if what == "multi_fw":
            for k in (0, 3, 10):
                fac = mod.spec_comps[k]['factor'][0]
                n = fac['FW'].shape[0]
                fac['FW'] = fac['FW'] + 0.2 * np.abs(np.random.RandomState(90 + k).randn(n, n))
                fac['FW_frdm_prior'] = 'free'
        else:
            mod.lambdaCorr = 0.2
            tb = {1: (4, 'free', 'free'), 11: (3, 'free', 'free')}
            _time_blobs(mod, tb)
    ll = m.estim_param_a_post_model()
    llo = o.estim_param_a_post_model()
    assert rel(ll, llo) < 1e-10
    for k in sorted(o.spec_comps):
        keys = ('FB', 'FW', 'TW', 'TB') if k in tb else ('FB', 'FW', 'TW')
        for key in keys:
            assert rel(m.spec_comps[k]['factor'][0][key], o.spec_comps[k]['factor'][0][key]) < 1e-8, \
                (k, key)
    for j in range(10):
        assert rel(m.spat_comps[j]['params'], o.spat_comps[j]['params']) < 1e-8
    groups = _spatial_groups(m)
    assert rel(np.abs(m.separated_images(groups)), np.abs(o.separated_images(X, groups))) < 1e-8


def test_fixed_components_vs_oracle():
    """frdm_prior 'fixed' paths: FB fixed, TW fixed, an instantaneous spatial
    component fixed (exercises the 'other' subtraction, audioModel.py:817-823)."""
    from pyfasst_amd import synthetic
    from pyfasst_amd.audioObject import SpectralAudio
    am = _am()
    F, T, J, K = 65, 90, 3, 6
    X = synthetic.stereo_mixture(F, T, J=J, K_true=3, rank=1, seed=4)
    np.random.seed(3)
    m = am.MultiChanNMFInst_FASST(SpectralAudio(X=X), nbComps=J, nbNMFComps=K, spatial_rank=1,
                                  iter_num=4, wlen=128, hopsize=32)
    o = R.RefFASST(iter_num=4)
    o.set_transform([X[0], X[1]])
    np.random.seed(3)
    R.init_nmf_inst(o, J, K, 1)
    for mod in (m, o):
        mod.spec_comps[0]['factor'][0]['FB_frdm_prior'] = 'fixed'
        mod.spec_comps[1]['factor'][0]['TW_frdm_prior'] = 'fixed'
        mod.spat_comps[2]['frdm_prior'] = 'fixed'
    ll = m.estim_param_a_post_model()
    llo = o.estim_param_a_post_model()
    assert rel(ll, llo) < 1e-10
    for j in range(J):
        assert rel(m.spat_comps[j]['params'], o.spat_comps[j]['params']) < 1e-8
        assert rel(m.spec_comps[j]['factor'][0]['FB'], o.spec_comps[j]['factor'][0]['FB']) < 1e-8
        assert rel(m.spec_comps[j]['factor'][0]['TW'], o.spec_comps[j]['factor'][0]['TW']) < 1e-8


@pytest.mark.parametrize("F,T,J,K,rank,iters,omega,which", [
    (129, 301, 4, 32, 2, 3, 1.0, "all"),    # C3 structure, every FW free
    (65, 77, 2, 20, 1, 4, 0.7, "first"),    # K not a multiple of 16, omega != 1, one source
    (97, 203, 3, 40, 2, 2, 1.0, "all"),     # K padded to 64
])
def test_free_fw_vs_oracle(F, T, J, K, rank, iters, omega, which):
    """FW_frdm_prior 'free' (audioModel.py:1578-1631) with a dense positive FW:
    the FW update between the FB and TW updates, against the oracle (itself
    pinned to the reference by the em_fw_free golden case)."""
    m, o, X = _c3_like(F, T, J, K, rank, iters)
    for mod in (m, o):
        mod.nmfUpdateCoeff = omega
        for j in range(J if which == "all" else 1):
            fac = mod.spec_comps[j]['factor'][0]
            rs = np.random.RandomState(50 + j)
            fac['FW'] = fac['FW'] + 0.2 * np.abs(rs.randn(K, K))
            fac['FW_frdm_prior'] = 'free'
        if which != "all":
            mod.spec_comps[J - 1]['factor'][0]['FB_frdm_prior'] = 'fixed'
    ll = m.estim_param_a_post_model()
    llo = o.estim_param_a_post_model()
    assert rel(ll, llo) < 1e-10
    for j in range(J):
        for key in ('FB', 'FW', 'TW'):
            assert rel(m.spec_comps[j]['factor'][0][key], o.spec_comps[j]['factor'][0][key]) < 1e-8, \
                (j, key)
        assert rel(m.spat_comps[j]['params'], o.spat_comps[j]['params']) < 1e-8
    assert rel(np.abs(m.separated_images()), np.abs(o.separated_images(X))) < 1e-8


@pytest.mark.parametrize("J,rank", [(6, 2), (8, 1), (8, 2), (12, 1), (16, 1), (12, 2)])
def test_inst_many_sources_vs_oracle(J, rank):
    """'inst' mixing with more than 4 sources (total rank up to 12): the
    f-averaged real R x R solve of update_mix_matrix (audioModel.py:808-839)."""
    from pyfasst_amd import synthetic
    from pyfasst_amd.audioObject import SpectralAudio
    am = _am()
    F, T, K = 65, 80, 6
    X = synthetic.stereo_mixture(F, T, J=J, K_true=3, rank=1, seed=7)
    np.random.seed(5)
    m = am.MultiChanNMFInst_FASST(SpectralAudio(X=X), nbComps=J, nbNMFComps=K,
                                  spatial_rank=rank, iter_num=3, wlen=128, hopsize=32)
    o = R.RefFASST(iter_num=3)
    o.set_transform([X[0], X[1]])
    np.random.seed(5)
    R.init_nmf_inst(o, J, K, rank)
    ll = m.estim_param_a_post_model()
    llo = o.estim_param_a_post_model()
    assert rel(ll, llo) < 1e-10
    for j in range(J):
        assert rel(m.spat_comps[j]['params'], o.spat_comps[j]['params']) < 1e-8
        assert rel(m.spec_comps[j]['factor'][0]['FB'], o.spec_comps[j]['factor'][0]['FB']) < 1e-8
        assert rel(m.spec_comps[j]['factor'][0]['TW'], o.spec_comps[j]['factor'][0]['TW']) < 1e-8
    assert rel(np.abs(m.separated_images()), np.abs(o.separated_images(X))) < 1e-8


def _split_spec(mod, splits, fixed=()):
    """Several spectral components per spatial component: source j's one
    component is cut into column blocks splits[j], the new keys interleaved
    over the sources (as tests/helpers.py 'multi_spec'); fixed = ((key,
    'FB' | 'TW'), ...) priors set to 'fixed'."""
    import copy
    pieces = {}
    for k in sorted(mod.spec_comps):
        j = mod.spec_comps[k]['spat_comp_ind']
        fac = mod.spec_comps[k]['factor'][0]
        a, pieces[j] = 0, []
        for n in splits[j]:
            f = copy.deepcopy(fac)
            f['FB'], f['FW'], f['TW'] = (np.array(fac['FB'][:, a:a + n]),
                                         np.array(fac['FW'][a:a + n, a:a + n]),
                                         np.array(fac['TW'][a:a + n]))
            pieces[j].append({'spat_comp_ind': j, 'factor': {0: f}})
            a += n
    new, key = {}, 0
    for pos in range(max(len(v) for v in pieces.values())):
        for j in sorted(pieces):
            if pos < len(pieces[j]):
                new[key] = pieces[j][pos]
                key += 1
    for key, which in fixed:
        new[key]['factor'][0][which + '_frdm_prior'] = 'fixed'
    mod.spec_comps = new


@pytest.mark.parametrize("F,T,J,K,rank,iters,splits,fixed,chunks", [
    # C3-like structure, 2-3 components per source incl. blocks not aligned to 16
    (129, 301, 3, 32, 2, 3, {0: [16, 16], 1: [10, 12, 10], 2: [32]}, (), None),
    # forced multi-chunk reductions (ragged last chunks), fixed FB / TW blocks
    (129, 301, 2, 24, 2, 2, {0: [5, 19], 1: [8, 8, 8]}, ((1, 'FB'), (2, 'TW')), (3, 3, 2)),
    # K_j = 64 (the padded maximum) in 4 components
    (65, 90, 2, 64, 1, 2, {0: [16, 16, 16, 16], 1: [30, 34]}, (), None),
])
def test_em_multi_components_vs_oracle(F, T, J, K, rank, iters, splits, fixed, chunks,
                                       monkeypatch):
    """Several spectral components per spatial component (comp_spat_comp_power's
    sum, audioModel.py:430-498, and the component-by-component FB / TW updates
    with V_j and V_k, :1479-1727) against the oracle, itself pinned to the
    reference by the em_multi / em_multi_inst golden cases."""
    if chunks:
        for name, v in zip(("FASST_NCHUNK_E", "FASST_NCHUNK_B", "FASST_NSPLIT_T"), chunks):
            monkeypatch.setenv(name, str(v))
    m, o, X = _c3_like(F, T, J, K, rank, iters)
    for mod in (m, o):
        _split_spec(mod, splits, fixed)
    ll = m.estim_param_a_post_model()
    llo = o.estim_param_a_post_model()
    assert rel(ll, llo) < 1e-10
    for j in range(J):
        assert rel(m.spat_comps[j]['params'], o.spat_comps[j]['params']) < 1e-8
    for k in sorted(o.spec_comps):
        for key in ('FB', 'FW', 'TW'):
            assert rel(m.spec_comps[k]['factor'][0][key], o.spec_comps[k]['factor'][0][key]) < 1e-8, \
                (k, key)
    # one source per spatial component (separate_spat_comps) ...
    groups = _spatial_groups(m)
    assert rel(np.abs(m.separated_images(groups)), np.abs(o.separated_images(X, groups))) < 1e-8
    # ... per spectral component (separate_comps' default), and mixed sources
    # (components of two spatial components; a subset: Sigma_x sums the
    # listed sources only, audioModel.py:1161-1164)
    keys = sorted(o.spec_comps)
    for sources in ({k: [k] for k in keys}, {0: [keys[0], keys[-1]], 1: keys[1:3]}):
        S = m.separated_images(sources)
        So = o.separated_images(X, sources)
        assert S.shape == So.shape
        assert rel(np.abs(S), np.abs(So)) < 1e-8


def test_multi_component_tw_restart_vs_oracle():
    """The TW restart test per spectral component (audioModel.py:2023-2028)
    when a spatial component holds several: only the dead component is
    redrawn, in key order."""
    m, o, X = _c3_like(33, 40, 2, 8, 1, 3)
    for mod in (m, o):
        _split_spec(mod, {0: [4, 4], 1: [3, 5]})
        mod.spec_comps[2]['factor'][0]['TW'][:] = 1e-30
    np.random.seed(12)
    ll = m.estim_param_a_post_model()
    np.random.seed(12)
    llo = o.estim_param_a_post_model()
    assert rel(ll, llo) < 1e-10
    for k in sorted(o.spec_comps):
        assert rel(m.spec_comps[k]['factor'][0]['TW'], o.spec_comps[k]['factor'][0]['TW']) < 1e-8


@pytest.mark.parametrize("omega", [1.0, 0.7])
def test_multi_component_free_fw_vs_oracle(omega):
    """Free FW (audioModel.py:1578-1631) on some of several spectral components
    per spatial component: the FW step of a component uses its own V_k
    (spec_comp_ind=[k]) between its FB and TW steps."""
    m, o, X = _c3_like(97, 150, 3, 24, 2, 3)
    for mod in (m, o):
        mod.nmfUpdateCoeff = omega
        _split_spec(mod, {0: [10, 14], 1: [8, 8, 8], 2: [24]}, ((4, 'FB'),))
        for k, seed in ((0, 60), (3, 61), (2, 62)):
            fac = mod.spec_comps[k]['factor'][0]
            n = fac['FW'].shape[0]
            fac['FW'] = fac['FW'] + 0.2 * np.abs(np.random.RandomState(seed).randn(n, n))
            fac['FW_frdm_prior'] = 'free'
    ll = m.estim_param_a_post_model()
    llo = o.estim_param_a_post_model()
    assert rel(ll, llo) < 1e-10
    for k in sorted(o.spec_comps):
        for key in ('FB', 'FW', 'TW'):
            assert rel(m.spec_comps[k]['factor'][0][key], o.spec_comps[k]['factor'][0][key]) < 1e-8, \
                (k, key)
    groups = _spatial_groups(m)
    assert rel(np.abs(m.separated_images(groups)), np.abs(o.separated_images(X, groups))) < 1e-8


@pytest.mark.parametrize("lam,splits,fw", [
    (0.3, None, False),                                  # one component per source
    (0.5, {0: [10, 14], 1: [8, 8, 8], 2: [24]}, False),  # several, keys interleaved
    (0.2, {0: [12, 12], 1: [24], 2: [6, 18]}, True),     # with free FW on some components
])
def test_lambda_corr_vs_oracle(lam, splits, fw):
    """lambdaCorr > 0 (audioModel.py:1484-1507 and the corrPen terms of the FB /
    FW / TW steps, :1544-1719): every component updated one at a time in key
    order against the powers of all sources, vs the oracle (pinned to the
    reference by the em_lambda / em_lambda_multi golden cases)."""
    m, o, X = _c3_like(97, 150, 3, 24, 2, 3)
    for mod in (m, o):
        mod.lambdaCorr = lam
        if splits:
            _split_spec(mod, splits, ((3, 'TW'),))
        if fw:
            for k, seed in ((0, 70), (4, 71)):
                fac = mod.spec_comps[k]['factor'][0]
                n = fac['FW'].shape[0]
                fac['FW'] = fac['FW'] + 0.2 * np.abs(np.random.RandomState(seed).randn(n, n))
                fac['FW_frdm_prior'] = 'free'
    ll = m.estim_param_a_post_model()
    llo = o.estim_param_a_post_model()
    assert rel(ll, llo) < 1e-10
    for k in sorted(o.spec_comps):
        for key in ('FB', 'FW', 'TW'):
            assert rel(m.spec_comps[k]['factor'][0][key], o.spec_comps[k]['factor'][0][key]) < 1e-8, \
                (k, key)
    for j in range(3):
        assert rel(m.spat_comps[j]['params'], o.spat_comps[j]['params']) < 1e-8
    groups = _spatial_groups(m)
    assert rel(np.abs(m.separated_images(groups)), np.abs(o.separated_images(X, groups))) < 1e-8


def _time_blobs(mod, spec):
    """Time blobs H = TW.TB on spectral components: spec = {key: (L, TB prior,
    TW prior)} (seeded, positive, H of the component's mean level)."""
    for k, (L, tb_prior, tw_prior) in spec.items():
        fac = mod.spec_comps[k]['factor'][0]
        n, T = fac['TW'].shape
        rs = np.random.RandomState(400 + k)
        TB = np.abs(rs.randn(L, T)) + 0.1
        TW = np.abs(rs.randn(n, L)) + 0.1
        TW *= fac['TW'].mean() / np.dot(TW, TB).mean()
        fac['TW'], fac['TB'] = TW, TB
        fac['TB_frdm_prior'], fac['TW_frdm_prior'] = tb_prior, tw_prior


@pytest.mark.parametrize("F,T,J,K,lam,splits,tb,omega", [
    # C3 structure, time blobs on every source (L up to 24), one fixed TB
    (129, 301, 4, 32, 0.0, None,
     {0: (8, 'free', 'free'), 1: (24, 'free', 'free'), 2: (5, 'fixed', 'free'),
      3: (3, 'free', 'fixed')}, 1.0),
    # several components per source, time blobs on some, omega != 1
    (97, 150, 3, 24, 0.0, {0: [10, 14], 1: [8, 8, 8], 2: [24]},
     {0: (6, 'free', 'free'), 4: (2, 'free', 'free'), 5: (40, 'free', 'fixed')}, 0.7),
    # with lambdaCorr (the corrPen terms of the TW / TB steps, :1650-1719, :1945-1973)
    (97, 150, 3, 24, 0.4, {0: [12, 12], 1: [24], 2: [6, 18]},
     {1: (4, 'free', 'free'), 3: (7, 'free', 'free'), 2: (64, 'free', 'free')}, 1.0),
])
def test_time_blobs_vs_oracle(F, T, J, K, lam, splits, tb, omega):
    """Time blobs (H = TW.TB, audioModel.py:486-487): the TW step through TB
    (:1665-1691), the TB step (:1931-1978) and their renormalisation
    (:2029-2033), vs the oracle (pinned to the reference by the em_tb golden
    case)."""
    m, o, X = _c3_like(F, T, J, K, 2, 3)
    for mod in (m, o):
        mod.lambdaCorr = lam
        mod.nmfUpdateCoeff = omega
        if splits:
            _split_spec(mod, splits)
        _time_blobs(mod, tb)
    ll = m.estim_param_a_post_model()
    llo = o.estim_param_a_post_model()
    assert rel(ll, llo) < 1e-10
    for k in sorted(o.spec_comps):
        keys = ('FB', 'FW', 'TW', 'TB') if k in tb else ('FB', 'FW', 'TW')
        for key in keys:
            assert rel(m.spec_comps[k]['factor'][0][key], o.spec_comps[k]['factor'][0][key]) < 1e-8, \
                (k, key)
    for j in range(J):
        assert rel(m.spat_comps[j]['params'], o.spat_comps[j]['params']) < 1e-8
    groups = _spatial_groups(m)
    assert rel(np.abs(m.separated_images(groups)), np.abs(o.separated_images(X, groups))) < 1e-8


def test_time_blobs_tw_restart_vs_oracle():
    """The restart test of a component with time blobs is sum(TW) < eps on its
    factor TW, not on H (audioModel.py:2023-2033): TW ~ 1e-12 with TB ~ 1e12
    keeps H (and the mixing solve) at a normal level but restarts TW; the host
    redraws TW, then renormalises TB.  The draws are bit-identical, so every
    parameter agrees to rounding after the restarting iteration."""
    for iters in (1, 3):
        m, o, X = _c3_like(33, 40, 3, 4, 1, iters)
        for mod in (m, o):
            _time_blobs(mod, {0: (3, 'free', 'free'), 2: (5, 'free', 'free')})
            fac = mod.spec_comps[0]['factor'][0]
            fac['TW'] *= 1e-12
            fac['TB'] *= 1e12
        np.random.seed(13)
        ll = m.estim_param_a_post_model()
        np.random.seed(13)
        llo = o.estim_param_a_post_model()
        # after the restart H sits ~1e5 above its level and the next
        # iterations amplify rounding: the oracle itself moves its FB / mixing
        # parameters by 3e-9 / 1e-8 after iteration 2 when Cx is perturbed by
        # 1e-15 relative noise (iteration 1: 4e-15), the GPU's reordered sums
        # by 3e-8 / 2e-7 after iteration 3
        tol = 1e-13 if iters == 1 else 1e-6
        assert rel(ll, llo) < max(tol, 1e-9)
        if iters == 1:
            assert o.restarted == [(0, 0)]
        for k in sorted(o.spec_comps):
            for key in ('FB', 'TW', 'TB') if k != 1 else ('FB', 'TW'):
                assert rel(m.spec_comps[k]['factor'][0][key],
                           o.spec_comps[k]['factor'][0][key]) < tol, (iters, k, key)
        for j in range(3):
            assert rel(m.spat_comps[j]['params'], o.spat_comps[j]['params']) < tol


def test_singular_mixing_raises_linalgerror():
    """A silent source makes hat_Rss[f] singular: LinAlgError('Singular Matrix')
    as the reference's conv solve (audioModel.py:855-861)."""
    m, o, X = _c3_like(33, 40, 2, 4, 2, 2)
    for mod in (m, o):
        mod.spec_comps[1]['factor'][0]['FB'][:] = 0.0
    with pytest.raises(np.linalg.LinAlgError):
        o.estim_param_a_post_model()
    with pytest.raises(np.linalg.LinAlgError):
        m.estim_param_a_post_model()


def test_tw_restart_vs_oracle():
    """sum(TW) < eps triggers the random TW restart (audioModel.py:2023-2028),
    drawn on the host RNG in the reference's order."""
    m, o, X = _c3_like(33, 40, 2, 4, 1, 3)
    for mod in (m, o):   # tiny but non-zero: the mixing solve stays regular
        mod.spec_comps[1]['factor'][0]['TW'][:] = 1e-30
    np.random.seed(11)
    ll = m.estim_param_a_post_model()
    np.random.seed(11)
    llo = o.estim_param_a_post_model()
    assert rel(ll, llo) < 1e-10
    for j in range(2):
        assert rel(m.spec_comps[j]['factor'][0]['TW'], o.spec_comps[j]['factor'][0]['TW']) < 1e-8


def test_sources_past_the_hip_path_fail_loudly():
    """More than 16 sources, or a total spatial rank above 32, raise instead of
    running."""
    for J, rank in ((17, 1), (16, [2] * 15 + [3])):
        with pytest.raises(NotImplementedError):
            m, o, X = _c3_like(33, 40, J, 4, rank, 1)
            m.estim_param_a_post_model()


def test_unsupported_structures_fail_loudly():
    m, o, X = _c3_like(33, 40, 2, 4, 1, 1)
    m.spec_comps[0]['factor'][0]['TW_constr'] = 'HMM'
    with pytest.raises(NotImplementedError):
        m.estim_param_a_post_model()


def test_mixed_types_free_conv_raises_as_reference(tmp_path):
    """A free 'conv' component next to any other component: the reference's
    conv solve (audioModel.py:856-857) passes the full hat_Rss[f].T against
    the free components' right-hand side and np.linalg.solve raises
    ValueError at the first M-step (the oracle restates it); the product
    raises the same exception type before running."""
    g = load("em_mixed")
    m = _product_model("em_mixed", g, tmp_path)
    m.spat_comps[2]['frdm_prior'] = 'free'
    with pytest.raises(ValueError):
        m.estim_param_a_post_model()
    o, _ = oracle_model_from_golden(g, "em_mixed")
    o.spat_comps[2]['frdm_prior'] = 'free'
    with pytest.raises(ValueError):
        o.estim_param_a_post_model()


def test_mixed_types_free_conv_refused_at_the_abi(tmp_path):
    """The same structure straight through the C ABI (no Python-side
    check): fasst_run refuses it (FASST_ERR_UNSUPPORTED) instead of
    updating the 'inst' rows and leaving the free 'conv' filters stale."""
    g = load("em_mixed")
    m = _product_model("em_mixed", g, tmp_path)
    m._upload()
    eng = m._engine
    eng.set_spatial(2, m.spat_comps[2]['params'], True)
    with pytest.raises(NotImplementedError, match="conv"):
        eng.run(np.ones((1, eng.F)), 1.0)


def test_full_size_config3_invariants():
    """BASELINE config 3 at full size (F=2049, T=10000, J=4, r=2, K=32):
    size-independent properties after two GEM iterations on the GPU."""
    from pyfasst_amd import synthetic
    from pyfasst_amd.audioObject import SpectralAudio
    am = _am()
    F, T = 2049, 10000
    X = synthetic.stereo_mixture(F, T, J=4, K_true=8, rank=2, seed=0)
    np.random.seed(1)
    m = am.MultiChanNMFConv(SpectralAudio(X=X), nbComps=4, nbNMFComps=32, spatial_rank=2,
                            iter_num=2, wlen=4096, hopsize=512)
    m.makeItConvolutive()
    ll = m.estim_param_a_post_model()
    assert np.all(np.isfinite(ll))
    for j in range(4):
        p = m.spat_comps[j]['params']
        assert p.shape == (2, 2, F)
        assert abs(np.mean(np.abs(p) ** 2) - 1.0) < 1e-12          # spatial renorm
        fac = m.spec_comps[j]['factor'][0]
        assert np.allclose(fac['FB'].max(axis=0), 1.0, rtol=0, atol=1e-15)  # FB col max
        np.testing.assert_array_equal(fac['FW'], 32.0 * np.eye(32))          # N6: FW = K I
        assert np.all(fac['TW'] >= 0) and np.all(np.isfinite(fac['TW']))
