"""Lead / accompaniment masks (SeparateLeadStereoTF.py:1762-1871) and the
SIMM-pipeline stft / istft (separateLeadFunctions.py:90-233) on the MI355X,
against the reference's golden vectors (tests/golden/lead.npz) and the
oracle (oracle/simm_ref.py).  FP64 FFTs differ from pocketfft in rounding
only: bound TIGHT relative (max-normalised); WAVs within 1 LSB.
"""
import os

import numpy as np
import pytest
import scipy.io.wavfile as wf

import simm_ref as S
from helpers import load, rel

pytestmark = pytest.mark.gpu

TIGHT = 1e-12
CFGS = ((128, 32, 128, 0, None), (256, 64, 512, 3, 17), (100, 25, 128, 0, None))


def _slf():
    from pyfasst_amd.SeparateLeadStereo import separateLeadFunctions as slf
    return slf


def _params():
    s = load("simm")
    return {'WF0': s['WF0'], 'HF0': s['st_HF0'], 'WGAMMA': s['WGAMMA'],
            'HGAMMA': s['st_HGAMMA'], 'HPHI': s['st_HPHI'], 'HM': s['st_HM'], 'WM': s['st_WM'],
            'alphaR': s['st_alphaR'], 'alphaL': s['st_alphaL'], 'betaR': s['st_betaR'],
            'betaL': s['st_betaL']}


@pytest.mark.parametrize("cfg", CFGS)
def test_simm_stft_istft_golden(cfg):
    g = load("lead")
    slf = _slf()
    wlen, hop, nfft, start, stop = cfg
    tag = '%d_%d_%d' % (wlen, hop, nfft)
    X, F, N = slf.stft(g['x'], window=slf.sinebell(wlen), hopsize=float(hop), nfft=float(nfft),
                       fs=8000., start=start, stop=stop)
    assert X.shape == g['X_' + tag].shape and rel(X, g['X_' + tag]) < TIGHT
    assert np.array_equal(F, g['F_' + tag]) and np.array_equal(N, g['N_' + tag])
    Xg = g['X_' + tag]
    y = slf.istft(Xg, window=slf.sinebell(wlen), hopsize=float(hop), nfft=float(nfft))
    assert y.shape == g['y_' + tag].shape and rel(y, g['y_' + tag]) < TIGHT
    y = slf.istft(Xg, analysisWindow=np.hanning(wlen), window=slf.sinebell(wlen),
                  hopsize=float(hop), nfft=float(nfft), originalDataLen=1000)
    assert y.shape == g['yh_' + tag].shape and rel(y, g['yh_' + tag]) < TIGHT


def test_lead_masks_and_wavs_golden(tmp_path):
    from pyfasst_amd.SeparateLeadStereo import SeparateLeadStereoTF as SL
    g = load("lead")
    P = _params()
    masks = SL.separate_lead_stfts(P, g['XR'], g['XL'])
    for name, m in zip(('vR', 'vL', 'mR', 'mL'), masks):
        assert rel(m, g['mask_' + name]) < TIGHT, name
    files = {'voc_output_file': os.path.join(str(tmp_path), 'voc.wav'),
             'mus_output_file': os.path.join(str(tmp_path), 'mus.wav')}
    proc = SL.SeparateLeadProcess(SIMMParams=P, stftParams={'windowSizeInSamples': 128,
                                                            'hopsize': 32., 'NFT': 128},
                                  XR=g['XR'], XL=g['XL'], files=files, fs=8000, scaleData=1.0,
                                  dataType=np.int16)
    (vR, vL), (mR, mL) = proc.separated_signals()
    for name, y in zip(('vR', 'vL', 'mR', 'mL'), (vR, vL, mR, mL)):
        assert rel(y, g['est_' + name]) < TIGHT, name
    proc.writeSeparatedSignals()
    for key, gk in (('voc_output_file', 'voc_wav'), ('mus_output_file', 'mus_wav')):
        d = wf.read(files[key])[1]
        assert d.shape == g[gk].shape
        assert np.abs(d.astype(int) - g[gk].astype(int)).max() <= 1


def test_lead_masks_vs_oracle_large():
    """F=1025 (nfft 2048), N=300 frames, R=12 shapes, NF0=180 combs."""
    from pyfasst_amd.SeparateLeadStereo import SeparateLeadStereoTF as SL
    rs = np.random.RandomState(4)
    F, N, NF0, P, K, R = 1025, 300, 180, 12, 4, 12
    Pm = {'WF0': rs.gamma(1, 1, (F, NF0)), 'HF0': rs.gamma(1, 1, (NF0, N)),
          'WGAMMA': rs.gamma(1, 1, (F, P)), 'HGAMMA': rs.gamma(1, 1, (P, K)),
          'HPHI': rs.gamma(1, 1, (K, N)), 'HM': rs.gamma(1, 1, (R, N)),
          'WM': rs.gamma(1, 1, (F, R)), 'alphaR': 0.7, 'alphaL': 0.3}
    b = rs.rand(R)
    Pm['betaR'], Pm['betaL'] = np.diag(b), np.diag(1 - b)
    XR = rs.randn(F, N) + 1j * rs.randn(F, N)
    XL = rs.randn(F, N) + 1j * rs.randn(F, N)
    got = SL.separate_lead_stfts(Pm, XR, XL)
    want = S.lead_masks(Pm, XR, XL)
    for a, w in zip(got, want):
        assert rel(a, w) < TIGHT
    slf = _slf()
    y = slf.istft(got[0], window=slf.sinebell(2048), hopsize=256., nfft=2048.)
    yo = S.slf_istft(want[0], window=S.sinebell(2048), hopsize=256., nfft=2048.)
    assert rel(y, yo) < 1e-11


def test_simm_istft_edge_cases():
    slf = _slf()
    X = np.ones((65, 2), dtype=complex)
    with pytest.raises(ValueError):       # shorter than two windows
        slf.istft(X, window=slf.sinebell(128), hopsize=32., nfft=128.)
    with pytest.raises(ValueError):
        slf.stft(np.ones(100), window=slf.sinebell(64), hopsize=16., nfft=64., stop=1000)
