"""C2's Wiener stage on the MI355X (BASELINE configs[1]): per-source mono
masks V_n / sum V * X on the IS-NMF model, and their iSTFT, against the
oracle restatement (oracle/fasst_ref.py mono_wiener_images, the one-channel
degenerate of audioModel.py:1327-1467).

PARITY UNPINNED by reference code: the reference's FASST raises for mono
signals, so the oracle restatement is the only checker;
the restatement's 2-channel parent (separated_images) is pinned to the
reference's golden outputs in tests/test_oracle_golden.py.  Tolerance 1e-12
relative (max-normalised): the GPU sums K products in a different order.
"""
import numpy as np
import pytest

import fasst_ref as R
from helpers import rel

pytestmark = pytest.mark.gpu


def _nmf():
    import pyfasst_amd.tools.nmf as nmf
    return nmf


def test_c2_mono_wiener_full_size():
    """F=1025, T=2000, K=64 IS-NMF (GPU), then the two sources' masks."""
    from pyfasst_amd import synthetic
    nmf = _nmf()
    F, T, K = 1025, 2000, 64
    X = synthetic.mono_stft(F, T, J=2, K_true=32, seed=0)
    np.random.seed(1)
    W, H = nmf.NMF_decomposition(np.abs(X) ** 2, nbComps=K, niter=5)
    comp = {0: list(range(32)), 1: list(range(32, 64))}
    S = nmf.NMF_wiener_images(X, W, H, comp)
    So = R.mono_wiener_images(X, W, H, comp)
    assert S.shape == (2, F, T)
    assert rel(S, So) < 1e-12, rel(S, So)
    # with no noise term the masks partition the mixture
    assert rel(S.sum(axis=0), X) < 1e-13
    w = np.hanning(2048)
    y = nmf.NMF_separate_waveforms(X, W, H, comp, w, 512)
    for n in range(2):
        yo = R.istft(So[n], w, w, 512, 2048)
        assert y[n].shape == yo.shape
        assert rel(y[n], yo) < 1e-12, rel(y[n], yo)


def test_mono_wiener_ragged_guard_and_grouping():
    """J = 3 sources over non-contiguous components, one unused component,
    a noise PSD, ragged F / T, and bins where Sigma_x = 0 (the determinant
    guard floors it to eps, so those images are exactly zero)."""
    nmf = _nmf()
    rs = np.random.RandomState(3)
    F, T, K = 97, 203, 13
    X = rs.randn(F, T) + 1j * rs.randn(F, T)
    W = rs.gamma(1.0, 1.0, size=(F, K))
    H = rs.gamma(0.5, 1.0, size=(K, T))
    W[5:9] = 0.0
    comp = {0: [0, 4, 7], 1: [1, 2, 11, 12], 2: [3, 5, 6, 8, 10]}   # 9 unused
    psd = rs.gamma(1.0, 0.1, size=F)
    psd[5:7] = 0.0
    for p in (None, psd):
        S = nmf.NMF_wiener_images(X, W, H, comp, psd=p)
        So = R.mono_wiener_images(X, W, H, [comp[0], comp[1], comp[2]], psd=p)
        assert rel(S, So) < 1e-12
    assert np.all(S[:, 5:7] == 0)
    with pytest.raises(ValueError):
        nmf.NMF_wiener_images(X, W, H, {0: [0, 1], 1: [1]})


def test_mono_wiener_large_k():
    nmf = _nmf()
    rs = np.random.RandomState(4)
    F, T, K = 129, 130, 200
    X = rs.randn(F, T) + 1j * rs.randn(F, T)
    W = rs.gamma(1.0, 1.0, size=(F, K))
    H = rs.gamma(0.5, 1.0, size=(K, T))
    comp = [list(range(0, K, 2)), list(range(1, K, 2))]
    S = nmf.NMF_wiener_images(X, W, H, comp)
    assert rel(S, R.mono_wiener_images(X, W, H, comp)) < 1e-12
    w = np.hanning(256)
    y = nmf.NMF_separate_waveforms(X, W, H, comp, w, 64)
    assert rel(y[1], R.istft(R.mono_wiener_images(X, W, H, comp)[1], w, w, 64, 256)) < 1e-12
