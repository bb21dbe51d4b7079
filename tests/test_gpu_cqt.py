"""CQT / MinQT front and back end on the GPU vs the reference and the oracle.

tests/golden/cqt.npz holds the reference's own outputs (tftransforms/minqt.py,
perfRast=1 as FASST builds it) for five geometries: MinQT with 12/24/48 bins
per octave (winNr = 1), CQT with several atoms per FFT frame (winNr = 5 and
3), hop factors 1/16 .. 1/2.  The GPU path is FP64 end to end; it differs
from NumPy by FFT algorithm (radix-2 in LDS vs pocketfft) and summation
order only, so it is held to 1e-10 of the largest magnitude.
"""
import numpy as np
import pytest

import cqt_ref
from helpers import CQT_CASES, load, rel

pytestmark = pytest.mark.gpu

TOL = 1e-10


def _product(kind, kw):
    from pyfasst_amd.tftransforms import minqt
    if kind == 'mqt':
        return minqt.MinQTransfo(perfRast=1, **kw)
    return minqt.CQTransfo(perfRast=1, **kw)


@pytest.mark.parametrize("name,kind,kw", CQT_CASES, ids=[c[0] for c in CQT_CASES])
def test_cqt_golden_gpu(name, kind, kw):
    g = load("cqt")
    t = _product(kind, kw)
    t.computeTransform(g['x'])
    X = t.transfo
    assert X.shape == g['X_' + name].shape
    np.testing.assert_array_equal(np.array(t.nframes), g['nframes_' + name])
    np.testing.assert_array_equal(t.freq_stamps, g['freqs_' + name])
    assert rel(X, g['X_' + name]) < TOL
    assert rel(np.abs(X), np.abs(g['X_' + name])) < TOL
    # inverse of the same spCQT (transfo setter -> invertTransform, as FASST's
    # separate_comps does, audioModel.py:1196-1203)
    t.transfo = g['X_' + name]
    y = t.invertTransform()
    assert y.shape == g['y_' + name].shape
    assert rel(y, g['y_' + name]) < TOL


def test_cell_view_matches_reference_cells():
    """spCQT2CellCQT (pure re-indexing) against the oracle's cells."""
    g = load("cqt")
    for name, kind, kw in CQT_CASES:
        t = _product(kind, kw)
        o = cqt_ref.RefCQT(kind, **kw)
        o.forward(g['x'])
        t.computeTransform(g['x'])
        t.transfo = g['X_' + name]
        cells = t.spCQT2CellCQT()
        for noct in range(int(o.octaveNr)):
            np.testing.assert_array_equal(cells[noct], o.sp_to_cell(g['X_' + name], noct))
        if kind == 'mqt':
            np.testing.assert_array_equal(cells['linear'], o.linear_cell(g['X_' + name]))


@pytest.mark.parametrize("fs,wlen,hop,secs", [
    (44100, 2048, 512, 6.0),    # FASST defaults: tfbpo 48, tffmin 25, 6 octaves, FFTLen 4096
    (44100, 4096, 512, 3.0),    # FFTLen 8192 (128 KB of LDS per frame)
])
def test_minqt_fasst_defaults_vs_oracle(fs, wlen, hop, secs):
    """MinQT as FASST builds it at 44.1 kHz (audioModel.py:206-214), seconds of
    audio, against the oracle restatement (forward and inverse)."""
    rs = np.random.RandomState(5)
    n = int(fs * secs)
    x = rs.randn(n) * np.sin(np.arange(n) / 5000.0) ** 2
    kw = dict(fmin=25, fmax=18000, bins=48, fs=fs, linFTLen=wlen, atomHopFactor=hop / float(wlen))
    t = _product('mqt', kw)
    t.computeTransform(x)
    o = cqt_ref.RefCQT('mqt', **kw)
    Xo = o.forward(x)
    assert t.transfo.shape == Xo.shape
    assert rel(t.transfo, Xo) < TOL
    y = t.invertTransform()
    yo = o.inverse(Xo)
    assert rel(y, yo) < TOL


def test_cqt_short_signal_raises():
    """A signal too short for the lowest octave's frames: the reference fails
    (negative nframes); the GPU path raises ValueError."""
    t = _product('cqt', dict(fmin=30, fmax=3000, bins=12, fs=8000, atomHopFactor=0.25))
    with pytest.raises(ValueError):
        t.computeTransform(np.zeros(0))


def test_filtfilt_matches_scipy_exactly_in_the_lowest_octaves():
    """The chunked filtfilt reproduces scipy's lfilter arithmetic: a CQT whose
    lowest octaves went through 6 filtfilt/decimation stages still matches the
    oracle (scipy) to 1e-10 of the peak, including the first frames."""
    rs = np.random.RandomState(9)
    x = rs.randn(30000)
    kw = dict(fmin=40, fmax=3500, bins=12, fs=8000, atomHopFactor=0.25)
    t = _product('cqt', kw)
    t.computeTransform(x)
    o = cqt_ref.RefCQT('cqt', **kw)
    Xo = o.forward(x)
    lo = slice(0, 12)          # rows of the lowest octave
    assert rel(t.transfo[lo], Xo[lo]) < TOL
    assert rel(t.transfo[lo, :40], Xo[lo, :40]) < TOL
