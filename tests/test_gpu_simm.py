"""SIMM / Stereo_SIMM on the MI355X vs the reference's golden vectors and the
CPU oracle (oracle/simm_ref.py; SIMM.py:46-943).

All compute goes through libfasst_hip.so (include/fasst_simm.h).  The FP64
GEMMs sum in a different order from NumPy/OpenBLAS, so results agree to
rounding, not bit-for-bit; TOL is the relative bound (max-normalised) held on
every returned parameter.
"""
import numpy as np
import pytest

import simm_ref
from helpers import load, rel

pytestmark = pytest.mark.gpu

TOL = 1e-9
ST_NAMES = ['alphaR', 'alphaL', 'HGAMMA', 'HPHI', 'HF0', 'betaR', 'betaL', 'HM', 'WM',
            'recoError']
MONO_NAMES = ['HGAMMA', 'HPHI', 'HF0', 'HM', 'WM', 'recoError']


def _S():
    from pyfasst_amd.SeparateLeadStereo.SIMM import SIMM as S
    return S


def _cmp(got, want, names, tol=TOL):
    for n, a, b in zip(names, got, want):
        assert np.shape(a) == np.shape(b), n
        assert rel(a, b) < tol, (n, rel(a, b))


def test_simm_native_library_loaded():
    from pyfasst_amd import _lib
    assert _lib.lib.simm_create is not None
    import pyfasst_amd.SeparateLeadStereo.SIMM.SIMM as mod
    assert mod._lib is _lib


def test_stereo_simm_golden():
    g = load("simm")
    S = _S()
    K, R = g['st_HGAMMA'].shape[1], g['st_HM'].shape[0]
    np.random.seed(1)
    out = S.Stereo_SIMM(g['SXR'], g['SXL'], g['WF0'], g['WGAMMA'], numberOfFilters=K,
                        numberOfAccompanimentSpectralShapes=R, numberOfIterations=4,
                        verbose=False)
    _cmp(out, [g['st_' + n] for n in ST_NAMES], ST_NAMES)


def test_stereo_simm_golden_compute_error_frozen_hgamma():
    g = load("simm")
    S = _S()
    K, R = g['st_HGAMMA'].shape[1], g['st_HM'].shape[0]
    np.random.seed(3)
    out = S.Stereo_SIMM(g['SXR'], g['SXL'], g['WF0'], g['WGAMMA'], numberOfFilters=K,
                        numberOfAccompanimentSpectralShapes=R, numberOfIterations=3,
                        updateRulePower=0.7, updateHGAMMA=False, computeError=True,
                        verbose=False)
    _cmp(out, [g['st2_' + n] for n in ST_NAMES], ST_NAMES)
    # the zero slots of recoError are zero exactly where the reference's are
    assert np.array_equal(out[-1] == 0, g['st2_recoError'] == 0)


@pytest.mark.parametrize("prefix,seed,R,n_iter", [("mono_", 2, 1, 4), ("monoN_", 4, None, 3)])
def test_mono_simm_golden(prefix, seed, R, n_iter):
    g = load("simm")
    S = _S()
    K = g['st_HGAMMA'].shape[1]
    R = g['SXR'].shape[1] if R is None else R
    np.random.seed(seed)
    out = S.SIMM(g['SXR'], g['WF0'], g['WGAMMA'], numberOfFilters=K,
                 numberOfAccompanimentSpectralShapes=R, numberOfIterations=n_iter, verbose=False)
    _cmp(out, [g[prefix + n] for n in MONO_NAMES], MONO_NAMES)


def _data(F, N, NF0, P, seed):
    rs = np.random.RandomState(seed)
    return (rs.gamma(0.8, 1.0, size=(F, N)), rs.gamma(0.8, 1.0, size=(F, N)),
            rs.gamma(1.0, 1.0, size=(F, NF0)), rs.gamma(1.0, 1.0, size=(F, P)))


# shapes that exercise ragged GEMM tiles and the split-K paths (F = 1025
# splits WF0^T X over f; N = 600 / 1300 split X HM^T over frames); R <= 48
# takes the fused skinny kernels (R = 40: the pipeline's numCompAccomp),
# R = 60 the materialised X, Y + general GEMM
SHAPES = [(257, 301, 97, 10, 4, 7), (1025, 130, 150, 12, 4, 10), (129, 600, 40, 5, 2, 3),
          (33, 17, 5, 3, 1, 1), (200, 1300, 30, 6, 2, 40), (97, 150, 20, 4, 2, 60),
          # K in (4, 8]: the 8-filter instantiations of the model-forming kernels
          (129, 333, 24, 7, 6, 48), (65, 90, 16, 5, 8, 52)]


@pytest.mark.parametrize("shape", SHAPES)
def test_stereo_simm_vs_oracle(shape):
    F, N, NF0, P, K, R = shape
    SXR, SXL, WF0, WG = _data(F, N, NF0, P, 5)
    S = _S()
    np.random.seed(7)
    got = S.Stereo_SIMM(SXR, SXL, WF0, WG, numberOfFilters=K,
                        numberOfAccompanimentSpectralShapes=R, numberOfIterations=5,
                        computeError=True, verbose=False)
    np.random.seed(7)
    want = simm_ref.stereo_simm(SXR, SXL, WF0, WG, K, R, numberOfIterations=5,
                                computeError=True)
    _cmp(got, want, ST_NAMES, tol=1e-8)


# The NF0-sized plain products (SF0 = WF0 HF0, WF0^T [num | den]) run on the
# hand-written k_dgemm2 by default (every test above, odd NF0 and odd N
# included: operands whose rows are not 16-byte aligned take its 4-byte load
# variant); FASST_SIMM_GEMM=2 selects the generic k_gemm, held to the same
# oracle.  The variable is read when the SIMM context is created.
@pytest.mark.parametrize("shape", [SHAPES[1], SHAPES[2]])
def test_stereo_simm_kgemm_path_vs_oracle(monkeypatch, shape):
    monkeypatch.setenv("FASST_SIMM_GEMM", "2")
    test_stereo_simm_vs_oracle(shape)


@pytest.mark.parametrize("shape", SHAPES[:2] + SHAPES[6:7])
def test_mono_simm_vs_oracle(shape):
    F, N, NF0, P, K, _ = shape
    SX, _, WF0, WG = _data(F, N, NF0, P, 6)
    S = _S()
    np.random.seed(8)
    got = S.SIMM(SX, WF0, WG, numberOfFilters=K, numberOfAccompanimentSpectralShapes=1,
                 numberOfIterations=5, verbose=False)
    np.random.seed(8)
    want = simm_ref.simm(SX, WF0, WG, K, 1, numberOfIterations=5)
    _cmp(got, want, MONO_NAMES, tol=1e-8)


def test_simm_given_initial_parameters_and_wrong_shapes():
    F, N, NF0, P, K, R = 65, 40, 24, 6, 3, 5
    SXR, SXL, WF0, WG = _data(F, N, NF0, P, 9)
    rs = np.random.RandomState(3)
    HG0, HPHI0, HF00 = rs.rand(P, K), rs.rand(K, N), rs.rand(NF0, N)
    S = _S()
    # a wrong-shaped WM0 is replaced by a random draw, as in the reference
    np.random.seed(5)
    got = S.Stereo_SIMM(SXR, SXL, WF0, WG, numberOfFilters=K,
                        numberOfAccompanimentSpectralShapes=R, HGAMMA0=HG0, HPHI0=HPHI0,
                        HF00=HF00, WM0=np.ones((F + 1, R)), numberOfIterations=3, verbose=False)
    np.random.seed(5)
    want = simm_ref.stereo_simm(SXR, SXL, WF0, WG, K, R, HGAMMA0=HG0, HPHI0=HPHI0, HF00=HF00,
                                WM0=np.ones((F + 1, R)), numberOfIterations=3)
    _cmp(got, want, ST_NAMES)


def test_simm_edge_cases():
    S = _S()
    SXR, SXL, WF0, WG = _data(33, 20, 6, 3, 1)
    # N7: mono HM *= sumWM only broadcasts for R == 1 or R == N
    with pytest.raises(ValueError):
        S.SIMM(SXR, WF0, WG, numberOfAccompanimentSpectralShapes=3, numberOfIterations=1)
    with pytest.raises(ValueError):
        S.Stereo_SIMM(SXR, SXL[:, :-1], WF0, WG, numberOfIterations=1)
    # WF0 with the wrong number of bins: the reference returns False
    assert S.Stereo_SIMM(SXR, SXL, WF0[:-1], WG, numberOfIterations=1) is False
    # zero iterations: the initial parameters come back unchanged
    np.random.seed(2)
    out = S.Stereo_SIMM(SXR, SXL, WF0, WG, numberOfFilters=2, numberOfIterations=0)
    np.random.seed(2)
    want = simm_ref.stereo_simm(SXR, SXL, WF0, WG, 2, 10, numberOfIterations=0)
    _cmp(out, want, ST_NAMES, tol=0.0 + 1e-300)


@pytest.mark.parametrize("shape", [SHAPES[1], SHAPES[6]])
def test_mono_simm_kgemm_vs_oracle(monkeypatch, shape):
    monkeypatch.setenv("FASST_SIMM_GEMM", "2")
    test_mono_simm_vs_oracle(shape)
