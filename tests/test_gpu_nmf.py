"""IS-NMF (tools/nmf.py:24-159) on the MI355X vs the reference's golden
vectors and the CPU oracle.  Compute goes through libfasst_hip.so
(include/fasst_nmf.h); GEMM summation order differs from OpenBLAS, so the
bound is relative (max-normalised) rounding agreement, TOL.
"""
import numpy as np
import pytest

import fasst_ref as R
from helpers import load, rel

pytestmark = pytest.mark.gpu

TOL = 1e-10


def _nmf():
    import pyfasst_amd.tools.nmf as nmf
    return nmf


def test_nmf_decomposition_golden():
    g = load("nmf")
    np.random.seed(1)
    W, H = _nmf().NMF_decomposition(g['SX'], nbComps=6, niter=7)
    assert rel(W, g['W']) < TOL and rel(H, g['H']) < TOL, (rel(W, g['W']), rel(H, g['H']))


def test_nmf_decomp_init_golden():
    g = load("nmf")
    nmf = _nmf()
    np.random.seed(2)
    W, H = nmf.NMF_decomp_init(g['SX'], nbComps=5, niter=6)
    assert rel(W, g['di_W']) < TOL and rel(H, g['di_H']) < TOL
    np.random.seed(3)
    W, H = nmf.NMF_decomp_init(g['SX'], nbComps=4, niter=5, Winit=g['Winit'], updateW=False)
    assert np.array_equal(W, g['dw_W'])          # frozen: returned untouched
    assert rel(H, g['dw_H']) < TOL
    np.random.seed(4)
    W, H = nmf.NMF_decomp_init(g['SX'], nbComps=4, niter=5, Hinit=g['Hinit'])
    assert rel(W, g['dh_W']) < TOL and rel(H, g['dh_H']) < TOL
    with pytest.raises(AttributeError):
        nmf.NMF_decomp_init(g['SX'], nbComps=4, niter=1, Hinit=np.ones((3, 3)))


# config 2 (F=1025, T=2000, K=64: fused contractions), ragged tiles on the
# fused path (K=16, 32, 48), the GEMM path (K=13, 80) and a single component
@pytest.mark.parametrize("F,N,K,niter", [(1025, 2000, 64, 3), (257, 301, 13, 6), (33, 17, 1, 4),
                                         (65, 40, 32, 4), (130, 77, 16, 3), (47, 211, 48, 3),
                                         (100, 90, 80, 2)])
def test_nmf_vs_oracle(F, N, K, niter):
    rs = np.random.RandomState(F + N)
    SX = rs.gamma(0.7, 1.0, size=(F, N)) * np.outer(rs.gamma(2, 1, F), np.ones(N))
    np.random.seed(5)
    W, H = _nmf().NMF_decomposition(SX, nbComps=K, niter=niter)
    np.random.seed(5)
    Wr, Hr = R.nmf_decomposition(SX, nbComps=K, niter=niter)
    assert rel(W, Wr) < 1e-9 and rel(H, Hr) < 1e-9, (rel(W, Wr), rel(H, Hr))
    # no H update
    np.random.seed(6)
    W, H = _nmf().NMF_decomp_init(SX, nbComps=K, niter=2, updateH=False)
    np.random.seed(6)
    Wr, Hr = R.nmf_decomp_init(SX, nbComps=K, niter=2, updateH=False)
    assert rel(W, Wr) < 1e-9 and rel(H, Hr) < 1e-9   # (H still takes the W column scale)


# frozen W on the fused path (K % 16 == 0, K <= 64: no W rescale, the H
# numerator kernel runs without the column-scale operand), ragged F and N
@pytest.mark.parametrize("F,N,K", [(131, 77, 16), (257, 203, 32), (90, 301, 64)])
def test_nmf_frozen_w_fused_vs_oracle(F, N, K):
    rs = np.random.RandomState(F * N)
    SX = rs.gamma(0.7, 1.0, size=(F, N))
    Winit = rs.gamma(1.0, 1.0, size=(F, K))
    np.random.seed(9)
    W, H = _nmf().NMF_decomp_init(SX, nbComps=K, niter=4, Winit=Winit, updateW=False)
    np.random.seed(9)
    Wr, Hr = R.nmf_decomp_init(SX, nbComps=K, niter=4, Winit=Winit, updateW=False)
    assert np.array_equal(W, Winit)
    assert rel(H, Hr) < 1e-9, rel(H, Hr)
