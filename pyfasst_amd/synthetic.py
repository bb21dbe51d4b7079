"""Synthetic STFT-domain workloads of BASELINE.json.

C3: stereo, J sources, each an NMF power V_j = W_j H_j with K_true comps
(W ~ Gamma(2,1), H ~ Gamma(0.5,1)), rank-2 convolutive mixing
A_j(f) ~ CN(0,1), X = sum_j A_j s_j + CN(0, 1e-6 mean V), s_j ~ CN(0, V_j).
Host-side data generation only (outside every timed region).
"""
import numpy as np


def _cn(rs, shape, var):
    return (rs.standard_normal(shape) + 1j * rs.standard_normal(shape)) * np.sqrt(var / 2.)


def stereo_mixture(F, T, J=4, K_true=8, rank=2, seed=0, dtype=np.complex128):
    """Channel STFTs X [2, F, T] of a random convolutive NMF mixture."""
    rs = np.random.RandomState(seed)
    X = np.zeros((2, F, T), dtype=dtype)
    vsum = 0.0
    for j in range(J):
        W = rs.gamma(2.0, 1.0, size=(F, K_true))
        H = rs.gamma(0.5, 1.0, size=(K_true, T))
        V = W @ H
        vsum += V.mean()
        A = _cn(rs, (rank, 2, F), 1.0)
        for r in range(rank):
            s = _cn(rs, (F, T), V)
            X[0] += A[r, 0][:, None] * s
            X[1] += A[r, 1][:, None] * s
        del V
    noise_var = 1e-6 * vsum / J
    X[0] += _cn(rs, (F, T), noise_var)
    X[1] += _cn(rs, (F, T), noise_var)
    return X


def mono_stft(F, T, J=2, K_true=32, seed=0):
    """Complex STFT X [F, T] of a mono NMF mixture (config C2):
    X ~ CN(0, sum_j W_j H_j), W ~ Gamma(2, 1), H ~ Gamma(0.5, 1)."""
    rs = np.random.RandomState(seed)
    V = np.zeros((F, T))
    for _ in range(J):
        V += rs.gamma(2.0, 1.0, size=(F, K_true)) @ rs.gamma(0.5, 1.0, size=(K_true, T))
    return _cn(rs, (F, T), V)


def mono_mixture(F, T, J=2, K_true=32, seed=0):
    """Power spectrogram SX = |X|^2 [F, T] of mono_stft (config C2)."""
    return np.abs(mono_stft(F, T, J, K_true, seed)) ** 2
