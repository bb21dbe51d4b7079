"""Window functions and helpers (tools/utils.py:12-72 of the reference).

Host-side parameter generators only; no signal compute happens here.
"""
import numpy as np


def db(val):
    """10 log10(val) (utils.py:16-22)."""
    return 10 * np.log10(val)


def ident(energy):
    """identity (utils.py:24-27)."""
    return energy


def nextpow2(i):
    """smallest power of two >= i, starting at 2 (utils.py:29-39)."""
    n = 2
    while n < i:
        n = n * 2
    return n


def sinebell(lengthWindow):
    """sin(pi t / L), t = 0..L-1 (utils.py:41-53)."""
    return np.sin((np.pi * (np.arange(lengthWindow))) / (1.0 * lengthWindow))


def hann(args):
    """numpy's Hann window (utils.py:55-61)."""
    return np.hanning(args)


def sqrt_blackmanharris(M):
    """sqrt of scipy's Blackman-Harris window (utils.py:63-69)."""
    import scipy.signal as spsig
    return np.sqrt(spsig.windows.blackmanharris(M))
