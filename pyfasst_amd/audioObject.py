"""Audio I/O (audioObject.py of the reference, its scipy.io.wavfile branch).

`AudioObject` is a lazily loaded WAV file whose samples are exposed divided
by max(1.1 max|x|, 1e-10) (audioObject.py:112-127), the scale the FASST model
code relies on; writing multiplies it back and picks the integer encoding as
the reference's `wavwrite` does (:83-98).  `SpectralAudio` is an addition: an
in-memory observation given directly in the STFT domain (channel STFTs X or
the packed covariance Cx), used for the synthetic STFT-domain benchmarks of
BASELINE.json.
"""
import warnings

import numpy as np
import scipy.io.wavfile as wav

from .tools.utils import nextpow2, sinebell, hann  # noqa: F401 (re-exported like the reference)

_INT_ENCODINGS = ('int16', 'int32', 'int8')


def _smallest_int_encoding(data):
    """The narrowest of int8 / int16 / int32 whose range the peak needs
    (thresholds 2**7 and 2**15, as the reference's wavwrite)."""
    peak = np.abs(data).max()
    for limit, enc in ((2 ** 15, 'int32'), (2 ** 7, 'int16')):
        if peak > limit:
            return enc
    return 'int8'


def wavread(filename, first=0, last=None):
    """(sample rate, samples[first:last], their dtype)."""
    rate, samples = wav.read(filename)
    samples = samples[first:last]
    return rate, samples, samples.dtype


def wavwrite(filename, rate, data, formattype='wav', formatenc='int16', formatend='file'):
    """Write `data` cast to `formatenc`; an encoding other than the three
    integer ones is replaced by the narrowest that holds the peak."""
    enc = formatenc if formatenc in _INT_ENCODINGS else _smallest_int_encoding(data)
    wav.write(filename, rate, np.array(data, dtype=enc))
    return 0


class AudioObject(object):
    """A WAV file read on first access to its data, rate or shape."""

    def __init__(self, filename, mode='rw'):
        self.filename = filename
        self.mode = mode

    # -- file access -------------------------------------------------------
    def _read(self):
        if 'r' not in self.mode:
            raise ValueError("Not in read mode.")
        rate, samples, enc = wavread(self.filename)
        self._samplerate, self._encoding = rate, enc
        self._nframes = samples.shape[0] if samples.ndim == 2 else samples.size
        self._channels = samples.shape[1] if samples.ndim == 2 else 1
        self._maxdata = np.maximum(1.1 * np.abs(samples).max(), 1e-10)
        self._data = samples / self._maxdata

    def _write(self):
        if 'w' not in self.mode:
            raise ValueError("Not in write mode.")
        if not (hasattr(self, '_samplerate') or hasattr(self, '_data')):
            raise AttributeError("Should set sample rate and have data in write mode.")
        wavwrite(filename=self.filename, rate=self._samplerate,
                 data=self._data * self._maxdata, formatenc=self._encoding)

    def _loaded(self, attr):
        if not hasattr(self, attr):
            self._read()
        return getattr(self, attr)

    # -- samples -------------------------------------------------------------
    def _get_data(self):
        return self._loaded('_data')

    def _set_data(self, data):
        rows, cols = data.shape[0], data.shape[1]
        # frames are rows: a wide array of more than two rows is transposed
        arr = np.array(data.T if (rows < cols and cols > 2) else data, order='C')
        self._encoding = arr.dtype.name
        self._maxdata = 1.1 * np.abs(arr).max()
        self._data = arr / self._maxdata

    def _del_data(self):
        self.__dict__.pop('_data', None)

    data = property(_get_data, _set_data, _del_data)

    # -- sample rate ---------------------------------------------------------
    def _get_samplerate(self):
        if 'r' in self.mode:
            return self._loaded('_samplerate')
        return self._samplerate

    def _set_samplerate(self, samplerate):
        if 'r' in self.mode:
            warnings.warn("Changing the sampling rate in read mode")
        self._samplerate = int(samplerate)

    samplerate = property(_get_samplerate, _set_samplerate)
    fs = samplerate

    # -- shape ---------------------------------------------------------------
    channels = property(lambda self: self._loaded('_channels'))
    nframes = property(lambda self: self._loaded('_nframes'))


class SpectralAudio(AudioObject):
    """Observation given in the STFT domain (no waveform).

    X: complex [C, F, T] channel STFTs (enables Wiener images), or
    Cx: complex [3, F, T] packed covariance (EM only).
    """

    def __init__(self, X=None, Cx=None, samplerate=44100, filename='spectral.wav'):
        super(SpectralAudio, self).__init__(filename, mode='r')
        if X is None and Cx is None:
            raise AttributeError("SpectralAudio needs X or Cx")
        self.X = None if X is None else np.asarray(X, dtype=np.complex128)
        self.Cx = None if Cx is None else np.asarray(Cx, dtype=np.complex128)
        self._samplerate = int(samplerate)
        self._channels = 2 if X is None else self.X.shape[0]
        shp = (self.X if X is not None else self.Cx).shape
        self.nbFreqs, self.nbFrames = shp[1], shp[2]
        self._nframes = 0
        self._maxdata = 1.0

    def _read(self):
        raise AttributeError("SpectralAudio has no waveform")
