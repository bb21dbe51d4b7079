"""Audio I/O (audioObject.py of the reference, scipy.io.wavfile branch).

`AudioObject` reads a WAV and rescales it by max(1.1*max|x|, 1e-10)
(audioObject.py:112-127); `_write` mirrors wavwrite's encoding choice
(:83-98).  `SpectralAudio` is an addition: an in-memory observation given
directly in the STFT domain (channel STFTs X or the packed covariance Cx),
used for the synthetic STFT-domain benchmarks of BASELINE.json.
"""
import warnings

import numpy as np
import scipy.io.wavfile as wav

from .tools.utils import nextpow2, sinebell, hann  # noqa: F401 (re-exported like the reference)


def wavread(filename, first=0, last=None):
    fs, data = wav.read(filename)
    data = data[first:last]
    return fs, data, data.dtype


def wavwrite(filename, rate, data, formattype='wav', formatenc='int16', formatend='file'):
    if formatenc not in ('int16', 'int32', 'int8'):
        if np.abs(data).max() > 2 ** 15:
            formatenc = 'int32'
        elif np.abs(data).max() > 2 ** 7:
            formatenc = 'int16'
        else:
            formatenc = 'int8'
    wav.write(filename, rate, np.array(data, dtype=formatenc))
    return 0


class AudioObject(object):
    def __init__(self, filename, mode='rw'):
        self.filename = filename
        self.mode = mode

    def _read(self):
        if 'r' not in self.mode:
            raise ValueError("Not in read mode.")
        self._samplerate, self._data, self._encoding = wavread(self.filename)
        if len(self._data.shape) == 2:
            self._nframes, self._channels = self._data.shape
        else:
            self._nframes = self._data.size
            self._channels = 1
        self._maxdata = np.maximum(1.1 * np.abs(self._data).max(), 1e-10)
        self._data = self._data / self._maxdata

    def _write(self):
        if 'w' not in self.mode:
            raise ValueError("Not in write mode.")
        if not hasattr(self, '_samplerate') and not hasattr(self, '_data'):
            raise AttributeError("Should set sample rate and have data in write mode.")
        wavwrite(filename=self.filename, rate=self._samplerate,
                 data=self._maxdata * self._data, formatenc=self._encoding)

    def _set_data(self, data):
        s = data.shape
        if s[0] < s[1] and s[1] > 2:
            self._data = np.array(data.T, order='C')
        else:
            self._data = np.array(data, order='C')
        self._maxdata = 1.1 * np.abs(self._data).max()
        self._encoding = self._data.dtype.name
        self._data = self._data / self._maxdata

    def _get_data(self):
        if not hasattr(self, '_data'):
            self._read()
        return self._data

    def _del_data(self):
        if hasattr(self, '_data'):
            del self._data

    data = property(_get_data, _set_data, _del_data)

    def _get_samplerate(self):
        if not hasattr(self, '_samplerate') and 'r' in self.mode:
            self._read()
        return self._samplerate

    def _set_samplerate(self, samplerate):
        if 'r' in self.mode:
            warnings.warn("Changing the sampling rate in read mode")
        self._samplerate = int(samplerate)

    samplerate = property(_get_samplerate, _set_samplerate)
    fs = samplerate

    @property
    def channels(self):
        if not hasattr(self, '_channels'):
            self._read()
        return self._channels

    @property
    def nframes(self):
        if not hasattr(self, '_nframes'):
            self._read()
        return self._nframes


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
