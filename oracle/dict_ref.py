"""CPU restatement of the SIMM dictionary generators (source and filter bases).

TEST INFRASTRUCTURE ONLY (the checker, never the product): imported by
tests/ and bench legs; the product package `pyfasst_amd` never imports it.

Restates SeparateLeadStereo/separateLeadFunctions.py:
  generate_ODGD_spec          :888-949   KLGLOTT88 glottal source as a
                                         harmonic sum, one F0
  generate_ODGD_spec_chirped  :1010-1072 the same with a linear F0 glide
  generate_WF0_TR_chirped     :696-886   WF0 = |transform(odgd)[:, mid]|^2
                                         for every F0 (and chirp), with the
                                         STFT transform SeparateLeadProcess.
                                         computeWF0 builds for
                                         tfrepresentation='stft'
                                         (SeparateLeadStereoTF.py:646-681)
  generateHannBasis           :1074-1146 WGAMMA, overlapping Hann bumps

As in the reference (numpy of its era): the odgd is complex and the STFT's
rfft discards its imaginary part (here: np.real before the rfft); the
analysis spectra odgdSpectrum are computed but unused by
generate_WF0_TR_chirped (not restated).  Pinned against tests/golden/wf0.npz.
"""
import numpy as np

import fasst_ref


def odgd_amplitudes(F0, Ot, partialMax):
    """KLGLOTT88 partial amplitudes (separateLeadFunctions.py:916-930)."""
    frequency_numbers = np.arange(1, partialMax + 1)
    temp_array = 1j * 2.0 * np.pi * frequency_numbers * Ot
    return (F0 * 27 / 4 * (np.exp(-temp_array) + (2 * (1 + 2 * np.exp(-temp_array)) / temp_array) -
                           (6 * (1 - np.exp(-temp_array)) / (temp_array ** 2))) / temp_array)


def generate_odgd(F0, Fs, lengthOdgd=2048, Ot=0.5, t0=0.0):
    """generate_ODGD_spec's time signal (:888-945)."""
    F0, Fs, Ot, t0 = np.double(F0), np.double(Fs), np.double(Ot), np.double(t0)
    partialMax = np.floor((Fs / 2) / F0)
    frequency_numbers = np.arange(1, partialMax + 1)
    amplitudes = odgd_amplitudes(F0, Ot, partialMax)
    timeStamps = np.arange(lengthOdgd) / Fs + t0 / F0
    odgd = (np.exp(np.outer(2.0 * 1j * np.pi * F0 * frequency_numbers, timeStamps)) *
            np.outer(amplitudes, np.ones(lengthOdgd)))
    return np.sum(odgd, axis=0)


def generate_odgd_chirped(F1, F2, Fs, lengthOdgd=2048, Ot=0.5, t0=0.0):
    """generate_ODGD_spec_chirped's time signal (:1010-1067)."""
    F1, F2 = np.double(F1), np.double(F2)
    F0 = np.double(F1 + F2) / 2.0
    Fs, Ot, t0 = np.double(Fs), np.double(Ot), np.double(t0)
    partialMax = np.floor((Fs / 2) / np.max([F1, F2]))
    frequency_numbers = np.arange(1, partialMax + 1)
    amplitudes = odgd_amplitudes(F0, Ot, partialMax)
    timeStamps = np.arange(lengthOdgd) / Fs + t0 / F0
    odgd = (np.exp(2.0 * 1j * np.pi * (np.outer(F1 * frequency_numbers, timeStamps) +
                                       np.outer((F2 - F1) * frequency_numbers, timeStamps ** 2) /
                                       (2 * lengthOdgd / Fs))) *
            np.outer(amplitudes, np.ones(lengthOdgd)))
    return np.sum(odgd, axis=0)


def f0_table(minF0, maxF0, stepNotes):
    """(:803-806)"""
    minF0, maxF0, stepNotes = np.double(minF0), np.double(maxF0), np.double(stepNotes)
    numberOfF0 = np.ceil(12.0 * stepNotes * np.log2(maxF0 / minF0)) + 1
    return minF0 * (2 ** (np.arange(numberOfF0, dtype=np.double) / (12 * stepNotes)))


def stft_mid_frame_power(odgd, window, hop, nfft, fs):
    """|STFT(odgd)[:, midindex]|^2 with the STFT class of tftransforms/stft.py
    (:339-394): midindex = argmin((L/2 - time_stamps)^2) (:845-847)."""
    L = odgd.size
    X = fasst_ref.stft(np.real(odgd), window, hop, nfft)
    time_stamps = np.arange(X.shape[1]) * hop / np.double(fs)
    time_stamps *= fs
    midindex = np.argmin((L / 2. - time_stamps) ** 2)
    return np.abs(X[:, midindex]) ** 2


def generate_wf0_tr_chirped_stft(ftlen, hop, window, fs, minF0, maxF0, stepNotes=4, Ot=0.5,
                                 perF0=1, depthChirpInSemiTone=0.5):
    """generate_WF0_TR_chirped (:696-886) with an STFT transform of ftlen bins
    (freqbins = ftlen/2 + 1, lengthWindow = (freqbins - 1) * 4)."""
    freqbins = ftlen // 2 + 1
    lengthWindow = (freqbins - 1) * 2 * 2
    F0Table = f0_table(minF0, maxF0, stepNotes)
    numberOfF0 = F0Table.size
    WF0 = np.zeros([freqbins, int(numberOfF0 * perF0)])
    for i in range(numberOfF0):
        odgd = generate_odgd(F0Table[i], fs, lengthOdgd=lengthWindow, Ot=Ot)
        WF0[:, i * perF0] = stft_mid_frame_power(odgd, window, hop, ftlen, fs)
        for c in range(perF0 - 1):
            F2 = F0Table[i] * (2 ** ((c + 1.0) * depthChirpInSemiTone / (12.0 * (perF0 - 1.0))))
            F1 = 2.0 * F0Table[i] - F2
            odgd = generate_odgd_chirped(F1, F2, fs, lengthOdgd=lengthWindow, Ot=Ot)
            WF0[:, i * perF0 + c + 1] = stft_mid_frame_power(odgd, window, hop, ftlen, fs)
    return F0Table, WF0


def generate_wf0_tr_chirped_cqt(t, minF0, maxF0, stepNotes=4, Ot=0.5, perF0=1,
                                depthChirpInSemiTone=0.5):
    """generate_WF0_TR_chirped (:696-886) with a CQT-type transform t
    (cqt_ref.RefCQT): lengthWindow = FFTLen * 2^(octaveNr - 1) (:742-744), the
    complex comb through the transform, |transfo[:, midindex]|^2 with
    midindex = argmin((datalen_init / 2 - time_stamps)^2) (:836-843) and the
    time stamps of minqt.py:676-689."""
    k = t.k
    fs = t.fs
    lengthWindow = int(k.FFTLen * (2 ** (t.octaveNr - 1)))
    F0Table = f0_table(minF0, maxF0, stepNotes)
    numberOfF0 = F0Table.size
    WF0 = np.zeros([int(t.freqbins), int(numberOfF0 * perF0)])

    def mid_power(odgd):
        sp = t.forward(odgd)
        time_stamps = (np.arange(t.nframes[0] * k.winNr) * k.atomHOP +
                       k.first_center * 2 ** (t.octaveNr - 1) - t.prefixZeros)
        midindex = np.argmin((t.datalen_init / 2. - time_stamps) ** 2)
        return np.abs(sp[:, midindex]) ** 2
    for i in range(numberOfF0):
        WF0[:, i * perF0] = mid_power(generate_odgd(F0Table[i], fs, lengthOdgd=lengthWindow, Ot=Ot))
        for c in range(perF0 - 1):
            F2 = F0Table[i] * (2 ** ((c + 1.0) * depthChirpInSemiTone / (12.0 * (perF0 - 1.0))))
            F1 = 2.0 * F0Table[i] - F2
            WF0[:, i * perF0 + c + 1] = mid_power(
                generate_odgd_chirped(F1, F2, fs, lengthOdgd=lengthWindow, Ot=Ot))
    return F0Table, WF0


def generate_hann_basis(numberFrequencyBins, sizeOfFourier, Fs, frequencyScale='linear',
                        numberOfBasis=20, overlap=.75):
    """generateHannBasis (:1074-1146), linear scale."""
    if frequencyScale != 'linear':
        return 0
    numberOfWindowsForUnit = np.ceil(1.0 / (1.0 - overlap))
    overlap = 1.0 - 1.0 / np.double(numberOfWindowsForUnit)
    lengthSineWindow = np.ceil(numberFrequencyBins / ((1.0 - overlap) * (numberOfBasis - 1) + 1 -
                                                      2.0 * overlap))
    lengthSineWindow = 2.0 * np.floor(lengthSineWindow / 2.0)
    mappingFrequency = np.arange(numberFrequencyBins)
    sizeBigWindow = 2.0 * numberFrequencyBins
    firstWindowCenter = -numberOfWindowsForUnit + 1
    lastWindowCenter = numberOfBasis - numberOfWindowsForUnit + 1
    sineCenters = np.round(np.arange(firstWindowCenter, lastWindowCenter) * (1 - overlap) *
                           np.double(lengthSineWindow) + lengthSineWindow / 2.0)
    prototypeSineWindow = np.hanning(int(lengthSineWindow))
    bigWindow = np.zeros([int(sizeBigWindow * 2), 1])
    bigWindow[int(sizeBigWindow - lengthSineWindow / 2.0):
              int(sizeBigWindow + lengthSineWindow / 2.0)] = np.vstack(prototypeSineWindow)
    WGAMMA = np.zeros([numberFrequencyBins, numberOfBasis])
    for p in np.arange(numberOfBasis):
        WGAMMA[:, p] = np.hstack(bigWindow[np.int32(mappingFrequency - sineCenters[p] +
                                                    sizeBigWindow)])
    return WGAMMA
