"""The whole lead/accompaniment pipeline on the GPU vs the reference.

SeparateLeadProcess(wav, ...).autoMelSepAndWrite(maxFrames=60) on the seeded
stereo signal of tests/golden/pipeline.npz (143 frames, 3 chunks): source
dictionary, chunked mono SIMM, Viterbi melody, chunked stereo SIMM with
per-chunk masks, overlap-add of the chunk WAVs (SeparateLeadStereoTF.py:
263-1897).  The melody path is integer output and must match exactly; the
separated int16 WAVs within a couple of LSB (FP64 SIMM updates and FFTs in a
different order than NumPy's).
"""
import os

import numpy as np
import pytest
import scipy.io.wavfile as wf

from helpers import load, rel

pytestmark = pytest.mark.gpu


def test_auto_melody_separation_vs_reference(tmp_path, monkeypatch):
    from pyfasst_amd.SeparateLeadStereo import SeparateLeadStereoTF as SL
    monkeypatch.chdir(tmp_path)
    g = load("pipeline")
    wav = os.path.join(str(tmp_path), "mix.wav")
    wf.write(wav, int(g['fs']), g['wav'])
    np.random.seed(3)
    proc = SL.SeparateLeadProcess(wav, windowSize=0.0464, nbIter=3, numCompAccomp=6, minF0=100,
                                  maxF0=800, stepNotes=4, K_numFilters=3, P_numAtomFilters=10,
                                  verbose=False, outputDirSuffix='out')
    np.testing.assert_array_equal(proc.SIMMParams['F0Table'], g['F0Table'])
    assert rel(proc.SIMMParams['WF0'], g['WF0']) < 1e-10
    np.testing.assert_array_equal(proc.SIMMParams['WGAMMA'], g['WGAMMA'])
    proc.autoMelSepAndWrite(maxFrames=60)
    assert int(proc.totFrames) == int(g['totFrames'])
    np.testing.assert_array_equal(proc.indexBestPath, g['indexBestPath'])
    np.testing.assert_array_equal(proc.freqMelody, g['freqMelody'])
    np.testing.assert_allclose(np.loadtxt(proc.files['pitch_output_file']), g['pitches'])
    assert rel(proc.SIMMParams['HF00'], g['HF00']) < 1e-8
    for key, ref in (('voc_output_file', g['lead']), ('mus_output_file', g['acc'])):
        y = wf.read(proc.files[key])[1].astype(np.int64)
        assert y.shape == ref.shape
        assert np.max(np.abs(y - ref.astype(np.int64))) <= 2


def test_auto_melody_separation_mqt_vs_reference(tmp_path, monkeypatch):
    """tfrepresentation='mqt' (the reference's MinQTSLStest,
    pyfasst_tests/pyfasst/SeparateLeadStereo/test_SeparateLeadStereoTF.py:40-47):
    WF0 on the MinQT, MinQT geometry (hop = atomHOP, window = FFTLen *
    2^(octaveNr-1)), startincqt realignment of each chunk, MinQT inverse of
    the masked chunks and the sine-bell^2 overlap-add; 315 frames, 3 chunks
    of 140, 140, 35
    (tests/golden/pipeline_mqt.npz)."""
    from pyfasst_amd.SeparateLeadStereo import SeparateLeadStereoTF as SL
    monkeypatch.chdir(tmp_path)
    g = load("pipeline_mqt")
    wav = os.path.join(str(tmp_path), "mix.wav")
    wf.write(wav, int(g['fs']), g['wav'])
    np.random.seed(3)
    proc = SL.SeparateLeadProcess(wav, windowSize=0.0464, nbIter=3, numCompAccomp=6, minF0=100,
                                  maxF0=800, stepNotes=4, K_numFilters=3, P_numAtomFilters=10,
                                  verbose=False, outputDirSuffix='out', tfrepresentation='mqt',
                                  cqtbins=12, cqtfmin=50)
    assert proc.stftParams['hopsize'] == float(g['hopsize'])
    assert proc.stftParams['windowSizeInSamples'] == float(g['window'])
    np.testing.assert_array_equal(proc.SIMMParams['F0Table'], g['F0Table'])
    assert rel(proc.SIMMParams['WF0'], g['WF0']) < 1e-10
    np.testing.assert_array_equal(proc.SIMMParams['WGAMMA'], g['WGAMMA'])
    proc.autoMelSepAndWrite(maxFrames=140)
    assert int(proc.totFrames) == int(g['totFrames'])
    np.testing.assert_array_equal(proc.indexBestPath, g['indexBestPath'])
    np.testing.assert_array_equal(proc.freqMelody, g['freqMelody'])
    np.testing.assert_allclose(np.loadtxt(proc.files['pitch_output_file']), g['pitches'])
    assert rel(proc.SIMMParams['HF00'], g['HF00']) < 1e-8
    for key, ref in (('voc_output_file', g['lead']), ('mus_output_file', g['acc'])):
        y = wf.read(proc.files[key])[1].astype(np.int64)
        assert y.shape == ref.shape
        assert np.max(np.abs(y - ref.astype(np.int64))) <= 2
