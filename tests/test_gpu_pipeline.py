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


def test_nnls_columns_vs_reference_chunks():
    """The batched GPU NNLS on each chunk's SX (the reference's per-frame
    scipy.optimize.nnls, tests/golden/pipeline_nnls.npz): same active set,
    values to 1e-10 of the column maximum, plus edge cases (an all-zero
    right-hand side, a right-hand side in the span of one column)."""
    from pyfasst_amd.tools.nnls import nnls_columns
    g = load("pipeline_nnls")
    W = g['WF0']
    for i in range(int(g['nchunks'])):
        X = nnls_columns(W, g['SX_%d' % i], add_eps=1e-9)
        ref = g['nnls_HF00_%d' % i]
        np.testing.assert_array_equal(X > 1e-9, ref > 1e-9)
        assert rel(X, ref) < 1e-10
    B = np.zeros((W.shape[0], 3))
    B[:, 1] = 2.5 * W[:, 7]
    B[:, 2] = -W[:, 3]
    X = nnls_columns(W, B)
    np.testing.assert_array_equal(X[:, 0], 0.0)
    np.testing.assert_array_equal(X[:, 2], 0.0)
    assert abs(X[7, 1] - 2.5) < 1e-10 and np.sum(np.abs(np.delete(X[:, 1], 7))) < 1e-10


def test_auto_melody_separation_nnls_init_vs_reference(tmp_path, monkeypatch):
    """initHF00='nnls' end to end (SeparateLeadStereoTF.py:982-993): the chunk
    HF00 of the mono SIMM from the batched GPU NNLS; melody path exact,
    WAVs within 2 LSB of the reference run (tests/golden/pipeline_nnls.npz)."""
    from pyfasst_amd.SeparateLeadStereo import SeparateLeadStereoTF as SL
    monkeypatch.chdir(tmp_path)
    g = load("pipeline_nnls")
    wav = os.path.join(str(tmp_path), "mix.wav")
    wf.write(wav, int(g['fs']), g['wav'])
    np.random.seed(3)
    proc = SL.SeparateLeadProcess(wav, windowSize=0.0464, nbIter=3, numCompAccomp=6, minF0=100,
                                  maxF0=800, stepNotes=4, K_numFilters=3, P_numAtomFilters=10,
                                  verbose=False, outputDirSuffix='out', initHF00='nnls')
    proc.autoMelSepAndWrite(maxFrames=60)
    np.testing.assert_array_equal(proc.indexBestPath, g['indexBestPath'])
    assert rel(proc.SIMMParams['HF00'], g['HF00']) < 1e-8
    for key, ref in (('voc_output_file', g['lead']), ('mus_output_file', g['acc'])):
        y = wf.read(proc.files[key])[1].astype(np.int64)
        assert y.shape == ref.shape
        assert np.max(np.abs(y - ref.astype(np.int64))) <= 2


def test_unvoiced_suimm_stages_vs_reference(tmp_path, monkeypatch):
    """The unvoiced-lead (SUIMM) stages (tests/golden/pipeline_suimm.npz):
    after autoMelSepAndWrite, estimStereoSUIMMParamsWriteSeps
    (SeparateLeadStereoTF.py:1585-1675: Stereo_SIMM per chunk on WUF0 = [WF0 |
    1], NF0 + 1 = 145 columns -- the odd-width path of the NF0-sized
    products -- with HGAMMA held fixed, '_VUIMM' masks, overlap-add); then
    setOutputFileNames and the un-chunked estimStereoSIMMParams /
    estimStereoSUIMMParams with their WAVs (:1677-1760).  WAVs within 2 LSB,
    parameters to 1e-8 of the reference run."""
    from pyfasst_amd.SeparateLeadStereo import SeparateLeadStereoTF as SL
    monkeypatch.chdir(tmp_path)
    g = load("pipeline_suimm")
    wav = os.path.join(str(tmp_path), "mix.wav")
    wf.write(wav, int(g['fs']), g['wav'])
    np.random.seed(3)
    proc = SL.SeparateLeadProcess(wav, windowSize=0.0464, nbIter=3, numCompAccomp=6, minF0=100,
                                  maxF0=800, stepNotes=4, K_numFilters=3, P_numAtomFilters=10,
                                  verbose=False, outputDirSuffix='out')
    proc.autoMelSepAndWrite(maxFrames=60)
    assert rel(proc.SIMMParams['HGAMMA'], g['HGAMMA_in']) < 1e-8
    proc.estimStereoSUIMMParamsWriteSeps(maxFrames=60)
    P = proc.SIMMParams
    assert P['WUF0'].shape[1] == P['WF0'].shape[1] + 1
    np.testing.assert_array_equal(P['WUF0'][:, -1], 1.0)
    assert rel(P['HGAMMA'], g['HGAMMA_suimm']) < 1e-8     # updateHGAMMA=False
    assert rel(P['WM'], g['WM_suimm']) < 1e-8

    def check_wav(path, ref):
        y = wf.read(path)[1].astype(np.int64)
        assert y.shape == ref.shape
        assert np.max(np.abs(y - ref.astype(np.int64))) <= 2, path
    check_wav(proc.files['voc_output_file'], g['lead'])
    check_wav(proc.files['voc_output_file'][:-4] + '_VUIMM.wav', g['lead_vuimm'])
    check_wav(proc.files['mus_output_file'][:-4] + '_VUIMM.wav', g['acc_vuimm'])
    proc.setOutputFileNames('out2')
    assert proc.files['outputDir'].endswith('/out2/') and os.path.isdir(proc.files['outputDir'])
    proc.estimStereoSIMMParams()
    assert rel(P['HF0'], g['whole_HF0']) < 1e-8
    assert rel(P['HGAMMA'], g['whole_HGAMMA']) < 1e-8
    assert abs(P['alphaR'] - g['whole_alphaR']) <= 1e-8 * abs(g['whole_alphaR'])
    proc.writeSeparatedSignals()
    check_wav(proc.files['voc_output_file'], g['whole_lead'])
    check_wav(proc.files['mus_output_file'], g['whole_acc'])
    proc.estimStereoSUIMMParams()
    assert rel(P['HUF0'], g['whole_HUF0']) < 1e-8
    assert rel(P['HGAMMA'], g['whole_HGAMMA_u']) < 1e-8
    assert rel(P['betaR'], g['whole_betaR_u']) < 1e-8
    proc.writeSeparatedSignalsWithUnvoice()
    check_wav(proc.files['voc_output_file'][:-4] + '_VUIMM.wav', g['whole_lead_vuimm'])
    check_wav(proc.files['mus_output_file'][:-4] + '_VUIMM.wav', g['whole_acc_vuimm'])



def test_nnls_drops_and_iteration_count_vs_scipy():
    """Columns whose active-set path drops coefficients (Lawson & Hanson's
    step E: the coefficient that sets alpha leaves the passive set at exactly
    zero): the GPU solution matches scipy.optimize.nnls (the reference's
    per-frame call, SeparateLeadStereoTF.py:988) and the iteration budget
    behaves as scipy's -- a column whose count is c (outer + inner passes)
    succeeds with maxiter c + 1 and fails with maxiter c, in both."""
    import scipy.optimize
    from pyfasst_amd.tools.nnls import nnls_columns
    rs = np.random.RandomState(1)      # 4 of the 40 columns take inner (drop) steps
    m, n = 15, 12
    A = rs.rand(m, n)
    B = rs.randn(m, 40)
    X = nnls_columns(A, B)
    for q in range(B.shape[1]):
        xs = scipy.optimize.nnls(A, B[:, q])[0]
        assert np.max(np.abs(X[:, q] - xs)) < 1e-10 * max(1.0, np.max(np.abs(xs)))
    import ctypes
    from pyfasst_amd import _lib
    info = np.empty(B.shape[1], dtype=np.int32)
    Xc = np.empty((n, B.shape[1]))
    Ac, Bc = np.ascontiguousarray(A), np.ascontiguousarray(B)
    _lib.check(_lib.lib.nnls_columns(_lib.default_device(), m, n, _lib.dptr(Ac), B.shape[1],
                                     _lib.dptr(Bc), 10.0 * max(m, n) * np.finfo(float).eps, 0.0,
                                     0, _lib.dptr(Xc), info.ctypes.data_as(_lib._ip)),
               "nnls_columns")
    drops = 0
    for q in range(B.shape[1]):
        c = int(info[q])
        if c == 0:      # A^T b <= 0: x = 0 with no pass (maxiter 0 means scipy's default)
            np.testing.assert_array_equal(Xc[:, q], 0.0)
            continue
        drops += c > int(np.sum(Xc[:, q] > 0))        # more passes than entries: a drop
        scipy.optimize.nnls(A, B[:, q], maxiter=c + 1)
        with pytest.raises(RuntimeError):
            scipy.optimize.nnls(A, B[:, q], maxiter=c)
        nnls_columns(A, B[:, q], maxiter=c + 1)
        with pytest.raises(Exception):
            nnls_columns(A, B[:, q], maxiter=c)
    assert drops > 0
