"""Build a scratch Python-3 translation of the reference pyfasst in /tmp.

TEST INFRASTRUCTURE ONLY.  Nothing here is shipped or imported by the
product package `pyfasst_amd`.  The scratch copy lives under /tmp, is never
committed, and never travels to the GPU box; it is used in this container
only to (i) pin the committed NumPy restatement `oracle/fasst_ref.py` and
(ii) generate the small golden fixtures under `tests/golden/`.

Recipe:
  1. copy /root/reference/pyfasst -> /tmp/pyfasst_scratch/pyfasst
  2. python -m lib2to3 -w -n
  3. fix the 2to3 artifacts and the Python-3 / NumPy-2 incompatibilities
     listed in PATCHES below (mechanical textual substitutions only).
The Cython Viterbi tracker is not needed by the EM / SIMM paths and is not
built.

Usage:  python oracle/make_scratch_ref.py  [dest_dir]
then    sys.path.insert(0, dest_dir); import pyfasst.audioModel
"""
import os
import re
import shutil
import subprocess
import sys

REF = "/root/reference/pyfasst"
DEFAULT_DEST = "/tmp/pyfasst_scratch"

# (file, regex, replacement).  Each is a mechanical py2->py3 / numpy-2 fix.
PATCHES = [
    # `from . import a.b as c` (2to3 artifact) -> `from .a import b as c`
    ("audioModel.py", r"from \. import (\w+)\.(\w+) as (\w+)", r"from .\1 import \2 as \3"),
    ("demixTF.py", r"from \. import (\w+)\.(\w+) as (\w+)", r"from .\1 import \2 as \3"),
    ("tftransforms/nsgt/unslicing.py", r"importcycle", "import cycle"),
    ("tftransforms/nsgt/nsigtf.py", r"importchain", "import chain"),
    ("tftransforms/nsgt/slicq.py", r"importcycle", "import cycle"),
    ("SeparateLeadStereo/SIMM/SIMM.py", r"from string import join\n", "\n"),
    ("SeparateLeadStereo/SIMM/SIMMopt.py", r"from string import join\n", "\n"),
    # integer divisions used as sizes/indices
    ("audioModel.py", r"self\.sig_repr_params\['fsize'\]/2\+1", "self.sig_repr_params['fsize']//2+1"),
    ("audioModel.py", r"nc \* \(nc \+ 1\) / 2", "nc * (nc + 1) // 2"),
    ("audioModel.py", r"'hopsize': self\.sig_repr_params\['wlen'\]/2", "'hopsize': self.sig_repr_params['wlen']//2"),
    # numpy 2 removed aliases
    ("audioModel.py", r"np\.complex\b", "complex"),
    ("tools/signalTools.py", r"np\.complex\b", "complex"),
    ("demixTF.py", r"np\.complex\b", "complex"),
    # stft.py float sizes/indices
    ("tftransforms/stft.py", r"np\.zeros\(lengthWindow/2\.0\)", "np.zeros(int(lengthWindow//2))"),
    ("tftransforms/stft.py", r"np\.zeros\(\[lengthWindow/2\.0, nc\]\)", "np.zeros([int(lengthWindow//2), nc])"),
    ("tftransforms/stft.py", r"np\.zeros\(newLengthData - data\.size\)", "np.zeros(int(newLengthData - data.size))"),
    ("tftransforms/stft.py", r"numberFrequencies = nfft / 2 \+ 1", "numberFrequencies = int(nfft // 2 + 1)"),
    ("tftransforms/stft.py", r"np\.zeros\(\[numberFrequencies, numberFrames\], dtype=complex\)",
     "np.zeros([numberFrequencies, int(numberFrames)], dtype=complex)"),
    ("tftransforms/stft.py", r"for n in np\.arange\(numberFrames\):", "for n in np.arange(int(numberFrames)):"),
    ("tftransforms/stft.py", r"beginFrame = n\*hopsize", "beginFrame = int(n*hopsize)"),
    ("tftransforms/stft.py", r"beginFrame = n \* hopsize", "beginFrame = int(n * hopsize)"),
    ("tftransforms/stft.py", r"endFrame = beginFrame\+lengthWindow", "endFrame = int(beginFrame+lengthWindow)"),
    ("tftransforms/stft.py", r"endFrame = beginFrame \+ lengthWindow", "endFrame = int(beginFrame + lengthWindow)"),
    ("tftransforms/stft.py", r"lengthData = hopsize\*\(numberFrames-1\) \+ lengthWindow",
     "lengthData = int(hopsize*(numberFrames-1) + lengthWindow)"),
    ("tftransforms/stft.py", r"\[\(lengthWindow/2\.0\):\]", "[int(lengthWindow//2):]"),
    ("tftransforms/stft.py", r"self\.freqbins = self\.ftlen / 2 \+ 1", "self.freqbins = self.ftlen // 2 + 1"),
    # SIMM-pipeline stft / istft (separateLeadFunctions.py:90-233) float sizes/indices
    ("SeparateLeadStereo/separateLeadFunctions.py", r"np\.zeros\(lengthWindow / 2\.0\)",
     "np.zeros(int(lengthWindow / 2.0))"),
    ("SeparateLeadStereo/separateLeadFunctions.py", r"np\.zeros\(\[newLengthData - lengthData\]\)",
     "np.zeros([int(newLengthData - lengthData)])"),
    ("SeparateLeadStereo/separateLeadFunctions.py", r"numberFrequencies = nfft / 2\.0 \+ 1",
     "numberFrequencies = int(nfft / 2.0 + 1)"),
    ("SeparateLeadStereo/separateLeadFunctions.py", r"        stop = numberFrames\n",
     "        stop = int(numberFrames)\n"),
    ("SeparateLeadStereo/separateLeadFunctions.py", r"beginFrame = n \* hopsize",
     "beginFrame = int(n * hopsize)"),
    ("SeparateLeadStereo/separateLeadFunctions.py", r"np\.fft\.rfft\(frameToProcess, nfft\)",
     "np.fft.rfft(frameToProcess, int(nfft))"),
    ("SeparateLeadStereo/separateLeadFunctions.py", r"np\.fft\.irfft\(X\[:,n\], nfft\)",
     "np.fft.irfft(X[:,n], int(nfft))"),
    ("SeparateLeadStereo/separateLeadFunctions.py",
     r"lengthData = hopsize \* \(numberFrames - 1\) \+ lengthWindow",
     "lengthData = int(hopsize * (numberFrames - 1) + lengthWindow)"),
    # the Cython tracker is not built: use the reference's own pure-Python
    # fallback (tracking/tracking.py), only needed at import time here
    ("SeparateLeadStereo/SeparateLeadStereoTF.py",
     r"from \.tracking\._tracking import viterbiTracking as viterbiTrackingArray",
     "from .tracking.tracking import viterbiTrackingArray"),
    # tftransforms/minqt.py (CQT / MinQT): numpy-2 aliases,
    # float sizes / indices, scipy >= 1.13 window location
    ("tftransforms/minqt.py", r"np\.complex\b", "complex"),
    ("tools/utils.py", r"spsig\.blackmanharris\(M\)", "spsig.windows.blackmanharris(M)"),
    ("tftransforms/minqt.py", r"np\.zeros\(\[bins \* winNr, FFTLen\],", "np.zeros([int(bins * winNr), int(FFTLen)],"),
    ("tftransforms/minqt.py", r"tempKernel = np\.zeros\(FFTLen, dtype=complex\)", "tempKernel = np.zeros(int(FFTLen), dtype=complex)"),
    ("tftransforms/minqt.py", r"winFct = winFunc\(Nk\)", "winFct = winFunc(int(Nk))"),
    ("tftransforms/minqt.py", r"tempKernel\[shift:\(Nk\+shift\)\] = tempKernelBin", "tempKernel[int(shift):int(Nk+shift)] = tempKernelBin"),
    ("tftransforms/minqt.py", r"self\.linBins = linFTLen/2 - Kmax \+ 1", "self.linBins = linFTLen//2 - Kmax + 1"),
    ("tftransforms/minqt.py", r"self\.cellCQT\[i\] = np\.zeros\(\[self\.cqtkernel\.bins \*\n\s+self\.cqtkernel\.winNr,\n\s+nframes\],",
     "self.cellCQT[i] = np.zeros([int(self.cqtkernel.bins * self.cqtkernel.winNr), int(nframes)],"),
    ("tftransforms/minqt.py", r"self\._spCQT = np\.zeros\(\[self\.cqtkernel\.bins\n\s+\* self\.octaveNr,\n\s+nframes \* atomNr\],",
     "self._spCQT = np.zeros([int(self.cqtkernel.bins * self.octaveNr), int(nframes * atomNr)],"),
    ("tftransforms/minqt.py", r"CQTframe = np\.zeros\(\[self\.cqtkernel\.bins \* atomNr, nframes\],",
     "CQTframe = np.zeros([int(self.cqtkernel.bins * atomNr), int(nframes)],"),
    ("tftransforms/minqt.py", r"XX = np\.zeros\(\[self\.cqtkernel\.FFTLen, nframes\],", "XX = np.zeros([int(self.cqtkernel.FFTLen), int(nframes)],"),
    ("tftransforms/minqt.py", r"for n in np\.arange\(nframes\):\n(\s+)if self\.verbose>2:", r"for n in np.arange(int(nframes)):\n\1if self.verbose>2:"),
    ("tftransforms/minqt.py", r"framestart = n \* self\.cqtkernel\.fftHOP\n", "framestart = int(n * self.cqtkernel.fftHOP)\n"),
    ("tftransforms/minqt.py", r"framestop = framestart \+ self\.cqtkernel\.FFTLen\n", "framestop = int(framestart + self.cqtkernel.FFTLen)\n"),
    ("tftransforms/minqt.py", r"XX\[:,n\]= np\.fft\.fft\(x\[framestart:framestop\],\n\s+n=cqtkernel\.FFTLen\)",
     "XX[:,n]= np.fft.fft(x[framestart:framestop], n=int(cqtkernel.FFTLen))"),
    ("tftransforms/minqt.py", r"for nshift in np\.arange\(2\*\*i\):", "for nshift in np.arange(int(2**i)):"),
    ("tftransforms/minqt.py", r"X,F,N = stft\(data=x\[self\.offsetSTFT:\],", "X,F,N = stft(data=x[int(self.offsetSTFT):],"),
    ("tftransforms/minqt.py", r"self\.cellCQT\['linear'\] = X\[self\.cqtkernel\.Kmax:,\n\s+:self\.nframes\[0\] \* self\.cqtkernel\.winNr\]",
     "self.cellCQT['linear'] = X[self.cqtkernel.Kmax:, :int(self.nframes[0] * self.cqtkernel.winNr)]"),
    ("tftransforms/minqt.py", r"self\._spCQT = np\.vstack\(\[\n\s+self\._spCQT,\n\s+np\.zeros\(\[self\.cqtkernel\.linBins,\n\s+self\._spCQT\.shape\[1\]\],\n\s+dtype=complex\)\]\)",
     "self._spCQT = np.vstack([self._spCQT, np.zeros([int(self.cqtkernel.linBins), self._spCQT.shape[1]], dtype=complex)])"),
    ("tftransforms/minqt.py", r"self\._spCQT\[\(self\.cqtkernel\.bins \* self\.octaveNr\):,", "self._spCQT[int(self.cqtkernel.bins * self.octaveNr):,"),
    ("tftransforms/minqt.py", r"self\.maxBlock = \(\n\s+cqtkernel\.FFTLen \*\n\s+\(2\*\*\(self\.octaveNr-1\)\)\)", "self.maxBlock = int(cqtkernel.FFTLen * (2**(self.octaveNr-1)))"),
    ("tftransforms/minqt.py", r"int\(nshift\):\(nframes\*nshifts\):nshifts\] = \(", "int(nshift):int(nframes*nshifts):nshifts] = ("),
    ("tftransforms/minqt.py", r"y = np\.zeros\(np\.ceil\(self\.datalen_init /\n\s+\(2\.\*\*\(self\.octaveNr-1\)\)\)\)",
     "y = np.zeros(int(np.ceil(self.datalen_init / (2.**(self.octaveNr-1)))))"),
    ("tftransforms/minqt.py", r"y = np\.concatenate\(\[y, np\.zeros\(ylen-y\.size\)\]\)", "y = np.concatenate([y, np.zeros(int(ylen-y.size))])"),
    ("tftransforms/minqt.py", r"yoct = np\.zeros\(self\.cqtkernel\.FFTLen\)", "yoct = np.zeros(int(self.cqtkernel.FFTLen))"),
    ("tftransforms/minqt.py", r"frastop = frastart \+ self\.cqtkernel\.FFTLen\n", "frastop = int(frastart + self.cqtkernel.FFTLen)\n"),
    ("tftransforms/minqt.py", r"frastart = n \* self\.cqtkernel\.fftHOP\n", "frastart = int(n * self.cqtkernel.fftHOP)\n"),
    ("tftransforms/minqt.py", r"np\.fft\.ifft\(Y\[:,n\], n=self\.cqtkernel\.FFTLen\)", "np.fft.ifft(Y[:,n], n=int(self.cqtkernel.FFTLen))"),
    ("tftransforms/minqt.py", r"self\._spCQT\[int\(self\.cqtkernel\.bins\*\(self\.octaveNr-noct-1\)\):\n(\s+)int\(self\.cqtkernel\.bins\*\(self\.octaveNr-noct\)\),\n(\s+):-1\] = \(",
     r"self._spCQT[int(self.cqtkernel.bins*(self.octaveNr-noct-1)):int(self.cqtkernel.bins*(self.octaveNr-noct)), :-1] = ("),
    ("tftransforms/minqt.py", r"newy = np\.zeros\(y\.size\*2\)", "newy = np.zeros(int(y.size*2))"),
    ("tftransforms/minqt.py", r"y = y\[self\.prefixZeros:\]", "y = y[int(self.prefixZeros):]"),
    ("tftransforms/minqt.py", r"y = y\[:self\.datalen_init\]", "y = y[:int(self.datalen_init)]"),
    ("tftransforms/minqt.py", r"np\.hstack\(\[np\.zeros\(\[self\.cqtkernel\.bins, dropped\]\),", "np.hstack([np.zeros([int(self.cqtkernel.bins), int(dropped)]),"),
    ("tftransforms/minqt.py", r"np\.zeros\(\[self\.cqtkernel\.bins,\n\s+np\.ceil\(X\.shape\[1\]/\n\s+self\.cqtkernel\.winNr\)\*\n\s+self\.cqtkernel\.winNr -\n\s+X\.shape\[1\]\]\)",
     "np.zeros([int(self.cqtkernel.bins), int(np.ceil(X.shape[1]/self.cqtkernel.winNr)*self.cqtkernel.winNr - X.shape[1])])"),
    ("tftransforms/minqt.py", r"np\.ascontiguousarray\(self\.cellCQT\[noct\]\[:,:self\.nframes\[noct\]\]\)", "np.ascontiguousarray(self.cellCQT[noct][:,:int(self.nframes[noct])])"),
    ("tftransforms/minqt.py", r"np\.hstack\(\[np\.zeros\(\[self\.cqtkernel\.linBins, dropped\]\),", "np.hstack([np.zeros([int(self.cqtkernel.linBins), int(dropped)]),"),
    ("tftransforms/minqt.py", r"self\.cellCQT\['linear'\]\[:,:\(self\.nframes\[0\]\*\n\s+self\.cqtkernel\.winNr\)\]",
     "self.cellCQT['linear'][:,:int(self.nframes[0]*self.cqtkernel.winNr)]"),
    ("tftransforms/minqt.py", r"Y = np\.zeros\(\[self\.cqtkernel\.linFTLen / 2 \+ 1,", "Y = np.zeros([self.cqtkernel.linFTLen // 2 + 1,"),
    ("tftransforms/minqt.py", r"y = y\[\(self\.prefixZeros-self\.offsetSTFT\):\]", "y = y[int(self.prefixZeros-self.offsetSTFT):]"),
    ("tftransforms/minqt.py", r"X\.shape\[1\]/self\.cqtkernel\.winNr, order='F'\)", "int(X.shape[1]//self.cqtkernel.winNr), order='F')"),
    ("tftransforms/minqt.py", r"np\.ceil\(X\.shape\[1\]/\n\s+self\.cqtkernel\.winNr\)\],", "int(np.ceil(X.shape[1]/self.cqtkernel.winNr))],"),
    ("tftransforms/minqt.py", r"CQTframe\[nb\*atomNr\+a\]", "CQTframe[int(nb*atomNr+a)]"),
    ("tftransforms/minqt.py", r"self\.cellCQT\[noct\]\[nb\*atomNr\+a\]", "self.cellCQT[noct][int(nb*atomNr+a)]"),
    ("tftransforms/minqt.py", r"self\.cellCQT\[noct\] = np\.zeros\(\[self\.cqtkernel\.bins \*\n\s+self\.cqtkernel\.winNr,",
     "self.cellCQT[noct] = np.zeros([int(self.cqtkernel.bins * self.cqtkernel.winNr),"),
    ("tftransforms/minqt.py", r"X\[nbin\]\.reshape\(\n\s+self\.cqtkernel\.winNr,", "X[nbin].reshape(int(self.cqtkernel.winNr),"),
    # tracking.py (the reference's pure-Python Viterbi, golden source for the
    # tracker): integer state paths
    ("SeparateLeadStereo/tracking/tracking.py", r"bestStatePath = zeros\(numberOfFrames\)",
     "bestStatePath = zeros(numberOfFrames, dtype=int)"),
    ("SeparateLeadStereo/SeparateLeadStereoTF.py", r"np\.Inf\b", "np.inf"),
    # SIMM dictionaries (separateLeadFunctions.py:696-1146): numpy < 1.13 let
    # rfft drop the imaginary part of the complex odgd (ComplexWarning) and
    # compared an array window with a string to False; float sizes
    ("tftransforms/stft.py", r"STFT\[:,n\] = np\.fft\.rfft\(frameToProcess, np\.int32\(nfft\)\)",
     "STFT[:,n] = np.fft.rfft(np.real(frameToProcess), np.int32(nfft))"),
    ("SeparateLeadStereo/separateLeadFunctions.py", r"    if analysisWindowType=='sinebell':\n",
     "    if not isinstance(analysisWindowType, str):\n        analysisWindow = analysisWindowType\n"
     "    elif analysisWindowType=='sinebell':\n"),
    ("SeparateLeadStereo/separateLeadFunctions.py", r"for fundamentalFrequency in np\.arange\(numberOfF0\):",
     "for fundamentalFrequency in np.arange(int(numberOfF0)):"),
    ("SeparateLeadStereo/separateLeadFunctions.py", r"WF0 = np\.zeros\(\[transform\.freqbins,\n\s+numberElementsInWF0\],",
     "WF0 = np.zeros([int(transform.freqbins), int(numberElementsInWF0)],"),
    ("SeparateLeadStereo/separateLeadFunctions.py", r"prototypeSineWindow = hann\(lengthSineWindow\)",
     "prototypeSineWindow = hann(int(lengthSineWindow))"),
    ("SeparateLeadStereo/separateLeadFunctions.py", r"bigWindow = np\.zeros\(\[sizeBigWindow \* 2, 1\]\)",
     "bigWindow = np.zeros([int(sizeBigWindow * 2), 1])"),
    ("SeparateLeadStereo/separateLeadFunctions.py", r"bigWindow\[\(sizeBigWindow - lengthSineWindow / 2\.0\):\\\n\s+\(sizeBigWindow \+ lengthSineWindow / 2\.0\)\]",
     "bigWindow[int(sizeBigWindow - lengthSineWindow / 2.0):int(sizeBigWindow + lengthSineWindow / 2.0)]"),
    # generate_WF0_TR_chirped on a CQT / MinQT transform (:742-815): the
    # window length FFTLen * 2**(octaveNr-1) is a float
    ("SeparateLeadStereo/separateLeadFunctions.py", r"    if hasattr\(transform, 'octaveNr'\):\n        lengthWindow = \(\n",
     "    if hasattr(transform, 'octaveNr'):\n        lengthWindow = int(\n"),
    ("SeparateLeadStereo/separateLeadFunctions.py", r"analysisWindow = transform\.winFunc\(lengthWindow\)",
     "analysisWindow = transform.winFunc(int(lengthWindow))"),
    # NMF initialisation (audioModel.py:2118-2177): float slice bounds
    ("audioModel.py", r"ind_start = np\.sum\(nbSpecComps\[:spec_ind\]\)",
     "ind_start = int(np.sum(nbSpecComps[:spec_ind]))"),
    # lead/accompaniment pipeline (SeparateLeadStereoTF.py:959-1897): py2
    # integer division on numpy ints, np.int, float slice bounds
    ("SeparateLeadStereo/SeparateLeadStereoTF.py", r"nChunks = totFrames / maxFrames \+ 1",
     "nChunks = totFrames // maxFrames + 1"),
    ("SeparateLeadStereo/SeparateLeadStereoTF.py", r"maxFrames = np\.int\(np\.ceil\(np\.double\(totFrames\)/nChunks\)\)",
     "maxFrames = int(np.ceil(np.double(totFrames)/nChunks))"),
    ("SeparateLeadStereo/SeparateLeadStereoTF.py", r"nChunks = totFrames/maxFrames \n",
     "nChunks = totFrames//maxFrames \n"),
    ("SeparateLeadStereo/SIMM/SIMM.py", r"F0Table\[np\.array\(imgYticks\)/chirpPerF0\]",
     "F0Table[np.array(imgYticks)//chirpPerF0]"),
    ("SeparateLeadStereo/SeparateLeadStereoTF.py", r"F0Table\[np\.array\(imgYticks\)/\n(\s+)self\.SIMMParams\['chirpPerF0'\]",
     r"F0Table[np.array(imgYticks)//\n\1self.SIMMParams['chirpPerF0']"),
    ("SeparateLeadStereo/SeparateLeadStereoTF.py", r"np\.ones\(chirpPerF0", "_ones_i(chirpPerF0"),
    ("SeparateLeadStereo/SeparateLeadStereoTF.py", r"\neps = 10 \*\* -9\n",
     "\neps = 10 ** -9\n_ones_i = lambda n, **kw: np.ones(int(n), **kw)  # py2 float sizes\n"),
    ("SeparateLeadStereo/SeparateLeadStereoTF.py", r"overlapSamp = wlen - hopsize\n",
     "overlapSamp = int(wlen - hopsize)\n"),
    ("SeparateLeadStereo/SeparateLeadStereoTF.py", r"data = np\.zeros\(\[nuDataLen, 2\], np\.int16\)",
     "data = np.zeros([int(nuDataLen), 2], np.int16)"),
    ("SeparateLeadStereo/SeparateLeadStereoTF.py", r"start = cumulframe - wlen \+ hopsize\n",
     "start = int(cumulframe - wlen + hopsize)\n"),
    # CQT-type chunks (:726-735, :810-818, :893-900): sample bounds are float
    # multiples of atomHOP, which numpy < 1.12 truncated as slice indices
    ("SeparateLeadStereo/SeparateLeadStereoTF.py", r"            data = data\[start:stop\]\n",
     "            data = data[int(start):int(stop)]\n"),
    ("SeparateLeadStereo/SeparateLeadStereoTF.py", r"'stft': self\.stftParams\['windowSizeInSamples'\] / 2,",
     "'stft': self.stftParams['windowSizeInSamples'] // 2,"),
]


def build(dest=DEFAULT_DEST):
    if not os.path.isdir(REF):
        raise RuntimeError("reference not present at %s" % REF)
    pkg = os.path.join(dest, "pyfasst")
    if os.path.isdir(dest):
        shutil.rmtree(dest)
    os.makedirs(dest)
    shutil.copytree(REF, pkg)
    for root, _, files in os.walk(pkg):
        os.chmod(root, 0o755)
        for f in files:
            os.chmod(os.path.join(root, f), 0o644)
    subprocess.check_call([sys.executable, "-m", "lib2to3", "-w", "-n", pkg],
                          stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    for rel, pat, rep in PATCHES:
        path = os.path.join(pkg, rel)
        with open(path) as fh:
            src = fh.read()
        new, n = re.subn(pat, rep, src)
        if n == 0:
            print("warning: patch had no effect: %s %s" % (rel, pat))
        with open(path, "w") as fh:
            fh.write(new)
    return dest


if __name__ == "__main__":
    d = build(sys.argv[1] if len(sys.argv) > 1 else DEFAULT_DEST)
    print(d)
