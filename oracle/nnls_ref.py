"""CPU oracle of the lead pipeline's initHF00='nnls' initialisation.

TEST INFRASTRUCTURE ONLY (imported by tests/ and never by pyfasst_amd).

The reference solves the NNLS problems with its dependency's routine
(SeparateLeadStereo/SeparateLeadStereoTF.py:982-993):
    HF00[:, n], _ = scipy.optimize.nnls(WF0, SX[:, n]);  HF00 += eps
so this oracle IS that call, column by column (scipy 1.15.3 in this image:
Lawson & Hanson's active-set NNLS, `scipy/optimize/_nnls.py`).  Pinned by
tests/golden/pipeline_nnls.npz, which records the HF00 the reference itself
handed to SIMM in a full pipeline run (tests/golden/make_golden.py
run_pipeline_nnls), bit for bit.
"""
import numpy as np
from scipy.optimize import nnls

EPS = 10 ** -9   # SeparateLeadStereoTF.py:31


def nnls_hf00(WF0, SX):
    """HF00 of one chunk as estimHF0 forms it (:984-993)."""
    HF00 = np.ones((WF0.shape[1], SX.shape[1]))
    for framenb in range(SX.shape[1]):
        HF00[:, framenb], _ = nnls(WF0, SX[:, framenb])
    HF00 += EPS
    return HF00
