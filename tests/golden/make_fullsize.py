"""Generate the BASELINE-size parity fixtures in tests/golden/ with the ORACLE.

Run in the build container (CPU only, minutes per case):

    python tests/golden/make_fullsize.py            # all cases
    python tests/golden/make_fullsize.py c3_full    # one case

The reference itself cannot run at these sizes in reasonable time (its E-step
materialises G[2,R,F,T]), so these fixtures come from the oracle restatement
(oracle/fasst_ref.py, oracle/simm_ref.py), which is itself pinned bit-exactly
to the reference on the small golden cases (tests/test_oracle_golden.py).
Inputs are synthetic and seeded (pyfasst_amd/synthetic.py, RandomState), so
the GPU box regenerates them bit-identically.  The outputs are stored
subsampled (every FSTEP-th bin, TSTEP-th frame) plus full-array sums, which
keeps each fixture under ~1 MB.  Each case runs in a fresh process (N2).

Cases (tests/helpers.py FULL_CASES mirrors the shapes):
  c3_full   BASELINE configs[2]: MultiChanNMFConv J=4 rank 2 K=32, F=2049,
            T=10000, data RandomState(0), init seed 1, 2 GEM iterations,
            separated images
  c3_t1000  the same structure at T=1000 (F-side chunking at full F), 3
            iterations
  c1_50     C1-shaped: MultiChanNMFInst_FASST J=2 rank 1 K=32, F=1025,
            T=1122 (tamy's STFT shape, synthetic), 50 GEM iterations
  c5_full   BASELINE configs[4]: Stereo_SIMM F=2049 N=20000 NF0=1092 P=30
            K=4 R=40 on gamma spectrograms (RandomState(0)), init seed 1,
            1 iteration
  c5_10     the same at the pipeline's default 10 iterations
            (SeparateLeadStereoTF.py:264)
"""
import os
import subprocess
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))
sys.path.insert(0, os.path.join(REPO, "tests"))

from helpers import FULL_CASES, sub_f, sub_t  # noqa: E402


def _fasst_case(name):
    import fasst_ref as R
    from pyfasst_amd import synthetic
    c = FULL_CASES[name]
    F, T, J, K, rank, conv, iters = (c[k] for k in ("F", "T", "J", "K", "rank", "conv", "iters"))
    X = synthetic.stereo_mixture(F, T, J=J, K_true=c["K_true"], rank=c["data_rank"],
                                 seed=c["data_seed"])
    o = R.RefFASST(iter_num=iters)
    o.set_transform([X[0], X[1]])
    np.random.seed(c["init_seed"])
    R.init_nmf_inst(o, J, K, rank)
    if conv:
        R.make_convolutive(o)
    t0 = time.time()
    ll = o.estim_param_a_post_model(
        callback=lambda i, m: print("  iter %d  %.1f s" % (i + 1, time.time() - t0), flush=True))
    out = {"logliks": ll, "final_psd": o.noise['PSD']}
    fs, ts = sub_f(F), sub_t(T)
    for j in range(J):
        p = o.spat_comps[j]['params']
        out["params_%d" % j] = p[..., fs] if conv else p
        fac = o.spec_comps[j]['factor'][0]
        out["FB_%d" % j] = fac['FB'][fs]
        out["TW_%d" % j] = fac['TW'][:, ts]
        out["FB_sum_%d" % j] = fac['FB'].sum()
        out["TW_sum_%d" % j] = fac['TW'].sum()
    S = np.abs(o.separated_images(X))
    out["absS"] = S[:, :, fs][:, :, :, ts]
    out["absS_sum"] = S.sum(axis=(2, 3))
    return out


def _simm_case(name):
    import simm_ref
    c = FULL_CASES[name]
    F, N, NF0, P, K, Rr = (c[k] for k in ("F", "N", "NF0", "P", "K", "R"))
    rs = np.random.RandomState(c["data_seed"])
    SXR = rs.gamma(0.8, 1.0, size=(F, N))
    SXL = rs.gamma(0.8, 1.0, size=(F, N))
    WF0 = rs.gamma(1.0, 1.0, size=(F, NF0))
    WG = rs.gamma(1.0, 1.0, size=(F, P))
    np.random.seed(c["init_seed"])
    t0 = time.time()
    res = simm_ref.stereo_simm(SXR, SXL, WF0, WG, K, Rr, numberOfIterations=c["iters"],
                               computeError=True)
    print("  stereo_simm %.1f s" % (time.time() - t0), flush=True)
    names = ['alphaR', 'alphaL', 'HGAMMA', 'HPHI', 'HF0', 'betaR', 'betaL', 'HM', 'WM',
             'recoError']
    out = {}
    fs, ts = sub_f(F), sub_t(N)
    for n, v in zip(names, res):
        v = np.asarray(v)
        out[n + "_sum"] = v.sum()
        if n in ('HPHI', 'HM'):
            v = v[:, ts]
        elif n == 'HF0':
            v = v[::8][:, ts]
        elif n == 'WM':
            v = v[fs]
        out[n] = v
    return out


def run_case(name):
    t0 = time.time()
    out = _simm_case(name) if name.startswith("c5") else _fasst_case(name)
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **out)
    print("%s: %.1f s" % (name, time.time() - t0), flush=True)


def main():
    names = sys.argv[1:] or sorted(FULL_CASES)
    if len(names) == 1:
        run_case(names[0])
        return
    for n in names:   # one process per case (N2)
        subprocess.check_call([sys.executable, os.path.abspath(__file__), n])


if __name__ == "__main__":
    main()
