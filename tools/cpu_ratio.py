"""Restatement-to-reference CPU time ratio for one GEM iteration at C3
(SURVEY.md §8(d) asks for it next to the CPU baseline).

BUILD-CONTAINER ONLY (needs /root/reference through the scratch py3
translation of oracle/make_scratch_ref.py; never runs on the GPU box).
Times ONE GEM_iteration of
  * the reference  (`pyfasst.audioModel.MultiChanNMFConv`, scratch translation)
  * the oracle     (`oracle/fasst_ref.py` RefFASST)
on the same C3 structure (F=2049, T=10000, J=4, spatial rank 2, K=32, conv),
each in its own process with the same BLAS thread count, and writes
profiles/r2_cpu_ratio.json.  bench.py's cpu_baseline reports the ratio next to
the oracle time it measures on the GPU box's host.

    python tools/cpu_ratio.py            # both legs + JSON
    python tools/cpu_ratio.py ref|oracle # one leg (prints seconds)
"""
import json
import os
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCRATCH = "/tmp/pyfasst_scratch"
FS, WLEN, HOP = 44100, 4096, 512
T_FRAMES, J, RANK, K = 10000, 4, 2, 32


def _wav():
    import scipy.io.wavfile as wf
    path = "/tmp/cpu_ratio_c3.wav"
    if not os.path.exists(path):
        n = (T_FRAMES - 2) * HOP   # ceil(n / hop) + 2 = T_FRAMES frames (stft.py:39)
        rs = np.random.RandomState(0)
        x = (rs.standard_normal((n, 2)) * 3000).astype(np.int16)
        wf.write(path, FS, x)
    return path


def leg_ref():
    import warnings
    warnings.simplefilter('ignore')
    sys.path.insert(0, SCRATCH)
    import pyfasst.audioModel as am
    np.random.seed(1)
    m = am.MultiChanNMFConv(_wav(), nbComps=J, nbNMFComps=K, spatial_rank=RANK, verbose=0,
                            iter_num=1, wlen=WLEN, hopsize=HOP)
    m.makeItConvolutive()
    m.noise['PSD'] = m.noise['ann_PSD_lim'][0]
    shape = m.Cx.shape
    t0 = time.perf_counter()
    m.GEM_iteration()
    return time.perf_counter() - t0, shape


def leg_oracle():
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    sys.path.insert(0, REPO)
    import fasst_ref as R
    from pyfasst_amd import synthetic
    X = synthetic.stereo_mixture(WLEN // 2 + 1, T_FRAMES, J=J, K_true=8, rank=RANK, seed=0)
    o = R.RefFASST(iter_num=1)
    o.set_transform([X[0], X[1]])
    del X
    np.random.seed(1)
    R.init_nmf_inst(o, J, K, RANK)
    R.make_convolutive(o)
    o.noise['PSD'] = o.annealed_psd(0)
    t0 = time.perf_counter()
    o.GEM_iteration()
    return time.perf_counter() - t0, (WLEN // 2 + 1, T_FRAMES)


def main():
    if len(sys.argv) > 1:
        dt, shape = (leg_ref if sys.argv[1] == "ref" else leg_oracle)()
        print(json.dumps({"seconds": dt, "shape": list(shape)}))
        return
    subprocess.check_call([sys.executable, os.path.join(REPO, "oracle", "make_scratch_ref.py")])
    res = {}
    for leg in ("ref", "oracle"):
        out = subprocess.check_output([sys.executable, os.path.abspath(__file__), leg], text=True)
        res[leg] = json.loads(out.strip().splitlines()[-1])
        print(leg, res[leg], flush=True)
    try:
        from threadpoolctl import threadpool_info
        threads = max([p.get('num_threads', 1) for p in threadpool_info()] + [1])
    except Exception:
        threads = None
    doc = {"what": "one GEM_iteration at C3 (F=2049, T=10000, J=4, rank 2, K=32, conv)",
           "reference_s": res["ref"]["seconds"], "oracle_s": res["oracle"]["seconds"],
           "ratio": res["oracle"]["seconds"] / res["ref"]["seconds"],
           "reference_shape": res["ref"]["shape"], "blas_threads": threads,
           "host": "build container (%d CPUs)" % os.cpu_count(),
           "script": "tools/cpu_ratio.py"}
    with open(os.path.join(REPO, "profiles", "r2_cpu_ratio.json"), "w") as f:
        json.dump(doc, f, indent=1)
    print(json.dumps(doc))


if __name__ == "__main__":
    main()
