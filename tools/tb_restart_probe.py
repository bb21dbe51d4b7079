"""Per-iteration GPU vs oracle differences on the time-blob restart case
(diagnostic for tests/test_gpu_parity.py::test_time_blobs_tw_restart_vs_oracle)."""
import sys
sys.path[:0] = ['.', 'oracle', 'tests']
import numpy as np
import test_gpu_parity as T
from helpers import rel

for n in (1, 2, 3):
    m, o, X = T._c3_like(33, 40, 3, 4, 1, n)
    for mod in (m, o):
        T._time_blobs(mod, {0: (3, 'free', 'free'), 2: (5, 'free', 'free')})
        mod.spec_comps[0]['factor'][0]['TW'] *= 1e-12
        mod.spec_comps[0]['factor'][0]['TB'] *= 1e12
    np.random.seed(13)
    ll = m.estim_param_a_post_model()
    np.random.seed(13)
    llo = o.estim_param_a_post_model()
    print("iters", n, "ll", rel(ll, llo), "oracle restarted", o.restarted)
    for k in sorted(o.spec_comps):
        f, g = m.spec_comps[k]['factor'][0], o.spec_comps[k]['factor'][0]
        print("  comp", k, {key: "%.2e" % rel(f[key], g[key]) for key in ('FB', 'FW', 'TW', 'TB')
                            if len(g[key])}, "sumTW %.3e" % np.sum(g['TW']))
    for j in range(3):
        print("  spat", j, "%.2e" % rel(m.spat_comps[j]['params'], o.spat_comps[j]['params']))
