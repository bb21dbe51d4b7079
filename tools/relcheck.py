import sys, os, tempfile
sys.path.insert(0, '.'); sys.path.insert(0, 'tests'); sys.path.insert(0, 'oracle')
import numpy as np
from helpers import CASES, load, rel, spec_keys
import test_gpu_parity as T
for case in ['em_conv', 'em_conv_j4', 'em_fw_free', 'em_multi', 'em_multi_inst', 'em_inst']:
    g = load(case); J = CASES[case][0]
    m = T._product_model(case, g, tempfile.mkdtemp())
    ll = m.estim_param_a_post_model()
    rp = max(rel(m.spat_comps[j]['params'], g['final_params_%d' % j]) for j in range(J))
    rs = max(max(rel(m.spec_comps[k]['factor'][0][x], g['final_%s_%d' % (x, k)]) for x in ('FB','TW','FW')) for k in spec_keys(g, J))
    print(case, 'll %.2e params %.2e spec %.2e' % (rel(ll, g['logliks']), rp, rs), flush=True)
