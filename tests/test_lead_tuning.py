"""SeparateLeadProcess.computeChroma / determineTuning
(SeparateLeadStereo/SeparateLeadStereoTF.py:1074-1128): host analysis of the
pipeline's HF0, on injected state (no GPU call).

The reference is Python 2 code: its `patterns.keys()` order (the row order
of scoresPerTuning, and which pattern wins a tie) is CPython 2.7's dict
order for the four names, recomputed here from that interpreter's string
hash and probe sequence rather than taken from the implementation; its
`/` on the argmax is integer division."""
import numpy as np
import pytest

from pyfasst_amd.SeparateLeadStereo.SeparateLeadStereoTF import SeparateLeadProcess

PATTERNS = {'minorHarmoPattern': [0, 2, 3, 5, 7, 8, 10],
            'minorMelodPattern': [0, 2, 3, 5, 7, 9, 11],
            'majorPattern': [0, 2, 4, 5, 7, 9, 11],
            'andalusPattern': [0, 1, 4, 5, 7, 8, 11]}
INSERTION = ['minorHarmoPattern', 'minorMelodPattern', 'majorPattern', 'andalusPattern']


def _py2_hash(s):
    """CPython 2.7 string_hash on 64-bit Linux (no -R)."""
    M = 1 << 64
    x = (ord(s[0]) << 7) % M
    for c in s:
        x = ((1000003 * x) % M) ^ ord(c)
    x ^= len(s)
    if x >= 1 << 63:
        x -= M
    return -2 if x == -1 else x


def _py2_dict_order(keys):
    """Iteration order of a CPython 2.7 dict filled by setitem in `keys`
    order (8-slot table, lookdict_string probing)."""
    assert len(keys) <= 5            # no resize below fill 2/3 of 8
    table, mask = [None] * 8, 7
    for k in keys:
        h = _py2_hash(k)
        i, perturb = h & mask, h % (1 << 64)
        while table[i & mask] is not None:
            i = ((i << 2) + i + perturb + 1) % (1 << 64)
            perturb >>= 5
        table[i & mask] = k
    return [k for k in table if k is not None]


def test_py2_hash_known_value():
    assert _py2_hash('a') == 12416037344     # CPython 2.7, 64-bit: hash('a')


def _proc(HF0, stepNotes):
    return SeparateLeadProcess(None, SIMMParams={'HF0': HF0, 'stepNotes': stepNotes},
                               N=HF0.shape[1], verbose=False)


def test_compute_chroma_folds_octaves_and_normalises():
    rng = np.random.RandomState(3)
    stepNotes, N = 2, 19
    HF0 = rng.rand(12 * stepNotes * 3 + 5, N)
    p = _proc(HF0, stepNotes)
    p.computeChroma()
    want = np.zeros([24, N])
    for n in range(24):
        rows = list(range(n, HF0.shape[0], 24))
        want[n] = sum(HF0[r] for r in rows) / len(rows)
    want /= want.sum(axis=0)
    np.testing.assert_allclose(p.chroma, want, rtol=1e-14)
    np.testing.assert_allclose(p.chroma.sum(axis=0), 1.0, rtol=1e-14)


def _scores(summary, stepNotes, order):
    out = np.zeros([len(order), 12 * stepNotes])
    for a, name in enumerate(order):
        for ntun in range(stepNotes):
            for nk in range(12):
                out[a, ntun + nk * stepNotes] = sum(
                    summary[((q + nk) * stepNotes + ntun) % summary.size] for q in PATTERNS[name])
    return out


@pytest.mark.parametrize("stepNotes", [1, 3])
def test_determine_tuning_vs_restatement(stepNotes):
    order = _py2_dict_order(INSERTION)
    rng = np.random.RandomState(stepNotes)
    p = _proc(rng.rand(12 * stepNotes * 4, 30), stepNotes)
    scores, tun, key, name = p.determineTuning()
    want = _scores(p.chroma.sum(axis=1), stepNotes, order)
    np.testing.assert_allclose(scores, want, rtol=1e-13)
    b = int(np.argmax(want))
    assert (name, key, tun) == (order[b // (12 * stepNotes)], (b % (12 * stepNotes)) // stepNotes,
                                b % stepNotes)


def test_determine_tuning_major_scale_tie_goes_to_the_relative_minor():
    """A C#-major scale (key 1) on tuning 1 of 2: the natural minor
    ('minorHarmoPattern' in the reference's table) on key 1 + 9 scores the
    same, and in the reference's Python 2 key order it comes first."""
    stepNotes, key, tun = 2, 1, 1
    HF0 = np.full([12 * stepNotes * 2, 8], 1e-6)
    for q in PATTERNS['majorPattern']:
        HF0[((q + key) % 12) * stepNotes + tun::12 * stepNotes] = 1.0
    p = _proc(HF0, stepNotes)
    scores, btun, bkey, name = p.determineTuning()
    assert _py2_dict_order(INSERTION).index('minorHarmoPattern') < \
        _py2_dict_order(INSERTION).index('majorPattern')
    assert (name, bkey, btun) == ('minorHarmoPattern', (key + 9) % 12, tun)
