"""The CPU oracle (oracle/pcabi_oracle.c) reproduces the reference's adapterAlignment text on
every golden vector produced by the reference itself (tests/golden/g1_alignments.tsv.gz,
tools/make_golden_g1.py) and on the reference's known answers."""
import pytest

from tests import golden_lib, oracle_lib


@pytest.mark.parametrize('which', ['g1', 'g1_long', 'g1_freegap'])
def test_oracle_matches_reference_vectors(which):
    rows = {'g1': golden_lib.g1_rows, 'g1_long': golden_lib.g1_long_rows, 'g1_freegap': golden_lib.g1_freegap_rows}[which]()
    assert len(rows) >= {'g1': 20000, 'g1_long': 1500, 'g1_freegap': 2000}[which]
    bad = []
    for sc, r, a, exp in rows:
        got = oracle_lib.result_string(r, a, sc)
        if exp.split(',')[0] == '-1':            # empty input: only field 0 is defined
            ok = got.split(',')[0] == '-1'
        else:
            ok = got == exp
        if not ok:
            bad.append((sc, r[:60], a, exp, got))
    assert not bad, bad[:5]


def test_known_answers():
    sc = (3, -6, -5, -2)
    cases = [('ACGTACGTAC', 'GTAC', '2,5,0,3,12,100.000000,100.000000'),
             ('AAAAAAAAAA', 'AAAA', '0,3,0,3,12,100.000000,100.000000'),
             ('AAAA', 'AAAAAAAAAA', '0,3,0,3,12,100.000000,40.000000'),
             ('GGGGGGGG', 'TTTT', '0,0,4,3,0,-nan,0.000000'),
             ('A', 'C', '0,0,1,0,0,-nan,0.000000'),
             ('AC--GT', 'ACGT', '0,5,0,3,5,66.666667,66.666667')]
    for r, a, exp in cases:
        assert oracle_lib.result_string(r, a, sc) == exp
    assert oracle_lib.result_string('', 'ACGT', sc).split(',')[0] == '-1'


def test_threaded_middle_loop_equals_python_loop():
    """The oracle's C middle loop (pcabi_oracle_middle_scan, threads over reads: the checker of
    the bench-sized middle-scan tests) == the reference's loop restated in Python on the oracle."""
    import random

    import numpy as np

    from custom_porechop_abi_amd import engine
    rng = random.Random(5)
    adps = ['AATGTACTTCGTTCAGTTACGTATTGCT', 'GCAATACGTAACTGAACGAAGT', ''.join(rng.choice('ACGT') for _ in range(150))]
    reads = []
    for k in range(60):
        r = ''.join(rng.choice('ACGT') for _ in range(rng.randint(0, 1500)))
        for _ in range(rng.choice([0, 1, 2, 3])):
            p = rng.randint(0, len(r))
            a = rng.choice(adps)
            r = r[:p] + a + (a if rng.random() < 0.2 else '') + r[p:]
        reads.append(r)
    pack = engine.SeqPack(reads)
    views = pack.views(np.zeros(len(reads), np.int64), pack.lengths)
    for sc in [(3, -6, -5, -2), (2, -1, -1, -1)]:
        a = oracle_lib.middle_scan_windows(views, adps, sc, 85.0)
        b = oracle_lib.middle_scan_threaded(views, adps, sc, 85.0, 4)
        assert a.shape[1] > 50 and np.array_equal(a, b)
