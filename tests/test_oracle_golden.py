"""The CPU oracle (oracle/pcabi_oracle.c) reproduces the reference's adapterAlignment text on
every golden vector produced by the reference itself (tests/golden/g1_alignments.tsv.gz,
tools/make_golden_g1.py) and on the reference's known answers."""
from tests import golden_lib, oracle_lib


def test_oracle_matches_reference_vectors():
    rows = golden_lib.g1_rows()
    assert len(rows) >= 20000
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
