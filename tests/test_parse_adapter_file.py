"""Custom adapter files (porechop_abi/parse_adapter_file.py:17-73): parsing, naming, the DNA
check and its exit, and the parsed sets through the batched drivers (long adapters included)."""
import subprocess
import sys

import pytest


def test_custom_adapter_file_sets(tmp_path):
    from custom_porechop_abi_amd.parse_adapter_file import get_adapters
    long_seq = 'ACGT' * 50                      # 200 bp: the striped core's range
    p = tmp_path / 'custom.txt'
    p.write_text('kit A\nAATGTACTTCGT\nGCAATACGTAAC\nstart only\nTTTTACGT\n\nend only\n\nCCCGGG\n'
                 'long\n%s\n%s\nincomplete\nACGT\n' % (long_seq, long_seq))
    sets = get_adapters(str(p))
    assert [a.name for a in sets] == ['kit A', 'start only', 'end only', 'long']
    assert sets[0].start_sequence == ('kit A_Top', 'AATGTACTTCGT')
    assert sets[0].end_sequence == ('kit A_Bottom', 'GCAATACGTAAC')
    assert sets[1].end_sequence == [] and sets[2].start_sequence == []
    assert sets[3].start_sequence[1] == long_seq and sets[3].best_start_or_end_score() == 0.0


@pytest.mark.parametrize('bad', ['ACGN', 'acgt', 'AC GT'])
def test_custom_adapter_file_rejects_non_dna(tmp_path, bad):
    p = tmp_path / 'bad.txt'
    p.write_text('x\n%s\n\n' % bad)
    code = ('import sys; sys.path.insert(0, %r); from custom_porechop_abi_amd.parse_adapter_file import get_adapters;'
            'get_adapters(%r)' % (str(__import__('os').path.dirname(__import__('os').path.dirname(
                __import__('os').path.abspath(__file__)))), str(p)))
    r = subprocess.run([sys.executable, '-c', code], capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and 'INVALID FORMAT' in r.stdout and ('Start: ' + bad) in r.stdout


@pytest.mark.gpu
def test_custom_long_adapters_through_the_drivers(gpu_lib, tmp_path):
    """A custom set with 200 bp sequences trims reads through find_adapters_at_read_ends exactly
    like the oracle-backed drivers (the reference's per-read rules on oracle alignments)."""
    import io
    import random
    from custom_porechop_abi_amd import engine, porechop_abi as P
    from custom_porechop_abi_amd.nanopore_read import NanoporeRead
    from custom_porechop_abi_amd.parse_adapter_file import get_adapters
    from tests import oracle_lib
    rng = random.Random(3)
    top = ''.join(rng.choice('ACGT') for _ in range(200))
    bottom = ''.join(rng.choice('ACGT') for _ in range(160))
    p = tmp_path / 'custom.txt'
    p.write_text('long kit\n%s\n%s\n' % (top, bottom))
    sets = get_adapters(str(p))

    def reads():
        out = []
        r2 = random.Random(5)
        for k in range(40):
            body = ''.join(r2.choice('ACGT') for _ in range(r2.randint(300, 900)))
            s = (top[r2.randint(0, 30):] if k % 2 else '') + body + (bottom[:160 - r2.randint(0, 30)] if k % 3 else '')
            out.append(NanoporeRead('r%d' % k, s, '+' * len(s)))
        return out
    got, exp = reads(), reads()
    P.find_adapters_at_read_ends(got, sets, 0, 260, 2, 75.0, (3, -6, -5, -2), io.StringIO(), 4, 1, False, 75.0, 5.0,
                                 False, None)
    saved = engine.align
    engine.align = oracle_lib.align_windows
    try:
        P.find_adapters_at_read_ends(exp, sets, 0, 260, 2, 75.0, (3, -6, -5, -2), io.StringIO(), 4, 1, False, 75.0,
                                     5.0, False, None)
    finally:
        engine.align = saved
    assert [(r.start_trim_amount, r.end_trim_amount) for r in got] == \
        [(r.start_trim_amount, r.end_trim_amount) for r in exp]
    assert sum(r.start_trim_amount > 0 for r in got) >= 15 and sum(r.end_trim_amount > 0 for r in got) >= 20
