"""The device DP core (custom_porechop_abi_amd/csrc/pcabi_dp.h), compiled for the HOST with g++,
against the oracle and the reference's golden vectors. This checks the exact arithmetic the
HIP kernels run (same source) without a GPU: the forward traceback-attribute propagation,
the pass-through padding rows of the fast core, the wrapped start-column field (reads longer
than 65 kb) and the exact "%f" identity rounding (pid6)."""
import ctypes
import os
import random
import subprocess
import tempfile

import pytest

from tests import golden_lib, oracle_lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope='module')
def model():
    out = os.path.join(tempfile.mkdtemp(prefix='pcabi_model_'), 'dp_model.so')
    subprocess.check_call(['g++', '-std=c++17', '-O2', '-shared', '-fPIC', '-o', out,
                           os.path.join(ROOT, 'tests', 'native', 'dp_model.cpp')])
    L = ctypes.CDLL(out)
    for fn in ('pcabi_model_align', 'pcabi_model_align_fast', 'pcabi_model_align_packed', 'pcabi_model_align_long'):
        getattr(L, fn).argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int] + \
            [ctypes.c_int] * 4 + [ctypes.c_void_p]
    L.pcabi_model_align_packed_rpl.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int,
                                               ctypes.c_int] + [ctypes.c_int] * 4 + [ctypes.c_void_p]
    L.pcabi_model_align_tagged.argtypes = L.pcabi_model_align_packed_rpl.argtypes
    L.pcabi_model_filter.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p,
                                     ctypes.c_int, ctypes.c_int] + [ctypes.c_int] * 4 + [ctypes.c_void_p]
    L.pcabi_model_filter_threshold.argtypes = [ctypes.c_int, ctypes.c_double] + [ctypes.c_int] * 4
    L.pcabi_model_align_chunked.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int] + \
        [ctypes.c_int] * 7 + [ctypes.c_void_p]
    L.pcabi_model_pid6.restype = ctypes.c_double
    L.pcabi_model_pid6.argtypes = [ctypes.c_int, ctypes.c_int]
    return L


def _run(model, fn, r, a, sc):
    out = (ctypes.c_int * 8)()
    rb, ab = r.encode(), a.encode()
    rc = getattr(model, fn)(rb, len(rb), ab, len(ab), *sc, out)
    return rc, list(out)


def _fmt(res):
    rs, re_, as_, ae, score, m, l1, l2 = res
    p1 = '-nan' if l1 == 0 else '%f' % (100.0 * m / l1)
    p2 = '-nan' if l2 == 0 else '%f' % (100.0 * m / l2)
    return '%d,%d,%d,%d,%d,%s,%s' % (rs, re_, as_, ae, score, p1, p2)


@pytest.mark.parametrize('fn', ['pcabi_model_align_packed', 'pcabi_model_align_fast', 'pcabi_model_align'])
def test_core_vs_reference_golden(model, fn):
    n_checked = 0
    for sc, r, a, exp in golden_lib.g1_rows():
        if not r or not a or len(a) > 128:
            continue
        rc, res = _run(model, fn, r, a, sc)
        if rc == -3:
            continue
        assert rc == 0
        assert _fmt(res) == exp, (sc, r, a, exp, res)
        n_checked += 1
    assert n_checked > (4000 if fn == 'pcabi_model_align_packed' else 15000)


@pytest.mark.parametrize('fn', ['pcabi_model_align_packed', 'pcabi_model_align_fast', 'pcabi_model_align'])
def test_core_fuzz_vs_oracle(model, fn):
    rng = random.Random(42)
    schemes = [(3, -6, -5, -2), (2, -1, -1, -1), (1, -1, -3, -1), (3, -6, -2, -5), (5, -4, -8, -6)]
    for _ in range(3000):
        sc = rng.choice(schemes)
        al = rng.choice(['A', 'AT', 'ACGT', 'ACGTN'])
        L = rng.randint(1, 128)
        a = ''.join(rng.choice(al) for _ in range(L))
        r = ''.join(rng.choice(al) for _ in range(rng.randint(1, 260)))
        rc, res = _run(model, fn, r, a, sc)
        if rc == -3:
            continue
        assert res == oracle_lib.align(r, a, sc), (sc, r, a)


def test_core_long_reads_wrapped_start_column(model):
    """Reads longer than the 16-bit start-column field: adapters placed past 65,536."""
    rng = random.Random(9)
    for k in range(4):
        n = 70000 + 30000 * k
        a = ''.join(rng.choice('ACGT') for _ in range(24))
        r = [rng.choice('ACGT') for _ in range(n)]
        p = n - 5000 if k % 2 else 66000
        r[p:p + 24] = list(a)
        r = ''.join(r)
        for sc in [(3, -6, -5, -2), (2, -1, -1, -1)]:
            exp = oracle_lib.align(r, a, sc)
            for fn in ('pcabi_model_align_fast', 'pcabi_model_align_packed'):
                rc, res = _run(model, fn, r, a, sc)
                assert rc == 0 and res == exp, fn


def _mutate(rng, s, rate):
    o = []
    for c in s:
        x = rng.random()
        if x < rate / 3:
            o.append(rng.choice('ACGT'))
        elif x < 2 * rate / 3:
            pass
        elif x < rate:
            o.append(c + rng.choice('ACGT'))
        else:
            o.append(c)
    return ''.join(o)


def test_packed_core_whole_reads(model):
    """Packed core on whole reads (the middle-adapter scan shape): the start diagonal is kept
    mod 256, so hits far into the read, gapped hits and adapters of 33..63 bp are the cases."""
    rng = random.Random(5)
    schemes = [(3, -6, -5, -2), (2, -1, -1, -1), (1, -1, -3, -1), (3, -6, -2, -5)]
    n_checked = 0
    for k in range(160):
        sc = schemes[k % len(schemes)]
        L = rng.choice([8, 22, 24, 31, 40, 52, 63])
        a = ''.join(rng.choice('ACGT') for _ in range(L))
        n = rng.randint(300, 2500)
        r = ''.join(rng.choice('ACGT') for _ in range(n))
        for _ in range(rng.randint(0, 3)):
            p = rng.randint(0, len(r))
            r = r[:p] + _mutate(rng, a, rng.choice([0.0, 0.05, 0.2])) + r[p:]
        rc, res = _run(model, 'pcabi_model_align_packed', r, a, sc)
        if rc == -3:
            continue
        assert rc == 0 and res == oracle_lib.align(r, a, sc), (sc, L, len(r))
        n_checked += 1
    assert n_checked > 100


def test_pid6_matches_text_round_trip(model):
    for l in range(1, 700):
        for m in range(0, l + 1):
            assert model.pcabi_model_pid6(m, l) == float('%f' % (100.0 * m / l))


def test_packed_core_extra_padding_rows(model):
    """Adapters run in a larger register bucket than their own (merged buckets): any number of
    pass-through padding rows above the adapter."""
    rng = random.Random(17)
    schemes = [(3, -6, -5, -2), (2, -1, -1, -1), (1, -1, -3, -1), (3, -6, -2, -5)]
    n_checked = 0
    for k in range(2500):
        sc = schemes[k % len(schemes)]
        al = rng.choice(['A', 'AT', 'ACGT', 'ACGTN'])
        L = rng.randint(1, 60)
        rpl = rng.choice([r for r in range(4, 68, 4) if r >= L])
        a = ''.join(rng.choice(al) for _ in range(L))
        r = ''.join(rng.choice(al) for _ in range(rng.randint(1, 260)))
        out = (ctypes.c_int * 8)()
        rc = model.pcabi_model_align_packed_rpl(r.encode(), len(r), a.encode(), L, rpl, *sc, out)
        if rc == -3:
            continue
        assert rc == 0 and list(out) == oracle_lib.align(r, a, sc), (sc, r, a, rpl)
        n_checked += 1
    assert n_checked > 2000


def _tagged(model, r, a, rpl, sc):
    out = (ctypes.c_int * 8)()
    rc = model.pcabi_model_align_tagged(r.encode(), len(r), a.encode(), len(a), rpl, *sc, out)
    return rc, list(out)


def test_tagged_core(model):
    """The run-tagged packed layout (pk::LayT: 7-bit run-counting tie tags, so the H key is
    stored without re-tagging, and c mod 128) against the oracle: tie-heavy alphabets, every small
    bucket with extra padding rows, long gap runs (adapters embedded with long insertions /
    deletions), and the reference's golden rows; layt_ok must accept the default scheme up to 31 bp
    in every bucket that holds the adapter (span bound L + 3L/2 <= 77 < 128, H runs <= 80 < the
    V-open tag 127 - rpl)."""
    rng = random.Random(23)
    schemes = [(3, -6, -5, -2), (1, -1, -3, -1), (3, -6, -2, -5), (5, -4, -8, -6), (2, -3, -5, -1), (2, -3, -2, -1)]
    for L in range(1, 32):
        for rpl in range((L + 3) & ~3, 33, 4):
            assert model.pcabi_model_align_tagged(b'A', 1, b'A' * L, L, rpl, 3, -6, -5, -2,
                                                  (ctypes.c_int * 8)()) == 0
    n_checked = 0
    for k in range(6000):
        sc = schemes[k % len(schemes)]
        al = rng.choice(['A', 'AT', 'ACGT', 'ACGTN'])
        L = rng.randint(1, 31)
        rpl = rng.choice([r for r in range(4, 33, 4) if r >= L])
        a = ''.join(rng.choice(al) for _ in range(L))
        if k % 3 == 0:
            r = ''.join(rng.choice(al) for _ in range(rng.randint(0, 60)))
            b = list(a)
            for _ in range(rng.randint(0, 3)):
                p = rng.randint(0, len(b))
                if rng.random() < 0.5:
                    b[p:p] = [rng.choice(al) for _ in range(rng.randint(1, 30))]
                else:
                    del b[p:p + rng.randint(1, 8)]
            r += ''.join(b) + ''.join(rng.choice(al) for _ in range(rng.randint(0, 60)))
            r = r or 'A'
        else:
            r = ''.join(rng.choice(al) for _ in range(rng.randint(1, 260)))
        rc, res = _tagged(model, r, a, rpl, sc)
        if rc == -3:
            continue
        assert rc == 0 and res == oracle_lib.align(r, a, sc), (sc, r, a, rpl)
        n_checked += 1
    assert n_checked > 4000
    # the longest gap runs: nothing matches, so H / V extend as far as the scores allow
    for sc in schemes:
        for L in (1, 8, 17, 24, 25, 26, 28, 30, 31):
            for n in (1, 60, 150, 400):
                a, r = 'C' * L, 'A' * n
                rc, res = _tagged(model, r, a, (L + 3) & ~3, sc)
                if rc == 0:
                    assert res == oracle_lib.align(r, a, sc), (sc, L, n)
    n_gold = 0
    for sc, r, a, exp in golden_lib.g1_rows():
        if not r or not a or len(a) > 31:
            continue
        rc, res = _tagged(model, r, a, (len(a) + 3) & ~3, sc)
        if rc == -3:
            continue
        assert rc == 0 and _fmt(res) == exp, (sc, r, a, exp, res)
        n_gold += 1
    assert n_gold > 1000


def test_cores_mismatch_outscoring_match(model):
    """Schemes where a mismatch scores as much as or more than a match (the reference takes any
    --scoring_scheme): every range and span bound uses max(match, mismatch), so the packed,
    run-tagged and fast cores either run exactly or decline (-3) -- never overflow."""
    rng = random.Random(31)
    schemes = [(1, 6, -5, -2), (2, 20, -5, -2), (1, 3, -5, -2), (0, 0, -1, -2), (2, 2, -3, -1), (-1, 4, -6, -3)]
    ran = {'packed': 0, 'tagged': 0, 'fast': 0}
    for k in range(1800):
        sc = schemes[k % len(schemes)]
        L = rng.randint(1, 63)
        a = ''.join(rng.choice('ACGT') for _ in range(L))
        r = ''.join(rng.choice('ACGT') for _ in range(rng.randint(1, 200)))
        exp = oracle_lib.align(r, a, sc)
        rc, res = _run(model, 'pcabi_model_align_packed', r, a, sc)
        if rc == 0:
            assert res == exp, ('packed', sc, r, a)
            ran['packed'] += 1
        rc, res = _run(model, 'pcabi_model_align_fast', r, a, sc)
        if rc == 0:
            assert res == exp, ('fast', sc, r, a)
            ran['fast'] += 1
        if L <= 31:
            rc, res = _tagged(model, r, a, (L + 3) & ~3, sc)
            if rc == 0:
                assert res == exp, ('tagged', sc, r, a)
                ran['tagged'] += 1
    assert min(ran.values()) > 100, ran


def test_packed_wide_core(model):
    """Wide register buckets (68..88 rows, pk::Lay<RPL > 64>: 9-bit score, count field m +
    (RPL + 1) nD): the 63-88 bp adapters -- the native barcoding "full sequence" adapters
    (porechop_abi/adapters.py:466-477) among them -- on end windows and whole reads, embedded
    mutated hits, extra padding rows, several scorings."""
    from custom_porechop_abi_amd import adapters as A
    full = []
    for i in (1, 7, 12):
        f = A.make_full_native_barcode_adapter(i)
        full += [f.start_sequence[1], f.end_sequence[1]]
    rng = random.Random(31)
    schemes = [(3, -6, -5, -2), (2, -1, -1, -1), (1, -1, -3, -1), (3, -6, -2, -5)]
    n_checked = 0
    for k in range(700):
        sc = schemes[k % len(schemes)]
        if k % 3 == 0:
            a = rng.choice(full)
        else:
            a = ''.join(rng.choice(rng.choice(['ACGT', 'AT', 'ACGTN'])) for _ in range(rng.randint(61, 88)))
        L = len(a)
        rpl = rng.choice([x for x in range(68, 92, 4) if x >= L])
        n = rng.choice([rng.randint(1, 150), 150, rng.randint(200, 1500)])
        r = ''.join(rng.choice('ACGT') for _ in range(n))
        for _ in range(rng.randint(0, 2)):
            p = rng.randint(0, len(r))
            r = r[:p] + _mutate(rng, a, rng.choice([0.0, 0.05, 0.15])) + r[p:]
        out = (ctypes.c_int * 8)()
        rc = model.pcabi_model_align_packed_rpl(r.encode(), len(r), a.encode(), L, rpl, *sc, out)
        if rc == -3:
            continue
        assert rc == 0 and list(out) == oracle_lib.align(r, a, sc), (sc, L, rpl, len(r))
        n_checked += 1
    assert n_checked > 500


def test_score_filter_wide_buckets(model):
    """The score filter at the wide register buckets (68..88 rows)."""
    rng = random.Random(37)
    schemes = [(3, -6, -5, -2), (2, -1, -1, -1), (3, -6, -2, -5)]
    for k in range(300):
        sc = schemes[k % len(schemes)]
        La, Lb = rng.randint(40, 88), rng.randint(1, 88)
        rpl = rng.choice([x for x in range(68, 92, 4) if x >= max(La, Lb)])
        a = ''.join(rng.choice('ACGT') for _ in range(La))
        b = ''.join(rng.choice('ACGT') for _ in range(Lb))
        r = ''.join(rng.choice('ACGT') for _ in range(rng.randint(1, 600)))
        if rng.random() < 0.5 and len(r) > 100:
            p = rng.randint(0, len(r) - 90)
            r = r[:p] + _mutate(rng, a, 0.05) + r[p:]
        out = (ctypes.c_int * 2)()
        rc = model.pcabi_model_filter(r.encode(), len(r), a.encode(), La, b.encode(), Lb, rpl, *sc, out)
        assert rc == 0
        assert list(out) == [oracle_lib.align(r, a, sc)[4], oracle_lib.align(r, b, sc)[4]], (sc, La, Lb, rpl)


def test_score_filter_equals_best_score(model):
    """The packed-16 score-only filter (two adapters per lane) returns exactly the best score the
    reference reports, for both halves, across scorings, paddings and read lengths."""
    rng = random.Random(23)
    schemes = [(3, -6, -5, -2), (2, -1, -1, -1), (1, -1, -3, -1), (3, -6, -2, -5)]
    n_checked = 0
    for k in range(1500):
        sc = schemes[k % len(schemes)]
        al = rng.choice(['A', 'AT', 'ACGT', 'ACGTN'])
        La, Lb = rng.randint(1, 60), rng.randint(1, 60)
        rpl = rng.choice([x for x in range(4, 68, 4) if x >= max(La, Lb)])
        a = ''.join(rng.choice(al) for _ in range(La))
        b = ''.join(rng.choice(al) for _ in range(Lb))
        r = ''.join(rng.choice(al) for _ in range(rng.randint(1, 400)))
        if rng.random() < 0.3 and len(r) > 70:
            p = rng.randint(0, len(r) - 60)
            r = r[:p] + a + r[p:]
        out = (ctypes.c_int * 2)()
        rc = model.pcabi_model_filter(r.encode(), len(r), a.encode(), La, b.encode(), Lb, rpl, *sc, out)
        if rc == -3:
            continue
        assert rc == 0
        assert list(out) == [oracle_lib.align(r, a, sc)[4], oracle_lib.align(r, b, sc)[4]], (sc, r, a, b, rpl)
        n_checked += 1
    assert n_checked > 1000


def test_score_filter_threshold_is_a_lower_bound(model):
    """Every alignment whose full identity reaches the threshold scores at least the filter's
    bound (checked on hits of mutated adapters, where the bound is tight)."""
    from custom_porechop_abi_amd.engine import pid6
    import numpy as np
    rng = random.Random(29)
    checked = 0
    for k in range(3000):
        sc = rng.choice([(3, -6, -5, -2), (2, -1, -1, -1), (1, -1, -3, -1), (3, -6, -2, -5)])
        thr = rng.choice([90.0, 85.0, 80.0, 95.0])
        L = rng.randint(8, 50)
        a = ''.join(rng.choice('ACGT') for _ in range(L))
        m = []
        for c in a:
            x = rng.random()
            if x < 0.04:
                m.append(rng.choice('ACGT'))
            elif x < 0.06:
                continue
            elif x < 0.08:
                m.append(c + rng.choice('ACGT'))
            else:
                m.append(c)
        r = ''.join(rng.choice('ACGT') for _ in range(rng.randint(0, 40))) + ''.join(m) + \
            ''.join(rng.choice('ACGT') for _ in range(rng.randint(0, 40)))
        res = oracle_lib.align(r, a, sc)
        if res[0] == -1:
            continue
        full = float(pid6(np.array([res[5]]), np.array([res[7]]))[0])
        if full >= thr:
            assert res[4] >= model.pcabi_model_filter_threshold(L, thr, *sc), (sc, thr, r, a, res)
            checked += 1
    assert checked > 500


@pytest.mark.parametrize('core', ['packed', 'generic', 'tagged'])
@pytest.mark.parametrize('sc', [(3, -6, -5, -2), (2, -1, -1, -1), (1, -1, -3, -1), (5, -4, -8, -6), (1, 2, -4, -2)])
def test_chunked_candidate_dp(model, sc, core):
    """The middle scan's chunked candidate DP (pcabi_dp.h sf::chunk_plan + align_lane_packed with
    CHUNK): reads split into chunks of C owned columns, each aligned alone, merged in read order.
    Whenever the whole-read best score reaches T (the bound every hit must reach) the merged
    result equals the whole-read result field for field; below T it stays below T. Chunk sizes
    down to a few columns put chunk boundaries inside adapter copies, at read ends and between
    equal-score copies (the first must win)."""
    rng = random.Random(sum(sc) * 31 + 7)
    n_hi = n_lo = n_multi = 0
    adps = ['AATGTACTTCGTTCAGTTACGTATTGCT', 'GCAATACGTAACTGAACGAAGT', 'ACGTTTAGGCATTGCA',
            ''.join(rng.choice('ACGT') for _ in range(40)), ''.join(rng.choice('ACGT') for _ in range(64))]
    if core == 'generic':   # long adapters (the 102 / 111 bp full rapid sequences) too
        adps += [''.join(rng.choice('ACGT') for _ in range(L)) for L in (102, 111)]
    if core == 'tagged':    # the run-tagged chunk kernels (k_align_chunk<.., TAGGED>): <= 31 bp
        adps = [x for x in adps if len(x) <= 31] + [''.join(rng.choice('ACGT') for _ in range(31))]
        if sc[2] == sc[3]:
            pytest.skip('the run-tagged layout is affine only')
    for it in range(1500 if core != 'generic' else 300):
        a = rng.choice(adps)
        n = rng.choice([rng.randint(1, 60), rng.randint(60, 600), rng.randint(600, 2500)])
        r = ''.join(rng.choice('ACGT') for _ in range(n))
        for _ in range(rng.choice([0, 1, 1, 2, 3])):
            copy = _mutate_cpu(rng, a, rng.choice([0.0, 0.05, 0.1, 0.2]))
            where = rng.random()
            if where < 0.2:
                r = copy[rng.randint(0, 5):] + r
            elif where < 0.4:
                r = r + copy[:max(1, len(copy) - rng.randint(0, 5))]
            else:
                p = rng.randint(0, len(r))
                r = r[:p] + copy + (copy if rng.random() < 0.3 else '') + r[p:]
        for thr in (90.0, 75.0):
            T = model.pcabi_model_filter_threshold(len(a), thr, *sc)
            if T <= 0:
                continue
            rc, whole = _run(model, 'pcabi_model_align_packed' if core == 'packed' else 'pcabi_model_align', r, a, sc)
            if rc == -3:
                continue
            C = rng.choice([1, 3, 17, 64, 200, 1000])
            out = (ctypes.c_int * 8)()
            rb, ab = r.encode(), a.encode()
            nc = model.pcabi_model_align_chunked(rb, len(rb), ab, len(ab), *sc, T, C,
                                                 {'packed': 0, 'generic': 1, 'tagged': 2}[core], out)
            if nc == -3 and core == 'tagged':
                continue
            assert nc > 0, (nc, sc, T, C)
            got = list(out)
            if whole[4] >= T:
                assert got == whole, (sc, thr, T, C, r, a, got, whole)
                n_hi += 1
                n_multi += nc > 1
            else:
                assert got[4] < T, (sc, thr, T, C, r, a, got, whole)
                n_lo += 1
    # mismatch outscoring match: nearly every read clears T, so few below-T cases exist
    assert n_hi > 40 and n_multi > 40 and (n_lo > 40 or sc[1] > sc[0]), (n_hi, n_lo, n_multi)


def _mutate_cpu(rng, s, rate):
    out = []
    for c in s:
        x = rng.random()
        if x < rate / 3:
            out.append(rng.choice('ACGT'))
        elif x < 2 * rate / 3:
            continue
        elif x < rate:
            out.append(c)
            out.append(rng.choice('ACGT'))
        else:
            out.append(c)
    return ''.join(out)


def test_long_two_pass_core(model):
    """The long buckets' two-pass packed core (pk::LayL, align_lane_packed_long: c / nD in one
    pass, m in the other, same scores and tie bits) vs the oracle: the reference's 89-111 bp
    golden rows, then random and tie-heavy reads against 89-128 bp adapters with embedded
    mutated copies, every scoring scheme that fits."""
    n_checked = 0
    for sc, r, a, exp in golden_lib.g1_rows():
        if not r or not a or not (88 < len(a) <= 128):
            continue
        rc, res = _run(model, 'pcabi_model_align_long', r, a, sc)
        if rc == -3:
            continue
        assert rc == 0 and _fmt(res) == exp, (sc, r, a, _fmt(res), exp)
        n_checked += 1
    rng = random.Random(77)
    for it in range(600):
        sc = rng.choice([(3, -6, -5, -2), (2, -1, -1, -1), (1, -1, -3, -1), (3, -6, -2, -5), (5, -4, -8, -6)])
        L = rng.choice([89, 96, 97, 102, 111, 112, 113, 128])
        alph = rng.choice(['ACGT', 'AT', 'ACGTN'])
        a = ''.join(rng.choice('ACGT') for _ in range(L))
        n = rng.choice([1, 5, 40, 150, rng.randint(1, 400)])
        r = ''.join(rng.choice(alph) for _ in range(n))
        if n > 30 and rng.random() < 0.7:
            cp = _mutate_cpu(rng, a, rng.choice([0.0, 0.05, 0.15]))
            p = rng.randint(-20, n)
            r = (r[:max(p, 0)] + cp[max(-p, 0):] + r[max(p, 0):])[:max(n, 1) + L]
        rc, res = _run(model, 'pcabi_model_align_long', r, a, sc)
        if rc == -3:
            continue
        assert rc == 0 and list(res) == oracle_lib.align(r, a, sc), (sc, r, a)
        n_checked += 1
    assert n_checked > 400


def _striped(model, r, a, sc, R, extra_pad=0, own_lo=1, own_hi=-1):
    model.pcabi_model_align_striped.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int] + \
        [ctypes.c_int] * 8 + [ctypes.c_void_p]
    out = (ctypes.c_int * 8)()
    rb, ab = r.encode(), a.encode()
    rc = model.pcabi_model_align_striped(rb, len(rb), ab, len(ab), R, extra_pad, *sc, own_lo, own_hi, out)
    assert rc == 0
    return list(out)


def test_striped_core_many_stripes(model):
    """The striped core (align_lane_striped: adapters of any length, row stripes of R rows, the
    boundary row through a per-lane buffer) with narrow stripes, so short adapters already cross
    many stripe boundaries: random and tie-heavy alphabets, every scheme (linear and affine,
    open cheaper than extend), whole padding stripes above the adapter."""
    rng = random.Random(101)
    schemes = [(3, -6, -5, -2), (2, -1, -1, -1), (1, -1, -3, -1), (3, -6, -2, -5), (5, -4, -8, -6)]
    for it in range(2500):
        sc = schemes[it % len(schemes)]
        al = rng.choice(['A', 'AT', 'ACGT', 'ACGTN'])
        L = rng.randint(1, 80)
        a = ''.join(rng.choice(al) for _ in range(L))
        r = ''.join(rng.choice(al) for _ in range(rng.randint(1, 220)))
        if rng.random() < 0.4 and len(r) > 20:
            p = rng.randint(0, len(r))
            r = r[:p] + _mutate_cpu(rng, a, rng.choice([0.0, 0.1])) + r[p:]
        R = rng.choice([8, 16, 32])
        got = _striped(model, r, a, sc, R, extra_pad=rng.choice([0, 0, 1, 2]))
        assert got == oracle_lib.align(r, a, sc), (sc, R, r, a)


def test_striped_core_long_adapters(model):
    """Adapters of 129-1200 bp (custom adapter files, ab-initio adapters with a large -sl) on end
    windows and longer reads, mutated copies (whole, cut at the read ends), the reference's
    golden rows above 128 bp."""
    n_gold = 0
    for sc, r, a, exp in golden_lib.g1_rows() + golden_lib.g1_long_rows():
        if not r or not a or len(a) <= 128:
            continue
        assert _fmt(_striped(model, r, a, sc, 32)) == exp, (sc, len(r), len(a))
        n_gold += 1
    assert n_gold >= 500
    rng = random.Random(103)
    schemes = [(3, -6, -5, -2), (2, -1, -1, -1), (1, -1, -3, -1), (3, -6, -2, -5), (5, -4, -8, -6)]
    for it in range(150):
        sc = schemes[it % len(schemes)]
        L = rng.choice([129, 200, 255, 256, 300, 512, 700])
        a = ''.join(rng.choice('ACGT') for _ in range(L))
        n = rng.choice([1, 40, 150, rng.randint(150, 1500)])
        r = ''.join(rng.choice('ACGT' if rng.random() < 0.8 else 'ACGTN') for _ in range(n))
        if rng.random() < 0.7:
            cp = _mutate_cpu(rng, a, rng.choice([0.0, 0.05, 0.15]))
            w = rng.random()
            if w < 0.25:
                r = cp[rng.randint(0, L // 2):] + r
            elif w < 0.5:
                r = r + cp[:rng.randint(1, len(cp))]
            else:
                p = rng.randint(0, len(r))
                r = r[:p] + cp + r[p:]
        got = _striped(model, r, a, sc, 32)
        assert got == oracle_lib.align(r, a, sc), (sc, L, len(r))


@pytest.mark.parametrize('sc', [(3, -6, -5, -2), (2, -1, -1, -1), (5, -4, -8, -6)])
def test_striped_core_chunks(model, sc):
    """The striped core in chunk mode (the middle scan's candidate DP on long adapters): chunks
    of C owned columns merged in read order equal the whole read whenever its score reaches T."""
    rng = random.Random(sum(sc) + 211)
    adps = [''.join(rng.choice('ACGT') for _ in range(L)) for L in (40, 150, 260)]
    n_hi = 0
    for it in range(60):
        a = rng.choice(adps)
        r = ''.join(rng.choice('ACGT') for _ in range(rng.randint(200, 2500)))
        for _ in range(rng.choice([1, 1, 2])):
            p = rng.randint(0, len(r))
            r = r[:p] + _mutate_cpu(rng, a, rng.choice([0.0, 0.05])) + r[p:]
        T = model.pcabi_model_filter_threshold(len(a), 85.0, *sc)
        D = len(a) + (len(a) * sc[0] - T + min(-sc[2], -sc[3]) - 1) // min(-sc[2], -sc[3]) + 2
        whole = oracle_lib.align(r, a, sc)
        C = rng.choice([7, 100, 512])
        best = None
        for lo in range(1, len(r) + 1, C):
            hi = lo + C
            start = max(0, lo - 1 - D)
            last = hi > len(r)
            seg = r[start:] if last else r[start:hi - 1]
            got = _striped(model, seg, a, sc, 32, own_lo=lo - start, own_hi=-1 if last else hi - start)
            if best is None or got[4] > best[4]:
                best = got[:]
                if best[0] >= 0:
                    best[0] += start
                    best[1] += start
            if last:
                break
        if whole[4] >= T:
            assert best == whole, (sc, len(a), C)
            n_hi += 1
        else:
            assert best[4] < T
    assert n_hi > 20


def test_cores_free_gap_schemes_golden(model):
    """Scorings with gap costs >= 0, match <= 0 or all zero (the reference accepts any four
    integers, porechop_abi/arg_parser.py:229-236), on the reference's own rows
    (tests/golden/g1_freegap.tsv.gz): the generic core (the register buckets such schemes get) on
    windows below 32 k, and the striped core -- where the engine routes windows of 32 k and more
    under a scoring with no path-span bound -- on every row, the 33-70 kb reads included."""
    n_gen = n_str = n_long = 0
    for sc, r, a, exp in golden_lib.g1_freegap_rows():
        if not r or not a:
            continue
        if len(a) <= 128 and len(r) < 32768 - 256:
            rc, res = _run(model, 'pcabi_model_align', r, a, sc)
            assert rc == 0 and _fmt(res) == exp, (sc, len(r), len(a), exp, res)
            n_gen += 1
        assert _fmt(_striped(model, r, a, sc, 32)) == exp, (sc, len(r), len(a))
        n_str += 1
        n_long += len(r) >= 32768
    assert n_gen >= 1500 and n_str >= 1800 and n_long >= 30


def test_row_split_core(model):
    """The row-split packed core (pcabi_dp.h LaneSplit, k_align_split: K lanes per window, each
    holding RPL / K rows, the lanes a systolic pipeline with the last column in K phases), run by
    the host model in lockstep: == the oracle for the run-tagged and packed layouts, K = 2 and 4,
    every bucket, tie-heavy alphabets, long gap runs, extra padding rows (whole padding lanes
    included), windows of 1 column and the reference's golden rows."""
    model.pcabi_model_align_split.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int] + \
        [ctypes.c_int] * 7 + [ctypes.c_void_p]

    def split(r, a, rpl, K, tagged, sc):
        out = (ctypes.c_int * 8)()
        rc = model.pcabi_model_align_split(r.encode(), len(r), a.encode(), len(a), rpl, K, tagged, *sc, out)
        return rc, list(out)

    rng = random.Random(77)
    schemes = [(3, -6, -5, -2), (2, -1, -1, -1), (1, -1, -3, -1), (3, -6, -2, -5), (5, -4, -8, -6), (2, -3, -5, -1),
               (1, 3, -5, -2)]
    n_checked = {(t, K): 0 for t in (0, 1) for K in (2, 4)}
    for k in range(8000):
        sc = schemes[k % len(schemes)]
        tagged = k % 2
        K = rng.choice([2, 4])
        al = rng.choice(['A', 'AT', 'ACGT', 'ACGTN'])
        L = rng.randint(1, 31 if tagged else 64)
        rpl = rng.choice([r for r in range(8, (33 if tagged else 65), 4) if r >= L and r % K == 0 and r // K >= 2])
        a = ''.join(rng.choice(al) for _ in range(L))
        if k % 3 == 0:
            b = list(a)
            for _ in range(rng.randint(0, 3)):
                p = rng.randint(0, len(b))
                if rng.random() < 0.5:
                    b[p:p] = [rng.choice(al) for _ in range(rng.randint(1, 30))]
                else:
                    del b[p:p + rng.randint(1, 8)]
            r = ''.join(rng.choice(al) for _ in range(rng.randint(0, 60))) + ''.join(b) + \
                ''.join(rng.choice(al) for _ in range(rng.randint(0, 60)))
            r = r or 'A'
        else:
            r = ''.join(rng.choice(al) for _ in range(rng.choice([1, 2, 3, rng.randint(1, 260)])))
        rc, res = split(r, a, rpl, K, tagged, sc)
        if rc == -3:
            continue
        assert rc == 0 and res == oracle_lib.align(r, a, sc), (sc, r, a, rpl, K, tagged)
        n_checked[(tagged, K)] += 1
    assert min(n_checked.values()) > 800, n_checked
    for sc in schemes:                                # the longest gap runs
        for L in (1, 8, 17, 24, 28, 31):
            for n in (1, 60, 150, 400):
                for K in (2, 4):
                    for tagged in (0, 1):
                        rpl = max(8, (L + 3) & ~3)
                        rpl += (-rpl) % (4 * K // 2)
                        rc, res = split('A' * n, 'C' * L, rpl, K, tagged, sc)
                        if rc == 0:
                            assert res == oracle_lib.align('A' * n, 'C' * L, sc), (sc, L, n, K, tagged)
    n_gold = 0
    for sc, r, a, exp in golden_lib.g1_rows():
        if not r or not a or len(a) > 64:
            continue
        rpl = max(8, (len(a) + 3) & ~3)
        for K in (2, 4):
            if rpl % K or rpl // K < 2:
                continue
            rc, res = split(r, a, rpl, K, int(len(a) <= 31), sc)
            if rc == -3 or (rc == -2 and len(a) <= 31):
                rc, res = split(r, a, rpl, K, 0, sc)
            if rc != 0:
                continue
            assert _fmt(res) == exp, (sc, r, a, exp, res, K)
            n_gold += 1
    assert n_gold > 2000


def test_row_split_chunk_core(model):
    """The row-split core in chunk mode (k_align_split_chunk: the middle scan's candidate DP with K
    lanes per chunk task): inner columns gated by the owned range (the lead-in columns cannot be
    the row-L best), then the K-phase last column for a read's last chunk (own_hi < 0) or the last
    lane's materialize for an inner chunk (reported as not at the read end). Field for field equal
    to the one-lane chunk core (align_lane_packed with CHUNK) on the same chunk, both layouts,
    K = 2 and 4, every bucket, owned ranges anywhere in the chunk (empty ones included)."""
    model.pcabi_model_split_chunk.argtypes = [ctypes.c_char_p, ctypes.c_int, ctypes.c_char_p, ctypes.c_int] + \
        [ctypes.c_int] * 9 + [ctypes.c_void_p, ctypes.c_void_p]
    rng = random.Random(91)
    schemes = [(3, -6, -5, -2), (2, -1, -1, -1), (1, -1, -3, -1), (3, -6, -2, -5), (5, -4, -8, -6), (2, -3, -5, -1)]
    n_checked = {(t, K, e): 0 for t in (0, 1) for K in (2, 4) for e in (0, 1)}
    for k in range(6000):
        sc = schemes[k % len(schemes)]
        tagged = k % 2
        K = rng.choice([2, 4])
        al = rng.choice(['AT', 'ACGT', 'ACGTN'])
        L = rng.randint(1, 31 if tagged else 64)
        rpl = rng.choice([r for r in range(8, (33 if tagged else 65), 4) if r >= L and r % K == 0 and r // K >= 2])
        a = ''.join(rng.choice(al) for _ in range(L))
        b = list(a)
        for _ in range(rng.randint(0, 2)):
            p = rng.randint(0, len(b))
            if rng.random() < 0.5:
                b[p:p] = [rng.choice(al) for _ in range(rng.randint(1, 6))]
            else:
                del b[p:p + rng.randint(1, 4)]
        r = ''.join(rng.choice(al) for _ in range(rng.randint(0, 80))) + ''.join(b) + \
            ''.join(rng.choice(al) for _ in range(rng.randint(0, 80)))
        r = r or 'A'
        n = len(r)
        at_end = rng.random() < 0.4
        own_lo = rng.randint(1, n + 1)
        own_hi = -1 if at_end else rng.randint(own_lo, n + 1)
        o_split, o_lane = (ctypes.c_int * 8)(), (ctypes.c_int * 8)()
        rc = model.pcabi_model_split_chunk(r.encode(), n, a.encode(), L, rpl, K, tagged, *sc, own_lo, own_hi,
                                           o_split, o_lane)
        if rc == -3:
            continue
        assert rc == 0 and list(o_split) == list(o_lane), (sc, r, a, rpl, K, tagged, own_lo, own_hi,
                                                             list(o_split), list(o_lane))
        n_checked[(tagged, K, int(at_end))] += 1
    assert min(n_checked.values()) > 300, n_checked
