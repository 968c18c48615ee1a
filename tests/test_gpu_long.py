"""GPU parity at the edges of the hot path, vs the CPU oracle (oracle/pcabi_oracle.c, pinned to
the reference by tests/test_oracle_golden.py):

  * adapters longer than 128 bp -- the striped core (pcabi_dp.h align_lane_striped,
    k_align_striped) -- in cross and pairs mode, through the legacy string ABI (the reference's
    own golden rows above 128 bp), in the middle scan (every round-1 path: seeds, score filter,
    full cross product) and in check_compatibility;
  * the legacy adapterAlignment symbol called from ThreadPool(16) workers, as the reference's
    phase drivers call it (porechop_abi.py:228, 418, 504);
  * the middle scan at BASELINE.json's read lengths: 20 kb-mean reads with reads past the 32 k
    and 65 k marks (configs[4]), and >= 1,000 reads x the 98-adapter middle list of the first 50
    adapter sets (the bench configuration, configs[2]).
"""
import random
from multiprocessing.dummy import Pool as ThreadPool

import numpy as np
import pytest

from tests import golden_lib, oracle_lib

SCHEMES = [(3, -6, -5, -2), (2, -1, -1, -1), (1, -1, -3, -1), (3, -6, -2, -5), (5, -4, -8, -6),
           (2, -1, 0, 0), (5, -4, -1, 0)]   # the last two: gap costs >= 0 (no path-span bound)
LONG_L = (129, 200, 255, 512, 1000)


def _rand(rng, n, alph='ACGT'):
    return ''.join(rng.choice(alph) for _ in range(n))


def _mutate(rng, s, rate):
    out = []
    for c in s:
        x = rng.random()
        if x < rate / 3:
            out.append(rng.choice('ACGT'))
        elif x < 2 * rate / 3:
            continue
        elif x < rate:
            out.append(c + rng.choice('ACGT'))
        else:
            out.append(c)
    return ''.join(out)


def _long_case(seed, n_reads):
    rng = random.Random(seed)
    adps = [_rand(rng, L) for L in LONG_L] + ['AATGTACTTCGTTCAGTTACGTATTGCT', _rand(rng, 60), _rand(rng, 111)]
    reads = []
    for k in range(n_reads):
        n = rng.choice([0, 1, 40, 150, 150, rng.randint(150, 1400)])
        r = _rand(rng, n, 'ACGT' if rng.random() < 0.8 else 'ACGTN')
        if n > 20 and rng.random() < 0.7:
            cp = _mutate(rng, rng.choice(adps), rng.choice([0.0, 0.05, 0.15]))
            w = rng.random()
            if w < 0.25:
                r = cp[rng.randint(0, len(cp) // 2):] + r
            elif w < 0.5:
                r = r + cp[:rng.randint(1, len(cp))]
            else:
                p = rng.randint(0, len(r))
                r = r[:p] + cp + r[p:]
        reads.append(r)
    return reads, adps


def _check(got, exp, reads, adps, n):
    ok = exp[0] != -1
    assert np.array_equal(got[0], exp[0])
    bad = np.nonzero(np.any(got[:, ok] != exp[:, ok], axis=0))[0]
    assert len(bad) == 0, 'first mismatch: pair %d len(read)=%d len(adapter)=%d got=%s exp=%s' % (
        int(np.nonzero(ok)[0][bad[0]]), len(reads[int(np.nonzero(ok)[0][bad[0]]) % n]),
        len(adps[int(np.nonzero(ok)[0][bad[0]]) // n]), got[:, ok][:, bad[0]], exp[:, ok][:, bad[0]])


@pytest.mark.gpu
@pytest.mark.parametrize('scheme', SCHEMES)
def test_long_adapters_cross_and_pairs(gpu_lib, scheme):
    """L in {129, 200, 255, 512, 1000} (the striped bucket) next to 28 / 60 / 111 bp adapters in
    one table: the cross product over ragged windows (empty, 1 bp, end windows of 150, whole reads
    up to ~2.4 kb) and explicit pairs, every integer field vs the oracle."""
    from custom_porechop_abi_amd import engine
    reads, adps = _long_case(sum(scheme) * 7 + 1, 48)
    pack = engine.SeqPack(reads)
    views = pack.views(np.zeros(len(reads), np.int64), pack.lengths)
    n = len(reads)
    got = engine.align(views, adps, scheme)
    exp = oracle_lib.align_many(reads, adps, (np.tile(np.arange(n), len(adps)), np.repeat(np.arange(len(adps)), n)),
                                scheme)
    _check(got, exp, reads, adps, n)
    rng = random.Random(sum(scheme))
    pr = np.array([rng.randrange(n) for _ in range(300)], np.int32)
    pa = np.array([rng.randrange(len(adps)) for _ in range(300)], np.int32)
    got = engine.align(views, adps, scheme, pairs=(pr, pa))
    exp = oracle_lib.align_many(reads, adps, (pr, pa), scheme)
    ok = exp[0] != -1
    assert np.array_equal(got[0], exp[0]) and np.array_equal(got[:, ok], exp[:, ok])


@pytest.mark.gpu
def test_long_adapters_legacy_abi_golden(gpu_lib):
    """adapterAlignment() text == the reference's own text on its golden rows with adapters of
    129-1200 bp (tests/golden/g1_long.tsv.gz, from oracle/_ref/cpp_functions.so)."""
    from custom_porechop_abi_amd import cpp_function_wrappers as w
    n = 0
    for sc, r, a, exp in golden_lib.g1_long_rows()[::3]:
        got = w.adapter_alignment(r, a, list(sc))
        if exp.split(',')[0] == '-1':
            assert got.split(',')[0] == '-1'
        else:
            assert got == exp, (sc, len(r), len(a))
        n += 1
    assert n >= 500


@pytest.mark.gpu
def test_legacy_abi_concurrent_threadpool(gpu_lib):
    """The reference calls adapterAlignment from ThreadPool(threads) workers
    (porechop_abi.py:228, 418, 504); the drop-in must be re-entrant (SURVEY §8b Threading):
    2,000 concurrent calls over 16 threads, mixed read / adapter lengths (long adapters
    included) and all five schemes, each == the oracle's text."""
    from custom_porechop_abi_amd import cpp_function_wrappers as w
    rng = random.Random(2024)
    jobs = []
    for k in range(2000):
        sc = SCHEMES[k % len(SCHEMES)]
        L = rng.choice([1, 8, 22, 24, 28, 50, 68, 111, 150, 300])
        a = _rand(rng, L)
        r = _rand(rng, rng.choice([1, 30, 150, rng.randint(1, 600)]), rng.choice(['ACGT', 'ACGTN', 'AT']))
        if len(r) > 20 and rng.random() < 0.5:
            p = rng.randint(0, len(r))
            r = r[:p] + _mutate(rng, a, 0.1) + r[p:]
        jobs.append((r, a, sc))
    exp = [oracle_lib.result_string(r, a, sc) for r, a, sc in jobs]
    with ThreadPool(16) as pool:
        got = pool.map(lambda j: w.adapter_alignment(j[0], j[1], list(j[2])), jobs, chunksize=7)
    bad = [k for k in range(len(jobs)) if got[k] != exp[k]]
    assert not bad, (len(bad), jobs[bad[0]][2], got[bad[0]], exp[bad[0]])


@pytest.mark.gpu
@pytest.mark.parametrize('mode', ['seeds', 'filter', 'cross'])
def test_long_adapters_middle_scan(gpu_lib, monkeypatch, mode):
    """The middle scan with long adapters (200 / 512 bp) among short ones, on each round-1 path:
    seeds (the long adapters are every read's candidates next to the seeded short ones), the
    score filter, and the full cross product with k_first_hit. Reads carry 0-3 copies (some
    repeated), so later rounds re-align masked reads against long adapters too."""
    from custom_porechop_abi_amd import engine
    if mode == 'seeds':
        monkeypatch.setenv('PCABI_MIDDLE_SEEDS', '2')
    elif mode == 'filter':
        monkeypatch.setenv('PCABI_MIDDLE_SEEDS', '0')
    else:
        monkeypatch.setenv('PCABI_MIDDLE_FILTER', '0')
    rng = random.Random(404)
    adps = ['AATGTACTTCGTTCAGTTACGTATTGCT', 'GCAATACGTAACTGAACGAAGT', _rand(rng, 200), 'ACGTTTAGGCATTGCA',
            _rand(rng, 512)]
    reads = []
    for k in range(90):
        r = _rand(rng, rng.choice([0, 5, rng.randint(200, 2500)]))
        for _ in range(rng.choice([0, 1, 2, 3])):
            a = _mutate(rng, rng.choice(adps), rng.choice([0.0, 0.02, 0.06]))
            p = rng.randint(0, len(r))
            r = r[:p] + a + (a if rng.random() < 0.2 else '') + r[p:]
        reads.append(r)
    pack = engine.SeqPack(reads)
    views = pack.views(np.zeros(len(reads), np.int64), pack.lengths)
    for sc in [(3, -6, -5, -2), (2, -1, -1, -1)]:
        exp = oracle_lib.middle_scan_threaded(views, adps, sc, 90.0)
        assert exp.shape[1] > 40 and np.isin([2, 4], exp[1]).all()
        got = engine.middle_scan(views, adps, sc, 90.0)
        og = np.lexsort((np.arange(got.shape[1]), got[0]))
        oe = np.lexsort((np.arange(exp.shape[1]), exp[0]))
        assert got.shape == exp.shape and np.array_equal(got[:, og], exp[:, oe])


def _middle_list(n_sets=50):
    from custom_porechop_abi_amd import adapters as A
    from custom_porechop_abi_amd.porechop_abi import middle_adapter_list
    sets = [a for a in A.fresh_adapters() if '(full sequence)' not in a.name][:n_sets]
    return [x[1] for x in middle_adapter_list(sets)[0]]


def _scan_vs_oracle(reads_codes, adps, sc, thr):
    from custom_porechop_abi_amd import engine, synth
    pack = engine.SeqPack([synth.codes_to_str(r) for r in reads_codes])
    views = pack.views(np.zeros(len(reads_codes), np.int64), pack.lengths)
    got = engine.middle_scan(views, adps, sc, thr)
    exp = oracle_lib.middle_scan_threaded(views, adps, sc, thr)
    og = np.lexsort((np.arange(got.shape[1]), got[0]))
    oe = np.lexsort((np.arange(exp.shape[1]), exp[0]))
    assert got.shape == exp.shape, (got.shape, exp.shape)
    assert np.array_equal(got[:, og], exp[:, oe])
    return exp


@pytest.mark.gpu
def test_middle_scan_20kb_reads_past_32k_and_65k(gpu_lib):
    """BASELINE.json configs[4] read shape: synthetic reads of mean 20 kb (SURVEY §8d recipe) plus
    reads of 40 kb, 70 kb and 120 kb carrying adapter copies past the 32 k mark (the non-packed
    cores' start-column field) and the 65 k mark (its 16-bit wrap), against the 98-adapter middle
    list: hits bit-exact vs the reference's loop on the oracle."""
    from custom_porechop_abi_amd import synth
    rng = np.random.default_rng(20)
    reads = synth.make_reads(120, 20000, seed=2020)
    top = synth._codes(synth.Y_TOP)
    bottom = synth._codes(synth.Y_BOTTOM)
    for n, marks in ((40000, (33000, 39000)), (70000, (32800, 66000, 69900)), (120000, (65600, 100000, 119950))):
        r = rng.integers(0, 4, n, dtype=np.uint8)
        for k, p in enumerate(marks):
            cp = synth.mutate(rng, top if k % 2 == 0 else bottom, 0.03)
            r = np.concatenate([r[:p], cp, r[p:]])
        reads.append(r)
    assert max(len(r) for r in reads) > 65536
    exp = _scan_vs_oracle(reads, _middle_list(), (3, -6, -5, -2), 90.0)
    assert (exp[2] > 65536).sum() >= 2 and (exp[2] > 32768).sum() >= 4


@pytest.mark.gpu
def test_middle_scan_bench_configuration(gpu_lib):
    """The bench's middle configuration (configs[2]) on 1,200 reads: mean 8 kb, the full
    98-adapter middle list of the first 50 adapter sets (the merged 8-mer seed table over all of
    them), threshold 90: every hit, in every round, equal to the reference loop on the oracle."""
    from custom_porechop_abi_amd import synth
    adps = _middle_list()
    assert len(adps) >= 90
    reads = synth.make_reads(1200, 8000, seed=777)
    exp = _scan_vs_oracle(reads, adps, (3, -6, -5, -2), 90.0)
    assert exp.shape[1] > 500 and len(np.unique(exp[1])) >= 2
