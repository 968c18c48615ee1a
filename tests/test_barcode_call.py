"""Barcode call epilogue (k_barcode_call, include/pcabi.h pcabi_barcode_call_*) vs the reference's
rules: NanoporeRead.determine_barcode (porechop_abi/nanopore_read.py:408-482) over the dicts that
find_start_trim / find_end_trim fill (:193-195, :215-217).

Scores are drawn from few (m, l2) values so equal identities -- where only the stable sorts
decide -- are the common case; barcode names repeat across sides and within a side (a dict keeps
a name's first position and its last value); failed alignments (rs == -1) score 0.0.
  * not gpu: a Python restatement of the kernel's slot scan (the algorithm) vs determine_barcode;
  * gpu    : the HIP kernel through the C ABI vs determine_barcode, and on the reference's
             barcoded test reads (G2 golden decisions) end to end.
"""
import random

import numpy as np
import pytest

from custom_porechop_abi_amd.adapters import Adapter
from custom_porechop_abi_amd.nanopore_read import NanoporeRead
from custom_porechop_abi_amd.porechop_abi import barcode_slots


def _pid6(m, l):
    return float('%f' % (100.0 * m / l))


def _random_case(seed, n_read):
    rng = random.Random(seed)
    fr = rng.choice(['forward', 'reverse'])
    nb = rng.randint(1, 6)

    def side_sets():
        sets = []
        for _ in range(rng.randint(0, 9)):
            kind = rng.random()
            if kind < 0.15:
                sets.append(Adapter('SQK-NSK007', start_sequence=('Y_Top', 'A'), end_sequence=('Y_Bottom', 'A')))
                continue
            b = rng.randint(1, nb)
            d = fr if kind < 0.85 else ('reverse' if fr == 'forward' else 'forward')
            nm = 'BC%02d' % b + ('_rev' if d == 'reverse' else '')
            sets.append(Adapter('Barcode %d (%s)' % (b, d), start_sequence=(nm, 'A'), end_sequence=(nm, 'A')))
        return sets

    sides = []
    for _ in range(2):
        sets = side_sets()
        res = np.zeros((8, max(1, len(sets)) * n_read), np.int32)
        ms = [rng.randint(0, 24) for _ in range(4)]
        ls = [rng.randint(20, 26) for _ in range(3)]
        for a in range(len(sets)):
            for r in range(n_read):
                i = a * n_read + r
                res[0, i] = -1 if rng.random() < 0.06 else rng.randint(0, 100)
                res[5, i] = rng.choice(ms)
                res[7, i] = rng.choice(ls)
        sides.append((sets, res[:, :len(sets) * n_read]))
    thr = rng.choice([0.0, 50.0, 75.0, 90.0])
    diff = rng.choice([0.0, 1.0, 5.0])
    return fr, sides, thr, diff


def _expected(fr, sides, n_read, thr, diff, require_two):
    calls = []
    for r in range(n_read):
        read = NanoporeRead('r', 'A', '')
        for side, (sets, res) in zip(('start', 'end'), sides):
            d = read.start_barcode_scores if side == 'start' else read.end_barcode_scores
            for a, s in enumerate(sets):
                if s.is_barcode() and s.barcode_direction() == fr:
                    i = a * n_read + r
                    d[s.get_barcode_name()] = 0.0 if res[0, i] == -1 else _pid6(res[5, i], res[7, i])
        read.determine_barcode(thr, diff, require_two)
        calls.append(read.barcode_call)
    return calls


def _scan(sides_slots, n_read, thr, diff, require_two):
    """Python restatement of k_barcode_call (csrc/pcabi_engine.hip): strict '>' scans in slot
    order. Returns barcode ids (-1 = 'none')."""
    out = []
    for r in range(n_read):
        def score(res, a):
            i = a * n_read + r
            return 0.0 if res[0, i] == -1 else _pid6(res[5, i], res[7, i])
        if require_two:
            best = []
            for res, (adp, name) in sides_slots:
                b = [0.0, 0.0]
                bn, cnt = -1, 0
                for a, nm in zip(adp.tolist(), name.tolist()):
                    x = score(res, a)
                    if cnt == 0 or x > b[0]:
                        if cnt:
                            b[1] = b[0]
                        b[0], bn = x, nm
                    elif cnt == 1 or x > b[1]:
                        b[1] = x
                    cnt += 1
                best.append((b, bn))
            (bs, ns), (be, ne) = best
            ok = bs[0] >= thr and be[0] >= thr and bs[0] >= bs[1] + diff and be[0] >= be[1] + diff and ns == ne
            out.append(ns if ok else -1)
        else:
            b1 = b2 = 0.0
            n1, has1, has2 = -1, False, False
            for res, (adp, name) in sides_slots:
                for a, nm in zip(adp.tolist(), name.tolist()):
                    x = score(res, a)
                    if not has1 or x > b1:
                        if has1 and n1 != nm:
                            b2, has2 = b1, True
                        b1, n1, has1 = x, nm, True
                    elif nm != n1 and (not has2 or x > b2):
                        b2, has2 = x, True
            out.append(n1 if (b1 >= thr and b1 >= b2 + diff and has1) else -1)
    return out


def _slots(fr, sides):
    ids = {}
    slots = [barcode_slots(sets, fr, ids) for sets, _ in sides]
    names = {v: k for k, v in ids.items()}
    return slots, names


@pytest.mark.parametrize('require_two', [False, True])
def test_slot_scan_restatement_matches_determine_barcode(require_two):
    n_read = 40
    for seed in range(150):
        fr, sides, thr, diff = _random_case(seed, n_read)
        slots, names = _slots(fr, sides)
        got = _scan([(res, sl) for (_, res), sl in zip(sides, slots)], n_read, thr, diff, require_two)
        got = [names.get(x, 'none') for x in got]
        assert got == _expected(fr, sides, n_read, thr, diff, require_two), seed


@pytest.mark.gpu
@pytest.mark.parametrize('require_two', [False, True])
def test_barcode_call_kernel_matches_determine_barcode(gpu_lib, require_two):
    from custom_porechop_abi_amd import engine
    n_read = 300
    for seed in range(60):
        fr, sides, thr, diff = _random_case(1000 + seed, n_read)
        slots, names = _slots(fr, sides)
        call = engine.barcode_call(sides[0][1], sides[1][1], slots[0], slots[1], n_read, thr, diff, require_two)
        got = [names.get(int(x), 'none') for x in call]
        assert got == _expected(fr, sides, n_read, thr, diff, require_two), seed


@pytest.mark.gpu
@pytest.mark.parametrize('case_name', ['barcodes', 'barcodes_two', 'choose_barcodes'])
def test_barcode_call_on_reference_reads(gpu_lib, case_name):
    """The reference's barcoded test reads: GPU alignments + GPU barcode call == the reference's
    barcode_call for every read (G2)."""
    import io
    from custom_porechop_abi_amd import adapters as A, engine, porechop_abi as P
    from tests import golden_lib
    case = [c for c in golden_lib.g2()['cases'] if c['case'] == case_name][0]
    opts = case['opts']
    sc = opts['scoring']
    recs = golden_lib.load_records(case['input'])
    reads = [NanoporeRead(n, s, q) for n, s, q in recs]
    sets = A.fresh_adapters()
    matching = P.find_matching_adapter_sets(reads[:10000], 0, opts['end_size'], sc, io.StringIO(),
                                            opts['adapter_threshold'], 1, adapter_sets=sets)
    matching = P.fix_up_1d2_sets(matching)
    fr = P.choose_barcoding_kit(matching, 0, io.StringIO())
    matching = P.add_full_barcode_adapter_sets(matching)
    starts = [a for a in matching if a.start_sequence]
    ends = [a for a in matching if a.end_sequence]
    pack = engine.SeqPack([r.seq for r in reads])
    sw, ew = engine.start_end_windows(pack, opts['end_size'])
    sres = engine.align(sw, [a.start_sequence[1] for a in starts], sc)
    eres = engine.align(ew, [a.end_sequence[1] for a in ends], sc)
    ids = {}
    ss, es = barcode_slots(starts, fr, ids), barcode_slots(ends, fr, ids)
    names = {v: k for k, v in ids.items()}
    call = engine.barcode_call(sres, eres, ss, es, len(reads), 75.0, 5.0, opts.get('require_two', False))
    exp = [r['barcode_call'] for r in case['reads']]
    assert [names.get(int(x), 'none') for x in call] == exp
    assert any(x != 'none' for x in exp)
