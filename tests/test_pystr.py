"""The drivers' native host helpers (custom_porechop_abi_amd/csrc/pystr.c, module _pystr) against
the Python passes they replace: str buffers, attribute lists, the trim max-update and the
alignment tuples appended per read (porechop_abi._end_decisions_batch)."""
import ctypes
import random

import numpy as np
import pytest

from custom_porechop_abi_amd import engine
from custom_porechop_abi_amd.nanopore_read import NanoporeRead

pytestmark = pytest.mark.skipif(engine._pystr is None, reason='_pystr not built (__graft_entry__.build)')


def test_ascii_buffers_addresses_and_lengths():
    rng = random.Random(1)
    seqs = [''.join(rng.choice('ACGTN') for _ in range(rng.randint(0, 300))) for _ in range(500)]
    addr, lens = engine.str_buffers(seqs)
    assert lens.tolist() == [len(s) for s in seqs]
    for s, a in zip(seqs[:50], addr[:50].tolist()):
        assert ctypes.string_at(a, len(s)).decode('ascii') == s
    # the slicing path's cases: a non-ASCII str, bytes, an empty list
    assert engine.str_buffers(seqs[:3] + ['ACGé']) is None
    assert engine.str_buffers([b'ACGT']) is None
    assert engine.str_buffers([]) is None


def test_windows_pack_same_with_and_without_buffers():
    rng = random.Random(2)
    seqs = [''.join(rng.choice('ACGT') for _ in range(rng.randint(5, 200))) for _ in range(300)]
    st = np.array([rng.randint(0, len(s) - 1) for s in seqs], np.int64)
    ln = np.array([rng.randint(0, len(s) - a) for s, a in zip(seqs, st)], np.int64)
    a = engine.SeqPack.windows(seqs, st, ln)
    b = engine.SeqPack([s[x:x + y] for s, x, y in zip(seqs, st.tolist(), ln.tolist())])
    assert np.array_equal(a.codes, b.codes) and np.array_equal(a.offsets, b.offsets)
    assert np.array_equal(a.lengths, b.lengths)
    with pytest.raises(ValueError):
        engine.SeqPack.windows(seqs, st, ln + 1000)


def test_attr_list_and_raise_trims():
    rng = random.Random(3)
    reads = [NanoporeRead('r%d' % i, 'ACGT' * 10, '') for i in range(200)]
    for r in reads:
        r.start_trim_amount = rng.randint(0, 30)
        r.end_trim_amount = rng.randint(0, 30)
    assert engine._pystr.attr_list(reads, 'name') == [r.name for r in reads]
    st = np.array([rng.randint(0, 40) for _ in reads], np.int32)
    et = np.array([rng.randint(0, 40) for _ in reads], np.int32)
    want = [(max(r.start_trim_amount, int(a)), max(r.end_trim_amount, int(b))) for r, a, b in zip(reads, st, et)]
    engine._pystr.raise_trims(reads, st, et)
    assert [(r.start_trim_amount, r.end_trim_amount) for r in reads] == want
    assert all(type(r.start_trim_amount) is int for r in reads)


class _Slotted(object):
    __slots__ = ('name', 'seq', 'start_trim_amount', 'end_trim_amount')

    def __init__(self, i):
        self.name, self.seq, self.start_trim_amount, self.end_trim_amount = 'r%d' % i, 'ACGT' * (i % 5), i % 7, i % 3


class _Prop(object):
    """Attributes behind a property and a class attribute (no instance-dict value to prefetch)."""
    end_trim_amount = 2

    def __init__(self, i):
        self._s = i % 11
        self.seq = 'A' * (i % 9)
        self.name = 'p%d' % i

    @property
    def start_trim_amount(self):
        return self._s

    @start_trim_amount.setter
    def start_trim_amount(self, v):
        self._s = v


def _mixed_objects(n=300, seed=5):
    """NanoporeReads (shared-key instance dicts), reads whose dicts were unshared by attributes set
    in another order, __slots__ objects and property-backed ones, interleaved: the helpers'
    prefetching (object, instance dict, its value array, the value) must follow each kind."""
    rng = random.Random(seed)
    out = []
    for i in range(n):
        k = rng.randrange(4)
        if k == 0:
            out.append(NanoporeRead('r%d' % i, 'ACGT' * (i % 6), ''))
        elif k == 1:
            r = NanoporeRead('u%d' % i, 'GATT' * (i % 4), '')
            r.__dict__ = dict(reversed(list(r.__dict__.items())))   # a combined (unshared) table
            r.extra = i
            out.append(r)
        elif k == 2:
            out.append(_Slotted(i))
        else:
            out.append(_Prop(i))
    return out


def test_helpers_on_every_object_layout():
    rng = random.Random(6)
    objs = _mixed_objects()
    for name in ('seq', 'name', 'start_trim_amount', 'end_trim_amount'):
        assert engine._pystr.attr_list(objs, name) == [getattr(o, name) for o in objs]
    out = np.empty(len(objs), np.int64)
    engine._pystr.int_attrs(objs, 'start_trim_amount', out)
    assert out.tolist() == [o.start_trim_amount for o in objs]
    st = np.array([rng.randint(0, 12) for _ in objs], np.int32)
    et = np.zeros(len(objs), np.int32)           # never above: end trims stay (the class attribute too)
    want = [(max(o.start_trim_amount, int(a)), o.end_trim_amount) for o, a in zip(objs, st)]
    engine._pystr.raise_trims(objs, st, et)
    assert [(o.start_trim_amount, o.end_trim_amount) for o in objs] == want
    with pytest.raises(AttributeError):
        engine._pystr.attr_list(objs + [object()], 'seq')


def test_append_rows_matches_python_tuples():
    rng = random.Random(4)
    reads = [NanoporeRead('r%d' % i, 'ACGT', '') for i in range(50)]
    objs = ['adapter%d' % k for k in range(7)]
    m = 400
    rd = np.sort(np.array([rng.randrange(50) for _ in range(m)], np.int64))
    ob = np.array([rng.randrange(7) for _ in range(m)], np.int64)
    f1 = np.array([rng.random() * 100 for _ in range(m)])
    f2 = np.array([rng.random() * 100 for _ in range(m)])
    i1 = np.array([rng.randrange(150) for _ in range(m)], np.int64)
    i2 = np.array([rng.randrange(150) for _ in range(m)], np.int64)
    reads[3].start_adapter_alignments.append(('kept', 1.0, 2.0, 3, 4))     # appended after what is there
    want = {i: list(r.start_adapter_alignments) for i, r in enumerate(reads)}
    for k in range(m):
        want[int(rd[k])].append((objs[ob[k]], float(f1[k]), float(f2[k]), int(i1[k]), int(i2[k])))
    engine._pystr.append_rows(reads, 'start_adapter_alignments', objs, rd, ob, f1, f2, i1, i2)
    assert {i: r.start_adapter_alignments for i, r in enumerate(reads)} == want
    assert reads[rd[0]].start_adapter_alignments[-1][0] is objs[ob[np.flatnonzero(rd == rd[0])[-1]]]
    with pytest.raises(IndexError):
        engine._pystr.append_rows(reads, 'start_adapter_alignments', objs, np.array([99], np.int64),
                                  ob[:1], f1[:1], f2[:1], i1[:1], i2[:1])


def test_nanopore_read_init_fast_paths_match_reference_rules():
    """NanoporeRead.__init__'s upper-case and RNA shortcuts against the reference's rules
    (nanopore_read.py:35-40: seq.upper(), RNA when count('U') > count('T'), then U -> T)."""
    rng = random.Random(5)
    alpha = 'ACGTNUacgtnu-xyzé'
    for _ in range(5000):
        s = ''.join(rng.choice(alpha[:rng.randint(1, len(alpha))]) for _ in range(rng.randint(0, 30)))
        r = NanoporeRead('n', s, '')
        su = s.upper()
        rna = su.count('U') > su.count('T')
        assert r.rna == rna and r.seq == (su.replace('U', 'T') if rna else su), s
