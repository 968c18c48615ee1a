"""Adapter sets (mirror of porechop_abi/adapters.py).

``Adapter`` keeps the reference's attribute names and methods (porechop_abi/adapters.py:18-52)
because the phase drivers and NanoporeRead use them. The sequence database itself is data:
custom_porechop_abi_amd/data/adapters.json, extracted from the reference by
tools/extract_adapters.py (119 sets, porechop_abi/adapters.py:77-463).
"""
import json
import os

_DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'data', 'adapters.json')


class Adapter(object):
    """One adapter set: optional (name, seq) start and end sequences plus the best identities
    seen during adapter-set discovery."""

    def __init__(self, name, start_sequence=None, end_sequence=None, both_ends_sequence=None):
        self.name = name
        if both_ends_sequence:
            start_sequence = end_sequence = both_ends_sequence
        self.start_sequence = start_sequence if start_sequence else []
        self.end_sequence = end_sequence if end_sequence else []
        self.best_start_score = 0.0
        self.best_end_score = 0.0

    def best_start_or_end_score(self):
        return max(self.best_start_score, self.best_end_score)

    def is_barcode(self):
        return self.name.startswith('Barcode ')

    def barcode_direction(self):
        return 'reverse' if '_rev' in self.start_sequence[0] else 'forward'

    def get_barcode_name(self):
        """Shortest of the set name and its sequence names, spaces -> underscores."""
        names = [self.name]
        if self.start_sequence:
            names.append(self.start_sequence[0])
        if self.end_sequence:
            names.append(self.end_sequence[0])
        return min(names, key=len).replace(' ', '_')

    def __repr__(self):
        return 'Adapter(%r)' % self.name


def _load():
    with open(_DATA) as f:
        d = json.load(f)
    sets = []
    for e in d['sets']:
        sets.append(Adapter(e['name'],
                            start_sequence=tuple(e['start']) if e['start'] else None,
                            end_sequence=tuple(e['end']) if e['end'] else None,
                            both_ends_sequence=tuple(e['both']) if e['both'] else None))
    return sets, d['full_barcode_flanks']


ADAPTERS, _FLANKS = _load()


def fresh_adapters():
    """A new list of Adapter objects (best scores reset), same order as ADAPTERS."""
    return _load()[0]


def _barcode(num, direction):
    name = 'Barcode %d (%s)' % (num, direction)
    return [x for x in ADAPTERS if x.name == name][0]


def make_full_native_barcode_adapter(barcode_num):
    """porechop_abi/adapters.py:466-476."""
    up, down, end_up, end_down = _FLANKS['make_full_native_barcode_adapter']
    bc = _barcode(barcode_num, 'reverse')
    return Adapter('Native barcoding %d (full sequence)' % barcode_num,
                   start_sequence=('NB%02d_start' % barcode_num, up + bc.start_sequence[1] + down),
                   end_sequence=('NB%02d_end' % barcode_num, end_up + bc.end_sequence[1] + end_down))


def make_old_full_rapid_barcode_adapter(barcode_num):
    """porechop_abi/adapters.py:479-487 (SQK-RBK001)."""
    a, b, tail = _FLANKS['make_old_full_rapid_barcode_adapter']
    bc = _barcode(barcode_num, 'forward')
    return Adapter('Rapid barcoding %d (full sequence, old)' % barcode_num,
                   start_sequence=('RB%02d_full' % barcode_num, a + b + bc.start_sequence[1] + tail))


def make_new_full_rapid_barcode_adapter(barcode_num):
    """porechop_abi/adapters.py:490-498 (SQK-RBK004)."""
    a, b, tail = _FLANKS['make_new_full_rapid_barcode_adapter']
    bc = _barcode(barcode_num, 'forward')
    return Adapter('Rapid barcoding %d (full sequence, new)' % barcode_num,
                   start_sequence=('RB%02d_full' % barcode_num, a + b + bc.start_sequence[1] + tail))
