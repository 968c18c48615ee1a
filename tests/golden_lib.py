"""Loaders for the committed golden fixtures (tests/golden/)."""
import gzip
import json
import os

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def g1_rows(name='g1_alignments.tsv.gz'):
    """[(scheme tuple, read, adapter, reference result string)] -- tools/make_golden_g1.py."""
    rows = []
    with gzip.open(os.path.join(GOLDEN, name), 'rt') as f:
        for line in f:
            line = line.rstrip('\n')
            if not line:
                continue
            sc, r, a, res = line.split('\t')
            rows.append((tuple(int(x) for x in sc.split(',')), r, a, res))
    return rows


def g1_long_rows():
    """The same for adapters longer than 128 bp -- tools/make_golden_g1_long.py."""
    return g1_rows('g1_long.tsv.gz')


def g1_freegap_rows():
    """The same under gap costs >= 0, match <= 0 and all-zero scorings, reads up to 70 kb --
    tools/make_golden_g1_freegap.py."""
    return g1_rows('g1_freegap.tsv.gz')


def g2():
    """Reference driver decisions -- tools/make_golden_g2.py."""
    with gzip.open(os.path.join(GOLDEN, 'g2_decisions.json.gz'), 'rt') as f:
        return json.load(f)


def load_records(fn):
    """(name, seq, quals) records of a fixture under tests/golden/data (gzipped FASTA/FASTQ),
    parsed the way porechop_abi/misc.py:123-168 does (first header token = name)."""
    with gzip.open(os.path.join(GOLDEN, 'data', fn + '.gz'), 'rt') as f:
        lines = [l.rstrip('\n') for l in f]
    out = []
    if lines[0].startswith('@'):
        for i in range(0, len(lines) - 3, 4):
            out.append((lines[i].strip()[1:].split()[0], lines[i + 1].strip(), lines[i + 3].strip()))
    else:
        name, seq = None, []
        for l in lines + ['>']:
            l = l.strip()
            if l.startswith('>'):
                if name is not None:
                    out.append((name, ''.join(seq), ''))
                name, seq = (l[1:].split()[0] if l[1:] else None), []
            elif l:
                seq.append(l)
    return out
