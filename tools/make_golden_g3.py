"""G3 golden vectors: sequence-file parsing and trimmed-read output produced by the REFERENCE'S
OWN Python code (porechop_abi.misc.load_fasta_or_fastq, porechop_abi.nanopore_read.NanoporeRead
normalisation and get_fasta / get_fastq with trims and middle splits).

Container-only generator (imports the reference the way tools/make_golden_g2.py does). Writes
  tests/golden/io/*          : small edge-case input files (data; generated here, seeded)
  tests/golden/g3_io.json.gz : per input file, the reference's records, NanoporeRead fields and
                               output strings for a set of seeded trim / split settings.
The reference's own test files (tests/golden/data/*.gz) are inputs too.
"""
import gzip
import json
import os
import random
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from make_golden_g2 import setup_reference  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
IO = os.path.join(ROOT, 'tests', 'golden', 'io')
DATA = os.path.join(ROOT, 'tests', 'golden', 'data')
OUT = os.path.join(ROOT, 'tests', 'golden', 'g3_io.json.gz')


def rand_seq(rng, n, alph='ACGT'):
    return ''.join(rng.choice(alph) for _ in range(n))


def edge_files(rng):
    """(file name, bytes) of the edge cases the parser must handle like the reference."""
    files = []
    # FASTQ: CRLF endings, lower case, tabs / spaces in headers, RNA reads, IUPAC, short quals
    recs = []
    for k in range(12):
        n = rng.randint(0, 300)
        alph = rng.choice(['ACGT', 'acgt', 'ACGU', 'ACGUU', 'ACGTNRYKM', 'acgun'])
        s = rand_seq(rng, n, alph)
        q = rand_seq(rng, n if k % 4 else max(0, n - rng.randint(1, 20)), '!#%&+5:?AI')
        name = rng.choice(['read%d' % k, 'read%d runid=abc ch=%d' % (k, k), 'read%d\tbarcode=BC01' % k,
                           ' read%d  lead' % k])
        recs.append('@%s\n%s\n+%s\n%s\n' % (name, s, rng.choice(['', name]), q))
    files.append(('crlf_mixed.fastq', ''.join(recs).replace('\n', '\r\n').encode()))
    files.append(('lone_cr.fastq', ''.join(recs[:5]).replace('\n', '\r').encode()))
    files.append(('plain_mixed.fastq', ''.join(recs).encode()))
    files.append(('no_final_newline.fastq', ''.join(recs)[:-1].encode()))
    files.append(('whitespace.fastq', ''.join('@  w%d x \n  %s \t\n+\n %s\x0c\n' % (k, rand_seq(rng, 40), 'I' * 40)
                                              for k in range(4)).encode()))
    # FASTA: multi-line, blank lines, empty header (sequence carries over), whitespace lines
    fa = ['>c1 first contig\n'] + [rand_seq(rng, 60) + '\n' for _ in range(5)] + ['\n', '  \n']
    fa += ['>\n', rand_seq(rng, 33) + '\n', '>c2\n', rand_seq(rng, 10, 'acgtu') + '\n', rand_seq(rng, 7) + '\n']
    fa += ['>c3\tx=1\n', '\n', '>c4 rna\n', rand_seq(rng, 150, 'ACGUUU') + '\n', '>c5 long\n']
    fa += [rand_seq(rng, 1000) + '\n']
    files.append(('multi.fasta', ''.join(fa).encode()))
    files.append(('multi_crlf.fasta', ''.join(fa).replace('\n', '\r\n').encode()))
    files.append(('multi.fasta.gz', gzip.compress(''.join(fa).encode(), mtime=0)))
    files.append(('plain_mixed.fastq.gz', gzip.compress(''.join(recs).encode(), mtime=0)))
    return files


def main():
    P, NR = setup_reference()
    import importlib
    M = importlib.import_module('porechop_abi.misc')
    rng = random.Random(2024)
    os.makedirs(IO, exist_ok=True)
    inputs = []
    for name, data in edge_files(rng):
        with open(os.path.join(IO, name), 'wb') as f:
            f.write(data)
        inputs.append(('io/' + name, os.path.join(IO, name)))
    for name in sorted(os.listdir(DATA)):
        inputs.append(('data/' + name, os.path.join(DATA, name)))
    cases = []
    for key, path in inputs:
        recs, kind = M.load_fasta_or_fastq(path)
        if kind == 'FASTA':
            reads = [NR.NanoporeRead(x[2], x[1], '') for x in recs]
        else:
            reads = [NR.NanoporeRead(x[4], x[1], x[3]) for x in recs]
        outs = []
        for setting in range(4):
            srng = random.Random(setting * 7919 + len(recs))
            trims, cuts = [], []
            for r in reads:
                n = len(r.seq)
                st = srng.choice([0, 0, srng.randint(0, 40), n + 5])
                et = srng.choice([0, 0, srng.randint(0, 40), n + 30])
                r.start_trim_amount, r.end_trim_amount = st, et
                r.middle_trim_positions = set()
                if setting >= 2 and n > 50 and srng.random() < 0.6:
                    for _ in range(srng.randint(1, 3)):
                        a = srng.randint(-20, n)
                        r.middle_trim_positions.update(range(a, a + srng.randint(1, 60)))
                trims.append([st, et])
                cuts.append(sorted(r.middle_trim_positions))
            min_split = [0, 1000, 10, 25][setting]
            discard = setting == 3
            untrimmed = setting == 1
            outs.append({'trims': trims, 'cuts': cuts, 'min_split': min_split, 'discard_middle': discard,
                         'untrimmed': untrimmed,
                         'fasta': ''.join(r.get_fasta(min_split, discard, untrimmed) for r in reads),
                         'fastq': ''.join(r.get_fastq(min_split, discard, untrimmed) for r in reads)
                         if kind == 'FASTQ' else None})
        cases.append({'file': key, 'type': kind, 'records': [list(x) for x in recs],
                      'reads': [[r.name, r.seq, r.quals, r.rna] for r in reads], 'outputs': outs})
    with gzip.open(OUT, 'wt') as f:
        json.dump({'generator': 'tools/make_golden_g3.py', 'cases': cases}, f)
    print('wrote', OUT, len(cases), 'cases')


if __name__ == '__main__':
    main()
