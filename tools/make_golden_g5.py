"""G5 golden vectors: the REFERENCE'S OWN ab-initio k-mer counter (oracle/_ref/approx_counter,
compiled by `make -C oracle ref` from porechop_abi/ab_initio_src/approx_counter.cpp and the
vendored SeqAn) on seeded synthetic read sets.

Container-only generator. The reference samples reads with std::random_device; every run here
asks for more reads than the file holds (-sn), so the whole set is used and the counts are
deterministic. Inputs (tests/golden/kmer/*.fasta.gz) carry start / end adapters (mutated), N
letters, lower case and short reads (IUPAC letters other than N make the reference's SeqAn
reader throw); parameter sets cover k 12 / 16 / 20, the limit, the
low-complexity threshold, forbidden k-mers, solid k-mers, two runs, and skip-end at verbosity 0
(the reference then recomputes the start into the .end file). Writes tests/golden/g5_kmer.json.gz.
"""
import gzip
import json
import os
import random
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KDIR = os.path.join(ROOT, 'tests', 'golden', 'kmer')
OUT = os.path.join(ROOT, 'tests', 'golden', 'g5_kmer.json.gz')
BIN = os.path.join(ROOT, 'oracle', '_ref', 'approx_counter')

Y_TOP = 'AATGTACTTCGTTCAGTTACGTATTGCT'
Y_BOT = 'GCAATACGTAACTGAACGAAGT'


def mutate(rng, s, r):
    o = []
    for c in s:
        x = rng.random()
        if x < r / 3:
            o.append(rng.choice('ACGT'))
        elif x < 2 * r / 3:
            pass
        elif x < r:
            o.append(c + rng.choice('ACGT'))
        else:
            o.append(c)
    return ''.join(o)


def make_input(path, seed, n):
    rng = random.Random(seed)
    with gzip.open(path, 'wt') as f:
        for k in range(n):
            body = ''.join(rng.choice('ACGT') for _ in range(rng.randint(120, 500)))
            if rng.random() < 0.05:
                p = rng.randint(0, len(body) - 10)
                body = body[:p] + rng.choice(['N', 'NNN', 'n']) + body[p + 1:]
            pre = ''.join(rng.choice('ACGT') for _ in range(rng.randint(0, 15)))
            suf = ''.join(rng.choice('ACGT') for _ in range(rng.randint(0, 15)))
            s = body
            if rng.random() < 0.75:
                s = pre + mutate(rng, Y_TOP, rng.choice([0.0, 0.05, 0.1])) + s
            if rng.random() < 0.6:
                s = s + mutate(rng, Y_BOT, rng.choice([0.0, 0.05, 0.1])) + suf
            if rng.random() < 0.1:
                s = s.lower()
            f.write('>read%d\n%s\n' % (k, s))


RUNS = [
    ('in1', ['-k', '16', '-lim', '60']),
    ('in1', ['-k', '12', '-lim', '40', '-lc', '1.5']),
    ('in1', ['-k', '20', '-lim', '30', '-sl', '80']),
    ('in2', ['-k', '16', '-lim', '80', '-lc', '0.6']),
    ('in2', ['-k', '16', '-lim', '50', '-fk', 'FORBID']),
    ('in2', ['-k', '16', '-sk', '200']),
    ('in1', ['-k', '16', '-lim', '25', '-mr', '2']),
    ('in2', ['-k', '14', '-lim', '30', '-se']),
]


def main():
    os.makedirs(KDIR, exist_ok=True)
    inputs = {'in1': os.path.join(KDIR, 'in1.fasta.gz'), 'in2': os.path.join(KDIR, 'in2.fasta.gz')}
    make_input(inputs['in1'], 11, 1500)
    make_input(inputs['in2'], 12, 2200)
    forbid = os.path.join(KDIR, 'forbidden.txt')
    with open(forbid, 'w') as f:
        f.write('ATGTACTTCGTTCAGT\nTCGTTCAGTTACGTAT\nNNNNACGTACGTACGT\nGCAATACGTAACTGAA\n')
    cases = []
    for name, args in RUNS:
        tmp = tempfile.mkdtemp(prefix='g5_')
        plain = os.path.join(tmp, 'reads.fasta')
        with gzip.open(inputs[name], 'rb') as src, open(plain, 'wb') as dst:
            dst.write(src.read())
        args = [forbid if a == 'FORBID' else a for a in args]
        cmd = [BIN, plain, '-o', os.path.join(tmp, 'out'), '-e', os.path.join(tmp, 'exact'), '-sn', '1000000',
               '-nt', '4', '-v', '0'] + args
        subprocess.run(cmd, check=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
        files = {}
        for fn in sorted(os.listdir(tmp)):
            if fn.startswith(('out', 'exact')):
                files[fn] = open(os.path.join(tmp, fn)).read()
        cases.append({'input': 'kmer/%s.fasta.gz' % name, 'args': [a if a != forbid else 'kmer/forbidden.txt'
                                                                   for a in args], 'files': files})
        print(name, args, {k: len(v.splitlines()) for k, v in files.items()})
    with gzip.open(OUT, 'wt') as f:
        json.dump({'generator': 'tools/make_golden_g5.py', 'cases': cases}, f)
    print('wrote', OUT)


if __name__ == '__main__':
    main()
