"""G2 golden vectors: per-read trimming decisions produced by the REFERENCE'S OWN Python drivers
(porechop_abi.porechop_abi.find_matching_adapter_sets / fix_up_1d2_sets /
choose_barcoding_kit / add_full_barcode_adapter_sets / find_adapters_at_read_ends /
find_adapters_in_read_middles) on top of the reference's SeqAn aligner compiled in place
(oracle/_ref/cpp_functions.so).

Container-only generator: it copies /root/reference/porechop_abi (Python files only) to a temp
dir, drops the compiled reference .so next to it and imports it from there. Output (committed
as data): tests/golden/g2_decisions.json.gz -- inputs (read names/sequences for the synthetic
set; the reference's own test FASTQs are under tests/golden/data/) and the decisions.
"""
import gzip
import importlib
import io
import json
import os
import random
import shutil
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_PKG = '/root/reference/porechop_abi'
OUT = os.path.join(ROOT, 'tests', 'golden', 'g2_decisions.json.gz')
DATA = os.path.join(ROOT, 'tests', 'golden', 'data')


def setup_reference():
    tmp = tempfile.mkdtemp(prefix='refpkg_')
    dst = os.path.join(tmp, 'porechop_abi')
    os.makedirs(dst)
    for f in os.listdir(REF_PKG):
        if f.endswith('.py'):
            shutil.copy(os.path.join(REF_PKG, f), dst)
    shutil.copy(os.path.join(ROOT, 'oracle', '_ref', 'cpp_functions.so'), os.path.join(dst, 'cpp_functions.so'))
    sys.path.insert(0, tmp)
    P = importlib.import_module('porechop_abi.porechop_abi')
    NR = importlib.import_module('porechop_abi.nanopore_read')
    return P, NR


def ranges(positions):
    """Sorted set of ints -> list of [start, end) runs."""
    out = []
    for p in sorted(positions):
        if out and out[-1][1] == p:
            out[-1][1] = p + 1
        else:
            out.append([p, p + 1])
    return out


def mutate(rng, s, rate):
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


def synthetic(n, seed, mean):
    """Small seeded set (SURVEY.md §8d recipe, scaled down) with start/end/middle adapters,
    plus short reads, N runs and lower-case bases to exercise edge paths."""
    rng = random.Random(seed)
    top, bot = 'AATGTACTTCGTTCAGTTACGTATTGCT', 'GCAATACGTAACTGAACGAAGT'
    bc = ['AAGAAAGTTGTCGGTGTCTTTGTG', 'TCGATTCCGTTTGTAGTCGTCTGT']
    reads = []
    for k in range(n):
        L = max(20, int(rng.lognormvariate(0, 0.5) * mean * 0.8825))
        body = ''.join(rng.choice('ACGT') for _ in range(L))
        if rng.random() < 0.05:
            p = rng.randint(0, len(body))
            body = body[:p] + 'N' * rng.randint(1, 40) + body[p:]
        if rng.random() < 0.25:
            p = rng.randint(0, len(body))
            body = body[:p] + mutate(rng, rng.choice([top, bot]), 0.05) + body[p:]
        if rng.random() < 0.08:
            p = rng.randint(0, len(body))
            body = body[:p] + mutate(rng, top, 0.03) + body[p:p + 300] + mutate(rng, top, 0.03) + body[p + 300:]
        pre = ''.join(rng.choice('ACGT') for _ in range(rng.randint(0, 20))) + mutate(rng, top, 0.1) \
            if rng.random() < 0.8 else ''
        if rng.random() < 0.15:
            pre = pre + mutate(rng, rng.choice(bc), 0.05)
        suf = mutate(rng, bot, 0.1) + ''.join(rng.choice('ACGT') for _ in range(rng.randint(0, 20))) \
            if rng.random() < 0.7 else ''
        seq = pre + body + suf
        if k % 37 == 0:
            seq = seq.lower()
        reads.append(('synth_%d' % k, seq, ''))
    return reads


def load(fn):
    """Parse a (gzipped) FASTA/FASTQ fixture into (name, seq, quals)."""
    with gzip.open(os.path.join(DATA, fn + '.gz'), 'rt') as f:
        lines = [l.rstrip('\n') for l in f]
    out = []
    if lines[0].startswith('@'):
        for i in range(0, len(lines) - 3, 4):
            out.append((lines[i][1:].split()[0], lines[i + 1].strip(), lines[i + 3].strip()))
    else:
        name, seq = None, []
        for l in lines + ['>']:
            if l.startswith('>'):
                if name is not None:
                    out.append((name, ''.join(seq), ''))
                name, seq = l[1:].split()[0] if l[1:] else None, []
            elif l.strip():
                seq.append(l.strip())
    return out


def run_case(P, NR, records, opts):
    devnull = io.StringIO()
    for a in P.ADAPTERS:
        a.best_start_score, a.best_end_score = 0.0, 0.0
    reads = [NR.NanoporeRead(n, s, q) for n, s, q in records]
    sc = opts['scoring']
    check = reads[:opts.get('check_reads', 10000)]
    matching = P.find_matching_adapter_sets(check, 0, opts['end_size'], sc, devnull, opts['adapter_threshold'], 1)
    matching = P.fix_up_1d2_sets(matching)
    fr = None
    if opts['barcodes']:
        fr = P.choose_barcoding_kit(matching, 0, devnull)
    set_scores = [[a.name, a.best_start_score, a.best_end_score]
                  for a in P.ADAPTERS if '(full sequence)' not in a.name]
    matching = P.add_full_barcode_adapter_sets(matching)
    if matching:
        P.find_adapters_at_read_ends(reads, matching, 0, opts['end_size'], opts['extra_end_trim'],
                                     opts['end_threshold'], sc, devnull, opts['min_trim_size'], 1,
                                     opts['barcodes'], 75.0, 5.0, opts.get('require_two', False), fr)
        P.find_adapters_in_read_middles(reads, matching, 0, opts['middle_threshold'], 10, 100, sc,
                                        devnull, 1, False)
    out = []
    for r in reads:
        out.append({
            'name': r.name,
            'start_trim': r.start_trim_amount, 'end_trim': r.end_trim_amount,
            'start_alns': [[a[0].name, a[1], a[2], a[3], a[4]] for a in r.start_adapter_alignments],
            'end_alns': [[a[0].name, a[1], a[2], a[3], a[4]] for a in r.end_adapter_alignments],
            'middle_pos': ranges(r.middle_adapter_positions),
            'middle_trim': ranges(r.middle_trim_positions),
            'middle_hit_str': r.middle_hit_str,
            'start_bc': list(r.start_barcode_scores.items()),
            'end_bc': list(r.end_barcode_scores.items()),
            'barcode_call': r.barcode_call,
        })
    return {'matching': [a.name for a in matching], 'forward_or_reverse': fr, 'set_scores': set_scores,
            'reads': out}


def main():
    P, NR = setup_reference()
    base = {'scoring': [3, -6, -5, -2], 'end_size': 150, 'extra_end_trim': 2, 'end_threshold': 75.0,
            'min_trim_size': 4, 'middle_threshold': 90.0, 'adapter_threshold': 90.0, 'barcodes': False}
    synth = synthetic(160, 7, 2500)
    cases = [
        ('one_adapter_set', 'test_one_adapter_set.fastq', dict(base)),
        ('two_adapter_sets', 'test_two_adapter_sets.fastq', dict(base)),
        ('barcodes', 'test_barcodes.fastq', dict(base, barcodes=True)),
        ('barcodes_two', 'test_barcodes.fastq', dict(base, barcodes=True, require_two=True)),
        ('choose_barcodes', 'test_choose_barcodes_1.fasta', dict(base, barcodes=True)),
        ('synthetic_default', None, dict(base)),
        ('synthetic_linear', None, dict(base, scoring=[2, -1, -1, -1], adapter_threshold=80.0,
                                        middle_threshold=85.0)),
        ('synthetic_endsize', None, dict(base, end_size=100, end_threshold=60.0, extra_end_trim=5,
                                         min_trim_size=10, check_reads=50)),
    ]
    result = {'synthetic_reads': synth, 'cases': []}
    for name, fn, opts in cases:
        records = synth if fn is None else load(fn)
        res = run_case(P, NR, records, opts)
        res.update({'case': name, 'input': fn or 'synthetic_reads', 'opts': opts})
        result['cases'].append(res)
        n_trim = sum(1 for r in res['reads'] if r['start_trim'] or r['end_trim'])
        n_mid = sum(1 for r in res['reads'] if r['middle_pos'])
        print('%-18s reads=%4d matching=%d trimmed=%d middle=%d' % (name, len(records), len(res['matching']),
                                                                 n_trim, n_mid))
    with gzip.open(OUT, 'wt') as f:
        json.dump(result, f)
    print('wrote', OUT)


if __name__ == '__main__':
    main()
