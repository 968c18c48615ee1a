"""G6 golden vectors: the text the REFERENCE'S OWN phase drivers print at verbosity 1, 2 and 3
(porechop_abi/porechop_abi.py:200-245, 359-438, 457-522: progress lines, the per-read
formatted_start_and_end_seq / full_start_end_output windows and middle_adapter_results, which come
from NanoporeRead's formatting methods, nanopore_read.py:254-406), run on top of the reference's
SeqAn aligner compiled in place (oracle/_ref/cpp_functions.so).

Container-only generator (imports the reference as tools/make_golden_g2.py does). For every G2 case
(the reference's test files and the seeded synthetic set) and verbosity 1 (threads 1 and 4: the
middle phase's thread-pool progress differs), 2 and 3, the output of each driver is recorded
separately: 'check' (find_matching_adapter_sets), 'ends' (find_adapters_at_read_ends) and
'middles' (find_adapters_in_read_middles). Output: tests/golden/g6_verbose.json.gz.
"""
import gzip
import io
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import make_golden_g2 as G2  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(ROOT, 'tests', 'golden', 'g6_verbose.json.gz')
G2_FILE = os.path.join(ROOT, 'tests', 'golden', 'g2_decisions.json.gz')


def run(P, NR, records, opts, verbosity, threads):
    for a in P.ADAPTERS:
        a.best_start_score, a.best_end_score = 0.0, 0.0
    reads = [NR.NanoporeRead(n, s, q) for n, s, q in records]
    sc = opts['scoring']
    out = {}
    buf = io.StringIO()
    matching = P.find_matching_adapter_sets(reads[:opts.get('check_reads', 10000)], verbosity, opts['end_size'], sc,
                                            buf, opts['adapter_threshold'], threads)
    out['check'] = buf.getvalue()
    matching = P.fix_up_1d2_sets(matching)
    fr = P.choose_barcoding_kit(matching, 0, io.StringIO()) if opts['barcodes'] else None
    matching = P.add_full_barcode_adapter_sets(matching)
    if matching:
        buf = io.StringIO()
        P.find_adapters_at_read_ends(reads, matching, verbosity, opts['end_size'], opts['extra_end_trim'],
                                     opts['end_threshold'], sc, buf, opts['min_trim_size'], threads,
                                     opts['barcodes'], 75.0, 5.0, opts.get('require_two', False), fr)
        out['ends'] = buf.getvalue()
        buf = io.StringIO()
        P.find_adapters_in_read_middles(reads, matching, verbosity, opts['middle_threshold'], 10, 100, sc, buf,
                                        threads, False)
        out['middles'] = buf.getvalue()
    return out


def main():
    P, NR = G2.setup_reference()
    with gzip.open(G2_FILE, 'rt') as f:
        g2 = json.load(f)
    result = {'runs': []}
    for case in g2['cases']:
        records = [tuple(x) for x in g2['synthetic_reads']] if case['input'] == 'synthetic_reads' \
            else G2.load(case['input'])
        for verbosity, threads in ((1, 1), (1, 4), (2, 1), (3, 1), (3, 4)):
            res = run(P, NR, records, case['opts'], verbosity, threads)
            result['runs'].append({'case': case['case'], 'verbosity': verbosity, 'threads': threads, 'out': res})
            print('%-18s v%d t%d %s' % (case['case'], verbosity, threads,
                                        {k: len(v) for k, v in res.items()}), flush=True)
    with gzip.open(OUT, 'wt') as f:
        json.dump(result, f)
    print('wrote', OUT, os.path.getsize(OUT))


if __name__ == '__main__':
    main()
