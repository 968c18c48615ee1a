"""G2-albacore golden output: the reference's CLI flow (porechop_abi.py:41-131: load_reads ->
find_matching_adapter_sets -> fix_up_1d2_sets -> choose_barcoding_kit ->
add_full_barcode_adapter_sets -> find_adapters_at_read_ends -> find_adapters_in_read_middles ->
filter_reads_by_adapter -> output_reads) on an Albacore output directory, run by the REFERENCE'S
OWN Python code over its SeqAn aligner compiled in place (oracle/_ref/cpp_functions.so), as
tools/make_golden_g2.py does. Container-only generator.

Input: the reference's own test fixture test/test_albacore_directory (four FASTQ files under
workspace/barcode01..03 and workspace/unclassified), committed as data under
tests/golden/data/albacore/ (gzipped: load_reads takes *.fastq.gz too). Outputs (committed):
tests/golden/g2_albacore.json.gz -- per run the barcode bins (-b: file name -> exact text) or the
trimmed output file, the matching sets, the check reads' count and the loaded read count.
"""
import gzip
import io
import json
import os
import shutil
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from make_golden_g2 import setup_reference  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = '/root/reference/test/test_albacore_directory'
DATA = os.path.join(ROOT, 'tests', 'golden', 'data', 'albacore')
OUT = os.path.join(ROOT, 'tests', 'golden', 'g2_albacore.json.gz')


def copy_fixture():
    for d, _, fs in os.walk(SRC):
        for f in fs:
            if not f.endswith('.fastq'):
                continue
            rel = os.path.relpath(os.path.join(d, f), SRC)
            dst = os.path.join(DATA, rel + '.gz')
            os.makedirs(os.path.dirname(dst), exist_ok=True)
            with open(os.path.join(d, f), 'rb') as a, gzip.GzipFile(dst, 'wb', mtime=0) as b:
                b.write(a.read())


def run(P, bins, check_reads=10000):
    for a in P.ADAPTERS:
        a.best_start_score, a.best_end_score = 0.0, 0.0
    sink = io.StringIO()
    reads, check, read_type = P.load_reads(DATA, 0, sink, check_reads)
    sc = [3, -6, -5, -2]
    matching = P.find_matching_adapter_sets(check, 0, 150, sc, sink, 90.0, 1)
    matching = P.fix_up_1d2_sets(matching)
    fr = P.choose_barcoding_kit(matching, 0, sink) if bins else None
    matching = P.add_full_barcode_adapter_sets(matching)
    names = [a.name for a in matching]
    if matching:
        P.find_adapters_at_read_ends(reads, matching, 0, 150, 2, 75.0, sc, sink, 4, 1, bins, 75.0, 5.0, False, fr)
        P.find_adapters_in_read_middles(reads, matching, 0, 90.0, 10, 100, sc, sink, 1, False)
        stdout = sys.stdout
        sys.stdout = io.StringIO()          # the fork's filter prints its count to stdout
        try:
            reads = P.filter_reads_by_adapter(reads)
        finally:
            sys.stdout = stdout
    tmp = tempfile.mkdtemp(prefix='albacore_out_')
    try:
        if bins:
            bdir = os.path.join(tmp, 'bins')
            P.output_reads(reads, 'fastq', None, read_type, 0, False, 1000, sink, bdir, DATA, False, 1, False)
            files = {f: open(os.path.join(bdir, f)).read() for f in sorted(os.listdir(bdir))}
            out = {'bins': files}
        else:
            path = os.path.join(tmp, 'out.fastq')
            P.output_reads(reads, 'fastq', path, read_type, 0, False, 1000, sink, None, DATA, False, 1, False)
            out = {'output': open(path).read()}
    finally:
        shutil.rmtree(tmp)
    out.update({'matching': names, 'forward_or_reverse': fr, 'check_reads': len(check), 'check_reads_arg': check_reads,
                'barcodes': bool(bins)})
    return out


def main():
    copy_fixture()
    P, _ = setup_reference()
    runs = [run(P, True), run(P, False), run(P, True, check_reads=20)]
    with gzip.open(OUT, 'wt') as f:
        json.dump({'runs': runs}, f)
    for r in runs:
        print('barcodes=%s check=%d matching=%s bins=%s' % (r['barcodes'], r['check_reads'], r['matching'][:4],
                                                            sorted(r.get('bins', {}))))
    print('wrote', OUT)


if __name__ == '__main__':
    main()
