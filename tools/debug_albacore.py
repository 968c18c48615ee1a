"""GPU-box debugging aid: FileTrimmer.trim() on the Albacore fixture vs the same decisions from the
batched drivers over the CPU oracle, read by read (prints the differing reads)."""
import io
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: F401
from custom_porechop_abi_amd import engine, misc, porechop_abi as P
from custom_porechop_abi_amd.pipeline import FileTrimmer
from tests import oracle_lib

d = os.path.join(ROOT, 'tests', 'golden', 'data', 'albacore')
check = misc.load_check_reads(d, 10000)
matching = P.find_matching_adapter_sets(check, 0, 150, (3, -6, -5, -2), io.StringIO(), 90.0, 1)
matching = P.fix_up_1d2_sets(matching)
fr = P.choose_barcoding_kit(matching, 0, io.StringIO())
matching = P.add_full_barcode_adapter_sets(matching)
print('matching', [a.name for a in matching], fr)
ft = FileTrimmer(matching, barcode_dir='/tmp/dbg_bins', forward_or_reverse_barcodes=fr)
for f, alb in misc.input_files(d):
    for b in misc.read_batches(f, max_reads=5):
        st, et, co, cu, hits, keep = ft.trim(b, albacore=alb)
        reads = b.nanopore_reads()
        for r in reads:
            r.albacore_barcode_call = alb
        saved = (engine.align, engine.end_decisions, engine.middle_scan)
        engine.align, engine.end_decisions = oracle_lib.align_windows, oracle_lib.end_decisions_windows
        engine.middle_scan = oracle_lib.middle_scan_windows
        try:
            P.find_adapters_at_read_ends(reads, matching, 0, 150, 2, 75.0, (3, -6, -5, -2), io.StringIO(), 4, 1, True,
                                         75.0, 5.0, False, fr)
            P.find_adapters_in_read_middles(reads, matching, 0, 90.0, 10, 100, (3, -6, -5, -2), io.StringIO(), 1, False)
        finally:
            engine.align, engine.end_decisions, engine.middle_scan = saved
        for i, r in enumerate(reads):
            rg = misc.positions_to_ranges(r.middle_trim_positions)
            mine = [(int(cu[2 * k]), int(cu[2 * k + 1])) for k in range(co[i], co[i + 1])]
            if (st[i], et[i]) != (r.start_trim_amount, r.end_trim_amount) or \
                    misc.positions_to_ranges(set(p for a, e in mine for p in range(a, e))) != rg:
                print('DIFF', r.name.split()[0], 'trims', (int(st[i]), int(et[i])), (r.start_trim_amount, r.end_trim_amount))
                print('   gpu cuts', mine)
                print('   ref ranges', rg, r.middle_hit_str.strip())
                print('   gpu hits', hits[:, hits[0] == i].T.tolist())
ft.close()
print('done')

# the file path: FileTrimmer.trim_file on the directory, bins vs the reference's golden bins
import gzip
import json
import shutil
shutil.rmtree('/tmp/dbg_bins2', ignore_errors=True)
with gzip.open(os.path.join(ROOT, 'tests', 'golden', 'g2_albacore.json.gz'), 'rt') as f:
    exp = json.load(f)['runs'][0]
ft = FileTrimmer(matching, barcode_dir='/tmp/dbg_bins2', forward_or_reverse_barcodes=fr)
ft.trim_file(d, '/tmp/unused.fastq', 'fastq', max_reads=5)
ft.close()
for name, txt in exp['bins'].items():
    got = open(os.path.join('/tmp/dbg_bins2', name)).read()
    if got != txt:
        g, w = got.split('\n'), txt.split('\n')
        print('BIN', name, len(g), len(w))
        for i in range(0, min(len(g), len(w)) - 1, 4):
            if g[i:i + 4] != w[i:i + 4]:
                print('  rec', i // 4, g[i][:60], len(g[i + 1]), '|', w[i][:60], len(w[i + 1]))
