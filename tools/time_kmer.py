"""Per-stage timing of one approx_counter run (GPU box): python tools/time_kmer.py"""
import os
import tempfile
import time

import numpy as np
import torch  # noqa: F401  (one HIP runtime)

from custom_porechop_abi_amd import approx_counter as AC, misc, synth

reads = synth.make_reads(40000, 1500, seed=3)
tmp = tempfile.mkdtemp()
p = os.path.join(tmp, 'r.fasta')
tab = np.array(list(b'ACGTN'), np.uint8)
with open(p, 'wb') as f:
    for k, r in enumerate(reads):
        f.write(b'>r%d\n%s\n' % (k, bytes(tab[r])))
b = misc.load_batch(p)
lct = AC.adjust_threshold(1.0, 16, 16)
for rep in range(3):
    t = {}
    for bottom in (False, True):
        t0 = time.perf_counter()
        s = AC.sample_sequences(b, 40000, 100, bottom, seed=1)
        t1 = time.perf_counter()
        km, cn = AC.count_kmers_top(s, 16, lct, set(), top=500)
        t2 = time.perf_counter()
        tk, tc = AC.most_frequent(km, cn, 500, 16)
        t3 = time.perf_counter()
        err = AC.error_count(s, tk, 16)
        t4 = time.perf_counter()
        ek, ec = AC.most_frequent(tk, err, 500, 16)
        AC.export_counter(ek, ec, 16, os.path.join(tmp, 'o'))
        t5 = time.perf_counter()
        for key, v in (('sample', t1 - t0), ('count_top', t2 - t1), ('rank', t3 - t2), ('error', t4 - t3),
                       ('rank2+export', t5 - t4)):
            t[key] = t.get(key, 0) + v * 1e3
    print({k: round(v, 2) for k, v in t.items()}, 'kept', len(km))
