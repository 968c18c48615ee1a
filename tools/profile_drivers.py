"""cProfile of the reference-API drivers (bench.py run_drivers) on 100k synthetic reads x 50 sets:
where the host time of find_adapters_at_read_ends / find_adapters_in_read_middles goes.
Usage (GPU box): python tools/profile_drivers.py [n_reads]"""
import cProfile
import io
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: F401  (one HIP runtime, as bench.py)
from custom_porechop_abi_amd import adapters as A, synth, porechop_abi as P
from custom_porechop_abi_amd.nanopore_read import NanoporeRead

SC = (3, -6, -5, -2)
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
seqs = [synth.codes_to_str(r) for r in synth.make_reads(n, 8000, seed=12345)]
sets = [a for a in A.fresh_adapters() if '(full sequence)' not in a.name][:50]
sink = io.StringIO()
warm = [NanoporeRead('r%d' % i, s, '') for i, s in enumerate(seqs[:2000])]
P.find_adapters_at_read_ends(warm, sets, 0, 150, 2, 75.0, SC, sink, 4, 1, False, 75.0, 5.0, False, None)
P.find_adapters_in_read_middles(warm, sets, 0, 90.0, 10, 100, SC, sink, 1, False)
reads = [NanoporeRead('r%d' % i, s, '') for i, s in enumerate(seqs)]
for name, fn in (('ends', lambda: P.find_adapters_at_read_ends(reads, sets, 0, 150, 2, 75.0, SC, sink, 4, 1,
                                                                False, 75.0, 5.0, False, None)),
                 ('middles', lambda: P.find_adapters_in_read_middles(reads, sets, 0, 90.0, 10, 100, SC, sink, 1,
                                                                     False))):
    pr = cProfile.Profile()
    t = time.perf_counter()
    pr.enable()
    fn()
    pr.disable()
    print('== %s %.1f ms' % (name, 1e3 * (time.perf_counter() - t)), flush=True)
    st = pstats.Stats(pr)
    st.sort_stats('tottime').print_stats(18)
    st.sort_stats('cumulative').print_stats(18)
