"""cProfile of the reference-API drivers (bench.py's drivers sub-record workload: 100k synthetic
8 kb reads as NanoporeRead objects x the first 50 adapter sets): one warm-up pass, then the end-trim
and middle drivers once each under the profiler; the top entries by own time go to stdout."""
import cProfile
import io
import pstats
import sys
import time

sys.path.insert(0, '.')
from custom_porechop_abi_amd import adapters as A, synth, porechop_abi as P  # noqa: E402
from custom_porechop_abi_amd.nanopore_read import NanoporeRead  # noqa: E402

SC = [3, -6, -5, -2]
n = int(sys.argv[1]) if len(sys.argv) > 1 else 100000
seqs = [synth.codes_to_str(r) for r in synth.make_reads(n, 8000, seed=12345)]
sets = [a for a in A.fresh_adapters() if '(full sequence)' not in a.name][:50]
sink = io.StringIO()


def ends(reads):
    P.find_adapters_at_read_ends(reads, sets, 0, 150, 2, 75.0, SC, sink, 4, 1, False, 75.0, 5.0, False, None)


def middles(reads):
    P.find_adapters_in_read_middles(reads, sets, 0, 90.0, 10, 100, SC, sink, 1, False)


warm = [NanoporeRead('r%d' % i, s, '') for i, s in enumerate(seqs[:2000])]
ends(warm)
middles(warm)
for name, fn in (('ends', ends), ('middles', middles)):
    reads = [NanoporeRead('r%d' % i, s, '') for i, s in enumerate(seqs)]
    if name == 'middles':
        ends(reads)
    t = time.perf_counter()
    fn(reads)
    print('%s plain: %.1f ms' % (name, 1e3 * (time.perf_counter() - t)), flush=True)
    reads = [NanoporeRead('r%d' % i, s, '') for i, s in enumerate(seqs)]
    if name == 'middles':
        ends(reads)
    pr = cProfile.Profile()
    pr.enable()
    fn(reads)
    pr.disable()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats('tottime').print_stats(25)
    print('==== %s ====' % name)
    print(s.getvalue()[:6000], flush=True)
