"""GPU replacement of the ab-initio k-mer counter (porechop_abi/ab_initio_src/approx_counter.cpp,
run by porechop_abi/abinitio.py:392-440 as a subprocess).

Same command line, config file and output files as the reference program:

    python -m custom_porechop_abi_amd.approx_counter INPUT [--config FILE] [-o OUT] [-e EXACT]
        [-k K] [-sl SL] [-sn SN] [-lim LIM] [-lc LC] [-fk FILE] [-sk SK] [-mr MR] [-se] [-v V] [-nt NT]

writes OUT_<run>.start / OUT_<run>.end ("KMER<TAB>count" lines, most frequent first) and, with
-e, EXACT_<run>.start / .end. The work (sampling aside) follows the reference step by step:
  sampleSequences (:415-476)    read starts (prefix of SL) / ends (the last SL + 1 bases) of reads
                                at least 2 SL long -- the reference shuffles with
                                std::random_device; here the shuffle is seeded (all reads are taken
                                when SN covers them, which is where the two agree exactly);
  count_kmers (:487-519)        GPU: pcabi_kmer_count_host (k_kmer_keys + radix sort + RLE);
  get_most_frequent (:396-405)  count descending, then DUST complexity ascending, then k-mer
                                value descending (CompareCount, :270-305); or get_solid_kmers;
  errorCount (:531-601)         GPU: pcabi_kmer_approx_host (Myers bit-vector edit distance);
  adjust_threshold (:183-186)   the low-complexity threshold scaled from k = 16.
"""
import argparse
import ctypes
import os
import sys

import numpy as np

from . import misc
from ._lib import check, lib

DNA = 'ACGT'


def _declare(L):
    if not getattr(L, '_kmer_declared', False):
        P, i64 = ctypes.c_void_p, ctypes.c_int64
        L.pcabi_kmer_count_host.argtypes = [ctypes.c_int, P, i64, P, P, i64, ctypes.c_int, ctypes.c_float, P, i64, P,
                                            P, i64]
        L.pcabi_kmer_count_host.restype = i64
        L.pcabi_kmer_approx_host.argtypes = [ctypes.c_int, P, i64, P, P, i64, ctypes.c_int, P, i64, P]
        L.pcabi_kmer_approx_host.restype = ctypes.c_int
        L.pcabi_kmer_top_host.argtypes = [ctypes.c_int, P, i64, P, P, i64, ctypes.c_int, ctypes.c_float, P, i64, i64,
                                          i64, P, P, i64]
        L.pcabi_kmer_top_host.restype = i64
        L.pcabi_gather_host.argtypes = [P, P, P, i64, P, P]
        L.pcabi_gather_host.restype = None
        L._kmer_declared = True
    return L


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p) if a is not None else None


def adjust_threshold(c_old, k_old, k_new):
    """approx_counter.cpp:183-186, in float like the reference."""
    ratio = ((k_new - 2 + 1) ** 2) / float((k_old - 2 + 1) ** 2)
    return float(np.float32(c_old) * np.float32(ratio))


def kmer_to_str(v, k):
    return ''.join(DNA[(int(v) >> (2 * (k - 1 - i))) & 3] for i in range(k))


def str_to_kmer(s):
    v = 0
    for c in s:
        v = (v << 2) | DNA.index(c)
    return v


def complexity(kmers, k):
    """getComplexity (:247-267) for an array of k-mers, float32 like the reference: sum over the
    16 dimers of v (v - 1) for the k - 1 dimers, / float(2 (k - 2))."""
    kmers = np.asarray(kmers, np.uint64)
    dim = [((kmers >> np.uint64(2 * i)) & np.uint64(15)).astype(np.int8) for i in range(k - 1)]
    s = np.zeros(len(kmers), np.int64)
    for v in range(16):
        c = np.zeros(len(kmers), np.int64)
        for d in dim:
            c += d == v
        s += c * (c - 1)
    return s.astype(np.float32) / np.float32(2 * (k - 2))


def most_frequent(kmers, counts, limit, k):
    """get_most_frequent (:396-405) with CompareCount: count desc, complexity asc, k-mer desc.
    Only the k-mers that can make the cut (count >= the limit-th largest) are ranked."""
    kmers = np.asarray(kmers, np.uint64)
    counts = np.asarray(counts, np.int64)
    if 0 < limit < len(counts):
        cut = np.partition(counts, len(counts) - limit)[len(counts) - limit]
        keep = counts >= cut
        kmers, counts = kmers[keep], counts[keep]
    comp = complexity(kmers, k)
    order = np.lexsort((np.uint64(0xFFFFFFFFFFFFFFFF) - kmers, comp, -counts))[:limit]
    return kmers[order], counts[order]


def solid_kmers(kmers, counts, solid_km):
    """get_solid_kmers (:372-388): counts >= solid_km, count descending (std::sort, not stable:
    equal counts keep no defined order in the reference -- here k-mer ascending)."""
    kmers = np.asarray(kmers, np.uint64)
    counts = np.asarray(counts, np.int64)
    keep = counts >= solid_km
    kmers, counts = kmers[keep], counts[keep]
    order = np.lexsort((kmers, -counts))
    return kmers[order], counts[order]


class Samples(object):
    """Sampled read ends in the engine layout (codes, offsets, lengths)."""

    def __init__(self, codes, offs, lens):
        self.codes, self.offs, self.lens = codes, offs, lens

    def __len__(self):
        return len(self.lens)


def sample_sequences(batch, nb_sample, cut_size, bottom, seed=0):
    """sampleSequences (:415-476): reads at least 2 * cut_size long, in a shuffled order, until
    nb_sample are taken; the start keeps the first cut_size bases, the end the suffix from
    len - 1 - cut_size (cut_size + 1 bases)."""
    n = batch.n
    order = np.random.default_rng(seed).permutation(n)
    lens = batch.lengths.astype(np.int64)
    ok = lens[order] >= 2 * cut_size
    take = order[ok][:nb_sample]
    cur = np.minimum(lens[take], cut_size)
    if bottom:
        start = lens[take] - 1 - cur
        ln = lens[take] - start
    else:
        start = np.zeros(len(take), np.int64)
        ln = cur
    # the sampled bases alone, packed (4-aligned starts, N padding), so only they go to the GPU
    ln = ln.astype(np.int64)
    offs = np.zeros(len(take), np.int64)
    if len(take):
        offs[1:] = np.cumsum((ln + 3) & ~3)[:-1]
    total = int(offs[-1] + ln[-1]) if len(take) else 0
    codes = np.full(((total + 3) & ~3) + 16, 4, np.uint8)
    src = np.ascontiguousarray(batch.code_off[take] + start, np.int64)
    ln32 = ln.astype(np.int32)
    _declare(lib()).pcabi_gather_host(_p(batch.codes), _p(src), _p(ln32), len(take), _p(codes), _p(offs))
    return Samples(codes, offs, ln32)


def count_kmers(samples, k, threshold, forbidden=(), device=0):
    """count_kmers (:487-519) on the GPU: (k-mers ascending, counts)."""
    L = _declare(lib())
    forb = np.array(sorted(set(int(x) for x in forbidden)), np.uint64)
    cap = int(max(1, samples.lens.astype(np.int64).sum()))
    km = np.zeros(cap, np.uint64)
    cn = np.zeros(cap, np.uint32)
    n = L.pcabi_kmer_count_host(device, _p(samples.codes), samples.codes.size, _p(samples.offs), _p(samples.lens),
                                len(samples), int(k), float(threshold), _p(forb) if len(forb) else None, len(forb),
                                _p(km), _p(cn), cap)
    if n < 0:
        check(int(n), 'pcabi_kmer_count_host')
    return km[:n].copy(), cn[:n].astype(np.int64)


def count_kmers_top(samples, k, threshold, forbidden=(), top=0, min_count=0, device=0):
    """count_kmers followed by the cut get_most_frequent (top) or get_solid_kmers (min_count)
    applies, on the GPU: every k-mer with count >= max(min_count, the top-th largest count),
    count descending (ties k-mer ascending) -- all the ranking below can keep."""
    L = _declare(lib())
    forb = np.array(sorted(set(int(x) for x in forbidden)), np.uint64)
    cap = max(4096, 4 * int(top))
    while True:
        km = np.empty(cap, np.uint64)
        cn = np.empty(cap, np.uint32)
        n = L.pcabi_kmer_top_host(device, _p(samples.codes), samples.codes.size, _p(samples.offs), _p(samples.lens),
                                  len(samples), int(k), float(threshold), _p(forb) if len(forb) else None, len(forb),
                                  int(top), int(min_count), _p(km), _p(cn), cap)
        if n < 0:
            check(int(n), 'pcabi_kmer_top_host')
        if n <= cap:
            return km[:n].copy(), cn[:n].astype(np.int64)
        cap = int(n)


def error_count(samples, kmers, k, device=0):
    """errorCount (:531-601) on the GPU: counts aligned with kmers."""
    L = _declare(lib())
    kmers = np.ascontiguousarray(kmers, np.uint64)
    out = np.zeros(len(kmers), np.uint64)
    step = 65535 * 64
    for a in range(0, len(kmers), step):
        part = np.ascontiguousarray(kmers[a:a + step])
        o = np.zeros(len(part), np.uint64)
        check(L.pcabi_kmer_approx_host(device, _p(samples.codes), samples.codes.size, _p(samples.offs),
                                       _p(samples.lens), len(samples), int(k), _p(part), len(part), _p(o)),
              'pcabi_kmer_approx_host')
        out[a:a + len(part)] = o
    return out.astype(np.int64)


def export_counter(kmers, counts, k, path):
    """exportCounter (:158-174)."""
    with open(path, 'w') as f:
        for v, c in zip(kmers.tolist(), counts.tolist()):
            f.write('%s\t%d\n' % (kmer_to_str(v, k), c))


def parse_config(path):
    """parse_config (:103-135): key=value lines, spaces dropped, '#' comments."""
    params = {}
    if not os.path.isfile(path):
        print('/!\\ WARNING: Could not open config file', file=sys.stderr)
        return params
    with open(path) as f:
        for line in f:
            line = line.rstrip('\n')
            if line.startswith('#'):
                continue
            arg, val, sep = '', '', False
            for c in line:
                if c == '=':
                    sep = True
                elif c != ' ':
                    if sep:
                        val += c
                    else:
                        arg += c
            params[arg] = val
    return params


def parse_kmer_list(path):
    """parse_kmer_list (:340-364): one k-mer per line, only ACGT ones kept."""
    out = set()
    with open(path) as f:
        for line in f:
            s = line.rstrip('\n').upper()
            if s and all(c in DNA for c in s):
                out.add(str_to_kmer(s))
    return out


def run(input_file, output='out.txt', exact_out='', k=16, sl=100, sn=40000, limit=500, lc=1.0, forbidden=None,
        solid_km=0, nb_of_runs=1, skip_end=False, v=1, seed=0, device=0):
    """The reference program's main loop (:679-958)."""
    if k < 2 or k > 32:
        raise ValueError('/!\\ ERROR: kmer size must be between 2 and 32 (included)')
    if k > sl:
        raise ValueError('/!\\ ERROR: kmer size must be smaller than the sampling length (k <= sl)')
    lct = adjust_threshold(lc, 16, k)
    kmer_set = parse_kmer_list(forbidden) if forbidden else set()
    batch = misc.load_batch(input_file)
    mr_v = 0 if (nb_of_runs > 1 and v < 2) else v
    written = []
    for run_i in range(nb_of_runs):
        suffix = '_%d' % run_i
        if sn > batch.n:
            sn = batch.n
        bottom = False
        for which in ('start', 'end'):
            sample = sample_sequences(batch, sn, sl, bottom, seed=seed + 2 * run_i + (1 if bottom else 0))
            # only the k-mers the cut can keep leave the device (pcabi_kmer_top_host)
            if solid_km:
                kmers, counts = count_kmers_top(sample, k, lct, kmer_set, top=0, min_count=solid_km, device=device)
            else:
                kmers, counts = count_kmers_top(sample, k, lct, kmer_set, top=limit, device=device)
            if solid_km:
                top_k, top_c = solid_kmers(kmers, counts, solid_km)
            else:
                top_k, top_c = most_frequent(kmers, counts, limit, k)
            if exact_out:
                export_counter(top_k, top_c, k, exact_out + suffix + '.' + which)
                written.append(exact_out + suffix + '.' + which)
            err = error_count(sample, top_k, k, device)
            ek, ec = most_frequent(top_k, err, limit, k)
            export_counter(ek, ec, k, output + suffix + '.' + which)
            written.append(output + suffix + '.' + which)
            # the reference's loop (:938-950): with skip_end the break only happens when verbose;
            # otherwise "end" is computed again from the read starts
            if skip_end:
                if mr_v > 0:
                    break
            else:
                bottom = True
    return written


def main(argv=None):
    ap = argparse.ArgumentParser(prog='approx_counter')
    ap.add_argument('input')
    ap.add_argument('-lc', '--low_complexity', dest='lc', type=float)
    ap.add_argument('-sn', '--sample_n', dest='sn', type=int)
    ap.add_argument('-sl', '--sample_length', dest='sl', type=int)
    ap.add_argument('-nt', '--nb_thread', dest='nt', type=int)
    ap.add_argument('-k', '--kmer_size', dest='k', type=int)
    ap.add_argument('-lim', '--limit', dest='lim', type=int)
    ap.add_argument('-mr', '--multi_run', dest='mr', type=int)
    ap.add_argument('-v', '--verbosity', dest='v', type=int)
    ap.add_argument('-e', '--exact_file', dest='e')
    ap.add_argument('-conf', '--config', dest='conf')
    ap.add_argument('-fk', '--forbidden_kmer', dest='fk')
    ap.add_argument('-sk', '--solid_km', dest='sk', type=int)
    ap.add_argument('-se', '--skip_end', dest='se', action='store_true')
    ap.add_argument('-o', '--out_file', dest='o')
    a = ap.parse_args(argv)
    # defaults, then the config file, then the command line (:700-760)
    cfg = dict(lc=1.0, k=16, v=1, sn=40000, sl=100, lim=500, sk=0, fk='', e='', mr=1, se=False, o='out.txt')
    if a.conf:
        p = parse_config(a.conf)
        for key, typ in (('lc', float), ('k', int), ('v', int), ('sn', int), ('sl', int), ('lim', int), ('sk', int),
                         ('mr', int)):
            if key in p:
                cfg[key] = typ(p[key])
        cfg['se'] = 'se' in p
        cfg['fk'] = p.get('fk', cfg['fk'])
        cfg['e'] = p.get('e', cfg['e'])
    for key in ('lim', 'lc', 'k', 'v', 'sl', 'sn', 'o', 'e', 'fk', 'sk', 'mr'):
        val = getattr(a, key)
        if val is not None:
            cfg[key] = val
    cfg['se'] = cfg['se'] or a.se
    run(a.input, output=cfg['o'], exact_out=cfg['e'], k=cfg['k'], sl=cfg['sl'], sn=cfg['sn'], limit=cfg['lim'],
        lc=cfg['lc'], forbidden=cfg['fk'] or None, solid_km=cfg['sk'], nb_of_runs=cfg['mr'], skip_end=cfg['se'],
        v=cfg['v'])
    return 0


if __name__ == '__main__':
    sys.exit(main())
