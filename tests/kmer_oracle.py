"""CPU restatement of approx_counter's two counting steps (TEST INFRASTRUCTURE ONLY), used to
check custom_porechop_abi_amd/approx_counter.py's host logic without a GPU. Pinned by
tests/golden/g5_kmer.json.gz (the reference program's own outputs).
  count_kmers : porechop_abi/ab_initio_src/approx_counter.cpp:487-519 (with is_DNA :313-321,
                haveLowComplexity :214-234, isForbiddenKmer :330-332)
  error_count : :531-601 as sum over sequences of 3 - d for the best substring edit distance
                d <= 2 (a plain DP over all sequences at once)."""
import numpy as np


def _seqs(samples):
    return [samples.codes[o:o + n] for o, n in zip(samples.offs.tolist(), samples.lens.tolist())]


def count_kmers(samples, k, threshold, forbidden=(), device=0):
    forbidden = set(int(x) for x in forbidden)
    counts = {}
    thr = np.float32(threshold)
    for s in _seqs(samples):
        s = s.astype(np.int64)
        for p in range(0, len(s) - k + 1):
            w = s[p:p + k]
            if (w >= 4).any():
                continue
            v = 0
            for x in w.tolist():
                v = (v << 2) | x
            dim = [(v >> (2 * i)) & 15 for i in range(k - 1)]
            c = np.bincount(dim, minlength=16)
            sc = np.float32(int((c * (c - 1)).sum())) / np.float32(2 * (k - 2))
            if sc >= thr or v in forbidden:
                continue
            counts[v] = counts.get(v, 0) + 1
    keys = np.array(sorted(counts), np.uint64)
    return keys, np.array([counts[int(x)] for x in keys], np.int64)


def error_count(samples, kmers, k, device=0):
    seqs = _seqs(samples)
    L = max([len(s) for s in seqs] + [1])
    a = np.full((len(seqs), L), 4, np.int64)
    ln = np.array([len(s) for s in seqs], np.int64)
    for i, s in enumerate(seqs):
        a[i, :len(s)] = s
    out = []
    for km in np.asarray(kmers, np.uint64).tolist():
        pat = [(km >> (2 * (k - 1 - i))) & 3 for i in range(k)]
        prev = np.tile(np.arange(k + 1), (len(seqs), 1))
        best = np.full(len(seqs), k)
        for j in range(L):
            c = a[:, j]
            cur = np.zeros_like(prev)
            for i in range(1, k + 1):
                cur[:, i] = np.minimum(np.minimum(prev[:, i - 1] + (c != pat[i - 1]), prev[:, i] + 1), cur[:, i - 1] + 1)
            live = j < ln
            best = np.where(live, np.minimum(best, cur[:, k]), best)
            prev = np.where(live[:, None], cur, prev)
        out.append(int(np.where(best <= 2, 3 - best, 0).sum()))
    return np.array(out, np.int64)


def count_kmers_top(samples, k, threshold, forbidden=(), top=0, min_count=0, device=0):
    """pcabi_kmer_top_host restated: count_kmers, then count descending (ties k-mer ascending),
    only the entries with count >= max(min_count, the top-th largest count)."""
    import numpy as np
    km, cn = count_kmers(samples, k, threshold, forbidden, device)
    km = np.asarray(km, np.uint64)
    cn = np.asarray(cn, np.int64)
    order = np.lexsort((km, -cn))
    km, cn = km[order], cn[order]
    thr = max(int(min_count), 0)
    if 0 < top <= len(cn):
        thr = max(thr, int(cn[top - 1]))
    keep = cn >= thr
    return km[keep], cn[keep]
