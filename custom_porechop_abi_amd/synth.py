"""Seeded synthetic ONT reads for benchmarks and large parity tests.

Recipe from SURVEY.md §8(d) / BASELINE.md ("Synthetic read recipe"), vectorised with numpy so
that 10^5-10^6 reads of mean 8 kb generate in seconds:
  * read length = max(200, int(lognormal(0, 0.5) * mean * 0.8825))  (mean ~= `mean`)
  * bases uniform over ACGT
  * p=0.8: 0-20 random bases + SQK-NSK007_Y_Top mutated at 10% (equal sub/del/ins) as prefix
  * p=0.7: SQK-NSK007_Y_Bottom mutated at 10% + 0-20 random bases as suffix
  * p=0.05: Y_Top mutated at 5% inserted at a uniform position
Reads are produced as Dna5 code arrays (uint8, A=0 C=1 G=2 T=3) -- the engine's native input.
"""
import numpy as np

Y_TOP = 'AATGTACTTCGTTCAGTTACGTATTGCT'
Y_BOTTOM = 'GCAATACGTAACTGAACGAAGT'
_CODE = {'A': 0, 'C': 1, 'G': 2, 'T': 3}


def _codes(s):
    return np.array([_CODE[c] for c in s], dtype=np.uint8)


def mutate(rng, codes, rate):
    """Substitute / delete / insert each base with probability rate/3 each."""
    u = rng.random(len(codes))
    out = []
    for k, c in enumerate(codes):
        x = u[k]
        if x < rate / 3:
            out.append(rng.integers(0, 4))
        elif x < 2 * rate / 3:
            continue
        elif x < rate:
            out.append(c)
            out.append(rng.integers(0, 4))
        else:
            out.append(c)
    return np.array(out, dtype=np.uint8)


def make_reads(n_reads, mean_len=8000, seed=12345, keep=None):
    """Return a list of uint8 code arrays.

    keep=None  -> full reads.
    keep=E     -> only what seq[:E] and seq[-E:] need: reads longer than 2E+64 are returned as
                  (head, tail, full_length) with the body between them elided (it is random
                  bases that no end window can see); shorter reads are returned whole.
    """
    rng = np.random.default_rng(seed)
    top, bottom = _codes(Y_TOP), _codes(Y_BOTTOM)
    lens = np.maximum(200, (rng.lognormal(0.0, 0.5, n_reads) * mean_len * 0.8825).astype(np.int64))
    has_start = rng.random(n_reads) < 0.8
    has_end = rng.random(n_reads) < 0.7
    has_mid = rng.random(n_reads) < 0.05
    out = []
    for k in range(n_reads):
        n = int(lens[k])
        pre = np.empty(0, np.uint8)
        suf = np.empty(0, np.uint8)
        if has_start[k]:
            pre = np.concatenate([rng.integers(0, 4, rng.integers(0, 21), dtype=np.uint8), mutate(rng, top, 0.10)])
        if has_end[k]:
            suf = np.concatenate([mutate(rng, bottom, 0.10), rng.integers(0, 4, rng.integers(0, 21), dtype=np.uint8)])
        body_len = max(0, n - len(pre) - len(suf))
        if keep is not None and n > 2 * keep + 64:
            head_body = rng.integers(0, 4, max(0, keep + 32 - len(pre)), dtype=np.uint8)
            tail_body = rng.integers(0, 4, max(0, keep + 32 - len(suf)), dtype=np.uint8)
            head = np.concatenate([pre, head_body])[:keep]
            tail = np.concatenate([tail_body, suf])[-keep:]
            full = len(pre) + body_len + len(suf)
            out.append((head, tail, full))
            continue
        body = rng.integers(0, 4, body_len, dtype=np.uint8)
        if has_mid[k] and body_len > 0:
            mid = mutate(rng, top, 0.05)
            p = int(rng.integers(0, body_len + 1))
            body = np.concatenate([body[:p], mid, body[p:]])
        out.append(np.concatenate([pre, body, suf]))
    return out


def pack_end_windows(reads, end_size, stride=None):
    """Dna5 start/end windows (seq[:end_size], seq[-end_size:]) of synthetic reads into one
    buffer with fixed 4-aligned stride: returns (codes, start_off, start_len, end_off, end_len)."""
    E = int(end_size)
    stride = stride or ((E + 3) & ~3)
    n = len(reads)
    buf = np.full(2 * n * stride + 16, 4, dtype=np.uint8)
    s_off = np.arange(n, dtype=np.int64) * (2 * stride)
    e_off = s_off + stride
    s_len = np.zeros(n, np.int32)
    e_len = np.zeros(n, np.int32)
    for k, r in enumerate(reads):
        if isinstance(r, tuple):
            head, tail, _ = r
        else:
            head, tail = r[:E], r[-E:] if E > 0 else r
        buf[s_off[k]:s_off[k] + len(head)] = head
        buf[e_off[k]:e_off[k] + len(tail)] = tail
        s_len[k] = len(head)
        e_len[k] = len(tail)
    return buf, s_off, s_len, e_off, e_len


_LETTERS = np.frombuffer(b'ACGTN', dtype=np.uint8)


def codes_to_str(c):
    return _LETTERS[np.asarray(c, dtype=np.intp)].tobytes().decode()


def revcomp_codes(c):
    return (3 - np.asarray(c, dtype=np.uint8)[::-1]).astype(np.uint8)


def make_barcoded_reads(n_reads, barcodes, mean_len=8000, seed=12345, keep=None):
    """Seeded barcoded reads for the demultiplexing workload (BASELINE.json configs[3]).

    barcodes: list of (start_seq, end_seq) strings, e.g. the 'Barcode k (forward)' sets of
    porechop_abi/adapters.py. Per read (lengths as make_reads):
      * p=0.9 barcoded with a uniform barcode b, else no barcode;
      * p=0.85: 0-20 random bases + Y_Top (10% mutated) + b's start sequence (10% mutated) prefix;
      * p=0.75: b's end sequence (10% mutated) + Y_Bottom (10% mutated) + 0-20 random bases suffix.
    Returns (reads, truth) with truth[k] = barcode index or -1; `keep` as in make_reads."""
    rng = np.random.default_rng(seed)
    top, bottom = _codes(Y_TOP), _codes(Y_BOTTOM)
    bcs = [(_codes(s), _codes(e)) for s, e in barcodes]
    lens = np.maximum(200, (rng.lognormal(0.0, 0.5, n_reads) * mean_len * 0.8825).astype(np.int64))
    barcoded = rng.random(n_reads) < 0.9
    which = rng.integers(0, len(bcs), n_reads)
    has_start = rng.random(n_reads) < 0.85
    has_end = rng.random(n_reads) < 0.75
    out, truth = [], []
    for k in range(n_reads):
        n = int(lens[k])
        b = int(which[k]) if barcoded[k] else -1
        pre = np.empty(0, np.uint8)
        suf = np.empty(0, np.uint8)
        if has_start[k]:
            parts = [rng.integers(0, 4, rng.integers(0, 21), dtype=np.uint8), mutate(rng, top, 0.10)]
            if b >= 0:
                parts.append(mutate(rng, bcs[b][0], 0.10))
            pre = np.concatenate(parts)
        if has_end[k]:
            parts = [mutate(rng, bcs[b][1], 0.10)] if b >= 0 else []
            parts += [mutate(rng, bottom, 0.10), rng.integers(0, 4, rng.integers(0, 21), dtype=np.uint8)]
            suf = np.concatenate(parts)
        body_len = max(0, n - len(pre) - len(suf))
        truth.append(b)
        if keep is not None and n > 2 * keep + 64:
            head = np.concatenate([pre, rng.integers(0, 4, max(0, keep + 32 - len(pre)), dtype=np.uint8)])[:keep]
            tail = np.concatenate([rng.integers(0, 4, max(0, keep + 32 - len(suf)), dtype=np.uint8), suf])[-keep:]
            out.append((head, tail, len(pre) + body_len + len(suf)))
            continue
        out.append(np.concatenate([pre, rng.integers(0, 4, body_len, dtype=np.uint8), suf]))
    return out, np.array(truth, np.int32)
