"""The pinned band bound of the middle scan's seeds (pcabi_seed.hip, k_seed_band_pin), restated on
the CPU: B = P + K * match + Q from two one-cell band DPs -- the suffix after the probe's K diagonal
matches run forwards, the prefix before them run backwards on the mirrored band -- must equal the
best score of the band DP constrained to pass through those K matches (the set of alignments the
seed argument needs: one whose piece p is exact). Host logic only: it pins the kernel's recurrences
and start rows (including the horizontal gaps next to the run), not the kernel itself (the GPU
parity tests of the middle scan cover that)."""
import numpy as np
import pytest

NEG = -10 ** 6


def _rows(S, V, adapter, read_at, E, sc):
    ma, mi, go, ge = sc
    W = 2 * E + 1
    for r, ab in enumerate(adapter, 1):
        h = sl = NEG
        nS, nV = [0] * W, [0] * W
        for x in range(W):
            dg = S[x] + (ma if read_at(r, x) == ab else mi)
            vu = max(V[x + 1] + ge, S[x + 1] + go) if x + 1 < W else NEG
            h = max(h + ge, sl + go)
            s = max(dg, vu, h)
            nS[x], nV[x], sl = s, vu, s
        S, V = nS, nV
    return S


def _start(E, sc):
    """A half's start row: the run's cell (0) and the horizontal gap next to it (kernel pin_start)."""
    go, ge = sc[2], sc[3]
    W = 2 * E + 1
    return [0 if x == E else (go + (x - E - 1) * ge if x > E else NEG) for x in range(W)], [NEG] * W


def pinned_bound(ac, rd, L, d0, E, o, K, sc):
    q = o + d0
    S, V = _start(E, sc)
    Q = max(_rows(S, V, list(ac[o + K:L]), lambda r, x: rd[q + K + (r - 1) + x - E], E, sc))
    S, V = _start(E, sc)
    P = max(_rows(S, V, [ac[o - r] for r in range(1, o + 1)], lambda r, x: rd[q - r + E - x], E, sc))
    return P + sc[0] * K + Q


def constrained_band(ac, rd, L, d0, E, o, K, sc):
    """The band DP of the whole adapter (free start in row 0, end anywhere in row L: an inside band)
    with rows o + 1 .. o + K forced onto the run's diagonal as matches; after the run the same row
    may continue with a horizontal gap."""
    ma, mi, go, ge = sc
    W = 2 * E + 1
    S, V = [0] * W, [NEG] * W
    for i in range(1, L + 1):
        ab = ac[i - 1]
        if o < i <= o + K:
            assert rd[i + d0 - 1] == ab
            nS = [NEG] * W
            nS[E] = S[E] + ma
            if i == o + K:
                for x in range(E + 1, W):
                    nS[x] = nS[E] + go + (x - E - 1) * ge
            S, V = nS, [NEG] * W
            continue
        h = sl = NEG
        nS, nV = [0] * W, [0] * W
        for x in range(W):
            j = i + d0 + x - E
            dg = S[x] + (ma if rd[j - 1] == ab else mi)
            vu = max(V[x + 1] + ge, S[x + 1] + go) if x + 1 < W else NEG
            h = max(h + ge, sl + go)
            s = max(dg, vu, h)
            nS[x], nV[x], sl = s, vu, s
        S, V = nS, nV
    return max(S)


@pytest.mark.parametrize('sc', [(3, -6, -5, -2), (2, -3, -4, -1), (1, -1, -2, -1), (5, -4, -3, -3)])
def test_pinned_bound_equals_constrained_band(sc):
    rng = np.random.default_rng(sum(abs(v) for v in sc))
    for _ in range(400):
        L = int(rng.integers(10, 40))
        E = int(rng.integers(1, 6))
        K = min(int(rng.integers(4, 9)), L)
        o = int(rng.integers(0, L - K + 1))
        ac = rng.integers(0, 4, L)
        rd = rng.integers(0, 4, L + 80)
        d0 = int(rng.integers(E + 2, 20))
        if rng.random() < 0.7:                    # a noisy copy of the adapter on the run's diagonal
            for i in range(L):
                if rng.random() < 0.85:
                    rd[d0 + i] = ac[i]
            if rng.random() < 0.5:                # an insertion next to the run
                p = d0 + o + K + int(rng.integers(0, 3))
                rd = np.concatenate([rd[:p], rng.integers(0, 4, int(rng.integers(1, 3))), rd[p:]])
        rd[o + d0:o + d0 + K] = ac[o:o + K]
        assert pinned_bound(ac, rd, L, d0, E, o, K, sc) == constrained_band(ac, rd, L, d0, E, o, K, sc)
