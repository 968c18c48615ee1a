"""Fuzz the oracle restatement (oracle/liboracle.so) against the reference compiled in place
(oracle/_ref/cpp_functions.so). Container-only tool: needs /root/reference (oracle/Makefile ref)."""
import ctypes, os, random, sys
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
ref = ctypes.CDLL(os.path.join(ROOT, 'oracle/_ref/cpp_functions.so'))
ora = ctypes.CDLL(os.path.join(ROOT, 'oracle/liboracle.so'))
for lib, fn, fr in ((ref, 'adapterAlignment', 'freeCString'), (ora, 'pcabi_oracle_adapter_alignment', 'pcabi_oracle_free')):
    getattr(lib, fn).argtypes = [ctypes.c_char_p, ctypes.c_char_p] + [ctypes.c_int] * 4
    getattr(lib, fn).restype = ctypes.c_void_p
    getattr(lib, fr).argtypes = [ctypes.c_void_p]

def call(lib, fn, fr, r, a, sc):
    p = getattr(lib, fn)(r.encode(), a.encode(), *sc)
    s = ctypes.cast(p, ctypes.c_char_p).value.decode()
    getattr(lib, fr)(p)
    return s

def main(n=20000, seed=1):
    rng = random.Random(seed)
    schemes = [(3, -6, -5, -2), (2, -1, -1, -1), (1, -1, -3, -1), (3, -6, -2, -5), (5, -4, -8, -6), (1, -2, -2, -2)]
    alph = ['A', 'AT', 'ACGT', 'ACGTN', 'ACGT-', 'AC']
    bad = 0
    for t in range(n):
        sc = rng.choice(schemes)
        al = rng.choice(alph)
        L = rng.choice([1, 2, 3, 5, 8, 13, 24, 30, 50, rng.randint(1, 120)])
        N = rng.choice([1, 2, 4, 10, 40, 150, rng.randint(1, 400)])
        a = ''.join(rng.choice(al) for _ in range(L))
        r = ''.join(rng.choice(al) for _ in range(N))
        if rng.random() < 0.3 and N > L:
            p = rng.randint(0, N - L)
            mut = ''.join(c if rng.random() > 0.15 else rng.choice('ACGT') for c in a)
            r = r[:p] + mut + r[p + L:]
        x = call(ref, 'adapterAlignment', 'freeCString', r, a, sc)
        y = call(ora, 'pcabi_oracle_adapter_alignment', 'pcabi_oracle_free', r, a, sc)
        if x != y:
            bad += 1
            if bad < 10:
                print('MISMATCH', sc, repr(r), repr(a), x, y)
    print('cases', n, 'mismatches', bad)
    return bad

if __name__ == '__main__':
    sys.exit(1 if main(int(sys.argv[1]) if len(sys.argv) > 1 else 20000) else 0)
