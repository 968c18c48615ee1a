"""C ABI of libpcabi.so (include/pcabi.h): the library loads without a GPU, exports every entry
point the header declares (the two legacy symbols of porechop_abi/include/adapter_align.h:12-16
included), and its host helpers are exact. No compute call needs a GPU here."""
import ctypes
import math
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    src = open(os.path.join(ROOT, 'include', 'pcabi.h')).read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    names = re.findall(r'^\s*(?:const\s+)?[A-Za-z_][\w]*\s*\**\s*\**\s*([A-Za-z_]\w*)\s*\(', src, flags=re.M)
    return sorted(set(n for n in names if n not in ('if', 'while', 'sizeof')))


def test_header_declares_legacy_symbols():
    names = declared_functions()
    assert 'adapterAlignment' in names and 'freeCString' in names
    assert len(names) >= 25


def test_library_exports_every_declared_symbol():
    from custom_porechop_abi_amd import _lib
    L = _lib.lib()
    so = ctypes.CDLL(_lib.LIB_PATH)
    for name in declared_functions():
        assert hasattr(so, name), name
    assert set(_lib.exported_symbols()) == set(declared_functions())
    assert L.pcabi_version() == 1
    assert L.pcabi_max_adapter_len() == 65535     # striped core: adapters of any practical length
    L.pcabi_io_release_cache()                    # host only: returns the cached batch mappings


def test_encode_dna5_matches_seqan_table():
    from custom_porechop_abi_amd import _lib, engine
    L = _lib.lib()
    src = bytes(range(256))
    out = np.zeros(256, np.uint8)
    L.pcabi_encode_dna5(ctypes.c_char_p(src), out.ctypes.data_as(ctypes.c_void_p), 256)
    exp = np.full(256, 4, np.uint8)
    for c, v in zip('ACGTUacgtu', [0, 1, 2, 3, 3, 0, 1, 2, 3, 3]):
        exp[ord(c)] = v
    assert np.array_equal(out, exp)
    assert np.array_equal(engine.DNA5, exp)


def test_pid6_host_exact():
    from custom_porechop_abi_amd import engine
    l = np.repeat(np.arange(1, 400), np.arange(2, 401)).astype(np.int32)
    m = np.concatenate([np.arange(0, k + 1) for k in range(1, 400)]).astype(np.int32)
    got = engine.pid6(m, l)
    exp = np.array([float('%f' % (100.0 * a / b)) for a, b in zip(m.tolist(), l.tolist())])
    assert np.array_equal(got, exp)
    assert math.isnan(engine.pid6(np.array([0], np.int32), np.array([0], np.int32))[0])


def test_compute_fails_loudly_without_device():
    from custom_porechop_abi_amd import _lib, cpp_function_wrappers as w, engine
    L = _lib.lib()
    if L.pcabi_device_count() > 0:
        pytest.skip('a GPU is visible')
    # no CPU fallback: the batch API raises ...
    pack = engine.SeqPack(['ACGTACGTAC'])
    with pytest.raises(_lib.PcabiError):
        engine.align(pack.views([0], pack.lengths), ['GTAC'], [3, -6, -5, -2])
    # ... and the legacy symbols, which have no error channel, stop the process with the reason
    # instead of answering "no alignment" (VERDICT r1); empty inputs keep the reference's "-1"
    assert w.adapter_alignment('', 'GTAC', [3, -6, -5, -2]).split(',')[0] == '-1'
    import subprocess
    import sys
    code = ('import sys; sys.path.insert(0, %r); from custom_porechop_abi_amd import cpp_function_wrappers as w; '
            'print(w.adapter_alignment("ACGTACGTAC", "GTAC", [3, -6, -5, -2]))' % ROOT)
    p = subprocess.run([sys.executable, '-c', code], capture_output=True, text=True, timeout=120)
    assert p.returncode != 0 and 'adapterAlignment failed' in p.stderr, (p.returncode, p.stdout, p.stderr[-400:])
    code = ('import sys; sys.path.insert(0, %r); from custom_porechop_abi_amd import _lib; '
            'print(_lib.lib().check_compatibility(b"ACGTACGTAC", b"ACGTAC"))' % ROOT)
    p = subprocess.run([sys.executable, '-c', code], capture_output=True, text=True, timeout=120)
    assert p.returncode != 0 and 'check_compatibility failed' in p.stderr, (p.returncode, p.stdout, p.stderr[-400:])


def test_window_views_match_python_slices():
    from custom_porechop_abi_amd import engine
    seqs = ['', 'A', 'ACGTN' * 50, 'acgu' * 100, 'GATTACA' * 7]
    pack = engine.SeqPack(seqs)
    for E in (150, 1, 0, 400):
        sw, ew = engine.start_end_windows(pack, E)
        for k, s in enumerate(seqs):
            for (codes, off, ln), sl in ((sw, s[:E]), (ew, s[-E:])):
                got = codes[off[k]:off[k] + ln[k]]
                assert off[k] + ln[k] + 16 <= len(codes)      # the ABI's tail padding
                assert np.array_equal(got, engine.encode_seq(sl))


def test_gathered_windows_equal_packed_slices():
    """SeqPack.windows (pcabi_encode_dna5_gather from the strs' own buffers) lays out exactly what
    SeqPack of the slices does: codes byte for byte, N padding included; non-ASCII input takes
    the slicing path. Covers the drivers' end windows and trimmed reads (porechop_abi.py)."""
    import random
    from custom_porechop_abi_amd import engine, porechop_abi as P
    from custom_porechop_abi_amd.nanopore_read import NanoporeRead
    rng = random.Random(7)
    seqs = [''.join(rng.choice('ACGTNacgu-xyz') for _ in range(rng.randint(0, 3000))) for _ in range(700)]
    seqs += ['', 'A', 'GATTACA' * 5000]
    st = [rng.randint(0, len(s)) for s in seqs]
    ln = [rng.randint(0, len(s) - a) for s, a in zip(seqs, st)]
    want = engine.SeqPack([s[a:a + l] for s, a, l in zip(seqs, st, ln)])
    for mixed in (False, True):
        q = seqs + (['ACGTé'] if mixed else [])
        got = engine.SeqPack.windows(q, st + [1] * mixed, ln + [3] * mixed)
        ref = want if not mixed else engine.SeqPack([s[a:a + l] for s, a, l in zip(q, st + [1], ln + [3])])
        assert np.array_equal(got.codes, ref.codes) and np.array_equal(got.offsets, ref.offsets)
        assert np.array_equal(got.lengths, ref.lengths)
    # 22 MB: the byte-balanced thread split (each thread starts at a segment boundary)
    big = engine.SeqPack.windows(['ACGT' * 3000000, 'TTGCA' * 2000000], [5, 17], [12000000 - 5, 9999983 - 17])
    assert np.array_equal(big.codes, engine.SeqPack([('ACGT' * 3000000)[5:], ('TTGCA' * 2000000)[17:9999983]]).codes)
    # the drivers' end windows for every sign of end_size, and the trimmed reads
    reads = [NanoporeRead('r%d' % i, s, '') for i, s in enumerate(seqs[:200])]
    for E in (150, 1, 0, -3, 5000):
        codes, (so, sl), (eo, el) = P.end_windows_pack(reads, E)
        ref = engine.SeqPack([r.seq[:E] for r in reads] + [r.seq[-E:] for r in reads])
        assert np.array_equal(codes, ref.codes)
        assert np.array_equal(np.concatenate([so, eo]), ref.offsets)
        assert np.array_equal(np.concatenate([sl, el]), ref.lengths)
    for r in reads:
        r.start_trim_amount, r.end_trim_amount = rng.randint(0, 400), rng.randint(0, 4000)
    a, l = P.trimmed_bounds(reads)
    got = engine.SeqPack.windows([r.seq for r in reads], a, l)
    ref = engine.SeqPack([r.get_seq_with_start_end_adapters_trimmed() for r in reads])
    assert np.array_equal(got.codes, ref.codes) and np.array_equal(got.lengths, ref.lengths)


def test_host_string_windows_checker_layout():
    """oracle_lib.seqs_windows -- how the checkers read the windows engine.middle_scan_seqs takes
    (host character addresses + lengths) -- gives SeqPack's layout of the same slices."""
    import random
    from custom_porechop_abi_amd import engine
    from tests import oracle_lib
    rng = random.Random(5)
    seqs = [''.join(rng.choice('ACGTNacgu-xyz') for _ in range(rng.randint(0, 900))) for _ in range(300)] + ['']
    st = [rng.randint(0, len(s)) for s in seqs]
    ln = [rng.randint(0, len(s) - a) for s, a in zip(seqs, st)]
    addr, have = engine.str_buffers(seqs)
    codes, offs, lens = oracle_lib.seqs_windows(addr + np.array(st, np.uint64), ln)
    ref = engine.SeqPack([s[a:a + l] for s, a, l in zip(seqs, st, ln)])
    assert np.array_equal(codes, ref.codes) and np.array_equal(offs, ref.offsets)
    assert np.array_equal(lens, ref.lengths)


def test_gathered_windows_reject_out_of_range():
    from custom_porechop_abi_amd import engine
    for st, ln in (([0], [5]), ([-1], [1]), ([2], [-1]), ([0, 0], [1, 1])):
        with pytest.raises(ValueError):
            engine.SeqPack.windows(['ACGT'], st, ln)
