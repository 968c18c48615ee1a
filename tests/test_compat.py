"""Ab-initio clustering link test: check_compatibility (porechop_abi/ab_initio_src/
compatibility.cpp:124-170, all-vs-all in consensus.py:72-100) vs the reference's own
compatibility.so outputs (tests/golden/g4_compat.json.gz, tools/make_golden_g4.py):
  * not gpu: the oracle restatement (oracle/pcabi_oracle.c pcabi_oracle_compat) and the device
    DP core compiled for the host + pcabi::compat_flag (the kernels' compat epilogue);
  * gpu    : the HIP kernels through pcabi_compat_host / the drop-in check_compatibility symbol
             and consensus.all_vs_all_matrix."""
import ctypes
import gzip
import json
import os

import numpy as np
import pytest

from tests import golden_lib, oracle_lib
from tests.test_dp_core_cpu import model  # noqa: F401  (host build of the device core)

G4 = json.load(gzip.open(os.path.join(golden_lib.GOLDEN, 'g4_compat.json.gz'), 'rt'))['pairs']
# both sequences > 128 bp: the striped core (tools/make_golden_g4.py --long)
G4L = json.load(gzip.open(os.path.join(golden_lib.GOLDEN, 'g4_compat_long.json.gz'), 'rt'))['pairs']


@pytest.mark.parametrize('which', ['g4', 'g4_long'])
def test_oracle_compat_matches_reference(which):
    lib = oracle_lib.load()
    lib.pcabi_oracle_compat.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    lib.pcabi_oracle_compat.restype = ctypes.c_int
    pairs = G4 if which == 'g4' else G4L
    bad = [(a, b, f) for a, b, f in pairs if lib.pcabi_oracle_compat(a.encode(), b.encode()) != f]
    assert not bad, bad[:3]


@pytest.mark.parametrize('which', ['g4', 'g4_long'])
def test_device_core_compat_matches_reference(model, which):  # noqa: F811
    model.pcabi_model_compat.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    model.pcabi_model_compat.restype = ctypes.c_int
    pairs = G4 if which == 'g4' else G4L
    bad = [(a, b, f) for a, b, f in pairs if model.pcabi_model_compat(a.encode(), b.encode()) != f]
    assert not bad, bad[:3]


@pytest.mark.gpu
@pytest.mark.parametrize('which', ['g4', 'g4_long'])
def test_compat_kernels_match_reference(gpu_lib, which):
    from custom_porechop_abi_amd import consensus
    pairs = G4 if which == 'g4' else G4L
    seqs = sorted({x for a, b, _ in pairs for x in (a, b)})
    idx = {s: k for k, s in enumerate(seqs)}
    pi = np.array([idx[a] for a, _, _ in pairs], np.int32)
    pj = np.array([idx[b] for _, b, _ in pairs], np.int32)
    got = consensus.compat_pairs(seqs, pi, pj)
    exp = np.array([f for _, _, f in pairs], np.int32)
    assert np.array_equal(got, exp), np.nonzero(got != exp)[0][:5]


@pytest.mark.gpu
def test_drop_in_symbol_and_all_vs_all(gpu_lib):
    from custom_porechop_abi_amd import _lib, consensus
    L = _lib.lib()
    for a, b, f in G4[:200]:
        assert L.check_compatibility(a.encode(), b.encode()) == f
    lib = oracle_lib.load()
    lib.pcabi_oracle_compat.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
    lib.pcabi_oracle_compat.restype = ctypes.c_int
    for a, b, f in G4L[:100]:
        assert L.check_compatibility(a.encode(), b.encode()) == f
    short = [a for a, _, _ in G4 if len(a) <= 128][:300]          # tiled cross mode
    # sequences > 128 bp as DP rows too: the striped bucket in the same cross product
    mixed = short[:120] + [s * 2 for s in short if len(s) > 70][:3] + [a for a, _, _ in G4L[:20]]
    assert sum(len(s) > 128 for s in mixed) > 10
    # equal-length pairs: the reference's row 0 is the first argument
    ties = [s for s in short if len(s) == 24][:20] + [s[::-1] for s in short if len(s) == 24][:20]
    for seqs in (short, mixed, ties):
        mat = consensus.all_vs_all_matrix(seqs)
        for i in range(len(seqs)):
            assert mat[i][i] == -1
            for j in range(i + 1, len(seqs)):
                o = lib.pcabi_oracle_compat(seqs[i].encode(), seqs[j].encode())
                if o >= 0:
                    assert mat[i][j] == mat[j][i] == o, (seqs[i], seqs[j])
