"""Ab-initio adapter clustering link test on the GPU (mirror of the compatibility part of
porechop_abi/consensus.py:72-100; the C++ it replaces is porechop_abi/ab_initio_src/
compatibility.cpp, bound there through ctypes as compatibility.so::check_compatibility).

all_vs_all_matrix(sequences) keeps the reference's signature and result: a list-of-lists
matrix, -1 on the diagonal, mat[i][j] = mat[j][i] = check_compatibility(seq_i, seq_j) in
{0, 1, 2}. All pairs run as ONE batch of the engine's DP kernels (pairs mode, scoring
2 / -1 / -1 linear, String<Dna> codes) with the compatibility epilogue on the device.
"""
import ctypes

import numpy as np

from ._lib import check, lib

# SeqAn String<Dna> (compatibility.h:23, S/basic/alphabet_residue_tabs.h:70-99): A C G T/U, else A
DNA4 = np.zeros(256, dtype=np.uint8)
for _c, _v in (('C', 1), ('G', 2), ('T', 3), ('U', 3)):
    DNA4[ord(_c)] = _v
    DNA4[ord(_c.lower())] = _v


def _declare(L):
    if not getattr(L, '_compat_declared', False):
        P = ctypes.c_void_p
        L.pcabi_compat_host.argtypes = [ctypes.c_int, P, ctypes.c_int64, P, P, ctypes.c_int64, P, P, ctypes.c_int64, P]
        L.pcabi_compat_host.restype = ctypes.c_int
        L.pcabi_compat_all_vs_all_host.argtypes = [ctypes.c_int, P, ctypes.c_int64, P, P, ctypes.c_int64, P]
        L.pcabi_compat_all_vs_all_host.restype = ctypes.c_int
        L.check_compatibility.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
        L.check_compatibility.restype = ctypes.c_int
        L._compat_declared = True
    return L


def _pack(sequences):
    raw = [s.encode('utf-8') if isinstance(s, str) else bytes(s) for s in sequences]
    lens = np.array([len(b) for b in raw], np.int32)
    offs = np.zeros(len(raw), np.int64)
    pos = 0
    parts = []
    for k, b in enumerate(raw):
        offs[k] = pos
        pad = (-len(b)) & 3
        parts.append(b + b'A' * pad)
        pos += len(b) + pad
    parts.append(b'A' * 16)
    codes = DNA4[np.frombuffer(b''.join(parts), dtype=np.uint8)]
    return np.ascontiguousarray(codes), offs, lens


def compat_pairs(sequences, pair_i, pair_j, device=0):
    """check_compatibility(sequences[pair_i[t]], sequences[pair_j[t]]) for every t (int32)."""
    L = _declare(lib())
    codes, offs, lens = _pack(sequences)
    pi = np.ascontiguousarray(pair_i, np.int32)
    pj = np.ascontiguousarray(pair_j, np.int32)
    out = np.zeros(len(pi), np.int32)
    if len(pi):
        p = lambda a: a.ctypes.data_as(ctypes.c_void_p)
        check(L.pcabi_compat_host(device, p(codes), codes.size, p(offs), p(lens), len(lens), p(pi), p(pj), len(pi),
                                  p(out)), 'pcabi_compat_host')
    return out


def all_vs_all_flags(sequences, device=0):
    """The flag matrix as an int32 (n, n) array (-1 on the diagonal): every sequence against
    every sequence in one tiled cross product on the device (pcabi_compat_all_vs_all_host)."""
    L = _declare(lib())
    codes, offs, lens = _pack(sequences)
    n = len(lens)
    mat = np.empty((n, n), np.int32) if n >= 2 else np.full((n, n), -1, np.int32)   # the library writes every entry
    if n >= 2:
        p = lambda a: a.ctypes.data_as(ctypes.c_void_p)
        check(L.pcabi_compat_all_vs_all_host(device, p(codes), codes.size, p(offs), p(lens), n, p(mat)),
              'pcabi_compat_all_vs_all_host')
    return mat


def all_vs_all_matrix(sequences):
    """consensus.py:72-100: the compatibility flag matrix of every pair (i < j, mirrored), as
    the reference's list of lists."""
    return all_vs_all_flags(sequences).tolist()
