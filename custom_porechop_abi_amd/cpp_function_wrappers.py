"""Drop-in for porechop_abi/cpp_function_wrappers.py: the same ``adapter_alignment`` entry point,
now bound to libpcabi.so (HIP, gfx950) instead of the reference's SeqAn cpp_functions.so.

Reference interface replaced: porechop_abi/cpp_function_wrappers.py:42-63 (ctypes binding of
``adapterAlignment`` / ``freeCString``, porechop_abi/include/adapter_align.h:12-16). Same
arguments, same return text ("rs,re,as,ae,score,pid1,pid2"), same ownership protocol.

Unlike the reference, a missing library is an exception rather than ``sys.exit``; there is
no CPU fallback.
"""
from ctypes import c_char_p, cast

from ._lib import lib


def adapter_alignment(read_sequence, adapter_sequence, scoring_scheme_vals):
    """Python wrapper for the adapterAlignment C ABI (one alignment, run on the GPU)."""
    match_score = scoring_scheme_vals[0]
    mismatch_score = scoring_scheme_vals[1]
    gap_open_score = scoring_scheme_vals[2]
    gap_extend_score = scoring_scheme_vals[3]
    L = lib()
    ptr = L.adapterAlignment(read_sequence.encode('utf-8'), adapter_sequence.encode('utf-8'),
                             match_score, mismatch_score, gap_open_score, gap_extend_score)
    return c_string_to_python_string(ptr)


def c_string_to_python_string(c_string):
    """Copy the malloc'd C string into Python and release it with freeCString."""
    text = cast(c_string, c_char_p).value.decode()
    lib().freeCString(c_string)
    return text
