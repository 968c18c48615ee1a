"""Loader for libpcabi.so, the MI355X adapter-alignment engine (C ABI: include/pcabi.h).

There is deliberately no CPU fallback: if the library or a gfx950 device is missing, compute
entry points raise PcabiError. The CPU restatement under oracle/ is test infrastructure only.

HIP runtime sharing: PyTorch-ROCm wheels bundle their own libamdhip64.so.7. If torch is already
imported (the multi-GPU path uses torch.distributed/RCCL), loading libpcabi.so after it binds
to the SAME runtime (identical SONAME), so one process never holds two HIP runtimes. Import
torch before this module whenever both are used (bench.py and shards.py do).
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('PCABI_LIB', os.path.join(_HERE, 'libpcabi.so'))

NFIELDS = 8
F_RS, F_RE, F_AS, F_AE, F_SCORE, F_M, F_L1, F_L2 = range(8)


class PcabiError(RuntimeError):
    pass


_lib = None


def lib():
    """Return the loaded ctypes library (loads and declares signatures on first use)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.isfile(LIB_PATH):
        raise PcabiError('libpcabi.so not found at %s - run __graft_entry__.build() '
                         '(hipcc --offload-arch=gfx950)' % LIB_PATH)
    L = ctypes.CDLL(LIB_PATH)
    c_int, c_i64, c_p, c_d = ctypes.c_int, ctypes.c_int64, ctypes.c_void_p, ctypes.c_double
    sig = {
        'adapterAlignment': ([ctypes.c_char_p, ctypes.c_char_p, c_int, c_int, c_int, c_int], c_p),
        'freeCString': ([c_p], None),
        'pcabi_last_error': ([], ctypes.c_char_p),
        'pcabi_version': ([], c_int),
        'pcabi_device_count': ([], c_int),
        'pcabi_max_adapter_len': ([], c_int),
        'pcabi_max_window_len': ([], c_int),
        'pcabi_encode_dna5': ([c_p, c_p, c_i64], None),
        'pcabi_encode_dna5_gather': ([c_p, c_p, c_p, c_i64, c_p, c_i64], None),
        'pcabi_pid6_host': ([c_p, c_p, c_i64, c_p], None),
        'pcabi_align_host': ([c_int, c_p, c_i64, c_p, c_p, c_i64, c_p, c_p, c_p, ctypes.c_int32,
                              c_p, c_p, c_i64, c_int, c_int, c_int, c_int, c_p], c_int),
        'pcabi_dev_set': ([c_int], c_int),
        'pcabi_dev_malloc': ([ctypes.POINTER(c_p), c_i64], c_int),
        'pcabi_dev_free': ([c_p], c_int),
        'pcabi_dev_h2d': ([c_p, c_p, c_i64], c_int),
        'pcabi_dev_d2h': ([c_p, c_p, c_i64], c_int),
        'pcabi_dev_memset': ([c_p, c_int, c_i64], c_int),
        'pcabi_dev_sync': ([], c_int),
        'pcabi_dev_copy_async': ([c_p, c_p, c_i64, c_int, c_p], c_int),
        'pcabi_stream_create': ([ctypes.POINTER(c_p)], c_int),
        'pcabi_stream_destroy': ([c_p], c_int),
        'pcabi_stream_sync': ([c_p], c_int),
        'pcabi_event_create': ([ctypes.POINTER(c_p)], c_int),
        'pcabi_event_destroy': ([c_p], c_int),
        'pcabi_event_record': ([c_p, c_p], c_int),
        'pcabi_stream_wait_event': ([c_p, c_p], c_int),
        'pcabi_event_elapsed_ms': ([ctypes.POINTER(ctypes.c_float), c_p, c_p], c_int),
        'pcabi_adapters_create': ([c_p, c_p, c_p, ctypes.c_int32, ctypes.POINTER(c_p)], c_int),
        'pcabi_adapters_create_scored': ([c_p, c_p, c_p, ctypes.c_int32, c_int, c_int, c_int, c_int,
                                          ctypes.POINTER(c_p)], c_int),
        'pcabi_adapters_destroy': ([c_p], None),
        'pcabi_tile_layout': ([c_p, c_i64, c_p], c_i64),
        'pcabi_tile_windows_dev': ([c_p, c_p, c_p, c_i64, c_p, c_i64, c_p, c_p], c_int),
        'pcabi_align_cross_dev': ([c_p, c_p, c_p, c_i64, ctypes.c_int32, c_p, c_int, c_int, c_int, c_int,
                                   c_p, c_i64, c_p], c_int),
        'pcabi_align_cross_dev_marked': ([c_p, c_p, c_p, c_i64, ctypes.c_int32, c_p, c_int, c_int, c_int, c_int,
                                          c_p, c_i64, c_p, c_p, c_p], c_int),
        'pcabi_align_cross_multi_dev': ([c_p, ctypes.c_int32, c_int, c_int, c_int, c_int, c_p, c_p, c_p], c_int),
        'pcabi_end_trim_dev': ([c_p, c_i64, ctypes.c_int32, c_p, c_i64, ctypes.c_int32, c_i64, c_int,
                                c_int, c_d, c_int, c_p, c_p, c_p, c_p, c_p], c_int),
        'pcabi_best_full_identity_dev': ([c_p, c_i64, c_i64, ctypes.c_int32, c_p, c_p], c_int),
        'pcabi_first_hits_host': ([c_int, c_p, c_i64, c_p, c_p, c_i64, c_p, c_p, c_p, ctypes.c_int32, c_int, c_int,
                                   c_int, c_int, c_d, c_p], c_int),
        'pcabi_first_hit_dev': ([c_p, c_i64, c_i64, ctypes.c_int32, c_d, c_p, c_i64, c_p], c_int),
        'pcabi_scan_create': ([c_p, ctypes.POINTER(c_p)], c_int),
        'pcabi_scan_destroy': ([c_p], None),
        'pcabi_middle_scan_dev': ([c_p, c_p, c_p, c_p, c_p, c_i64, c_int, c_int, c_int, c_int, c_d, c_p, c_i64, c_p],
                                  c_i64),
        'pcabi_middle_scan_host': ([c_int, c_p, c_i64, c_p, c_p, c_i64, c_p, c_p, c_p, ctypes.c_int32, c_int, c_int,
                                    c_int, c_int, c_d, c_p, c_i64], c_i64),
        'pcabi_middle_scan_seqs': ([c_int, c_p, c_p, c_i64, c_p, c_p, c_p, ctypes.c_int32, c_int, c_int, c_int, c_int,
                                    c_d, c_p, c_i64], c_i64),
        'pcabi_middle_seed_runs': ([], c_i64),
        'pcabi_middle_requeues': ([c_p], c_i64),
        'pcabi_scan_profile': ([c_p, ctypes.c_int32, c_p, ctypes.c_int32], ctypes.c_int32),
        'pcabi_set_side_streams': ([c_int], c_int),
        'pcabi_stream_side_streams': ([c_p, c_int], c_int),
        'pcabi_io_release_cache': ([], None),
        'pcabi_best_full_identity_host': ([c_int, c_p, c_i64, c_p, c_p, c_i64, c_p, c_p, c_p, ctypes.c_int32, c_int,
                                           c_int, c_int, c_int, c_p, c_int], c_int),
        'pcabi_middle_cuts_dev': ([c_p, c_i64, c_i64, c_i64, c_p, c_p, c_int, c_int, c_p, c_p, c_p], c_int),
        'pcabi_middle_cuts_host': ([c_int, c_p, c_i64, c_i64, c_i64, c_p, c_p, ctypes.c_int32, c_int, c_int, c_p, c_p],
                                   c_int),
        'pcabi_barcode_call_dev': ([c_p, c_i64, c_p, c_p, ctypes.c_int32, c_p, c_i64, c_p, c_p, ctypes.c_int32,
                                    c_i64, c_d, c_d, c_int, c_p, c_p, c_p], c_int),
        'pcabi_barcode_call_host': ([c_int, c_p, ctypes.c_int32, c_p, c_p, ctypes.c_int32, c_p, ctypes.c_int32, c_p,
                                     c_p, ctypes.c_int32, c_i64, c_d, c_d, c_int, c_p, c_p], c_int),
        'pcabi_end_decisions_host': ([c_int, c_p, c_i64, c_p, c_p, c_p, c_p, c_i64, c_p, c_p, c_p, ctypes.c_int32,
                                      c_p, c_p, c_p, ctypes.c_int32, c_int, c_int, c_int, c_int, c_int, c_int, c_d,
                                      c_int, c_p, c_p, c_p, c_p, c_i64, c_p, c_p, ctypes.c_int32, c_p,
                                      ctypes.c_int32, c_p], c_int),
        'pcabi_stage_seqs_host': ([c_int, c_p, c_p, c_i64, c_p, c_i64], c_int),
        'pcabi_end_decisions_seqs': ([c_int, c_p, c_p, c_i64, c_p, c_p, c_p, ctypes.c_int32, c_p, c_p, c_p,
                                      ctypes.c_int32, c_int, c_int, c_int, c_int, c_int, c_int, c_d, c_int, c_p, c_p,
                                      c_p, c_p, c_i64, c_p, c_p, ctypes.c_int32, c_p, ctypes.c_int32, c_p], c_int),
        'pcabi_flag_list_dev': ([c_p, ctypes.c_int32, c_i64, c_p, c_i64, c_p, c_i64, c_p, c_p], c_int),
        'pcabi_trim_views_dev': ([c_p, c_p, c_p, c_p, c_i64, c_p, c_p, c_p], c_int),
    }
    for name, (argtypes, restype) in sig.items():
        fn = getattr(L, name)
        fn.argtypes = argtypes
        fn.restype = restype
    _lib = L
    return L


def exported_symbols():
    """Names every ABI entry point declared in include/pcabi.h (checked by tests)."""
    lib()
    return ['adapterAlignment', 'freeCString', 'pcabi_last_error', 'pcabi_version',
            'pcabi_device_count', 'pcabi_max_adapter_len', 'pcabi_max_window_len',
            'pcabi_encode_dna5', 'pcabi_encode_dna5_gather', 'pcabi_pid6_host', 'pcabi_align_host', 'pcabi_dev_set',
            'pcabi_dev_malloc', 'pcabi_dev_free', 'pcabi_dev_h2d', 'pcabi_dev_d2h',
            'pcabi_dev_memset', 'pcabi_dev_sync', 'pcabi_dev_copy_async', 'pcabi_stream_create', 'pcabi_stream_destroy',
            'pcabi_stream_sync', 'pcabi_event_create', 'pcabi_event_destroy', 'pcabi_event_record',
            'pcabi_stream_wait_event', 'pcabi_event_elapsed_ms', 'pcabi_adapters_create', 'pcabi_adapters_create_scored', 'pcabi_adapters_destroy',
            'pcabi_tile_layout', 'pcabi_tile_windows_dev', 'pcabi_align_cross_dev', 'pcabi_align_cross_dev_marked',
            'pcabi_align_cross_multi_dev', 'pcabi_end_trim_dev',
            'pcabi_best_full_identity_dev', 'pcabi_first_hits_host', 'pcabi_first_hit_dev', 'pcabi_scan_create',
            'pcabi_scan_destroy', 'pcabi_middle_scan_dev', 'pcabi_middle_scan_host', 'pcabi_middle_scan_seqs', 'pcabi_middle_seed_runs',
            'pcabi_middle_requeues', 'pcabi_scan_profile', 'pcabi_set_side_streams', 'pcabi_stream_side_streams',
            'pcabi_barcode_call_dev',
            'pcabi_barcode_call_host', 'pcabi_fastx_open', 'pcabi_fastx_type', 'pcabi_fastx_next',
            'pcabi_fastx_close', 'pcabi_fastx_remaining', 'pcabi_fastx_load', 'pcabi_reads_count', 'pcabi_reads_type', 'pcabi_reads_views',
            'pcabi_reads_free', 'pcabi_reads_write', 'check_compatibility', 'pcabi_compat_host',
            'pcabi_compat_all_vs_all_host', 'pcabi_kmer_count_host', 'pcabi_kmer_top_host', 'pcabi_gather_host',
            'pcabi_kmer_approx_host', 'pcabi_io_release_cache', 'pcabi_best_full_identity_host',
            'pcabi_middle_cuts_dev', 'pcabi_middle_cuts_host', 'pcabi_fastx_record_start', 'pcabi_fastx_set_range', 'pcabi_fastx_next_text',
            'pcabi_end_decisions_host', 'pcabi_end_decisions_seqs', 'pcabi_stage_seqs_host', 'pcabi_flag_list_dev', 'pcabi_trim_views_dev']


class CrossRegion(ctypes.Structure):
    """include/pcabi.h pcabi_cross_region: one cross product of pcabi_align_cross_multi_dev."""
    _fields_ = [('tiles', ctypes.c_void_p), ('tile_off', ctypes.c_void_p), ('win_len', ctypes.c_void_p),
                ('n_win', ctypes.c_int64), ('max_win_len', ctypes.c_int32), ('adps', ctypes.c_void_p),
                ('out', ctypes.c_void_p), ('out_stride', ctypes.c_int64)]


def cross_regions(regions):
    """A ctypes array of CrossRegion from (tiles, tile_off, win_len, n_win, max_win_len, adps, out,
    out_stride) tuples (device pointers as ints or c_void_p)."""
    arr = (CrossRegion * len(regions))()
    for k, r in enumerate(regions):
        vals = [x.value if isinstance(x, ctypes.c_void_p) else x for x in r]
        arr[k] = CrossRegion(*vals)
    return arr


def check(rc, what):
    if rc != 0:
        msg = lib().pcabi_last_error()
        raise PcabiError('%s failed (%d): %s' % (what, rc, msg.decode() if msg else ''))
