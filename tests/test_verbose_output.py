"""The phase drivers' verbose output vs the text the REFERENCE'S OWN drivers print
(tests/golden/g6_verbose.json.gz, tools/make_golden_g6.py): progress lines at verbosity 1 (the
middle phase's thread-pool variant included), the per-read windows at verbosity 2
(NanoporeRead.formatted_start_and_end_seq, nanopore_read.py:315-328) and 3 (full_start_end_output,
:330-360), and the middle hits with their highlighted context (middle_adapter_results /
formatted_middle_seq, :362-406), colour codes included -- so a reference test that greps the
verbose output (test/test_one_adapter_set.py:60-68) passes after the level-2 swap.
  * not gpu: the drivers with the CPU oracle standing in for the kernels (host logic + text);
  * gpu    : the same drivers on the HIP kernels.
"""
import gzip
import io
import json
import os

import pytest

from tests import golden_lib, oracle_lib

_G6 = None


def g6():
    global _G6
    if _G6 is None:
        with gzip.open(os.path.join(os.path.dirname(__file__), 'golden', 'g6_verbose.json.gz'), 'rt') as f:
            _G6 = json.load(f)
    return _G6


G2 = golden_lib.g2()
RUNS = [(r['case'], r['verbosity'], r['threads']) for r in g6()['runs']]


def _drivers_output(case_name, verbosity, threads):
    from custom_porechop_abi_amd import adapters as A, porechop_abi as P
    from custom_porechop_abi_amd.nanopore_read import NanoporeRead
    case = next(c for c in G2['cases'] if c['case'] == case_name)
    opts = case['opts']
    recs = [tuple(x) for x in G2['synthetic_reads']] if case['input'] == 'synthetic_reads' \
        else golden_lib.load_records(case['input'])
    reads = [NanoporeRead(n, s, q) for n, s, q in recs]
    sc = opts['scoring']
    out = {}
    buf = io.StringIO()
    matching = P.find_matching_adapter_sets(reads[:opts.get('check_reads', 10000)], verbosity, opts['end_size'], sc,
                                            buf, opts['adapter_threshold'], threads, adapter_sets=A.fresh_adapters())
    out['check'] = buf.getvalue()
    matching = P.fix_up_1d2_sets(matching)
    fr = P.choose_barcoding_kit(matching, 0, io.StringIO()) if opts['barcodes'] else None
    matching = P.add_full_barcode_adapter_sets(matching)
    if matching:
        buf = io.StringIO()
        P.find_adapters_at_read_ends(reads, matching, verbosity, opts['end_size'], opts['extra_end_trim'],
                                     opts['end_threshold'], sc, buf, opts['min_trim_size'], threads, opts['barcodes'],
                                     75.0, 5.0, opts.get('require_two', False), fr)
        out['ends'] = buf.getvalue()
        buf = io.StringIO()
        P.find_adapters_in_read_middles(reads, matching, verbosity, opts['middle_threshold'], 10, 100, sc, buf,
                                        threads, False)
        out['middles'] = buf.getvalue()
    return out


def _expected(case_name, verbosity, threads):
    return next(r['out'] for r in g6()['runs']
                if (r['case'], r['verbosity'], r['threads']) == (case_name, verbosity, threads))


def _oracle_backend(monkeypatch):
    from custom_porechop_abi_amd import engine
    monkeypatch.setattr(engine, 'align', oracle_lib.align_windows)
    monkeypatch.setattr(engine, 'end_decisions', oracle_lib.end_decisions_windows)
    monkeypatch.setattr(engine, 'best_full_identity', oracle_lib.best_full_identity_windows)
    monkeypatch.setattr(engine, 'first_hits', oracle_lib.first_hits_windows)
    monkeypatch.setattr(engine, 'middle_scan', oracle_lib.middle_scan_windows)
    monkeypatch.setattr(engine, 'middle_scan_seqs', oracle_lib.middle_scan_seqs_windows)


@pytest.mark.parametrize('case_name,verbosity,threads', RUNS)
def test_verbose_output_matches_reference_with_oracle_backend(monkeypatch, case_name, verbosity, threads):
    _oracle_backend(monkeypatch)
    got = _drivers_output(case_name, verbosity, threads)
    exp = _expected(case_name, verbosity, threads)
    assert sorted(got) == sorted(exp)
    for phase in exp:
        assert got[phase] == exp[phase], phase


def test_reference_verbosity_2_window_strings(monkeypatch):
    """test/test_one_adapter_set.py:60-68: the two formatted window strings and the phase heading
    appear in the verbosity-2 output."""
    _oracle_backend(monkeypatch)
    out = ''.join(_drivers_output('one_adapter_set', 2, 1).values())
    assert 'Trimming adapters from read ends' in out
    assert 'CGCACCTCTCCCCTCTGCGTCCTAGGCACTAGATCCAAACCTAGTTCGCCTGAAATTTACTGATGCTAGACCG' \
           'AAACTTCGCGCCGACTACTCCATGGTT' in out
    assert 'GCCCGTATCCACGTAAGAGTGCATCTCATTGCGCACAGGTATATCTGCCAGATAAGACGTCGAGG' in out


def test_formatting_methods_edge_cases():
    """The slices of the formatting methods at their edges (expected strings from the reference's own
    methods, nanopore_read.py:254-313, run in the container):
    no trim, trims that cover the whole read, a trim of only the extra bases, short middles."""
    from custom_porechop_abi_amd.misc import RED, YELLOW, END_FORMATTING as E
    from custom_porechop_abi_amd.nanopore_read import NanoporeRead
    r = NanoporeRead('r', 'ACGTACGTAC', '')
    assert r.formatted_whole_seq(2) == r.seq and r.formatted_start_seq(5, 2) == 'ACGTA'
    r.start_trim_amount = 2                       # only the extra trim: no red part
    assert r.formatted_start_seq(5, 2) == YELLOW + 'AC' + E + 'GTA'
    r.end_trim_amount = 2                         # red_bases == 0: the reference's [-2:-0] slice is empty
    assert r.formatted_end_seq(5, 2) == 'CGT' + YELLOW + E
    r.start_trim_amount, r.end_trim_amount = 7, 7  # red parts cover the read
    assert r.formatted_whole_seq(2) == RED + r.seq + E
    r.start_trim_amount, r.end_trim_amount = 4, 0
    assert r.formatted_whole_seq(2) == RED + 'AC' + E + YELLOW + 'GT' + E + 'ACGTAC'
    r.start_trim_amount, r.end_trim_amount = 5, 5  # middle of 4 <= 2 * extra: all yellow
    assert r.formatted_whole_seq(2) == RED + 'ACG' + E + YELLOW + 'TACG' + E + RED + 'TAC' + E
    assert r.formatted_middle_seq() is None and r.middle_adapter_results(2) == ''


@pytest.mark.gpu
@pytest.mark.parametrize('case_name,verbosity,threads', [x for x in RUNS if x[1] >= 2])
def test_verbose_output_matches_reference_on_gpu(gpu_lib, case_name, verbosity, threads):
    got = _drivers_output(case_name, verbosity, threads)
    exp = _expected(case_name, verbosity, threads)
    for phase in exp:
        assert got[phase] == exp[phase], phase
