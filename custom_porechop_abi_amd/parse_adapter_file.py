"""Custom adapter files (mirror of porechop_abi/parse_adapter_file.py:17-73, the CLI's
--custom_adapters): three lines per adapter set -- name, start sequence, end sequence (an empty
line for a missing side); the sequences must be DNA (A, C, G, T only). Sets are named after the
file's name line, their sequences "<name>_Top" / "<name>_Bottom". Adapters of any length go
through the engine (the striped core takes those past 128 bp).
"""
import re
import sys

from .adapters import Adapter

_DNA = re.compile(r'^[ATCG]+$')


def err_log(msg):
    print('/!\\\t' + msg)


def get_adapters(infile):
    """The custom adapter sets of `infile`, in file order. A trailing incomplete group (fewer
    than three lines) is ignored, and a sequence that is not DNA ends the program with the
    reference's message and exit status 1."""
    with open(infile) as f:
        lines = [x.rstrip('\n') for x in f]
    adapters = []
    for i in range(0, len(lines) - len(lines) % 3, 3):
        name, start, end = lines[i], lines[i + 1], lines[i + 2]
        if (start and not _DNA.match(start)) or (end and not _DNA.match(end)):
            for m in ('INVALID FORMAT', 'Unable to parse DNA sequences from inputs', 'Start: ' + start,
                      'End: ' + end, 'Expected format:', 'line 1: Adapter name',
                      'line 2: Start sequence (DNA or empty line)', 'line 3: End sequence (DNA or empty line)',
                      '--- repeat ---'):
                err_log(m)
            sys.exit(1)
        adapters.append(Adapter(name, start_sequence=(name + '_Top', start) if start else [],
                                end_sequence=(name + '_Bottom', end) if end else []))
    return adapters
