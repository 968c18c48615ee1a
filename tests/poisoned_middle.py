"""Test infrastructure (run by tests/test_gpu_middle_paths.py::test_poisoned_scratch, in a child
process started with PCABI_POISON=1 or =0x3f): every device scratch buffer this
process allocates starts as 0xFF (every int -1) or 0x3F bytes (every int32 / int64 a huge positive count,
small enough that a quarter more does not overflow int64: 0x7F bytes did, and hid the r05 bug)
instead of the zeros fresh hipMalloc memory usually holds, and the
middle scan's product paths and an end-trim cross product must still equal the oracle:

  * round-1 overflow, growth and requeue from tiny initial buffers (PCABI_MIDDLE_INIT_CAPS);
  * faults injected into rounds 1-3 (PCABI_MIDDLE_FAULT), with and without candidate windows;
  * the shadow arena that has to grow, the caller's pack left intact, three scans of one pack;
  * candidate windows on 20 kb reads (the certificate's second plan);
  * an end-trim cross product (the tiled cross ABI) vs the oracle.

A kernel or host path that reads scratch it never wrote (r05: the plans' `need2`) sees garbage
here. Exit status 0 when every case matches; one line per case on stdout."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (one HIP runtime per process, custom_porechop_abi_amd/_lib.py)

from custom_porechop_abi_amd import _lib, engine  # noqa: E402
from tests import oracle_lib  # noqa: E402
from tests.test_gpu_middle_paths import ADPS, SC, _dev_scan, _reads, _requeues, _sorted  # noqa: E402


def case(name, ok):
    print('%-60s %s' % (name, 'ok' if ok else 'MISMATCH'), flush=True)
    if not ok:
        sys.exit(1)


def setenv(**kw):
    for k in ('PCABI_MIDDLE_INIT_CAPS', 'PCABI_MIDDLE_FAULT', 'PCABI_MIDDLE_WINDOWS', 'PCABI_MIDDLE_DEVROUNDS'):
        os.environ.pop(k, None)
    os.environ.update({k: v for k, v in kw.items()})


def main():
    assert os.environ.get('PCABI_POISON', '0') != '0', 'run with PCABI_POISON=1 (0xFF) or a hex byte'
    L = _lib.lib()
    assert L.pcabi_device_count() >= 1
    os.environ['PCABI_MIDDLE_SEEDS'] = '2'
    reads = _reads(7, 160, 8000, 90.0)
    pack = engine.SeqPack(reads)
    views = pack.views(np.zeros(len(reads), np.int64), pack.lengths)
    exp = _sorted(oracle_lib.middle_scan_threaded(views, ADPS, SC, 90.0))

    for caps in ('256,64,128', '256,0,0', '0,0,128'):
        setenv(PCABI_MIDDLE_INIT_CAPS=caps)
        n0, _ = _requeues(L)
        got = _dev_scan(L, views, ADPS, SC, 90.0)
        n1, _ = _requeues(L)
        case('round-1 growth from caps %s (requeues %d)' % (caps, n1 - n0), n1 > n0 and np.array_equal(_sorted(got), exp))

    for windows in ('0', '1'):
        for fault in ('0:7,1:4,2:2', '1:4', '0:8', '2:15'):
            setenv(PCABI_MIDDLE_FAULT=fault, PCABI_MIDDLE_WINDOWS=windows)
            n0, _ = _requeues(L)
            got = engine.middle_scan(views, ADPS, SC, 90.0)
            n1, _ = _requeues(L)
            case('fault %s, windows %s (requeues %d)' % (fault, windows, n1 - n0),
                 n1 - n0 >= len(fault.split(',')) and np.array_equal(_sorted(got), exp))

    for devrounds in ('1', '0'):
        setenv(PCABI_MIDDLE_INIT_CAPS='0,0,0,4096', PCABI_MIDDLE_DEVROUNDS=devrounds)
        intact = []
        got = _dev_scan(L, views, ADPS, SC, 90.0, calls=3, intact=intact, stream=devrounds == '1')
        case('growing shadow arena, devrounds %s, 3 calls, pack intact' % devrounds,
             intact == [True, True, True] and np.array_equal(_sorted(got), exp))

    setenv(PCABI_MIDDLE_WINDOWS='1')
    r20 = _reads(21090, 60, 20000, 90.0)
    p20 = engine.SeqPack(r20)
    v20 = p20.views(np.zeros(len(r20), np.int64), p20.lengths)
    e20 = _sorted(oracle_lib.middle_scan_threaded(v20, ADPS, SC, 90.0))
    got = engine.middle_scan(v20, ADPS, SC, 90.0)
    case('candidate windows on 20 kb reads', e20.shape[1] > 30 and np.array_equal(_sorted(got), e20))

    setenv()
    rng = np.random.default_rng(5)
    wins = [''.join(rng.choice(list('ACGT'), size=int(rng.integers(0, 151)))) for _ in range(700)]
    wins[3] = ADPS[0][4:] + wins[3][:120]
    wp = engine.SeqPack(wins)
    wv = wp.views(np.zeros(len(wins), np.int64), wp.lengths)
    adps = ADPS + ['ACGTTGCAACGTACGATCGATCGA', 'GGCATTACGGATCGATTTACG']
    got = engine.align(wv, adps, SC)
    want = oracle_lib.align_windows(wv, adps, SC)
    ok = want[0] != -1          # empty window: only field 0 is defined by the reference
    case('end-trim cross product (%d windows x %d adapters)' % (len(wins), len(adps)),
         np.array_equal(got[0], want[0]) and np.array_equal(got[:, ok], want[:, ok]) and (~ok).sum() > 0)
    print('all cases ok', flush=True)


if __name__ == '__main__':
    main()
