"""Timeline of one bench phase from a rocprofv3 kernel trace (run_kernel_trace.csv): per step, the
kernels between a start marker and the next step's first kernel -- busy time (union of the
kernels' intervals over all streams), wall span, idle gaps, and per-kernel totals. Host-side
analysis only (no GPU).

    python tools/trace_timeline.py gpurun_out/prof_mid8000 [--after k_end_trim] [--until k_tile_windows]
"""
import argparse
import collections
import csv
import glob
import os
import re


def load(path):
    files = glob.glob(os.path.join(path, '**', '*kernel_trace.csv'), recursive=True) if os.path.isdir(path) else [path]
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name']))
    rows.sort()
    return rows


def short(name):
    name = re.sub(r'\(.*', '', name)
    name = re.sub(r'^void ', '', name)
    name = re.sub(r'pcabi_eng::\(anonymous namespace\)::|pcabi_seed::\(anonymous namespace\)::|pcabi_eng::|pcabi_seed::', '', name)
    return name[:70]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('path')
    ap.add_argument('--after', default='k_end_trim')
    ap.add_argument('--until', default='k_tile_windows')
    ap.add_argument('--gap-us', type=float, default=15.0)
    a = ap.parse_args()
    rows = load(a.path)
    steps = []
    cur = None
    for s, e, n in rows:
        if a.after in n:
            if cur:
                steps.append(cur)
            cur = []
            continue
        if cur is not None:
            if a.until in n:
                steps.append(cur)
                cur = None
            else:
                cur.append((s, e, n))
    if cur:
        steps.append(cur)
    steps = [st for st in steps if st]
    print('%d phases' % len(steps))
    tot = collections.Counter()
    cnt = collections.Counter()
    for i, st in enumerate(steps):
        t0 = st[0][0]
        t1 = max(e for _, e, _ in st)
        busy = 0
        hi = t0
        gaps = []
        for s, e, n in st:
            if s > hi:
                if (s - hi) / 1e3 >= a.gap_us:
                    gaps.append(((hi - t0) / 1e3, (s - hi) / 1e3, short(n)))
                busy += e - s
            else:
                busy += max(0, e - hi)
            hi = max(hi, e)
            tot[short(n)] += e - s
            cnt[short(n)] += 1
        print('phase %d: %d kernels, wall %.1f us, busy %.1f us, %d gaps >= %.0f us (%.1f us)'
              % (i, len(st), (t1 - t0) / 1e3, busy / 1e3, len(gaps), a.gap_us, sum(g[1] for g in gaps)))
        if i == len(steps) - 1:
            for at, g, n in gaps[:40]:
                print('   gap at +%8.1f us: %7.1f us before %s' % (at, g, n))
    ns = max(1, len(steps))
    print('per phase, by kernel (us, launches):')
    for n, t in tot.most_common(40):
        print('  %9.1f  %6.1f  %s' % (t / 1e3 / ns, cnt[n] / ns, n))


if __name__ == '__main__':
    main()
