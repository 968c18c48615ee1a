"""Timeline of the last step in a rocprofv3 kernel trace: every kernel from the last occurrence of
START (a kernel-name substring, default k_end_trim) to the end of the trace, with its queue, start,
duration, and the device's idle gaps (no kernel running on any queue) between them -- where a
step's wall time goes beyond its kernels (launch latency, fork / join events, host round trips).

    python tools/trace_busy.py run_kernel_trace.csv [START] [--all] [--prev]

--prev: the step before the last (from the second-to-last START to the last one) -- the last step of
a bench run with a per-phase profile step after the timed ones is that profile step."""
import csv
import sys


def main():
    path = sys.argv[1]
    start_pat = sys.argv[2] if len(sys.argv) > 2 and not sys.argv[2].startswith('--') else 'k_end_trim'
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    idx = [i for i, r in enumerate(rows) if start_pat in r['Kernel_Name']]
    if not idx:
        print('no kernel matching', start_pat)
        return
    if '--prev' in sys.argv and len(idx) > 1:
        sel = rows[idx[-2]:idx[-1]]
    else:
        sel = rows[idx[-1]:]
    t0 = int(sel[0]['Start_Timestamp'])
    busy_end = t0
    idle = 0
    by_name = {}
    for r in sel:
        s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
        gap = max(0, s - busy_end)
        idle += gap
        busy_end = max(busy_end, e)
        name = r['Kernel_Name'].split('(')[0].replace('void ', '')[:60]
        by_name[name] = by_name.get(name, 0) + (e - s)
        if '--all' in sys.argv:
            print('%9.1f %8.1f %6.1f q%s %s' % ((s - t0) / 1e3, (e - s) / 1e3, gap / 1e3, r['Queue_Id'], name))
    span = busy_end - t0
    print('span %.1f us, idle (no kernel on any queue) %.1f us, kernels %d' % (span / 1e3, idle / 1e3, len(sel)))
    for k, v in sorted(by_name.items(), key=lambda x: -x[1])[:25]:
        print('  %8.1f us  %s' % (v / 1e3, k))


if __name__ == '__main__':
    main()
