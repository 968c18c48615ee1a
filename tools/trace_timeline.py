"""Print the kernel timeline of the last bench step from a rocprofv3 --kernel-trace CSV.

usage: python tools/trace_timeline.py gpurun_out/trace_mid/run_kernel_trace.csv [marker]
The timeline starts `back` dispatches (default 8) before the last dispatch of `marker` (default
k_end_trim, once per step), so it covers the step's end-trim launches and everything after.
"""
import csv
import sys


def main():
    path = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else 'k_end_trim'
    back = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    idx = [i for i, r in enumerate(rows) if marker in r['Kernel_Name']]
    first = max(idx[-1] - back, 0) if idx else 0
    t0 = int(rows[first]['Start_Timestamp'])
    for r in rows[first:]:
        name = r['Kernel_Name'].replace('(anonymous namespace)::', '')
        name = name.split('(')[0] if not name.startswith('void ') else name[5:].split('(')[0]
        s = (int(r['Start_Timestamp']) - t0) / 1e6
        e = (int(r['End_Timestamp']) - t0) / 1e6
        print('%9.3f %9.3f %8.3f  q%-3s grid %-9s %s' % (s, e, e - s, r['Queue_Id'], r['Grid_Size_X'], name[:60]))


if __name__ == '__main__':
    main()
