"""Summarise rocprofv3 --pmc passes (tools/gpu_pmc.sh output) per kernel: counters summed over
the kernel's dispatches, divided by the dispatch count (per-launch values).

    python tools/pmc_report.py [gpurun_out/pmc] [kernel-substring ...]

Derived lines: VALU issue utilisation, HBM bytes per launch with the gfx950 FETCH_SIZE x2
correction (MI355X_MICROARCH.md, HBM/rocprofv3 section)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(d):
    per = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for f in sorted(glob.glob(os.path.join(d, 'p*', 'run_counter_collection.csv'))):
        for r in csv.DictReader(open(f)):
            k = r['Kernel_Name']
            per[k][r['Counter_Name']] += float(r['Counter_Value'])
            disp[(k, r['Counter_Name'])].add((f, r['Dispatch_Id']))
    out = {}
    for k, cs in per.items():
        out[k] = {c: v / max(1, len(disp[(k, c)])) for c, v in cs.items()}
    return out


def main():
    d = sys.argv[1] if len(sys.argv) > 1 and os.path.isdir(sys.argv[1]) else 'gpurun_out/pmc'
    subs = [a for a in sys.argv[1:] if not os.path.isdir(a)] or ['k_align']
    res = load(d)
    report = {}
    for k, cs in sorted(res.items(), key=lambda kv: -kv[1].get('SQ_BUSY_CYCLES', 0)):
        if not any(s in k for s in subs):
            continue
        name = k.replace('void (anonymous namespace)::', '').split('(')[0]
        print('==', name)
        for c in sorted(cs):
            print('   %-24s %16.1f' % (c, cs[c]))
        der = {}
        if 'SQ_ACTIVE_INST_VALU' in cs and 'SQ_BUSY_CYCLES' in cs and cs['SQ_BUSY_CYCLES']:
            # SQ counters are per SE-summed; report ratios only
            der['valu_active_per_busy_cycle'] = cs['SQ_ACTIVE_INST_VALU'] / cs['SQ_BUSY_CYCLES']
        if 'SQ_WAIT_INST_ANY' in cs and 'SQ_WAVE_CYCLES' in cs and cs['SQ_WAVE_CYCLES']:
            der['wait_inst_frac'] = cs['SQ_WAIT_INST_ANY'] / cs['SQ_WAVE_CYCLES']
            der['wait_any_frac'] = cs.get('SQ_WAIT_ANY', 0) / cs['SQ_WAVE_CYCLES']
            der['active_inst_frac'] = cs.get('SQ_ACTIVE_INST_ANY', 0) / cs['SQ_WAVE_CYCLES']
        if 'FETCH_SIZE' in cs:
            der['hbm_read_bytes_corrected'] = cs['FETCH_SIZE'] * 1024 * 2
        if 'WRITE_SIZE' in cs:
            der['hbm_write_bytes'] = cs['WRITE_SIZE'] * 1024
        if 'TCC_EA0_RDREQ_sum' in cs:
            der['ea_rdreq_x64B'] = cs['TCC_EA0_RDREQ_sum'] * 64
        for c, v in der.items():
            print('   > %-22s %16.4f' % (c, v))
        report[name] = {'counters': cs, 'derived': der}
    if '--json' in sys.argv:
        print(json.dumps(report))


if __name__ == '__main__':
    main()
