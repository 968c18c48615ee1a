"""One-screen summary of a bench.py JSON line: the headline, its roofline, and each sub-record's
step time, phases and parity check (tools/gpu_r06_record.sh)."""
import json
import sys

d = json.load(open(sys.argv[1]))
print(json.dumps({k: d.get(k) for k in ('value', 'ms_per_step', 'roofline')}))
for k in ('per_side_schedule', 'host_path', 'reference_job', 'middle', 'middle_20kb', 'barcodes', 'config2_10k_119sets',
          'drivers', 'check_phase', 'e2e', 'compat', 'kmer'):
    v = d.get(k) or {}
    print(k, json.dumps({x: v.get(x) for x in ('value', 'ms_per_step', 'middle_ms_per_step', 'ms_per_phase', 'error',
                                               'parity_spot_check', 'step_vs_slowest_stage')})[:900])
