#!/bin/bash
# GPU-box script (r04): the new middle-path and verbose-output GPU tests, then the reference_job
# sub-record of the bench and a kernel-stats profile of it; each step time-limited, stop at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_middle_paths.py::test_seed_scan_bytemap_equals_bitmap_scan tests/test_gpu_middle_paths.py::test_barcode_call_96_sets_random_scores tests/test_gpu_middle_paths.py::test_barcode_call_96_sets_on_barcoded_reads tests/test_gpu_middle_paths.py::test_candidate_windows_at_the_certificate_bound tests/test_verbose_output.py 'tests/test_gpu_parity.py::test_row_split_cross_product' > $OUT/t_mid.log 2>&1 || { echo "pytest failed rc=$?"; tail -30 $OUT/t_mid.log; exit 1; }
tail -2 $OUT/t_mid.log
timeout -k 10 300 python bench.py --only-subs reference_job --steps 6 --warmup 2 --cpu-sample 0 > $OUT/refjob.json 2> $OUT/refjob.err || { echo "bench failed rc=$?"; tail -20 $OUT/refjob.err; exit 1; }
python -c "import json; d0=json.load(open('$OUT/refjob.json')); print(json.dumps({k: d0.get(k) for k in ('value','ms_per_step','roofline')})); d=d0['reference_job']; print(json.dumps({k: d.get(k) for k in ('value','ms_per_step','ms_per_phase','kept_sets','kept_adapters','end_trim_gcups','roofline','parity_spot_check','error')}))"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_rj -o run -- python3 $R/bench.py --only-subs reference_job --steps 3 --warmup 1 --cpu-sample 0 --check 0 > $OUT/prof_rj.json 2> $OUT/prof_rj.err || { echo "rocprof failed rc=$?"; tail -20 $OUT/prof_rj.err; exit 1; }
head -30 $OUT/prof_rj/run_kernel_stats.csv | cut -d, -f1-5
cd $R
timeout -k 10 300 python bench.py --workload middle --steps 5 --warmup 2 --cpu-sample 0 > $OUT/mid8.json 2> $OUT/mid8.err || { echo "mid8 failed rc=$?"; tail -20 $OUT/mid8.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/mid8.json')); print(json.dumps({k: d.get(k) for k in ('value','ms_per_step','middle_ms_per_step','middle_phases','parity_spot_check')}))"
PCABI_SEED_BYTEMAP=0 timeout -k 10 300 python bench.py --workload middle --steps 5 --warmup 2 --cpu-sample 0 > $OUT/mid8_bits.json 2> $OUT/mid8_bits.err || { echo "mid8 bits failed rc=$?"; tail -20 $OUT/mid8_bits.err; exit 1; }
python -c "import json; d=json.load(open('$OUT/mid8_bits.json')); print('bitmap scan', json.dumps({k: d.get(k) for k in ('value','ms_per_step','middle_ms_per_step','middle_phases')}))"
