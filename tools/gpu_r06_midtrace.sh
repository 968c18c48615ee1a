#!/bin/bash
# r06: kernel trace of the middle bench (8 kb and 20 kb) and the last step's timeline from the end
# trim on (tools/trace_busy.py): where the middle scan's wall time goes beyond its kernels
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${TAG:-r06midtrace}
mkdir -p $OUT
export TMPDIR=/tmp
for L in 8000 20000; do
  cd /tmp
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/t$L -o run -- python3 $R/bench.py --workload middle --mean-len $L --steps 3 --warmup 2 --cpu-sample 0 --check 0 > $OUT/t$L.log 2>&1 || { echo "trace $L failed rc=$?"; tail -5 $OUT/t$L.log; exit 1; }
  cd $R
  f=$(ls $OUT/t$L/*kernel_trace.csv $OUT/t$L/*/*kernel_trace.csv 2>/dev/null | head -1)
  python tools/trace_busy.py $f k_end_trim --all > $OUT/timeline_$L.txt
  tail -30 $OUT/timeline_$L.txt
done
