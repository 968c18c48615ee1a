set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_long.py > gpurun_out/pytest_long.log 2>&1; rc=$?
tail -25 gpurun_out/pytest_long.log
exit $rc
