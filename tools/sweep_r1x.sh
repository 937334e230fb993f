#!/bin/bash
# hipBLASLt wide-batch path (blas.hip): numerics tests, then bench at 256 trials/GPU with the path on vs off.
set -o pipefail
mkdir -p gpurun_out/r1x
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_lt_gpu.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r1x/pytest_lt.log 2>&1
rc=$?; tail -3 gpurun_out/r1x/pytest_lt.log; [ $rc -ne 0 ] && exit $rc
for lt in 128 0; do
  CAIN_LT_MIN_ROWS=$lt timeout -k 10 400 python bench.py --steps 1 --warmup 1 > gpurun_out/r1x/bench_lt$lt.log 2>&1 || exit 1
  echo "bench lt=$lt $(tail -1 gpurun_out/r1x/bench_lt$lt.log | cut -c1-260)"
done
