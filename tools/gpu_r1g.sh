#!/bin/bash
# Default 4-deep rings on the narrow 128-row bodies: tests, bench, rocprofv3 kernel stats of one bench step.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py tests/test_engine_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r1g.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r1g.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_r1g.log 2>&1
rc=$?; tail -1 gpurun_out/bench_r1g.log; [ $rc -ne 0 ] && exit $rc
OUT=prof_r1g ARGS="--steps 1 --warmup 0" bash tools/profile.sh
