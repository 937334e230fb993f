#!/bin/bash
# Full-line activation staging: correctness, 32/64/128-row sweep, bench.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py tests/test_engine_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r1d.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r1d.log; [ $rc -ne 0 ] && exit $rc
out=gpurun_out/sweep_r1d.jsonl
: > $out
timeout -k 10 300 python tools/bench_kernels.py --norm --rows 32,64,128 --gemm-only >> $out || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench_r1d.log 2>&1
rc=$?; tail -1 gpurun_out/bench_r1d.log; exit $rc
