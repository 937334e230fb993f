#!/bin/bash
# Round-1 GPU pass A: kernel + engine tests after the KV layout change, kernel sweeps, two benches.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py tests/test_engine_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r1a.log 2>&1
rc=$?; tail -5 gpurun_out/pytest_r1a.log; [ $rc -ne 0 ] && exit $rc
bash tools/sweep_r1.sh > gpurun_out/sweep_r1.log 2>&1
rc=$?; tail -3 gpurun_out/sweep_r1.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_r1a_default.log 2>&1
rc=$?; tail -1 gpurun_out/bench_r1a_default.log; [ $rc -ne 0 ] && exit $rc
CAIN_BGEMM_D=4 CAIN_ATTN_SPLIT_BLOCKS=16 timeout -k 10 300 python bench.py > gpurun_out/bench_r1a_d4s16.log 2>&1
rc=$?; tail -1 gpurun_out/bench_r1a_d4s16.log; exit $rc
