#!/bin/bash
# 256-row decode: tests, 256-row GEMM microbench, bench at 128 and 256 trials per GPU.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py tests/test_engine_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r1h.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r1h.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/bench_kernels.py --norm --rows 256 --gemm-only > gpurun_out/gemm256_r1h.jsonl || exit 1
timeout -k 10 300 python tools/bench_kernels.py --attn-only --attn "256:700,256:1400" --attn-splits auto >> gpurun_out/gemm256_r1h.jsonl || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench_r1h_128.log 2>&1
rc=$?; tail -1 gpurun_out/bench_r1h_128.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --batch 256 > gpurun_out/bench_r1h_256.log 2>&1
rc=$?; tail -1 gpurun_out/bench_r1h_256.log; exit $rc
