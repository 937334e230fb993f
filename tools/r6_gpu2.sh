#!/usr/bin/env bash
# round 6: Q4 kernel after the staging change: numerics, per-shape in-graph us (fp4 / q4_0 / q4_k), batch-1 rates
set -o pipefail
mkdir -p gpurun_out/r6q
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_q4_gpu.py > gpurun_out/r6q/q4_tests.log 2>&1 || { tail -30 gpurun_out/r6q/q4_tests.log; exit 1; }
tail -2 gpurun_out/r6q/q4_tests.log
timeout -k 10 300 python tools/w4_bench.py --dtypes fp4,q4_0,q4_k --variants rule > gpurun_out/r6q/w4_bench_llama.jsonl || exit 1
cat gpurun_out/r6q/w4_bench_llama.jsonl
timeout -k 10 300 python tools/b1_ab.py --models llama3.1:8b,qwen2:1.5b,gemma:2b --dtype fp4,q4_k,q4_0 --label q4b --out gpurun_out/r6q/b1_q4.jsonl
