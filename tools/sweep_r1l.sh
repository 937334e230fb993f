#!/bin/bash
# Skinny GEMM: every slice up front for short k-ranges. Tests, 1-row sweep (new vs pipelined), batch-1 benches.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py tests/test_engine_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r1l.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r1l.log; [ $rc -ne 0 ] && exit $rc
out=gpurun_out/sweep_r1l.jsonl
: > $out
for m in qwen2:1.5b llama3.1:8b gemma:2b; do
  timeout -k 10 300 python tools/bench_kernels.py --model $m --norm --rows 1,8 --gemm-only --waves 0 | sed "s/}\$/, \"env\": \"default\"}/" >> $out || exit 1
  CAIN_SKINNY_PP=0 timeout -k 10 300 python tools/bench_kernels.py --model $m --norm --rows 1,8 --gemm-only --waves 0 | sed "s/}\$/, \"env\": \"PP0\"}/" >> $out || exit 1
done
for m in qwen2:1.5b llama3.1:8b; do
  timeout -k 10 300 python bench.py --batch 1 --model $m --words 500 --steps 2 --warmup 1 > gpurun_out/bench_r1l_$m.log 2>&1 || exit 1
  tail -1 gpurun_out/bench_r1l_$m.log | cut -c1-130
done
