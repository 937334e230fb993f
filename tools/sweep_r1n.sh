#!/bin/bash
# 8-wave attention workgroups for few (row, kv head) pairs: tests, single-stream kernel durations, benches.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py tests/test_engine_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r1n.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r1n.log; [ $rc -ne 0 ] && exit $rc
for m in qwen2:1.5b llama3.1:8b; do
  name=qs_aw8_${m%%:*}
  mkdir -p gpurun_out/$name
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$name -o run -- python3 bench.py --no-energy --batch 1 --model $m --words 1000 --steps 1 --warmup 0 > gpurun_out/$name/bench.log 2>&1 || exit 1
  find gpurun_out/$name -name "*kernel_trace.csv" -delete
  grep attn_decode gpurun_out/$name/run_kernel_stats.csv | cut -c1-40,150-260
done
for m in qwen2:1.5b llama3.1:8b gemma:2b; do
  timeout -k 10 300 python bench.py --batch 1 --model $m --words 1000 --steps 1 --warmup 1 > gpurun_out/bench_r1n_$m.log 2>&1 || exit 1
  tail -1 gpurun_out/bench_r1n_$m.log | cut -c1-120
done
