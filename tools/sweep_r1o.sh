#!/bin/bash
# fp8-weight (W8A16) decode: kernel + engine tests, bf16 regression tests (shared epilogue header),
# single-stream kernel durations under rocprofv3, bf16 vs fp8 bench lines at batch 1 and 64.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_w8_gpu.py tests/test_ops_gpu.py tests/test_engine_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r1o.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_r1o.log; [ $rc -ne 0 ] && exit $rc
for m in qwen2:1.5b llama3.1:8b; do
  name=qs_w8_${m%%:*}
  mkdir -p gpurun_out/$name
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$name -o run -- python3 bench.py --no-energy --weights fp8 --batch 1 --model $m --words 1000 --steps 1 --warmup 0 > gpurun_out/$name/bench.log 2>&1 || exit 1
  find gpurun_out/$name -name "*kernel_trace.csv" -delete
  cut -c1-60,150-260 gpurun_out/$name/run_kernel_stats.csv | head -12
done
for m in qwen2:1.5b llama3.1:8b gemma:2b; do
  for w in fp8 bf16; do
    timeout -k 10 300 python bench.py --weights $w --batch 1 --model $m --words 1000 --steps 1 --warmup 1 > gpurun_out/bench_r1o_${m}_${w}_b1.log 2>&1 || exit 1
    echo "$m $w b1: $(tail -1 gpurun_out/bench_r1o_${m}_${w}_b1.log | cut -c1-100)"
  done
done
for w in fp8 bf16; do
  timeout -k 10 300 python bench.py --weights $w --batch 64 --model llama3.1:8b --words 1000 --steps 1 --warmup 1 > gpurun_out/bench_r1o_llama_${w}_b64.log 2>&1 || exit 1
  echo "llama $w b64: $(tail -1 gpurun_out/bench_r1o_llama_${w}_b64.log | cut -c1-100)"
done
