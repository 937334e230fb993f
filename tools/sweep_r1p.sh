#!/bin/bash
# fp8-weight GEMM variants: waves x pairs-in-flight at 1 row, 1 vs 2 row blocks per workgroup at 64 rows.
set -o pipefail
mkdir -p gpurun_out/r1p
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_w8_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_r1p.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_r1p.log; [ $rc -ne 0 ] && exit $rc
run() {  # name batch model
  local name=$1 b=$2 m=$3
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r1p/$name -o run -- python3 bench.py --no-energy --weights fp8 --batch $b --model $m --words 300 --steps 1 --warmup 0 > gpurun_out/r1p/$name.log 2>&1 || exit 1
  find gpurun_out/r1p/$name -name "*kernel_trace.csv" -delete
  echo "$name $(tail -1 gpurun_out/r1p/$name.log | cut -c70-100)"
}
for m in llama3.1:8b qwen2:1.5b; do
  for w in 4 8; do for u in 2 4; do
    CAIN_W8_WAVES=$w CAIN_W8_U=$u run b1_${m%%:*}_w${w}_u${u} 1 $m
  done; done
  run b1_${m%%:*}_auto 1 $m
done
for nb in 1 2; do
  CAIN_W8_NB=$nb run b64_llama_nb$nb 64 llama3.1:8b
  CAIN_W8_NB=$nb run b32_llama_nb$nb 32 llama3.1:8b
done
