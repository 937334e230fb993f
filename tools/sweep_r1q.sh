#!/bin/bash
# fp8-weight GEMM: 1/2/4 16-row tiles of N per workgroup (activation fragments shared across tiles) at 1 row.
set -o pipefail
mkdir -p gpurun_out/r1q
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
run() {  # name batch model
  local name=$1 b=$2 m=$3
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r1q/$name -o run -- python3 bench.py --no-energy --weights fp8 --batch $b --model $m --words 300 --steps 1 --warmup 0 > gpurun_out/r1q/$name.log 2>&1 || exit 1
  find gpurun_out/r1q/$name -name "*kernel_trace.csv" -delete
}
for nt in 2 4; do
  CAIN_W8_NT=$nt CAIN_W8_NB=1 timeout -k 10 300 python -u -m pytest tests/test_w8_gpu.py -x -q -k "not engine" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r1q/pytest_nt$nt.log 2>&1
  rc=$?; tail -1 gpurun_out/r1q/pytest_nt$nt.log; [ $rc -ne 0 ] && exit $rc
done
for m in llama3.1:8b qwen2:1.5b; do
  for nt in 1 2 4; do
    CAIN_W8_NT=$nt run b1_${m%%:*}_nt${nt} 1 $m
    CAIN_W8_NT=$nt CAIN_W8_WAVES=4 run b1_${m%%:*}_nt${nt}_w4 1 $m
  done
done
