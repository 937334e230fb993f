#!/bin/bash
# Batched GEMM wave grid: WM = 2 wave rows x 2 tiles (half the LDS fragment reads) vs WM = 1, at 128 / 256 rows;
# 256-row fused-norm bodies with 2-slice weight groups (no spills).
set -o pipefail
mkdir -p gpurun_out/r1s
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
CAIN_BGEMM_WM=2 timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -x -q -k "batched or qkv" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r1s/pytest_wm2.log 2>&1
rc=$?; tail -1 gpurun_out/r1s/pytest_wm2.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -x -q -k "batched or qkv" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r1s/pytest_wm1.log 2>&1
rc=$?; tail -1 gpurun_out/r1s/pytest_wm1.log; [ $rc -ne 0 ] && exit $rc
for wm in 1 2; do
  CAIN_BGEMM_WM=$wm timeout -k 10 240 python tools/bench_kernels.py --rows 128,256 --roles qkv,o,gateup,down,lm_head --gemm-only --norm --waves 0 > gpurun_out/r1s/wm$wm.jsonl 2>&1 || exit 1
  echo "wm=$wm"; python3 -c "
import json
for l in open('gpurun_out/r1s/wm$wm.jsonl'):
    if l.startswith('{'):
        r=json.loads(l); print('  ',r['role'],r['M'],r['us'],r['TBps'])
"
done
for wm in 1 2; do
  CAIN_BGEMM_WM=$wm timeout -k 10 400 python bench.py --steps 1 --warmup 1 > gpurun_out/r1s/bench_wm$wm.log 2>&1 || exit 1
  echo "bench wm=$wm $(tail -1 gpurun_out/r1s/bench_wm$wm.log | cut -c60-130)"
done
