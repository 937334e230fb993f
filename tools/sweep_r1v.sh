#!/bin/bash
# Batched GEMM at 256 rows: 16-wave workgroups (8 columns x 2 rows, 4 waves per SIMD) vs the 8-wave body.
set -o pipefail
mkdir -p gpurun_out/r1v
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
CAIN_BGEMM_WM=3 timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -x -q -k "batched or qkv" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r1v/pytest_wm3.log 2>&1
rc=$?; tail -1 gpurun_out/r1v/pytest_wm3.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -x -q -k "batched or qkv" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r1v/pytest_wm1.log 2>&1
rc=$?; tail -1 gpurun_out/r1v/pytest_wm1.log; [ $rc -ne 0 ] && exit $rc
for wm in 1 3; do
  CAIN_BGEMM_WM=$wm timeout -k 10 240 python tools/bench_kernels.py --rows 256 --roles qkv,o,gateup,down,lm_head --gemm-only --norm --waves 0 > gpurun_out/r1v/wm$wm.jsonl 2>&1 || exit 1
  echo "wm=$wm"; python3 -c "
import json
for l in open('gpurun_out/r1v/wm$wm.jsonl'):
    if l.startswith('{'):
        r=json.loads(l); print('  ',r['role'],r['M'],r['us'],r['TBps'])
"
done
for wm in 1 3; do
  CAIN_BGEMM_WM=$wm timeout -k 10 400 python bench.py --steps 1 --warmup 1 > gpurun_out/r1v/bench_wm$wm.log 2>&1 || exit 1
  echo "bench wm=$wm $(tail -1 gpurun_out/r1v/bench_wm$wm.log | cut -c60-130)"
done
