#!/bin/bash
# Batched GEMM at 128/256 rows: workgroup target (k-split count) sweep.
set -o pipefail
mkdir -p gpurun_out/r1r
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
for cfg in "0 8" "256 8" "512 8" "512 16" "1024 16"; do
  set -- $cfg
  CAIN_BGEMM_WG=$1 CAIN_BGEMM_KSMAX=$2 timeout -k 10 240 python tools/bench_kernels.py --rows 128,256 --roles qkv,o,gateup,down,lm_head --gemm-only --norm --waves 0 > gpurun_out/r1r/wg$1_ks$2.jsonl 2>&1 || exit 1
  echo "wg=$1 ksmax=$2"; python3 -c "
import json,sys
for l in open('gpurun_out/r1r/wg$1_ks$2.jsonl'):
    if l.startswith('{'):
        r=json.loads(l); print('  ',r.get('role'),r.get('M'),r.get('us'),r.get('TBps'))
"
done
