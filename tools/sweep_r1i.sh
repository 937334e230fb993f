#!/bin/bash
# 256 rows: 8 waves x 1 tile vs 4 waves x 2 tiles, without the fused norm (its staging sums spill the latter).
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/sweep_r1i.jsonl
: > $out
run() {
  env "$@" timeout -k 10 300 python tools/bench_kernels.py --rows ${ROWS:-256} --gemm-only \
    --roles ${ROLES:-qkv,o,gateup,down,lm_head} | sed "s/}\$/, \"env\": \"$*\"}/" >> $out
}
run CAIN_BGEMM_NTW=0 || exit 1
run CAIN_BGEMM_NTW=2 || exit 1
ROWS=128 run CAIN_BGEMM_NTW=0 || exit 1
ROWS=128 run CAIN_BGEMM_D=4 || exit 1
echo done
