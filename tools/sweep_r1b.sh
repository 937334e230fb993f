#!/bin/bash
# 128-row GEMM: activation + weight register rings (CAIN_BGEMM_D) vs the default pipeline.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
out=gpurun_out/sweep_r1b.jsonl
: > $out
run() {
  env "$@" timeout -k 10 300 python tools/bench_kernels.py --norm --rows ${ROWS:-128} --gemm-only \
    --roles ${ROLES:-qkv,o,gateup,down,lm_head} | sed "s/}\$/, \"env\": \"$*\"}/" >> $out
}
run CAIN_BGEMM_D=0 || exit 1
run CAIN_BGEMM_D=4 || exit 1
run CAIN_BGEMM_D=6 || exit 1
run CAIN_BGEMM_D=8 || exit 1
run CAIN_BGEMM_D=4 CAIN_BGEMM_W=8 || exit 1
run CAIN_BGEMM_D=4 CAIN_BGEMM_W=4 || exit 1
run CAIN_BGEMM_D=8 CAIN_BGEMM_W=4 || exit 1
echo done
