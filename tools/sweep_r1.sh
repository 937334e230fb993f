#!/bin/bash
# Attention split sweep (fragment-major KV cache) and 128-row GEMM register-ring depth sweep.
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
out=gpurun_out/sweep_r1.jsonl
: > $out
timeout -k 10 300 python tools/bench_kernels.py --attn-only --attn "64:700,128:350,128:700,128:1400,1:1400" \
  --attn-splits auto,1,2,3,4,6,8 >> $out || exit $?
run() {
  env "$@" timeout -k 10 300 python tools/bench_kernels.py --norm --rows ${ROWS:-128} --gemm-only \
    --roles ${ROLES:-qkv,o,gateup,down,lm_head} | sed "s/}\$/, \"env\": \"$*\"}/" >> $out
}
run CAIN_BGEMM_D=0 || exit 1
run CAIN_BGEMM_D=4 || exit 1
run CAIN_BGEMM_D=8 || exit 1
run CAIN_BGEMM_D=8 CAIN_BGEMM_W=8 || exit 1
run CAIN_BGEMM_D=4 CAIN_BGEMM_W=8 || exit 1
echo done
