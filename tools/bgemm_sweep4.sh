#!/bin/bash
# After the copy-free ping-pong weight pipeline: chunk depth / waves per shape at M = 32, 64, 128.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/bgemm_sweep4.jsonl
: > $out
run() {
  env "$@" timeout -k 10 300 python tools/bench_kernels.py --norm --rows ${ROWS:-32,64,128} --gemm-only \
    --roles ${ROLES:-qkv,o,gateup,down,lm_head} | sed "s/}\$/, \"env\": \"$*\"}/" >> $out
}
run CAIN_BGEMM_CK=0 || exit 1
run CAIN_BGEMM_CK=4 || exit 1
run CAIN_BGEMM_CK=8 || exit 1
run CAIN_BGEMM_W=8 || exit 1
run CAIN_BGEMM_W=4 || exit 1
echo done
