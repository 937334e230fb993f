#!/bin/bash
# 128-row batched GEMM variants (LDS chunk depth, waves per workgroup, k-split target).
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/bgemm_sweep3.jsonl
: > $out
run() {
  env "$@" timeout -k 10 300 python tools/bench_kernels.py --norm --rows ${ROWS:-128} --gemm-only \
    --roles ${ROLES:-qkv,o,gateup,down,lm_head} | sed "s/}\$/, \"env\": \"$*\"}/" >> $out
}
run CAIN_BGEMM_CK=4 || exit 1
run CAIN_BGEMM_CK=8 || exit 1
run CAIN_BGEMM_CK=8 CAIN_BGEMM_W=8 || exit 1
run CAIN_BGEMM_CK=4 CAIN_BGEMM_WG=256 || exit 1
run CAIN_BGEMM_CK=8 CAIN_BGEMM_WG=512 || exit 1
echo done
