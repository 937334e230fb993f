#!/bin/bash
# Second batched-GEMM sweep: waves per workgroup (W), LDS chunk depth (CK) and k-split caps.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/bgemm_sweep2.jsonl
: > $out
run() {  # env assignments...
  env "$@" timeout -k 10 300 python tools/bench_kernels.py --norm --rows ${ROWS:-32,64} --gemm-only \
    --roles ${ROLES:-qkv,o,gateup,down} | sed "s/}\$/, \"env\": \"$*\"}/" >> $out
}
run CAIN_BGEMM_W=8 || exit 1
for ksm in 4 8 16; do
  run CAIN_BGEMM_W=4 CAIN_BGEMM_KSMAX=$ksm || exit 1
  run CAIN_BGEMM_CK=16 CAIN_BGEMM_KSMAX=$ksm || exit 1
  run CAIN_BGEMM_KSMAX=$ksm CAIN_BGEMM_WG=512 || exit 1
done
echo done
