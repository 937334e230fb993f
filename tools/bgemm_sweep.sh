#!/bin/bash
# Sweep the batched-GEMM launch heuristics (env-tunable) on the flagship decode shapes.
# Usage: ROWS=32,64 bash tools/bgemm_sweep.sh   -> gpurun_out/bgemm_sweep.jsonl
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/bgemm_sweep.jsonl
: > $out
for ntw in ${NTWS:-1 2}; do
  for wg in ${WGS:-128 256 512}; do
    for ksm in ${KSMAXS:-2 4 8}; do
      CAIN_BGEMM_NTW=$ntw CAIN_BGEMM_WG=$wg CAIN_BGEMM_KSMAX=$ksm timeout -k 10 300 \
        python tools/bench_kernels.py --rows ${ROWS:-32,64} --gemm-only --roles ${ROLES:-qkv,o,gateup,down,lm_head} \
        | sed "s/}\$/, \"ntw\": $ntw, \"wg\": $wg, \"ksmax\": $ksm}/" >> $out || exit $?
    done
  done
done
echo done
