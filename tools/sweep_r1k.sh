#!/bin/bash
# Single-stream shapes: skinny vs batched (split-K) GEMM at 1 row, attention split count at 1 row.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/sweep_r1k.jsonl
: > $out
for m in qwen2:1.5b llama3.1:8b; do
  timeout -k 10 300 python tools/bench_kernels.py --model $m --norm --rows 1 --gemm-only --waves 0 | sed "s/}\$/, \"env\": \"default\"}/" >> $out || exit 1
  CAIN_BGEMM_MIN_M=0 timeout -k 10 300 python tools/bench_kernels.py --model $m --norm --rows 1 --gemm-only --waves 0 | sed "s/}\$/, \"env\": \"CAIN_BGEMM_MIN_M=0\"}/" >> $out || exit 1
  timeout -k 10 300 python tools/bench_kernels.py --model $m --attn-only --attn "1:333,1:700,1:1400" --attn-splits auto,1,2,4,6,8,12,16 >> $out || exit 1
done
echo done
