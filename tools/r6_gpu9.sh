#!/usr/bin/env bash
# round 6: batch-1 attention split count with the one-round-trip combine up to 16 splits: cap 8 (the rule) / 12 /
# 16 (>= 3 blocks per split at full context), interleaved on qwen2:1.5b, llama3.1:8b, gemma:2b MXFP4
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r6_splits${TAG:-}; mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k attention \
  > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -1 $out/tests.log
for rep in 1 2; do
  for ns in 8 12 16; do
    CAIN_ATTN_FEW_SPLITS=$ns CAIN_ATTN_MIN_BLOCKS=3 timeout -k 10 400 python -u tools/b1_ab.py \
      --models qwen2:1.5b,llama3.1:8b,gemma:2b --trials 3 --label ns$ns --out $out/b1.jsonl > /dev/null || exit 1
  done
done
cat $out/b1.jsonl
