#!/usr/bin/env bash
# round 6: the 8-deep QKV ring (gemm_w4.hip w4_qkv_deep) -- W4 GPU tests, then batch-1 A/B on one box (deep on / off,
# interleaved) on the models whose QKV K > 2,048, and qwen2:1.5b as the unaffected control
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r6_qkvdeep${TAG:-}; mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_w4_gpu.py \
  > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for rep in 1 2; do
  for deep in 0 1; do
    CAIN_W4_QKV_DEEP=$deep timeout -k 10 400 python -u tools/b1_ab.py --models llama3.1:8b,qwen2:7b,gemma:7b,qwen2:1.5b \
      --trials 3 --label deep$deep --out $out/b1.jsonl > /dev/null || exit 1
  done
done
cat $out/b1.jsonl
d=$out/prof; mkdir -p $d
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o b1 -- python3 tools/b1_ab.py \
  --models llama3.1:8b --dtype fp4 --trials 1 --label prof > $d/b1.log 2>&1 || exit 1
find $out -name "*kernel_trace.csv" -size +20M -delete
