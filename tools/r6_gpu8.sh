#!/usr/bin/env bash
# round 6: the MXFP4 batch-1 layer chain (gemm_w4.hip w4_chain_kernel) -- its test, then batch-1 A/B chain off / on,
# interleaved, on the chain-eligible models and qwen2:1.5b (not eligible: control), and a kernel profile with it on
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r6_chain${TAG:-}; mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_w4_gpu.py -k "chain" \
  > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for rep in 1 2; do
  for on in 0 1; do
    CAIN_W4_CHAIN=$on timeout -k 10 400 python -u tools/b1_ab.py --models llama3.1:8b,mistral:7b,qwen2:7b,phi3:3.8b,qwen2:1.5b \
      --trials 3 --label chain$on --out $out/b1.jsonl > /dev/null || exit 1
  done
done
cat $out/b1.jsonl
d=$out/prof; mkdir -p $d
CAIN_W4_CHAIN=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o b1 -- python3 tools/b1_ab.py \
  --models llama3.1:8b --dtype fp4 --trials 1 --label prof > $d/b1.log 2>&1 || exit 1
find $out -name "*kernel_trace.csv" -size +20M -delete
