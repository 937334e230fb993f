#!/usr/bin/env bash
# round 6: one-round-trip split combine in the decode attention -- attention tests, then batch-1 A/B against the
# previous attention (ab/libcain_kernels_attnbase2.so), interleaved, and a kernel profile
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r6_attn${TAG:-}; mkdir -p $out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k attention \
  tests/test_engine_gpu.py > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
for rep in 1 2; do
  CAIN_KERNELS_LIB=ab/libcain_kernels_attnbase2.so timeout -k 10 400 python -u tools/b1_ab.py \
    --models gemma:2b,llama3.1:8b --trials 3 --label base --out $out/b1.jsonl > /dev/null || exit 1
  timeout -k 10 400 python -u tools/b1_ab.py --models gemma:2b,llama3.1:8b --trials 3 --label new \
    --out $out/b1.jsonl > /dev/null || exit 1
done
cat $out/b1.jsonl
d=$out/prof; mkdir -p $d
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o b1 -- python3 tools/b1_ab.py \
  --models llama3.1:8b --dtype fp4 --trials 1 --label prof > $d/b1.log 2>&1 || exit 1
find $out -name "*kernel_trace.csv" -size +20M -delete
