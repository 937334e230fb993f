#!/usr/bin/env bash
# round 6: the lean chunk-maximum sampler -- GPU tests, phase trace, then batch-1 A/B (sampler mode 2 = two-stage
# kernel at one row, 3 = lean kernel) on llama3.1:8b and qwen2:1.5b fp4, interleaved, then a kernel profile of mode 3
set -o pipefail
export TMPDIR=/tmp
out=gpurun_out/r6_lean${TAG:-}; mkdir -p $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_sample_lean_gpu.py \
  "tests/test_ops_gpu.py::test_sample_chunk_max_matches" > $out/tests.log 2>&1 || { tail -30 $out/tests.log; exit 1; }
tail -2 $out/tests.log
timeout -k 10 200 python -u tools/sample_lean_trace.py > $out/trace.log 2>&1 || { tail $out/trace.log; exit 1; }
grep -v amdgpu.ids $out/trace.log
for mode in 2 3 2 3; do
  timeout -k 10 300 python -u tools/b1_ab.py --models llama3.1:8b,qwen2:1.5b --dtype fp4 --trials 3 --sample-cm $mode \
    --label cm$mode --out $out/b1.jsonl || exit 1
done
d=$out/prof_cm3; mkdir -p $d
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o b1 -- python3 tools/b1_ab.py \
  --models llama3.1:8b --dtype fp4 --trials 1 --sample-cm 3 --label prof > $d/b1.log 2>&1 || exit 1
find $out -name "*kernel_trace.csv" -size +20M -delete
