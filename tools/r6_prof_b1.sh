#!/usr/bin/env bash
# round 6: batch-1 kernel profiles of the final library (gemma:2b, qwen2:1.5b MXFP4)
set -o pipefail
export TMPDIR=/tmp
for m in gemma:2b qwen2:1.5b; do
  d=gpurun_out/r6prof_final/b1_${m/:/_}; mkdir -p $d
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o b1 -- python3 tools/b1_ab.py \
    --models $m --dtype fp4 --trials 1 --label prof > $d/b1.log 2>&1 || exit 1
done
find gpurun_out/r6prof_final -name "*kernel_trace.csv" -size +20M -delete
