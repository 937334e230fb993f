#!/usr/bin/env bash
# round 6 profiles: batch-1 MXFP4 llama3.1:8b and qwen2:1.5b (graph-replayed decode), kernel stats only.
# (The headline profile, profiles/r6/prof/headline_kernel_stats.csv, came from
#  `CAIN_WGEMM_INLINE=0 bash tools/prof_bench.sh r6prof/headline_inl0 --steps 1 --warmup 1 --no-single --no-energy`.)
set -o pipefail
export TMPDIR=/tmp
for m in llama3.1:8b qwen2:1.5b; do
  d=gpurun_out/r6prof/b1_${m/:/_}; mkdir -p $d
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o b1 -- python3 tools/b1_ab.py --models $m --dtype fp4 --trials 1 --label prof > $d/b1.log 2>&1 || exit 1
done
find gpurun_out/r6prof -name "*kernel_trace.csv" -size +20M -delete
