#!/bin/bash
# rocprofv3 kernel stats of the headline bench configuration (llama3.1:8b, 300 words (400 tokens), 256 trials/GPU).
set -o pipefail
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out/prof_b256
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_b256 -o run -- python3 bench.py --no-energy --words 300 --steps 1 --warmup 0 > gpurun_out/prof_b256/bench.log 2>&1 || exit 1
find gpurun_out/prof_b256 -name "*kernel_trace.csv" -delete
tail -1 gpurun_out/prof_b256/bench.log | cut -c1-160
cut -c1-70 gpurun_out/prof_b256/run_kernel_stats.csv | head -14
