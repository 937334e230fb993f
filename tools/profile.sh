#!/bin/bash
# rocprofv3 kernel-trace + stats of the bench (kernel time breakdown). Usage: ARGS="..." OUT=name bash tools/profile.sh
# Keeps only the stats CSV (the per-dispatch trace of a long generation is tens of MB).
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-prof}
mkdir -p gpurun_out/$OUT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$OUT -o run -- python3 bench.py --no-energy ${ARGS:-} > gpurun_out/$OUT/bench.log 2>&1
rc=$?; tail -3 gpurun_out/$OUT/bench.log
find gpurun_out/$OUT -name "*kernel_trace.csv" -delete
find gpurun_out/$OUT -name "*kernel_stats.csv" | head -1 | xargs -I{} head -25 {}
exit $rc
