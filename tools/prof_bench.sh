#!/bin/bash
# rocprofv3 kernel trace + per-kernel stats of bench.py -> gpurun_out/<tag>/ (stats CSV kept, trace dropped)
# usage: tools/prof_bench.sh <tag> <bench.py args...>
set -o pipefail
export TMPDIR=/tmp
tag=$1; shift
out=gpurun_out/$tag; mkdir -p $out
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out -o run -- python3 bench.py "$@" > $out/bench.log 2>&1
rc=$?
find $out -name "*kernel_trace.csv" -size +20M -delete
exit $rc
