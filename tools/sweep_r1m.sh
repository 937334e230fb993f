#!/bin/bash
# Single-stream kernel durations under rocprofv3 (the Python microbench is host-launch-bound at these sizes):
# qwen2:1.5b batch 1 with default knobs, the split-K batched GEMM at 1 row, and attention split counts.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name, env...
  local name=$1; shift
  mkdir -p gpurun_out/$name
  env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/$name -o run -- python3 bench.py --no-energy --batch 1 --model qwen2:1.5b --words 500 --steps 1 --warmup 0 > gpurun_out/$name/bench.log 2>&1 || return 1
  find gpurun_out/$name -name "*kernel_trace.csv" -delete
  python3 - "$name" <<'PY'
import csv, glob, sys
f = glob.glob(f"gpurun_out/{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(sys.argv[1], "total ms", round(tot / 1e6, 2))
for r in rows[:7]:
    print(f"   {r['Name'][:58]:58s} {r['Calls']:>6} {float(r['AverageNs'])/1e3:7.2f} us")
PY
}
run qs_default || exit 1
run qs_bgemm CAIN_BGEMM_MIN_M=0 || exit 1
run qs_ns1 CAIN_ATTN_NSPLIT=1 || exit 1
run qs_ns4 CAIN_ATTN_NSPLIT=4 || exit 1
