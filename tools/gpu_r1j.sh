#!/bin/bash
# Single-stream (batch 1) profiles: qwen2:1.5b and llama3.1:8b kernel stats; bench lines.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --batch 1 --model qwen2:1.5b --words 500 --steps 2 --warmup 1 > gpurun_out/bench_r1j_qwen_b1.log 2>&1 || exit 1
tail -1 gpurun_out/bench_r1j_qwen_b1.log | cut -c1-160
timeout -k 10 300 python bench.py --batch 1 --words 500 --steps 2 --warmup 1 > gpurun_out/bench_r1j_llama_b1.log 2>&1 || exit 1
tail -1 gpurun_out/bench_r1j_llama_b1.log | cut -c1-160
OUT=prof_r1j_qwen ARGS="--batch 1 --model qwen2:1.5b --words 500 --steps 1 --warmup 0" bash tools/profile.sh > /dev/null || exit 1
python3 - <<'PY'
import csv
rows=list(csv.DictReader(open([l for l in __import__('glob').glob('gpurun_out/prof_r1j_qwen/**/*kernel_stats.csv', recursive=True)][0])))
for r in rows[:12]:
    print(f"{r['Name'][:60]:60s} {r['Calls']:>6} {float(r['AverageNs'])/1e3:8.2f} us {float(r['Percentage']):6.2f}%")
PY
