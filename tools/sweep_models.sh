#!/bin/bash
# Trial-batched bench for every study model and requested length (bench.py JSON lines).
# usage: bash tools/sweep_models.sh "<models>" [batch]
set -o pipefail
mkdir -p gpurun_out/models
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
B=${2:-256}
for m in $1; do
  for w in 100 500 1000; do
    timeout -k 10 400 python bench.py --model $m --words $w --batch $B --steps 1 --warmup 1 > gpurun_out/models/${m}_${w}_b$B.log 2>&1 || { tail -5 gpurun_out/models/${m}_${w}_b$B.log; exit 1; }
    echo "$m $w: $(tail -1 gpurun_out/models/${m}_${w}_b$B.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["J_per_token"], r["vs_baseline"], r["vs_baseline_J_per_token"])')"
  done
done
