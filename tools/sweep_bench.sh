#!/bin/bash
# Sweep bench.py over trial batch sizes (and request lengths). Each run bounded; stops at first failure.
set -o pipefail
mkdir -p gpurun_out
OUT=gpurun_out/sweep.jsonl
: > $OUT
for words in ${WORDS:-1000}; do
  for b in ${BATCHES:-1 16 32 64}; do
    timeout -k 10 400 python bench.py --steps ${STEPS:-1} --warmup 1 --batch $b --words $words ${EXTRA:-} >> $OUT 2> gpurun_out/sweep_err.log || { tail -20 gpurun_out/sweep_err.log; exit 1; }
    tail -1 $OUT | cut -c1-220
  done
done
