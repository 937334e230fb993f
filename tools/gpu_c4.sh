#!/bin/bash
# Config 4 (seven-model single-stream sweep) with one repetition per cell, no cooldown.
set -o pipefail
mkdir -p gpurun_out/study
export PYTHONUNBUFFERED=1
CAIN_STUDY_REPETITIONS=1 CAIN_STUDY_COOLDOWN_MS=0 CAIN_STUDY_RESULTS_DIR=gpurun_out/study \
  timeout -k 10 1000 python -m cain_amd experiments/c4_seven_model_sweep.py > gpurun_out/study/c4.log 2>&1
rc=$?; tail -5 gpurun_out/study/c4.log; cat gpurun_out/study/c4_seven_model_sweep/analysis/per_model.md 2>/dev/null; exit $rc
