#!/usr/bin/env bash
# One session of the full MI355X study (7 models x 2 arms x 3 lengths x 30 repetitions = 1,260 runs) on one GPU
# through the data-parallel fan-out (RCCL at world 1), with the engine server on the same GPU as the remote arm.
# Sessions are chunked by CAIN_RUN_BUDGET_S (a gpurun call is limited to 20 min): the results of earlier sessions
# travel in the tree under study_resume/ and the runner resumes their TODO rows (same seed, same run table).
# usage (inside gpurun): bash tools/study_chunk.sh [budget_s]
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/study_r3
mkdir -p "$OUT"
if [ -d study_resume/full_factorial_r3 ] && [ ! -d "$OUT/full_factorial_r3" ]; then
  cp -r study_resume/full_factorial_r3 "$OUT/"
fi
export CAIN_STUDY_RESULTS_DIR="$PWD/$OUT" CAIN_STUDY_NAME=full_factorial_r3 CAIN_STUDY_REMOTE=local:0 \
       CAIN_STUDY_COOLDOWN_MS=1000 CAIN_STUDY_SEED=2025 CAIN_ASSUME_YES=1 CAIN_RUN_BUDGET_S="${1:-960}"
timeout -k 30 1140 python -u -m cain_amd experiments/study.py --gpus 1 --yes > "$OUT/session_$(date +%s).log" 2>&1
rc=$?
grep -c ",DONE," "$OUT/full_factorial_r3/run_table.csv" || true
# one archive instead of ~5k per-run files: gpurun merges back at most 2,000 files, and a partial merge once lost
# the run table of two sessions (unpack with: tar xzf gpurun_out/study_r3/full_factorial_r3.tgz -C gpurun_out/study_r3)
tar czf "$OUT/full_factorial_r3.tgz" -C "$OUT" full_factorial_r3 && rm -rf "$OUT/full_factorial_r3"
exit $rc
