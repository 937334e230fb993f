#!/usr/bin/env bash
# One session of an MI355X study through the data-parallel fan-out (RCCL at world 1) on one GPU, with the engine
# server on the same GPU as the remote arm.  Sessions are chunked by CAIN_RUN_BUDGET_S (a gpurun call is limited to
# 20 min): the results of earlier sessions travel in the tree under study_resume/ and the runner resumes their TODO
# rows (same seed, same run table).
#
#   STUDY_NAME     run-table name (default full_factorial_r3: round 3's 1,260-run design at a 1 s cooldown)
#   COOLDOWN_MS    rest between runs (round 4: 10000, from profiles/r4/energy/cooldown.json -- the board is back
#                  within 2 % of its idle floor 5-8 s after a 1,000-word on-device run)
#   METHODS        arms (default remote,on_device)
#   REPS           repetitions per (model, arm, length) cell (default 30)
#   IDLE_SETTLE_S  rest before each session's idle baseline (default 5; round 4: 12)
#   SEED           shuffle seed (default 2025; a second replicate of a design uses another seed and name)
#
# usage (inside gpurun): bash tools/study_chunk.sh [budget_s]
set -o pipefail
export TMPDIR=/tmp
NAME="${STUDY_NAME:-full_factorial_r3}"
OUT=gpurun_out/study_${NAME}
mkdir -p "$OUT"
if [ -d "study_resume/$NAME" ] && [ ! -d "$OUT/$NAME" ]; then
  cp -r "study_resume/$NAME" "$OUT/"
fi
export CAIN_STUDY_RESULTS_DIR="$PWD/$OUT" CAIN_STUDY_NAME="$NAME" CAIN_STUDY_REMOTE=local:0 \
       CAIN_STUDY_COOLDOWN_MS="${COOLDOWN_MS:-1000}" CAIN_STUDY_SEED="${SEED:-2025}" CAIN_ASSUME_YES=1 \
       CAIN_STUDY_METHODS="${METHODS:-remote,on_device}" CAIN_STUDY_REPETITIONS="${REPS:-30}" \
       CAIN_STUDY_IDLE_SETTLE_S="${IDLE_SETTLE_S:-5}" CAIN_RUN_BUDGET_S="${1:-960}"
log="$OUT/session_$(date +%s).log"
# provenance: which kernel library this session ran (CAIN_KERNELS_LIB or the in-tree build)
echo "kernels $(md5sum "${CAIN_KERNELS_LIB:-cain_amd/ops/libcain_kernels.so}")" > "$log"
timeout -k 30 1140 python -u -m cain_amd experiments/study.py --gpus 1 --yes >> "$log" 2>&1
rc=$?
grep -c ",DONE," "$OUT/$NAME/run_table.csv" || true
# one archive instead of ~5k per-run files: gpurun merges back at most 2,000 files, and a partial merge once lost
# the run table of two sessions (unpack with: tar xzf gpurun_out/study_<name>/<name>.tgz -C gpurun_out/study_<name>)
tar czf "$OUT/$NAME.tgz" -C "$OUT" "$NAME" && rm -rf "$OUT/$NAME"
exit $rc
