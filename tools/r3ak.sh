set -o pipefail
export TMPDIR=/tmp
tools/gpu_steps.sh r3ak \
 "prof_w8|300|CAIN_W8_WAVES=8 bash tools/prof_bench.sh r3ak/prof_fp8_w8 --batch 1 --weights fp8 --steps 1 --warmup 1 --no-single --no-energy" \
 "prof_w4|300|CAIN_W8_WAVES=4 bash tools/prof_bench.sh r3ak/prof_fp8_w4 --batch 1 --weights fp8 --steps 1 --warmup 1 --no-single --no-energy"
