set -o pipefail
export TMPDIR=/tmp
tools/gpu_steps.sh r3ae \
 "b128|300|python3 bench.py --batch 128 --steps 2 --warmup 1 --no-single --no-energy" \
 "prof128|300|bash tools/prof_bench.sh r3ae/prof_b128 --batch 128 --steps 1 --warmup 1 --no-single --no-energy"
