set -o pipefail
export TMPDIR=/tmp
B="python3 bench.py --batch 1 --steps 2 --warmup 1 --no-single --no-energy"
tools/gpu_steps.sh r3ap \
 "l|300|$B" \
 "l16|300|CAIN_SKINNY_W16=256 $B" \
 "lb|300|$B" \
 "l16b|300|CAIN_SKINNY_W16=256 $B" \
 "prof|300|CAIN_SKINNY_W16=256 bash tools/prof_bench.sh r3ap/prof_b1_llama_w16 --batch 1 --steps 1 --warmup 1 --no-single --no-energy"
