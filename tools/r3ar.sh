set -o pipefail
export TMPDIR=/tmp
B="python3 bench.py --batch 1 --steps 2 --warmup 1 --no-single --no-energy"
tools/gpu_steps.sh r3ar \
 "l|300|$B" \
 "l4|300|CAIN_SKINNY_W4=1000 $B" \
 "lb|300|$B" \
 "l4b|300|CAIN_SKINNY_W4=1000 $B" \
 "q|300|$B --model qwen2:1.5b" \
 "q4|300|CAIN_SKINNY_W4=1000 $B --model qwen2:1.5b"
